"""Summarise tools/kt_single.sh (rocprofv3 --kernel-trace --stats of non-pipelined single
batches, tools/phase_timing.py) into profiles/<round>/rocprof_single/: the stats CSV, a top
list, and kernel_single.json with the average k_accumulate + k_fixup duration that bench.py's
roofline.kernel_ms (single-batch HIP events around the same two kernels) must agree with.

python3 tools/summarize_single.py gpurun_out/kt_single profiles/r01/rocprof_single
"""
import csv
import glob
import json
import os
import shutil
import sys

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(dst, exist_ok=True)
stats = glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True)[0]
shutil.copy(stats, os.path.join(dst, "kernel_stats_single_batch.csv"))
rows = sorted(csv.DictReader(open(stats)), key=lambda r: -float(r["TotalDurationNs"]))
with open(os.path.join(dst, "kernel_stats_top.txt"), "w") as f:
    f.write("# rocprofv3 --kernel-trace --stats -- python3 tools/phase_timing.py --reps 4 (n = 2^20 BLS12-381,\n"
            "# one batch at a time: per-kernel durations without pipeline time-sharing)\n")
    f.write("%-70s %8s %14s\n" % ("kernel", "calls", "avg_us"))
    for r in rows[:24]:
        f.write("%-70s %8s %14.1f\n" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))


def avg_ns(prefix):
    hit = [r for r in rows if r["Name"].startswith(prefix)]
    return float(hit[0]["AverageNs"]) if hit else 0.0


acc = avg_ns("void kzgmi::k_accumulate<kzgmi::Bls12_381>")
fix = avg_ns("void kzgmi::k_fixup<kzgmi::Bls12_381>")
out = {"command": "rocprofv3 --kernel-trace --stats -- python3 tools/phase_timing.py --reps 4 (n = 2^20)",
       "k_accumulate_avg_ms": acc / 1e6, "k_fixup_avg_ms": fix / 1e6, "accumulate_phase_avg_ms": (acc + fix) / 1e6}
json.dump(out, open(os.path.join(dst, "kernel_single.json"), "w"), indent=1)
print(json.dumps(out))
