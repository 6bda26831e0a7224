"""Summarise tools/prof.sh kernel (rocprofv3 --kernel-trace --stats of non-pipelined single
batches, tools/phase_timing.py) into profiles/<round>/rocprof_single/: the stats CSV, a top
list, and kernel_single.json with the average k_accumulate + k_fixup + k_fixup_crowded duration that bench.py's
roofline.kernel_ms (single-batch HIP events around the same two kernels) must agree with.

python3 tools/summarize_single.py gpurun_out/prof_single profiles/r06/rocprof_single [Bn254 "n = 2^22"]
"""
import csv
import glob
import json
import os
import shutil
import sys

src, dst = sys.argv[1], sys.argv[2]
CV = sys.argv[3] if len(sys.argv) > 3 else "Bls12_381"  # Bn254 for a BN254 trace
LABEL = sys.argv[4] if len(sys.argv) > 4 else "n = 2^20"
os.makedirs(dst, exist_ok=True)
stats = sorted(glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True))[0]
shutil.copy(stats, os.path.join(dst, "kernel_stats_single_batch.csv"))
rows = sorted(csv.DictReader(open(stats)), key=lambda r: -float(r["TotalDurationNs"]))
with open(os.path.join(dst, "kernel_stats_top.txt"), "w") as f:
    f.write("# rocprofv3 --kernel-trace --stats -- python3 tools/phase_timing.py --reps 4 (%s %s,\n" % (LABEL, CV))
    f.write("# one batch at a time: per-kernel durations without pipeline time-sharing)\n")
    f.write("%-70s %8s %14s\n" % ("kernel", "calls", "avg_us"))
    for r in rows[:24]:
        f.write("%-70s %8s %14.1f\n" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))


def avg_ns(prefix):
    hit = [r for r in rows if r["Name"].startswith(prefix)]
    return float(hit[0]["AverageNs"]) if hit else 0.0


acc = avg_ns("void kzgmi::k_accumulate<kzgmi::%s>" % CV)
fix = avg_ns("void kzgmi::k_fixup<kzgmi::%s>" % CV)
# the crowded-bucket joins (msm.hpp k_fixup_crowded, launched behind every k_fixup since round 5)
crowd = avg_ns("void kzgmi::k_fixup_crowded<kzgmi::%s>" % CV)
f29 = avg_ns("void kzgmi::k_from29<kzgmi::%s>" % CV)  # builds before the records fed the reduction directly
out = {"command": "rocprofv3 --kernel-trace --stats -- python3 tools/phase_timing.py --reps 4 (%s, %s)" % (CV, LABEL),
       "k_accumulate_avg_ms": acc / 1e6, "k_fixup_avg_ms": fix / 1e6, "k_fixup_crowded_avg_ms": crowd / 1e6,
       **({"k_from29_avg_ms": f29 / 1e6} if f29 else {}),
       "accumulate_phase_avg_ms": (acc + f29 + fix + crowd) / 1e6,
       "accumulate_phase": "k_accumulate + k_fixup + k_fixup_crowded: the kernels between the accumulate "
                           "phase's two HIP events in csrc/api.hip (bench.py roofline.kernel_ms)"}
json.dump(out, open(os.path.join(dst, "kernel_single.json"), "w"), indent=1)
print(json.dumps(out))


# ---- PMC passes of tools/prof.sh kernel / traffic (absent for the plain kt_single.sh trace)
def per_launch(kind, counter=None):
    files = glob.glob(os.path.join(src, kind, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        return None
    vals = {}
    for r in csv.DictReader(open(files[0])):
        if r["Kernel_Name"].startswith("void kzgmi::k_accumulate<kzgmi::Bls12_381>") and \
                (counter is None or r["Counter_Name"] == counter):
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


fetch, write = per_launch("fetch_size"), per_launch("write_size")
if fetch and write:
    n = 1 << 20
    entries = 32 * n  # window terms of one batch
    fetch_kib, write_kib = sum(fetch) / len(fetch), sum(write) / len(write)
    hit, miss = per_launch("tcc_hit_sum", "TCC_HIT_sum"), per_launch("tcc_hit_sum", "TCC_MISS_sum")
    pmc = {
        "kernel": "k_accumulate<Bls12_381>",
        "command": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE | TCC_HIT_sum TCC_MISS_sum (separate passes) "
                   "-- python3 tools/phase_timing.py --reps 2 (n = 2^20, single batches)",
        "launches_fetch": len(fetch), "launches_write": len(write),
        "FETCH_SIZE_KiB_per_launch_raw": fetch_kib,
        "WRITE_SIZE_KiB_per_launch": write_kib,
        "traffic_bytes_per_launch": (2 * fetch_kib + write_kib) * 1024,
        "traffic_bytes_per_launch_raw": (fetch_kib + write_kib) * 1024,
        "correction": "FETCH_SIZE x 2 + WRITE_SIZE, as MI355X_MICROARCH.md's HBM section prescribes (gfx950 "
                      "tallies 128-B requests at 64 B); calibrated in our own 16-B-per-lane access pattern: "
                      "k_pts_to29 reads 268.4 MB of 128-B point slots and FETCH_SIZE reports 142.5 MB (x1.88, "
                      "profiles/r02/pmc_sq_accumulate.json).  Infinity-Cache hits are counted, so this is "
                      "L2-miss traffic, an upper bound on HBM bytes",
        "algorithmic_bytes_per_launch": 256 * n,
        "gather_model_bytes_per_launch": entries * (112 + 4),
        "gather_model": "every window term gathers its 112-B radix-2^29 affine point (x, y: 2 x 14 words "
                        "of a 128-B slot) and streams its 4-B sorted value (32 terms per tuple): the traffic "
                        "Pippenger accumulation touches by construction",
        "tcc_hit_rate": (sum(hit) / (sum(hit) + sum(miss))) if hit and miss else None,
        "k_accumulate_avg_ms": acc / 1e6,
    }
    json.dump(pmc, open(os.path.join(dst, "pmc_accumulate_single.json"), "w"), indent=1)
    print(json.dumps(pmc, indent=1))
