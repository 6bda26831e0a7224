"""Summarise tools/prof.sh pipelined output into profiles/<round>/rocprof/:
kernel_stats.csv (rocprofv3 --stats), kernel_stats_top.txt and pmc_accumulate_pipelined.json (per-launch
HBM traffic of k_accumulate: FETCH_SIZE x 2 per MI355X_MICROARCH.md 'HBM' (gfx950 tallies
128-B read requests at 64 B) + WRITE_SIZE; FETCH/WRITE_SIZE are in KiB)."""
import csv
import glob
import json
import os
import shutil
import sys

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(dst, exist_ok=True)
stats = glob.glob(os.path.join(src, "kt", "**", "*kernel_stats.csv"), recursive=True)[0]
shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
rows = sorted(csv.DictReader(open(stats)), key=lambda r: -float(r["TotalDurationNs"]))
with open(os.path.join(dst, "kernel_stats_top.txt"), "w") as f:
    f.write("%-70s %8s %14s %8s\n" % ("kernel", "calls", "avg_us", "pct"))
    for r in rows[:16]:
        f.write("%-70s %8s %14.1f %8s\n" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3,
                                          r.get("Percentage", "")))


def per_launch(kind):
    f = glob.glob(os.path.join(src, kind, "**", "*counter_collection.csv"), recursive=True)[0]
    vals = {}
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("void kzgmi::k_accumulate<"):
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


fetch, write = per_launch("fetch"), per_launch("write")
fetch_kib = sum(fetch) / len(fetch)
write_kib = sum(write) / len(write)
acc = [r for r in rows if r["Name"].startswith("void kzgmi::k_accumulate<kzgmi::Bls12_381>")][0]
out = {
    "kernel": "k_accumulate<Bls12_381>",
    "command": "bench.py --steps 24 --warmup 8 --no-cpu --msm-steps 0 --fs-steps 0 --compressed-steps 0 --trusted-steps 0 --commit-steps 0 (n = 2^20)",
    "launches_fetch": len(fetch), "launches_write": len(write),
    "FETCH_SIZE_KiB_per_launch_raw": fetch_kib,
    "WRITE_SIZE_KiB_per_launch": write_kib,
    "traffic_bytes_per_launch": (2 * fetch_kib + write_kib) * 1024,
    "correction": "FETCH_SIZE x 2 (gfx950 counts 128-B read requests at 64 B, MI355X_MICROARCH.md HBM); "
                  "the kernel's 16-B-per-lane loads are gathers, not streams: absolute is approximate",
    "rocprof_avg_duration_ns": float(acc["AverageNs"]),
    "algorithmic_bytes_per_launch": 256 * (1 << 20),
}
out["note"] = ("pipelined run: 16 batches share the chip, so durations include queueing and the counters "
               "include concurrently running kernels; the judged per-launch traffic is the single-batch "
               "profiles/r01/rocprof_single/pmc_accumulate_single.json")
json.dump(out, open(os.path.join(dst, "pmc_accumulate_pipelined.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
