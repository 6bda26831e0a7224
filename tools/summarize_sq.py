"""Summarise tools/prof.sh sq (SQ counters of k_accumulate on single batches) into
profiles/<round>/pmc_sq_accumulate.json: per-launch averages and the per-addition VALU count.

python3 tools/summarize_sq.py gpurun_out/prof_sq profiles/r06/pmc_sq_accumulate.json [n] [Bn254]
"""
import collections
import csv
import glob
import json
import os
import sys

src, dst = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20
CV = sys.argv[4] if len(sys.argv) > 4 else "Bls12_381"  # Bn254: 32 n window terms as well (GLV halves)
per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
    acc = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"].split("(")[0].replace("void ", ""), r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, _, c), v in acc.items():
        per[k][c].append(v)
out = {"command": "tools/prof.sh sq: rocprofv3 --pmc <SQ counters> | FETCH_SIZE | WRITE_SIZE (separate passes, "
                  "--kernel-include-regex) -- python3 tools/phase_timing.py --reps 2 (n = %d %s, single batches)" % (n, CV),
       "per_launch": {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}}
acc = out["per_launch"].get("kzgmi::k_accumulate<kzgmi::%s>" % CV)
if acc and "SQ_INSTS_VALU" in acc:
    wc = acc["SQ_WAVE_CYCLES"]
    out["k_accumulate"] = {
        "valu_instructions_per_mixed_addition": acc["SQ_INSTS_VALU"] * 64 / (32 * n),
        "waves": acc["SQ_WAVES"],
        "wave_cycle_split": {"active_valu": acc["SQ_ACTIVE_INST_VALU"] / wc,
                             "issue_stall (SQ_WAIT_INST_ANY)": acc["SQ_WAIT_INST_ANY"] / wc,
                             "parked on waitcnt/barrier (SQ_WAIT_ANY)": acc["SQ_WAIT_ANY"] / wc},
        "note": "SQ_INSTS_VALU counts wave-instructions: x 64 lanes / 32 n additions = per-addition VALU count " +
                ("(3544 of them v_mad_u64_u32: 8 radix-29 products x 392 + 2 squarings x 301 - 196 saved by the Y3 pair's "
                 "shared reduction). " if CV == "Bls12_381" else "(9-limb radix-2^29 products: 162 mads each). ") + "Wait counters "
                "overlap across the 4 waves per SIMD (a parked wave's SIMD issues for the others)."}
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out.get("k_accumulate"), indent=1))
