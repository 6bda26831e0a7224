"""Summarise tools/prof.sh valu (SQ_INSTS_VALU / SQ_INSTS_SALU / SQ_WAVES of every kernel of
single batches) into the per-batch VALU issue budget: for each kernel the wave-instructions per
batch and the whole-chip issue time they cost at the measured issue rate -- what a kernel takes
from the pipelined step when every slot's kernels share the CUs.

python3 tools/summarize_valu.py gpurun_out/prof_valu profiles/r04/pmc_valu_per_batch.json [step_ms]
"""
import collections
import csv
import glob
import json
import os
import sys

ISSUE_NS = 1 / 0.4474  # ns per wave-instruction per SIMD (profiles/r02/probes/mad_rate_blocks.txt, 4 waves/SIMD)
SIMDS = 1024

src, dst = sys.argv[1], sys.argv[2]
step_ms = float(sys.argv[3]) if len(sys.argv) > 3 else None
per = collections.defaultdict(lambda: collections.defaultdict(float))  # kernel -> counter -> sum
disp = collections.defaultdict(set)
for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((f, r["Dispatch_Id"]))
acc = [k for k in per if k.startswith("kzgmi::k_accumulate")]
if not acc:
    sys.exit("no k_accumulate dispatch in %s" % src)
batches = len(disp[acc[0]])  # one accumulation launch per batch
rows = {}
for k, cs in per.items():
    valu = cs.get("SQ_INSTS_VALU", 0.0) / batches
    rows[k] = {"launches_per_batch": len(disp[k]) / batches, "valu_wave_instr_per_batch": valu,
               "salu_wave_instr_per_batch": cs.get("SQ_INSTS_SALU", 0.0) / batches,
               "waves_per_batch": cs.get("SQ_WAVES", 0.0) / batches,
               "whole_chip_issue_ms": valu * ISSUE_NS / SIMDS / 1e6}
rows = dict(sorted(rows.items(), key=lambda kv: -kv[1]["valu_wave_instr_per_batch"]))
SETUP = ("k_gen_tuples", "k_gen_table", "k_precompute_lines", "k_g2_mul", "k_convert_g2", "k_set_generator",
         "k_probe")  # once per run (test data, SRS), not per batch
for k, r in rows.items():
    r["per_batch"] = not any(t in k for t in SETUP) and r["launches_per_batch"] >= 0.99
total = sum(r["whole_chip_issue_ms"] for r in rows.values() if r["per_batch"])
out = {"command": "tools/prof.sh valu: rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -- python3 "
                  "tools/phase_timing.py --reps 2 (n = 2^20 BLS12-381, single batches)",
       "batches": batches, "issue_ns_per_wave_instr_per_simd": ISSUE_NS, "simds": SIMDS,
       "total_whole_chip_issue_ms_per_batch": total, "kernels": rows,
       "note": "whole_chip_issue_ms = VALU wave-instructions per batch x the measured issue time per "
               "wave-instruction / 1024 SIMDs: the time the batch's VALU work occupies the whole chip "
               "when the pipeline keeps every SIMD busy (the pipelined step's floor); setup kernels "
               "(tuple generation, line precomputation) run once per run, not per batch"}
if step_ms:
    out["pipelined_step_ms"] = step_ms
    out["issue_frac_of_step"] = total / step_ms
json.dump(out, open(dst, "w"), indent=1)
for k, r in list(rows.items())[:12]:
    print("%-60s %8.3f ms  %.2f launches" % (k[:60], r["whole_chip_issue_ms"], r["launches_per_batch"]))
print("total %.3f ms per batch" % total)
