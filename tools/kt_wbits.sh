#!/bin/bash
# kernel trace of single 2^17 batches at both window widths (KZGMI_WBITS=16 / 13)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for w in 16 13; do
  OUT=$R/gpurun_out/kt_w$w; mkdir -p $OUT
  KZGMI_WBITS=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o kt -- python3 $R/tools/phase_timing.py --reps 4 --n 131072 > $OUT/run.log 2>&1 || { tail -20 $OUT/run.log; exit 1; }
  python3 - $OUT $w <<'P'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:14]:
    if 'gen_' in r['Name'] or 'lines' in r['Name'] or 'g2_mul' in r['Name']: continue
    print('w=' + sys.argv[2], r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
P
done
