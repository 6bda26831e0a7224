cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt28" -o run -- python3 "$R/tools/phase_timing.py" --reps 2 > "$R/gpurun_out/kt28.log" 2>&1 || { tail -20 "$R/gpurun_out/kt28.log"; exit 1; }
python3 - <<'PY'
import csv, os
R = os.environ["GRAFT_REPO_ROOT"]
import glob
f = glob.glob(R + "/gpurun_out/kt28/**/*kernel_stats*", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:60], r["Calls"], r["AverageNs"])
PY
