set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof/hot_r05n -o run -- python3 scripts/hot_receiver_bench.py > gpurun_out/hot_r05n.jsonl 2>&1 || exit $?
python3 - <<'PY'
import csv, glob
rows=[]
for f in glob.glob("gpurun_out/prof/hot_r05n/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
rows.sort()
t0=rows[0][0]
for s,e,n in rows:
    if any(k in n for k in ("k_step","k_hot","k_carry","k_spill","k_zone","k_inject","k_pending","k_fold","k_sparse")):
        print(f"{(s-t0)/1e3:10.1f} {(e-s)/1e3:8.2f} us  {n}")
PY
