# kernel trace of the reference-schedule PPO loop (fused MFMA minibatch step)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/ppo_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ppo_trace -- python tools/ppo_bench.py --mode reference --iters 2 --warmup 1 > gpurun_out/ppo_trace.log 2>&1 || exit 2
f=$(find gpurun_out/ppo_trace -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1000, 1), "us avg", round(float(r["TotalDurationNs"]) / 1e6, 2), "ms")
PY
