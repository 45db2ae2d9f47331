# Development aid: kernel trace of the reference-schedule PPO loop (TunableOp off, so no tuning
# kernels in the trace)
set -o pipefail
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_rows -o ppo -- python3 $GRAFT_REPO_ROOT/tools/ppo_bench.py --mode reference --iters 2 --warmup 1 --no-tune > $GRAFT_REPO_ROOT/gpurun_out/prof_rows.log 2>&1 || exit 6
find $GRAFT_REPO_ROOT/gpurun_out/prof_rows -name "*kernel_stats.csv" | head -1 > /tmp/ks.txt
cut -c1-160 $(cat /tmp/ks.txt) | grep -v Cijk | head -14
