# PPO column-split rows kernel session: the PPO GPU tests, per-phase stamps of both rows
# kernels (tools/mlp_timing.py), the reference-schedule loop with each (reference default
# colliders; the split one also with the all-capsule hand), the split loop's kernel trace.
# usage (on the box, via gpurun): bash tools/gpu_ppo_split.sh <prefix>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=${1:-ppo}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${P}_tests.log 2>&1
RC=$?
echo "PYTEST_EXIT $RC" >> gpurun_out/${P}_tests.log
if [ $RC -ne 0 ]; then tail -40 gpurun_out/${P}_tests.log; exit 1; fi
timeout -k 10 120 python tools/mlp_timing.py > gpurun_out/${P}_mlp_timing_split.txt 2>&1 || exit 2
PIANORL_MLP_SPLIT=0 timeout -k 10 120 python tools/mlp_timing.py > gpurun_out/${P}_mlp_timing_tile.txt 2>&1 || exit 3
timeout -k 10 200 python tools/ppo_bench.py --mode reference --iters 3 --warmup 2 > gpurun_out/${P}_ppo_split.jsonl 2>/dev/null || exit 4
timeout -k 10 200 python tools/ppo_bench.py --mode reference --iters 3 --warmup 2 --hand authored >> gpurun_out/${P}_ppo_split.jsonl 2>/dev/null || exit 4
PIANORL_MLP_SPLIT=0 timeout -k 10 200 python tools/ppo_bench.py --mode reference --iters 3 --warmup 2 > gpurun_out/${P}_ppo_tile.jsonl 2>/dev/null || exit 5
rm -rf gpurun_out/${P}_ppo_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${P}_ppo_trace -- python tools/ppo_bench.py --mode reference --iters 2 --warmup 1 --no-tune > gpurun_out/${P}_ppo_trace.log 2>&1 || exit 6
find gpurun_out/${P}_ppo_trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/${P}_ppo_kernel_stats.csv \;
cat gpurun_out/${P}_mlp_timing_split.txt
echo DONE
