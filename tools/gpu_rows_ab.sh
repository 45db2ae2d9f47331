# Development aid: PPO minibatch step A/B (fused gather vs PIANORL_GATHER=1): PPO GPU tests, the
# reference-schedule loop, the rows kernel's phase stamps and a kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py -q -x -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_ppo.log 2>&1 || { tail -40 gpurun_out/pytest_ppo.log; exit 9; }
tail -2 gpurun_out/pytest_ppo.log
for v in fused gather; do
  unset PIANORL_GATHER
  if [ $v = gather ]; then export PIANORL_GATHER=1; fi
  timeout -k 10 200 python tools/ppo_bench.py --mode reference --iters 5 --warmup 2 > gpurun_out/ppo_$v.jsonl 2> gpurun_out/ppo_$v.err || exit 3
  python -c "
import json
d=json.loads(open('gpurun_out/ppo_$v.jsonl').read().strip().splitlines()[-1]); print('$v', round(d['value']), d.get('minibatch_step_ms'), d.get('phases_ms'))
"
done
unset PIANORL_GATHER
timeout -k 10 120 python tools/mlp_timing.py > gpurun_out/mlp_timing.txt 2>&1 || exit 5
grep -v amdgpu.ids gpurun_out/mlp_timing.txt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_rows -o ppo -- python3 $GRAFT_REPO_ROOT/tools/ppo_bench.py --mode reference --iters 2 --warmup 1 --no-tune > $GRAFT_REPO_ROOT/gpurun_out/prof_rows.log 2>&1 || exit 6
find $GRAFT_REPO_ROOT/gpurun_out/prof_rows -name "*kernel_stats.csv" -exec cat {} \; | grep -v Cijk | cut -c1-150 | head -14
