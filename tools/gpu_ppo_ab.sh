# Development aid: PPO GPU tests, then the reference-schedule loop with the fused grad-norm
# partials (default) and with the separate norm pass (PIANORL_SUMSQ=1); the returns kernel test
# and the bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_returns.py -q -x -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_ppo.log 2>&1 || { tail -40 gpurun_out/pytest_ppo.log; exit 9; }
tail -2 gpurun_out/pytest_ppo.log
for v in fused sumsq; do
  unset PIANORL_SUMSQ
  if [ $v = sumsq ]; then export PIANORL_SUMSQ=1; fi
  timeout -k 10 200 python tools/ppo_bench.py --mode reference --iters 5 --warmup 2 > gpurun_out/ppo_$v.jsonl 2> gpurun_out/ppo_$v.err || exit 3
  python -c "
import json
d=json.loads(open('gpurun_out/ppo_$v.jsonl').read().strip().splitlines()[-1]); print('$v', round(d['value']), d.get('minibatch_step_ms'))
"
done
unset PIANORL_SUMSQ
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || exit 4
python -c "
import json
d=json.loads(open('gpurun_out/bench_ab.json').read().strip().splitlines()[-1]); print('bench', round(d['value']), d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['config']['hull_hand']['value'])
"
