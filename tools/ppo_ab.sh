# PPO minibatch step: GPU tests, then the reference-schedule loop with the fused MFMA step and
# without it (PIANORL_NO_MFMA=1), one box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_ppo_dp.py -q -x -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_ppo.log 2>&1
RC=$?
tail -3 gpurun_out/pytest_ppo.log
if [ $RC -gt 1 ]; then exit 9; fi
timeout -k 10 200 python tools/ppo_bench.py --mode reference --iters 3 --warmup 2 > gpurun_out/ppo_mfma.jsonl 2> gpurun_out/ppo_mfma.err || exit 3
PIANORL_NO_MFMA=1 timeout -k 10 200 python tools/ppo_bench.py --mode reference --iters 3 --warmup 2 > gpurun_out/ppo_nomfma.jsonl 2> gpurun_out/ppo_nomfma.err || exit 4
python -c "
import json
for f in ('gpurun_out/ppo_mfma.jsonl','gpurun_out/ppo_nomfma.jsonl'):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, round(d['value']), d.get('minibatch_step_ms'), d.get('phases_ms'))
"
timeout -k 10 120 python tools/mlp_timing.py > gpurun_out/mlp_timing.txt 2>&1 || exit 5
cat gpurun_out/mlp_timing.txt
cd /tmp && export TMPDIR=/tmp
PIANORL_LIB=$GRAFT_REPO_ROOT/diffusion-piano_amd/libpianorl.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_ppo -o ppo -- python3 $GRAFT_REPO_ROOT/tools/mlp_timing.py > $GRAFT_REPO_ROOT/gpurun_out/prof_ppo.log 2>&1 || exit 6
find $GRAFT_REPO_ROOT/gpurun_out/prof_ppo -name "*kernel_stats.csv" -exec head -12 {} \;
