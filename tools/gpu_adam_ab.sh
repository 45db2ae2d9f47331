# Development aid: PPO loop A/B over libpianorl builds (args: lib file names in
# diffusion-piano_amd/), the PPO GPU tests on the default build first, and each build's kernel
# trace (the clip+Adam kernel's average).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py -q -x -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_ppo.log 2>&1 || { tail -40 gpurun_out/pytest_ppo.log; exit 9; }
tail -2 gpurun_out/pytest_ppo.log
for L in "$@"; do
  PIANORL_LIB=diffusion-piano_amd/$L timeout -k 10 200 python tools/ppo_bench.py --mode reference --iters 5 --warmup 2 > gpurun_out/ppoab_$L.jsonl 2> gpurun_out/ppoab_$L.err || exit 3
  python -c "
import json
d=json.loads(open('gpurun_out/ppoab_$L.jsonl').read().strip().splitlines()[-1]); print('$L', round(d['value']), d.get('minibatch_step_ms'))
"
  rm -rf gpurun_out/ppoab_tr_$L
  PIANORL_LIB=diffusion-piano_amd/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ppoab_tr_$L -- python tools/ppo_bench.py --mode reference --iters 2 --warmup 1 --no-tune > gpurun_out/ppoab_tr_$L.log 2>&1 || exit 4
  python -c "
import csv,glob
f=glob.glob('gpurun_out/ppoab_tr_$L/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'adam' in r['Name'] or 'mlp_' in r['Name']: print('  $L', r['Calls'], r['AverageNs'], r['Name'][:60])
"
done
