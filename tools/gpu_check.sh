# GPU suite + quick A/B throughput of a variant library + PPO loop (development aid).
# usage (on the box, via gpurun): bash tools/gpu_check.sh [variant .so under diffusion-piano_amd/]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_all.log 2>&1
RC=$?
echo "EXIT $RC" >> gpurun_out/pytest_all.log
grep -E "passed|failed|^FAILED|^E  .*(Error|assert)" gpurun_out/pytest_all.log | tail -20
if [ $RC -gt 1 ]; then exit 9; fi
timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 > gpurun_out/tp_base.txt 2>&1 || exit 6
cat gpurun_out/tp_base.txt
if [ -n "$1" ]; then
  PIANOSIM_LIB=diffusion-piano_amd/$1 timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 > gpurun_out/tp_var.txt 2>&1 || exit 7
  cat gpurun_out/tp_var.txt
fi
timeout -k 10 200 python tools/ppo_bench.py --mode reference --iters 3 --warmup 2 > gpurun_out/ppo.jsonl 2> gpurun_out/ppo.err || exit 8
tail -1 gpurun_out/ppo.jsonl | cut -c1-300
