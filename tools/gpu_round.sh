# One GPU session: parity tests (+ drift report), bench, rocprofv3 kernel trace and the two
# PMC passes (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in separate passes).
# usage (on the box, via gpurun): bash tools/gpu_round.sh <prefix, e.g. r03_v1>
# (SKIP_HULL=1: without the box/hull-hand bench, profiles and throughput; PART=1: the tests, bench
# and capsule-hand profiles only; PART=2: throughput, PPO, LDL' and hull parts only - two calls
# when one would not fit gpurun's time limit)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=${1:-r01}
SONG=crossing_field
mkdir -p gpurun_out profiles
rm -rf gpurun_out/${P}_trace gpurun_out/${P}_fetch gpurun_out/${P}_write gpurun_out/${P}_sq
if [ "${PART:-all}" != 2 ]; then
PIANOSIM_REPORT=profiles/${P}_drift.json timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
RC=$?
echo "PYTEST_EXIT $RC" >> gpurun_out/pytest_gpu.log
# 0 = green, 1 = a failed assertion; anything else (fault, abort, time limit) ends the call
if [ $RC -gt 1 ]; then exit 9; fi
cp profiles/${P}_drift.json profiles/drift_latest.json 2>/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${P}_trace -- python bench.py --no-cpu-baseline --no-hull-leg --steps 20 > gpurun_out/${P}_trace.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${P}_fetch -- python bench.py --no-cpu-baseline --no-hull-leg --steps 10 > gpurun_out/${P}_fetch.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${P}_write -- python bench.py --no-cpu-baseline --no-hull-leg --steps 10 > gpurun_out/${P}_write.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/${P}_sq -- python bench.py --no-cpu-baseline --no-hull-leg --steps 10 > gpurun_out/${P}_sq.log 2>&1 || exit 7
python tools/collect_pmc.py gpurun_out/${P}_trace gpurun_out/${P}_fetch gpurun_out/${P}_write 4096 $SONG $P 5 gpurun_out/${P}_sq > gpurun_out/pmc.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
cp gpurun_out/bench.json profiles/${P}_bench.json
# per-phase cycle split from the -DPS_TIMING build (built on the CPU side beforehand)
if [ -f diffusion-piano_amd/libpianosim_timing.so ]; then
  (echo "# tools/phase_timing.py 4096 crossing_field (PIANOSIM_LIB=libpianosim_timing.so, -DPS_TIMING), MI355X, random actions";
   PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so timeout -k 10 120 python tools/phase_timing.py 4096 crossing_field) > profiles/${P}_phase_timing.txt 2>/dev/null || exit 5
fi
if [ -f diffusion-piano_amd/libpianosim_timing.so ]; then
  PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so timeout -k 10 120 python tools/tail_timing.py 1024 twinkle > profiles/${P}_tail_1024.txt 2>/dev/null || exit 5
fi
fi
if [ "${PART:-all}" != 1 ]; then
timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 16384 > profiles/${P}_throughput.txt 2>/dev/null || exit 6
timeout -k 10 200 python tools/throughput.py twinkle 1024 4096 >> profiles/${P}_throughput.txt 2>/dev/null || exit 6
timeout -k 10 200 python tools/ppo_bench.py --mode reference --iters 3 --warmup 2 > profiles/${P}_ppo_bench.jsonl 2>/dev/null || exit 8
# the PPO loop's kernels (TunableOp off: no GEMM tuning launches in the trace)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${P}_ppo_trace -- python tools/ppo_bench.py --mode reference --iters 2 --warmup 1 --no-tune > gpurun_out/${P}_ppo_trace.log 2>&1 || exit 8
find gpurun_out/${P}_ppo_trace -name "*kernel_stats.csv" -exec cp {} profiles/${P}_ppo_kernel_stats.csv \;
# the coupled-block LDL' on the matrix cores against the register method (tools/ldl_bench.hip)
if [ -f tools/libldlbench.so ]; then
  timeout -k 10 120 python tools/ldl_bench.py > profiles/${P}_ldl_bench.jsonl 2>/dev/null || exit 8
fi
# the reference's default collider kinds (palm boxes, hull fingertips): pianosim_kernel<true>
if [ -z "$SKIP_HULL" ]; then
  H=${P}_hull
  timeout -k 10 300 python bench.py --hand hull --no-cpu-baseline > profiles/${H}_bench.json 2> gpurun_out/${H}_bench.err || exit 10
  export PIANOSIM_HULL=1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${H}_trace -- python bench.py --hand hull --no-cpu-baseline --steps 20 > gpurun_out/${H}_trace.log 2>&1 || exit 11
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${H}_fetch -- python bench.py --hand hull --no-cpu-baseline --steps 10 > gpurun_out/${H}_fetch.log 2>&1 || exit 12
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${H}_write -- python bench.py --hand hull --no-cpu-baseline --steps 10 > gpurun_out/${H}_write.log 2>&1 || exit 13
  python tools/collect_pmc.py gpurun_out/${H}_trace gpurun_out/${H}_fetch gpurun_out/${H}_write 4096 $SONG $H 5 > gpurun_out/pmc_hull.log 2>&1
  if [ -f diffusion-piano_amd/libpianosim_timing.so ]; then
    (echo "# PIANOSIM_HULL=1 tools/phase_timing.py 4096 crossing_field (box/hull hand, -DPS_TIMING), MI355X, random actions";
     PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so timeout -k 10 120 python tools/phase_timing.py 4096 crossing_field) > profiles/${H}_phase_timing.txt 2>/dev/null || exit 14
  fi
  timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 16384 > profiles/${H}_throughput.txt 2>/dev/null || exit 15
  unset PIANOSIM_HULL
fi
fi
rm -rf gpurun_out/profiles_new && cp -r profiles gpurun_out/profiles_new
echo DONE
