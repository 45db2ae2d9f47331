# One GPU session: parity tests (+ drift report), bench, rocprofv3 kernel trace and the PMC
# passes (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in separate passes) of the bench's
# default workload (the reference's default colliders: palm boxes + hull fingertips).
# usage (on the box, via gpurun): bash tools/gpu_round.sh <prefix, e.g. r05_v1>
# PART=1: the tests, bench and the headline's profiles; PART=2: throughput per collider set,
# phase / tail timing, PPO and LDL' parts (two calls when one would not fit gpurun's limit);
# NOTEST=1: PART 1 without the GPU test suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=${1:-r05}
SONG=crossing_field
mkdir -p gpurun_out profiles
rm -rf gpurun_out/${P}_trace gpurun_out/${P}_fetch gpurun_out/${P}_write gpurun_out/${P}_sq gpurun_out/${P}_cap_trace
if [ "${PART:-all}" != 2 ]; then
if [ -z "$NOTEST" ]; then
PIANOSIM_REPORT=profiles/${P}_drift.json timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
RC=$?
echo "PYTEST_EXIT $RC" >> gpurun_out/pytest_gpu.log
cp gpurun_out/pytest_gpu.log profiles/${P}_pytest_gpu.log
# 0 = green, 1 = a failed assertion; anything else (fault, abort, time limit) ends the call
if [ $RC -gt 1 ]; then exit 9; fi
cp profiles/${P}_drift.json profiles/drift_latest.json 2>/dev/null
fi
B="python bench.py --no-cpu-baseline --no-legs"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${P}_trace -- $B --steps 20 > gpurun_out/${P}_trace.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${P}_fetch -- $B --steps 10 > gpurun_out/${P}_fetch.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${P}_write -- $B --steps 10 > gpurun_out/${P}_write.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/${P}_sq -- $B --steps 10 > gpurun_out/${P}_sq.log 2>&1 || exit 7
PIANOSIM_HAND=hull python tools/collect_pmc.py gpurun_out/${P}_trace gpurun_out/${P}_fetch gpurun_out/${P}_write 4096 $SONG $P 5 gpurun_out/${P}_sq > gpurun_out/pmc.log 2>&1
# the all-capsule hand's kernel trace (its own instantiation) for the record
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${P}_cap_trace -- $B --hand authored --steps 20 > gpurun_out/${P}_cap_trace.log 2>&1 || exit 2
find gpurun_out/${P}_cap_trace -name "*kernel_stats.csv" -exec cp {} profiles/${P}_capsule_kernel_stats.csv \;
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
cp gpurun_out/bench.json profiles/${P}_bench.json
fi
if [ "${PART:-all}" != 1 ]; then
# per-phase cycle split from the -DPS_TIMING build (built on the CPU side beforehand)
for H in hull authored; do
  (echo "# PIANOSIM_HAND=$H tools/phase_timing.py 4096 crossing_field (PIANOSIM_LIB=libpianosim_timing.so, -DPS_TIMING), MI355X, random actions";
   PIANOSIM_HAND=$H PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so timeout -k 10 120 python tools/phase_timing.py 4096 crossing_field) > profiles/${P}_${H}_phase_timing.txt 2>/dev/null || exit 5
done
PIANOSIM_HAND=hull PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so timeout -k 10 120 python tools/tail_timing.py 1024 twinkle > profiles/${P}_hull_tail_1024.txt 2>/dev/null || exit 5
rm -f profiles/${P}_throughput.txt
for H in hull primitive authored; do
  PIANOSIM_HAND=$H timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 16384 | sed "s/^/$H /" >> profiles/${P}_throughput.txt 2>/dev/null || exit 6
done
if [ -z "$NOPPO" ]; then
timeout -k 10 200 python tools/ppo_bench.py --mode reference --iters 3 --warmup 2 > profiles/${P}_ppo_bench.jsonl 2>/dev/null || exit 8
timeout -k 10 200 python tools/ppo_bench.py --mode reference --iters 3 --warmup 2 --hand authored >> profiles/${P}_ppo_bench.jsonl 2>/dev/null || exit 8
# the PPO loop's kernels (TunableOp off: no GEMM tuning launches in the trace)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${P}_ppo_trace -- python tools/ppo_bench.py --mode reference --iters 2 --warmup 1 --no-tune > gpurun_out/${P}_ppo_trace.log 2>&1 || exit 8
find gpurun_out/${P}_ppo_trace -name "*kernel_stats.csv" -exec cp {} profiles/${P}_ppo_kernel_stats.csv \;
fi
fi
rm -rf gpurun_out/profiles_new && cp -r profiles gpurun_out/profiles_new
echo DONE
