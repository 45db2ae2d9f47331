# Development aid: hull-hand tests + the whole-block test, throughput of both hands, a short bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_colliders.py tests/test_gpu_solver.py::test_newton_whole_c_block_overlapping_hands tests/test_gpu_task_kwargs.py -q -m gpu --timeout 300 --timeout-method thread -s > gpurun_out/pytest_sel.log 2>&1
RC=$?
echo "PYTEST_EXIT $RC" >> gpurun_out/pytest_sel.log
grep -E "passed|failed|^FAILED|: n [0-9]+, median|max coupled|calm of|^E  " gpurun_out/pytest_sel.log | head -40
if [ $RC -gt 1 ]; then exit 9; fi
PIANOSIM_HULL=1 timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 16384 > gpurun_out/tp.txt 2>&1 || exit 6
grep N= gpurun_out/tp.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/bench_short.json 2> gpurun_out/bench_short.err || exit 7
cat gpurun_out/bench_short.json
