# Development aid (round 5): end-of-round confirmation of the committed tree as the driver runs it
# (GPU suite with -x, smoke(), default bench.py line and its kernel trace).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/fin_tests.log 2>&1 || { echo TESTS_FAIL; exit 3; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/fin_smoke.log 2>&1 || { echo SMOKE_FAIL; exit 4; }
timeout -k 10 400 python bench.py > gpurun_out/fin_bench.json 2> gpurun_out/fin_bench.err || { echo BENCH_FAIL; exit 5; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin_prof -o fin -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/fin_prof.log 2>&1 || { echo PROF_FAIL; exit 6; }
echo DONE
