set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; echo "PYTEST_EXIT $?" >> gpurun_out/pytest_gpu.log
timeout -k 10 200 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -- python bench.py --no-cpu-baseline --steps 20 > gpurun_out/prof_trace.log 2>&1 || exit 2
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -- python bench.py --no-cpu-baseline --steps 10 > gpurun_out/prof_fetch.log 2>&1 || exit 3
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -- python bench.py --no-cpu-baseline --steps 10 > gpurun_out/prof_write.log 2>&1 || exit 4
python tools/collect_pmc.py gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write 4096 r01 > gpurun_out/pmc.log 2>&1
cp profiles/r01_pmc.json profiles/pmc_latest.json gpurun_out/ 2>/dev/null
timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/bench2.json 2>&1
echo DONE
