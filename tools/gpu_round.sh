# One GPU session: parity tests (+ drift report), bench, rocprofv3 kernel trace and the two
# PMC passes (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in separate passes).
# usage (on the box, via gpurun): bash tools/gpu_round.sh <prefix, e.g. r01_v2>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=${1:-r01}
SONG=crossing_field
mkdir -p gpurun_out profiles
rm -rf gpurun_out/${P}_trace gpurun_out/${P}_fetch gpurun_out/${P}_write
PIANOSIM_REPORT=profiles/${P}_drift.json timeout -k 10 500 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
RC=$?
echo "PYTEST_EXIT $RC" >> gpurun_out/pytest_gpu.log
# 0 = green, 1 = a failed assertion; anything else (fault, abort, time limit) ends the call
if [ $RC -gt 1 ]; then exit 9; fi
cp profiles/${P}_drift.json profiles/drift_latest.json 2>/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${P}_trace -- python bench.py --no-cpu-baseline --steps 20 > gpurun_out/${P}_trace.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${P}_fetch -- python bench.py --no-cpu-baseline --steps 10 > gpurun_out/${P}_fetch.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${P}_write -- python bench.py --no-cpu-baseline --steps 10 > gpurun_out/${P}_write.log 2>&1 || exit 4
python tools/collect_pmc.py gpurun_out/${P}_trace gpurun_out/${P}_fetch gpurun_out/${P}_write 4096 $SONG $P > gpurun_out/pmc.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
cp gpurun_out/bench.json profiles/${P}_bench.json
cp -r profiles gpurun_out/profiles_new
echo DONE
