set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -s > gpurun_out/pytest_gpu.log 2>&1
RC=$?
echo "PYTEST_EXIT $RC" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
if [ $RC -gt 1 ]; then exit 9; fi
CASES="bench coupled heavy trace random guren" timeout -k 10 300 python -u tools/parity_probe.py > gpurun_out/probe.jsonl 2>gpurun_out/probe.err || exit 8
cat gpurun_out/probe.jsonl
for L in libpianosim_base.so libpianosim.so libpianosim_base.so libpianosim.so; do
  PIANOSIM_LIB=diffusion-piano_amd/$L timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 >> gpurun_out/tp.txt 2>&1 || exit 6
done
for L in libpianosim_base.so libpianosim.so; do
  PIANOSIM_HULL=1 PIANOSIM_LIB=diffusion-piano_amd/$L timeout -k 10 200 python tools/throughput.py crossing_field 4096 >> gpurun_out/tp.txt 2>&1 || exit 6
done
grep N= gpurun_out/tp.txt
