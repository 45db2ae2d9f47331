# Development aid: box/hull hand after parking the lane state around its collision: collider
# tests, hull phase split, hull and capsule throughput
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_colliders.py > gpurun_out/park_tests.log 2>&1 || { tail -30 gpurun_out/park_tests.log; exit 3; }
tail -2 gpurun_out/park_tests.log
bash tools/gpu_xphase.sh libpianosim_timing.so || exit 5
PIANOSIM_HULL=1 timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 16384 > gpurun_out/park_tp.txt 2>&1 || exit 4
timeout -k 10 200 python tools/throughput.py crossing_field 4096 >> gpurun_out/park_tp.txt 2>&1 || exit 4
grep -v amdgpu.ids gpurun_out/park_tp.txt
