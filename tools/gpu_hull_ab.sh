# Development aid: hull narrow-phase change check: collider parity tests, hull and capsule
# throughput, hull phase split with MPR rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_colliders.py > gpurun_out/hull_ab_tests.log 2>&1 || { tail -30 gpurun_out/hull_ab_tests.log; exit 3; }
tail -3 gpurun_out/hull_ab_tests.log
PIANOSIM_HULL=1 timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 16384 2>&1 | grep -v amdgpu.ids || exit 4
timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 2>&1 | grep -v amdgpu.ids || exit 4
PIANOSIM_HULL=1 PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so timeout -k 10 120 python tools/phase_timing.py 4096 crossing_field > gpurun_out/hull_phase.txt 2>&1 || exit 5
head -26 gpurun_out/hull_phase.txt | grep -v amdgpu.ids
