# Development aid: the sensitive parity gates (teacher-forced control steps, coupled hands,
# full contact capacity) on two builds: old = previous commit, pt = paired MPR + cell tables.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in old pt; do
PIANOSIM_LIB=diffusion-piano_amd/libpianosim_$L.so timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_colliders.py tests/test_gpu_solver.py -k "teacher_forced or coupled_hands" > gpurun_out/ab3_${L}tests.log 2>&1
echo "$L tests rc $?"
done
