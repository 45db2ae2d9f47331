# Throughput of several prebuilt step-kernel libraries on one box, interleaved so clock drift
# hits all of them (development aid). Optional parity selection first (PARITY=tests/...).
# usage (on the box, via gpurun): bash tools/ab_multi.sh libA.so libB.so ...  (names under diffusion-piano_amd/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$PARITY" ]; then
  for L in "$@"; do
    PIANOSIM_LIB=diffusion-piano_amd/$L timeout -k 10 400 python -u -m pytest $PARITY -q -m gpu -x --timeout 200 --timeout-method thread > gpurun_out/ab_pytest_$L.log 2>&1
    RC=$?
    echo "$L PYTEST_EXIT $RC"; tail -2 gpurun_out/ab_pytest_$L.log
    if [ $RC -gt 1 ]; then exit 9; fi
  done
fi
: > gpurun_out/ab.txt
for i in 1 2; do
  for L in "$@"; do
    PIANOSIM_LIB=diffusion-piano_amd/$L timeout -k 10 200 python tools/throughput.py crossing_field ${NS:-1024 4096 16384} >> gpurun_out/ab.txt 2>&1 || exit 6
  done
done
cat gpurun_out/ab.txt
