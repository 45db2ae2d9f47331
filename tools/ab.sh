# A/B of a kernel change on one box (development aid): parity tests of the new build, then
# throughput of libpianosim_base.so (the previous commit's kernel, built beforehand) and of
# the new libpianosim.so, interleaved so clock drift hits both, plus the phase split when
# libpianosim_timing.so exists.
# usage (on the box, via gpurun): bash tools/ab.sh [pytest selection, default the parity file]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SEL=${1:-tests/test_gpu_parity.py}
timeout -k 10 400 python -u -m pytest $SEL -q -m gpu -x --timeout 200 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1
RC=$?
echo "PYTEST_EXIT $RC" >> gpurun_out/ab_pytest.log
tail -3 gpurun_out/ab_pytest.log
if [ $RC -gt 1 ]; then exit 9; fi
: > gpurun_out/ab.txt
for i in 1 2; do
  for L in libpianosim_base.so libpianosim.so; do
    PIANOSIM_LIB=diffusion-piano_amd/$L timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 16384 >> gpurun_out/ab.txt 2>&1 || exit 6
  done
done
cat gpurun_out/ab.txt
if [ -f diffusion-piano_amd/libpianosim_timing.so ]; then
  PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so timeout -k 10 120 python tools/phase_timing.py 4096 > gpurun_out/ab_phase.txt 2>&1 || exit 5
  head -20 gpurun_out/ab_phase.txt
fi
