# Development aid: bitwise state A/B of two builds (libpianosim_old.so vs libpianosim.so, hull
# hand), the paired-narrow-phase xcheck test, then throughput A/B and the new build's phases.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PIANOSIM_HAND=hull PIANOSIM_LIB=diffusion-piano_amd/libpianosim_old.so timeout -k 10 120 python tools/ab_state.py gpurun_out/ab_old.npz 1024 20 > /dev/null 2>&1 || exit 2
PIANOSIM_HAND=hull PIANOSIM_LIB=diffusion-piano_amd/libpianosim.so timeout -k 10 120 python tools/ab_state.py gpurun_out/ab_new.npz 1024 20 > /dev/null 2>&1 || exit 3
python -c "
import numpy as np
a=np.load('gpurun_out/ab_old.npz'); b=np.load('gpurun_out/ab_new.npz')
for k in a.files:
    d=(a[k]!=b[k]); print(k, 'differ', int(d.sum()), 'of', d.size)
" > gpurun_out/pm_ab.txt
PS_XCHECK_DIAG=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_colliders.py -q -s --timeout 200 --timeout-method thread -k "narrow_phase" > gpurun_out/pm_tests.log 2>&1
rm -f gpurun_out/pm_tp.txt
for L in old new old new; do
  if [ $L = old ]; then LIB=diffusion-piano_amd/libpianosim_old.so; else LIB=diffusion-piano_amd/libpianosim.so; fi
  PIANOSIM_LIB=$LIB PIANOSIM_HAND=hull timeout -k 10 200 python tools/throughput.py crossing_field 4096 2>/dev/null | sed "s/^/$L hull /" >> gpurun_out/pm_tp.txt || exit 5
done
(PIANOSIM_HAND=hull PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so timeout -k 10 120 python tools/phase_timing.py 4096 crossing_field) > gpurun_out/pm_hull_phase.txt 2>/dev/null || exit 7
cat gpurun_out/pm_ab.txt gpurun_out/pm_tp.txt
tail -3 gpurun_out/pm_tests.log
