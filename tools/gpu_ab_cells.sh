# Development aid (round 5): hull support cells - bitwise A/B against the previous build, hull
# throughput old / new / polish interleaved, parity probe of the polish experiment, xcheck test.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/ab_cells.txt
: > $O
for L in old cells new; do
  F=libpianosim_$L.so; [ $L = new ] && F=libpianosim.so
  PIANOSIM_HAND=hull PIANOSIM_LIB=diffusion-piano_amd/$F timeout -k 10 120 python tools/ab_state.py gpurun_out/ab_$L.npz >> $O 2>&1 || exit 2
done
python -c "
import numpy as np
a, b = np.load('gpurun_out/ab_old.npz'), np.load('gpurun_out/ab_cells.npz')
for k in a.files:
    d = np.abs(a[k].astype(np.float64) - b[k].astype(np.float64))
    print(k, 'bitwise equal' if np.array_equal(a[k], b[k]) else f'DIFFER max {d.max():.3e} rows {int((d.reshape(len(d), -1).max(1) > 0).sum())}')
" >> $O 2>&1
timeout -k 10 300 python -u -m pytest -q -s --timeout 120 --timeout-method thread tests/test_gpu_colliders.py -k "narrow or one_substep or duplicates" >> $O 2>&1
timeout -k 10 300 python -u tools/parity_probe.py hull >> $O 2>/dev/null
for rep in 1 2; do
  for L in old cells new polish; do
    F=libpianosim_$L.so; [ $L = new ] && F=libpianosim.so
    PIANOSIM_HAND=hull PIANOSIM_LIB=diffusion-piano_amd/$F timeout -k 10 200 python tools/throughput.py crossing_field 4096 2>/dev/null | sed "s/^/hull $L /" >> $O || exit 5
  done
  for L in new polish; do
    F=libpianosim_$L.so; [ $L = new ] && F=libpianosim.so
    PIANOSIM_LIB=diffusion-piano_amd/$F timeout -k 10 200 python tools/throughput.py crossing_field 4096 2>/dev/null | sed "s/^/capsule $L /" >> $O || exit 5
  done
done
PIANOSIM_LIB=diffusion-piano_amd/libpianosim_polish.so timeout -k 10 900 python -u tools/parity_probe.py bench coupled trace heavy guren random > gpurun_out/ab_polish_probe.jsonl 2>/dev/null || exit 6
(PIANOSIM_HAND=hull PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so timeout -k 10 120 python tools/phase_timing.py 4096 crossing_field) > gpurun_out/ab_cells_phase.txt 2>/dev/null || exit 7
echo DONE
