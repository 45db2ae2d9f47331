# Development aid (round 5): the step library built for gfx950:xnack- (the pool runs with XNACK
# off; the default gfx950 target is xnack-any) against the product build: bitwise state, then
# throughput interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/ab_xnack.txt
: > $O
for H in hull authored; do
  PIANOSIM_HAND=$H timeout -k 10 200 python tools/ab_state.py /tmp/a_$H.npz 4096 8 > /dev/null 2>&1 || exit 5
  PIANOSIM_HAND=$H PIANOSIM_LIB=diffusion-piano_amd/libpianosim_xn.so timeout -k 10 200 python tools/ab_state.py /tmp/b_$H.npz 4096 8 > /dev/null 2>&1 || exit 5
  python -c "
import numpy as np
a, b = np.load('/tmp/a_$H.npz'), np.load('/tmp/b_$H.npz')
bad = [k for k in a.files if not np.array_equal(a[k], b[k], equal_nan=True)]
print('$H bitwise' if not bad else '$H DIFF ' + str(bad))" >> $O
done
for rep in 1 2 3; do
  for L in new xn; do
    F=libpianosim_$L.so; [ $L = new ] && F=libpianosim.so
    PIANOSIM_HAND=hull PIANOSIM_LIB=diffusion-piano_amd/$F timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 2>/dev/null | sed "s/^/hull $L /" >> $O || exit 5
    PIANOSIM_LIB=diffusion-piano_amd/$F timeout -k 10 200 python tools/throughput.py crossing_field 4096 2>/dev/null | sed "s/^/capsule $L /" >> $O || exit 5
  done
done
echo DONE
