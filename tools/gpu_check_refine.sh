# Development aid (round 5): the one-wave dispatch and the solver_refine option - bitwise state
# of the product build against the previous build (libpianosim_base.so) at 1024 envs (one-wave
# instantiation) and 4096 envs (two-wave), the GPU suite (verbose, every gate's numbers), and
# throughput.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/ck_bitwise.txt
: > $O
for H in hull authored; do
  for N in 1024 4096; do
    PIANOSIM_HAND=$H PIANOSIM_LIB=diffusion-piano_amd/libpianosim_base.so timeout -k 10 200 python tools/ab_state.py /tmp/a_$H$N.npz $N 12 >> $O 2>/dev/null || exit 5
    PIANOSIM_HAND=$H timeout -k 10 200 python tools/ab_state.py /tmp/b_$H$N.npz $N 12 >> $O 2>/dev/null || exit 5
    python -c "
import numpy as np
a, b = np.load('/tmp/a_$H$N.npz'), np.load('/tmp/b_$H$N.npz')
bad = [k for k in a.files if not np.array_equal(a[k], b[k], equal_nan=True)]
print('$H', $N, 'bitwise' if not bad else 'DIFF ' + str(bad))" >> $O
  done
done
timeout -k 10 1000 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ck_tests.log 2>&1
RC=$?
echo "PYTEST_EXIT $RC" >> gpurun_out/ck_tests.log
if [ $RC -gt 1 ]; then exit 9; fi
T=gpurun_out/ck_throughput.txt
: > $T
for H in hull authored; do
  PIANOSIM_HAND=$H timeout -k 10 200 python tools/throughput.py twinkle 1024 4096 | sed "s/^/$H /" >> $T || exit 6
  PIANOSIM_HAND=$H timeout -k 10 200 python tools/throughput.py crossing_field 1024 4096 | sed "s/^/$H /" >> $T || exit 6
  PIANOSIM_REFINE=1 PIANOSIM_HAND=$H timeout -k 10 200 python tools/throughput.py crossing_field 4096 | sed "s/^/$H refine1 /" >> $T || exit 6
done
echo DONE
