# Development aid (round 5): the uncoupled factor's pivot pairs in the box/hull kernel
# (PS_HULL_PAIR=1, tools/build_variants.py hp hpt) against the product build: phase timing,
# throughput interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/ab_hullpair.txt
: > $O
for L in timing hpt; do
  (PIANOSIM_HAND=hull PIANOSIM_LIB=diffusion-piano_amd/libpianosim_$L.so timeout -k 10 120 python tools/phase_timing.py 4096 crossing_field) 2>/dev/null | grep -E "^total|nt:factor|Newton:" | sed "s/^/hull $L /" >> $O || exit 7
done
for rep in 1 2 3; do
  for L in new hp; do
    F=libpianosim_$L.so; [ $L = new ] && F=libpianosim.so
    PIANOSIM_HAND=hull PIANOSIM_LIB=diffusion-piano_amd/$F timeout -k 10 200 python tools/throughput.py crossing_field 4096 2>/dev/null | sed "s/^/hull $L /" >> $O || exit 5
  done
done
echo DONE
