# Development aid: hull-hand throughput of library variants (VARS), interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/${OUT:-ab_vars}.txt
: > $O
for rep in 1 2; do
  for L in new $VARS; do
    F=libpianosim_$L.so; [ $L = new ] && F=libpianosim.so
    PIANOSIM_HAND=${HAND:-hull} PIANOSIM_LIB=diffusion-piano_amd/$F timeout -k 10 200 python tools/throughput.py crossing_field 4096 2>/dev/null | sed "s/^/$L /" >> $O || exit 5
  done
done
echo DONE
