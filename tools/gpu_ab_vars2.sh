# Development aid: box/hull-hand throughput of build variants against the product build,
# interleaved on one box. usage: VARS="vpair vglob" bash tools/gpu_ab_vars2.sh <out prefix>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=${1:-abv}
mkdir -p gpurun_out
rm -f gpurun_out/${P}_tp.txt
for r in 1 2; do
  for L in new $VARS; do
    if [ $L = new ]; then LIB=diffusion-piano_amd/libpianosim.so; else LIB=diffusion-piano_amd/libpianosim_$L.so; fi
    PIANOSIM_LIB=$LIB PIANOSIM_HAND=${HAND:-hull} timeout -k 10 200 python tools/throughput.py crossing_field 4096 2>/dev/null | sed "s/^/$L /" >> gpurun_out/${P}_tp.txt || exit 5
  done
done
cat gpurun_out/${P}_tp.txt
