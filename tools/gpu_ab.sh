# Development aid: throughput of step-library variants against the product build, interleaved on
# one box (replaces the one-off gpu_ab_*.sh scripts of rounds 3-5, which are in the git history).
# Variants are built beforehand with tools/build_variants.py (diffusion-piano_amd/libpianosim_<v>.so).
# usage (via gpurun): VARS="v1 v2" HAND=hull ENVS="4096" REPS=2 bash tools/gpu_ab.sh <out prefix>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=${1:-ab}
mkdir -p gpurun_out
rm -f gpurun_out/${P}_tp.txt
for r in $(seq ${REPS:-2}); do
  for L in new $VARS; do
    if [ $L = new ]; then LIB=diffusion-piano_amd/libpianosim.so; else LIB=diffusion-piano_amd/libpianosim_$L.so; fi
    PIANOSIM_LIB=$LIB PIANOSIM_HAND=${HAND:-hull} timeout -k 10 200 python tools/throughput.py ${SONG:-crossing_field} ${ENVS:-4096} 2>/dev/null | sed "s/^/$L /" >> gpurun_out/${P}_tp.txt || exit 5
  done
done
cat gpurun_out/${P}_tp.txt
