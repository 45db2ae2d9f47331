# Development aid (round 5): gated polish variants (tools/build_variants.py) against the default
# build: parity probe per variant, then throughput interleaved (hull and capsule hands, 4096 envs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
VARS=${VARS:-"new pol1 g3 g4 n3 a3"}
O=gpurun_out/ab_polish.txt
: > $O
for L in $VARS; do
  F=libpianosim_$L.so; [ $L = new ] && F=libpianosim_base.so
  echo "== $L" >> gpurun_out/ab_polish_probe.jsonl
  PIANOSIM_LIB=diffusion-piano_amd/$F timeout -k 10 400 python -u tools/parity_probe.py ${CASES:-coupled heavy guren trace bench} >> gpurun_out/ab_polish_probe.jsonl 2>gpurun_out/ab_polish_probe.err || exit 6
done
for rep in 1 2; do
  for L in $VARS; do
    F=libpianosim_$L.so; [ $L = new ] && F=libpianosim_base.so
    PIANOSIM_HAND=hull PIANOSIM_LIB=diffusion-piano_amd/$F timeout -k 10 200 python tools/throughput.py crossing_field 4096 2>/dev/null | sed "s/^/hull $L /" >> $O || exit 5
    PIANOSIM_LIB=diffusion-piano_amd/$F timeout -k 10 200 python tools/throughput.py crossing_field 4096 2>/dev/null | sed "s/^/capsule $L /" >> $O || exit 5
  done
done
# one wave per SIMD (no scratch, AGPR spills) against the default build at and below one round
# of resident waves
W=gpurun_out/ab_w1.txt
: > $W
for rep in 1 2; do
  for L in new w1; do
    F=libpianosim_$L.so; [ $L = new ] && F=libpianosim_base.so
    PIANOSIM_HAND=hull PIANOSIM_LIB=diffusion-piano_amd/$F timeout -k 10 200 python tools/throughput.py twinkle 1024 2048 2>/dev/null | sed "s/^/hull $L /" >> $W || exit 5
    PIANOSIM_LIB=diffusion-piano_amd/$F timeout -k 10 200 python tools/throughput.py twinkle 1024 2048 2>/dev/null | sed "s/^/capsule $L /" >> $W || exit 5
  done
done
echo DONE
