# Development aid (round 5): full Newton steps after a failed piece check (PS_NT_FULLSTEPS=1 / 2,
# tools/build_variants.py f1 f2 f1t f2t) against the product build: Newton iterations per substep
# (timing builds), throughput interleaved, parity probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/ab_full.txt
: > $O
for L in timing f1t f2t; do
  (PIANOSIM_HAND=hull PIANOSIM_LIB=diffusion-piano_amd/libpianosim_$L.so timeout -k 10 120 python tools/phase_timing.py 4096 crossing_field) 2>/dev/null | grep -E "^total|Newton" | sed "s/^/hull $L /" >> $O || exit 7
done
for rep in 1 2; do
  for L in new f1 f2; do
    F=libpianosim_$L.so; [ $L = new ] && F=libpianosim.so
    PIANOSIM_HAND=hull PIANOSIM_LIB=diffusion-piano_amd/$F timeout -k 10 200 python tools/throughput.py crossing_field 4096 2>/dev/null | sed "s/^/hull $L /" >> $O || exit 5
    PIANOSIM_LIB=diffusion-piano_amd/$F timeout -k 10 200 python tools/throughput.py crossing_field 4096 2>/dev/null | sed "s/^/capsule $L /" >> $O || exit 5
  done
done
for L in f1 f2; do
  echo "== $L" >> gpurun_out/ab_full_probe.jsonl
  PIANOSIM_LIB=diffusion-piano_amd/libpianosim_$L.so timeout -k 10 300 python -u tools/parity_probe.py coupled bench >> gpurun_out/ab_full_probe.jsonl 2>/dev/null || exit 6
done
echo DONE
