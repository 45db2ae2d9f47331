cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for L in new m8 m16; do
  if [ $L = new ]; then LIB=diffusion-piano_amd/libpianosim.so; else LIB=diffusion-piano_amd/libpianosim_$L.so; fi
  PIANOSIM_LIB=$LIB timeout -k 10 200 python tools/parity_probe.py coupled heavy guren > gpurun_out/abr_$L.txt 2>&1 || exit 3
  PIANOSIM_LIB=$LIB PIANOSIM_HAND=hull timeout -k 10 100 python tools/throughput.py crossing_field 4096 2>/dev/null | sed "s/^/$L /" >> gpurun_out/abr_tp.txt || exit 4
done
PIANOSIM_LIB=diffusion-piano_amd/libpianosim.so PIANOSIM_REFINE=0 PIANOSIM_HAND=hull timeout -k 10 100 python tools/throughput.py crossing_field 4096 2>/dev/null | sed "s/^/r0 /" >> gpurun_out/abr_tp.txt
cat gpurun_out/abr_tp.txt; grep -h case gpurun_out/abr_*.txt | cut -c1-160
