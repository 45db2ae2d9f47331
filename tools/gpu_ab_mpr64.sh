# Development aid (round 6): the fp64 MPR (PS_MPR_F64=1, the product build) against the fp32 one
# (libpianosim_f32mpr.so, tools/build_variants.py f32mpr=-DPS_MPR_F64=0): box/hull throughput
# interleaved, the contact-list comparison and the benched-workload parity test of each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab64_tp.txt
for r in 1 2; do
  for L in new f32mpr; do
    if [ $L = new ]; then LIB=diffusion-piano_amd/libpianosim.so; else LIB=diffusion-piano_amd/libpianosim_$L.so; fi
    PIANOSIM_LIB=$LIB PIANOSIM_HAND=hull timeout -k 10 100 python tools/throughput.py crossing_field 4096 2>/dev/null | sed "s/^/$L /" >> gpurun_out/ab64_tp.txt || exit 5
  done
done
for L in new f32mpr; do
  if [ $L = new ]; then LIB=diffusion-piano_amd/libpianosim.so; else LIB=diffusion-piano_amd/libpianosim_$L.so; fi
  PIANOSIM_LIB=$LIB timeout -k 10 200 python tools/contact_diff.py 20 4096 > gpurun_out/ab64_cd_$L.log 2>&1 || exit 6
  PIANOSIM_LIB=$LIB timeout -k 10 300 python -u -m pytest -q -s --timeout 280 tests/test_gpu_colliders.py -k "benched or one_substep or teacher_forced" -m gpu > gpurun_out/ab64_t_$L.log 2>&1
done
cat gpurun_out/ab64_tp.txt
grep -h mismatches gpurun_out/ab64_cd_*.log | cut -c1-300
grep -h "n [0-9]*, median" gpurun_out/ab64_t_*.log | cut -c1-330
