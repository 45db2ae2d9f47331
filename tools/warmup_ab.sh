# A/B of the exact solve's warm-up sweep count (throughput + per-env tail), one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for W in 8 0 2 4 6 12; do
  PIANOSIM_WARMUP=$W timeout -k 10 150 python tools/throughput.py crossing_field 1024 4096 >> gpurun_out/warmup_ab.txt 2>&1 || exit 3
done
cat gpurun_out/warmup_ab.txt
