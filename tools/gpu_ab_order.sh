# Development aid (round 5): the step launch's dispatch-order key - measured cycles of each
# env's last step (PIANOSIM_ORDER_KEY=1, the default) against its Newton iterations (0) and no
# ordering - same library, interleaved, both hands, 4096 / 8192 envs; the bench line last.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/ab_order.txt
: > $O
for rep in 1 2 3; do
  for K in 1 0 none; do
    if [ $K = none ]; then X="PIANOSIM_NO_ORDER=1"; else X="PIANOSIM_ORDER_KEY=$K"; fi
    env $X PIANOSIM_HAND=hull timeout -k 10 200 python tools/throughput.py crossing_field 4096 8192 2>/dev/null | sed "s/^/hull key=$K /" >> $O || exit 5
    env $X timeout -k 10 200 python tools/throughput.py crossing_field 4096 2>/dev/null | sed "s/^/capsule key=$K /" >> $O || exit 5
  done
done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_order_bench.json 2> gpurun_out/ab_order_bench.err || exit 1
echo DONE
