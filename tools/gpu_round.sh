# one GPU call: Newton solver tests, phase timing, bench (outputs under gpurun_out/)
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py -v --timeout 300 --timeout-method thread -s > gpurun_out/solver.log 2>&1; echo rc=$? >> gpurun_out/solver.log
PIANOSIM_LIB=diffusion-piano_amd/libpianosim_timing.so timeout -k 10 300 python -u tools/phase_timing.py 4096 > gpurun_out/phase.txt 2>&1; echo rc=$? >> gpurun_out/phase.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1; echo rc=$? >> gpurun_out/bench.log
