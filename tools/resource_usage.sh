# Development aid: register / scratch / LDS use of the step kernel's instantiations, from the
# compiler's resource-usage remarks on a device-only compile with the product flags
# (__graft_entry__._hipcc_lib). usage: bash tools/resource_usage.sh [extra hipcc flags]
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-value --cuda-device-only -c \
  -fno-hip-fp32-correctly-rounded-divide-sqrt -falign-loops=64 -mllvm -amdgpu-sched-strategy=max-ilp \
  -Rpass-analysis=kernel-resource-usage "$@" -o /tmp/ps_dev.o diffusion-piano_amd/csrc/pianosim.hip 2>&1 |
  grep -E "Function Name|VGPRs:|AGPRs:|ScratchSize|Occupancy|LDS Size" | sed 's/.*remark: //' |
  paste - - - - - - | grep pianosim_kernel
