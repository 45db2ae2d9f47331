# builds tools/libxcheck.so (narrow-phase test harness; not part of the product)
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-value \
  -fno-hip-fp32-correctly-rounded-divide-sqrt -o tools/libxcheck.so tools/xcheck.hip
