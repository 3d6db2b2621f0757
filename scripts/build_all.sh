#!/bin/bash
# Build the product library and the diagnostic (stamps) variant in-tree.
set -e
cd "$(dirname "$0")/.."
python -c "import sys; sys.path.insert(0,'convex-mpc-unitree-go2_amd'); from cmpc.build import build_library; build_library(force=True)" 2>&1 | grep -v "occupancy\|solve_bin_kernel(KParams\|\^\|warning generated" || true
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form -DCMPC_STAMPS -Iinclude -Iconvex-mpc-unitree-go2_amd/csrc convex-mpc-unitree-go2_amd/csrc/cmpc_host.hip -o convex-mpc-unitree-go2_amd/cmpc/lib/libcmpc_stamps.so 2>&1 | grep -i " error" || true
ls -la convex-mpc-unitree-go2_amd/cmpc/lib/
