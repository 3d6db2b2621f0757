#!/bin/bash
# Build a variant of libcmpc.so with extra compile flags (A/B experiments).
#   usage: bash scripts/build_variant.sh <name> [-DFLAG ...]  -> cmpc/lib/libcmpc_<name>.so
set -e
cd "$(dirname "$0")/.."
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form "$@" \
  -Iinclude -Iconvex-mpc-unitree-go2_amd/csrc convex-mpc-unitree-go2_amd/csrc/cmpc_host.hip \
  -o convex-mpc-unitree-go2_amd/cmpc/lib/libcmpc_$name.so
