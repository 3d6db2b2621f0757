#!/bin/bash
# Build a variant of libcmpc.so with extra compile flags (A/B experiments).
#   usage: bash scripts/build_variant.sh <name> [-DFLAG ...]  -> cmpc/lib/libcmpc_<name>.so
#   (NO_VFORM=1: without -amdgpu-mfma-vgpr-form)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
VFORM="-mllvm -amdgpu-mfma-vgpr-form"; [ "${NO_VFORM:-0}" = "1" ] && VFORM=""
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fno-slp-vectorize ${VFORM} "$@" \
  -Iinclude -Iconvex-mpc-unitree-go2_amd/csrc convex-mpc-unitree-go2_amd/csrc/cmpc_host.hip \
  -o convex-mpc-unitree-go2_amd/cmpc/lib/libcmpc_$name.so
