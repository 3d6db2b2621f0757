// cmpc_device.h -- device-side parameter block shared by the kernels and the host launcher.
#pragma once
#include <stdint.h>

namespace cmpc {

// Kernel-argument copy of cmpc_params with the reference's factor 2 folded in
// (H = diag(2Q, 2R), centroidal_mpc.py:178-201).
struct KParams {
  int N;
  float Q2[12];
  float R2[12];
  float mu, fz_min;
  float rho0, sigma, alpha;
  float eps_abs, eps_rel;
  float polish_tol;
  float r2_min;         // min_i R2[i]: strong-convexity modulus of the condensed objective
  int max_iter;
  int adaptive_interval;
  int polish_stable;
  int polish_refine;
  int polish_repairs;
  int check_every;      // termination (polish trigger) test every this many ADMM iterations
  int latency_mode;  // set per launch: at most one wave per SIMD (small batch), see condense_tiles
};

// Device pointers of one cmpc_solve call (layouts: include/cmpc.h).
struct Inputs {
  const float* Ad;
  const float* Bd;
  const float* gd;
  const float* x0;
  const float* xref;
  const uint8_t* contact;
  const float* w_init;  // nullable: primal warm start, cmpc_solve_warm's w layout
  const float* y_init;  // nullable: dual warm start [B][12N] (force layout)
  const float* lam_init;  // nullable: the reference's warm duals [B][52N] = [lam_x | lam_a]
};
struct Outputs {
  float* w;
  int32_t* status;
  int32_t* iters;
  float* y;             // nullable: the dual at the returned forces [B][12N]
  float* lam;           // nullable: the reference's multipliers [B][52N] = [lam_x | lam_a]
  // nullable: per-plan cumulative counters (cmpc_plan_stats): [0] loose acceptances, [1] status 2
  // because the certified face bound was missed, [2] checks on a stalled downdated refinement
  // redone on a fresh factorization
  unsigned long long* stats;
};

// Free-variable capacities of the LDS bins (3 forces per stance (step, leg)).  Solve kernels
// (register classes, cmpc_wave.hip solve_group_kernel): bins 1 + 0 (NC 128, 96: two waves per
// SIMD), bins 3 + 2 (NC 160, 144: one wave per SIMD), bin 4 (NC 192: one wave per SIMD, its own
// kernel so that the rare > 160 instances do not size the NC <= 160 kernel's registers).
constexpr int kNumBins = 5;
constexpr int kBinCap[kNumBins] = {96, 128, 144, 160, 192};

}  // namespace cmpc
