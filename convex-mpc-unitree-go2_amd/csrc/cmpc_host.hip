// cmpc_host.hip -- C-ABI (include/cmpc.h): plan management and kernel launches.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "cmpc.h"
#include "cmpc_device.h"

#include "cmpc_wave.hip"      // solve kernels: same translation unit
#include "cmpc_dynamics.hip"  // QP-data (discrete dynamics) kernel
#include "cmpc_traj.hip"      // reference trajectory / contact table / foot levers kernel
#include "cmpc_leg.hip"       // leg controller (stance torque mapping, swing) kernel
#include "cmpc_sim.hip"       // single-rigid-body plant (closed-loop stand-in for MuJoCo)

constexpr int kNumGroups = 3;  // solve kernels (register classes), see solve_group_kernel
static_assert(kNumGroups == CMPC_NUM_SOLVE_KERNELS, "one timing slot per solve kernel");

struct cmpc_plan {
  cmpc_params p;
  cmpc::KParams kp;
  int device;
  int cus = 0;      // compute units of the device
  int* d_counters;  // counts[kNumBins], heads[kNumBins]
  unsigned long long* d_stats = nullptr;  // CMPC_NUM_STATS cumulative counters (cmpc_plan_stats)
  int* d_lists;     // kNumBins * max_batch
  float* d_work;    // per-wave park slabs; group k's region starts at work_off[k] (groups overlap)
  size_t work_off[kNumGroups];
  int grid[kNumGroups];      // persistent grid of each group's one-wave kernel
  size_t slab[kNumGroups];   // park slab per wave (floats)
  // small batches (B <= team_max_batch): one kernel for all bins, kTeamWaves waves per QP
  // (cmpc_team.hip), on the caller's stream
  int team_grid = 0;    // workgroups resident at two per CU (solve_team_kernel<W, 2>)
  int team_grid1 = 0;   // at one per CU (<W, 1>: B <= CUs)
  size_t team_slab = 0;
  int64_t team_max_batch = -1;  // -1: automatic (B <= 4 x CUs: at most one wave per SIMD)
  // batches of B >= heavy_first_min_batch submit the NC >= 160 class first
  int64_t heavy_first_min_batch = -1;  // -1: automatic (B > 16 x CUs), 0: never
  // The solve kernels (cmpc_wave.hip solve_group_kernel: the NC <= 128 class, the NC 144 / 160
  // class, the NC 192 bin) run concurrently: one class on the caller's stream, the other on a
  // plan stream, the NC 192 kernel on a second plan stream, both forked from / joined to the
  // caller's.  Three streams in total stay within the device's hardware queues
  // (GPU_MAX_HW_QUEUES = 4), so the kernels overlap instead of sharing a queue.
  hipStream_t side = nullptr;
  hipStream_t top = nullptr;
  hipEvent_t fork = nullptr;
  hipEvent_t join = nullptr;
  hipEvent_t join_top = nullptr;
  // timing hooks
  bool timing = false;
  struct Rec { hipEvent_t a, b; int group; };
  std::vector<Rec> recs;       // recorded (pending) pairs
  std::vector<Rec> pool;       // free event pairs
};

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(CMPC_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

using KernelFn = void (*)(cmpc::KParams, cmpc::Inputs, cmpc::Outputs, const int*, const int*,
                          const int*, int*, int, float*, size_t);

// The plan's workspace, streams and events belong to the device current at cmpc_plan_create:
// every launch must run there (the Python layer makes the tensors' device current).
int check_device(const cmpc_plan* pl, const char* what) {
  int dev = -1;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  if (dev != pl->device)
    return fail(CMPC_E_INVALID, std::string(what) + ": the current device is not the plan's device");
  return CMPC_OK;
}

// group 0: bins 1 (NC 128) then 0 (NC 96), two waves per SIMD; group 1: bins 3 (NC 160) then
// 2 (NC 144), one wave per SIMD; group 2: bin 4 (NC 192) alone, one wave per SIMD.  qa = the
// group's first (larger) bin.
int group_first_bin(int k) { return k == 0 ? 1 : (k == 1 ? 3 : 4); }

constexpr int kTeamWaves = 4;

KernelFn group_fn(int k) {
  return k == 0 ? cmpc::solve_group_kernel<128, 96>
                : (k == 1 ? cmpc::solve_group_kernel<160, 144> : cmpc::solve_group_kernel<192, 0>);
}

const char* group_name(int k) {
  static const char* names[kNumGroups] = {"solve_group_kernel<128, 96>",
                                          "solve_group_kernel<160, 144>",
                                          "solve_group_kernel<192, 0>"};
  return names[k];
}

// park slab per wave (floats): the one-wave inverse
size_t group_slab(int k) {
  return k == 0 ? std::max(cmpc::Cfg<128>::SLAB, cmpc::Cfg<96>::SLAB)
                : (k == 1 ? std::max(cmpc::Cfg<160>::SLAB, cmpc::Cfg<144>::SLAB) : cmpc::Cfg<192>::SLAB);
}

// which solve kernels a horizon can need: the NC >= 144 class once the horizon can hold more
// than 128 free forces, the NC 192 kernel once more than 160
bool has_group(const cmpc_plan* pl, int k) {
  return k == 0 || cmpc::kBinCap[k == 1 ? 1 : 3] < 12 * pl->kp.N;
}

}  // namespace

extern "C" {

void cmpc_params_default(cmpc_params* p) {
  if (!p) return;
  memset(p, 0, sizeof(*p));
  p->abi_version = CMPC_ABI_VERSION;
  p->N = 16;
  const float Q[12] = {1, 1, 50, 10, 20, 1, 2, 2, 1, 1, 1, 1};  // centroidal_mpc.py:12
  for (int i = 0; i < 12; ++i) {
    p->Q[i] = Q[i];
    p->R[i] = 1e-5f;  // centroidal_mpc.py:13
  }
  p->mu = 0.8f;        // centroidal_mpc.py:15
  p->fz_min = 10.f;    // centroidal_mpc.py:127
  p->eps_abs = 1e-4f;  // centroidal_mpc.py:25-26
  p->eps_rel = 1e-4f;
  p->max_iter = 1000;  // centroidal_mpc.py:27
  p->rho = 1e-4f;
  p->sigma = 1e-6f;    // OSQP default
  p->alpha = 1.6f;     // OSQP default
  p->adaptive_rho_interval = 25;  // centroidal_mpc.py:32
  p->polish_stable = 3;
  p->polish_refine = 2;  // (round 6: 4 -> 2 with the LDL' solve; profiles/r06d_*)
  p->polish_tol = 1e-5f;
  p->polish_repairs = 6;
  p->reserved0 = 0;
  p->check_termination = 1;  // (reference OPTS: 10, accepted; see include/cmpc.h)
  p->max_batch = 65536;
}

int cmpc_plan_create(const cmpc_params* p, cmpc_plan** out) {
  if (!p || !out) return fail(CMPC_E_INVALID, "cmpc_plan_create: null argument");
  *out = nullptr;
  if (p->abi_version != CMPC_ABI_VERSION)
    return fail(CMPC_E_INVALID, "cmpc_plan_create: abi_version mismatch");
  if (p->N < 1 || p->N > 16) return fail(CMPC_E_INVALID, "cmpc_plan_create: N must be in 1..16");
  for (int i = 0; i < 12; ++i) {
    if (!(p->Q[i] >= 0.f) || !std::isfinite(p->Q[i]))
      return fail(CMPC_E_INVALID, "cmpc_plan_create: Q must be finite and >= 0");
    if (!(p->R[i] > 0.f) || !std::isfinite(p->R[i]))
      return fail(CMPC_E_INVALID, "cmpc_plan_create: R must be finite and > 0");
  }
  if (!(p->mu > 0.f) || !std::isfinite(p->mu)) return fail(CMPC_E_INVALID, "cmpc_plan_create: mu must be > 0");
  if (!std::isfinite(p->fz_min)) return fail(CMPC_E_INVALID, "cmpc_plan_create: fz_min must be finite");
  if (p->max_iter < 1) return fail(CMPC_E_INVALID, "cmpc_plan_create: max_iter must be >= 1");
  if (!(p->rho > 0.f) || !(p->sigma >= 0.f) || !(p->alpha > 0.f && p->alpha < 2.f))
    return fail(CMPC_E_INVALID, "cmpc_plan_create: need rho > 0, sigma >= 0, 0 < alpha < 2");
  if (p->polish_stable < 1 || p->polish_refine < 1 || !(p->polish_tol > 0.f) ||
      p->polish_repairs < 0 || p->check_termination < 1)
    return fail(CMPC_E_INVALID, "cmpc_plan_create: polish settings out of range");
  if (p->adaptive_rho_interval < 0 || p->max_batch < 1 || p->max_batch > (1LL << 30))
    return fail(CMPC_E_INVALID, "cmpc_plan_create: adaptive_rho_interval/max_batch out of range");
  if (p->reserved0 != 0)
    return fail(CMPC_E_INVALID, "cmpc_plan_create: reserved0 must be 0 (ABI 4's ipm_facts: the "
                                "interior-point fallback was removed)");

  cmpc_plan* pl = new cmpc_plan();
  pl->p = *p;
  cmpc::KParams& k = pl->kp;
  k.N = p->N;
  k.r2_min = 2.f * p->R[0];
  for (int i = 0; i < 12; ++i) {
    k.Q2[i] = 2.f * p->Q[i];
    k.R2[i] = 2.f * p->R[i];
    k.r2_min = std::min(k.r2_min, k.R2[i]);
  }
  k.mu = p->mu;
  k.fz_min = p->fz_min;
  k.rho0 = p->rho;
  k.sigma = p->sigma;
  k.alpha = p->alpha;
  k.eps_abs = p->eps_abs;
  k.eps_rel = p->eps_rel;
  k.polish_tol = p->polish_tol;
  k.max_iter = p->max_iter;
  k.adaptive_interval = p->adaptive_rho_interval;
  k.polish_stable = p->polish_stable;
  k.polish_refine = p->polish_refine;
  k.polish_repairs = p->polish_repairs;
  k.check_every = p->check_termination;

  hipError_t e = hipGetDevice(&pl->device);
  if (e != hipSuccess) { delete pl; return hip_fail(e, "hipGetDevice"); }
  int cus = 0;
  e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, pl->device);
  pl->cus = cus;
  if (e != hipSuccess) { delete pl; return hip_fail(e, "hipDeviceGetAttribute"); }
  // persistent grids: resident workgroups per CU x CUs
  size_t work_floats = 0;
  for (int k = 0; k < kNumGroups; ++k) {
    int nb = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, group_fn(k), 64, 0);
    if (e != hipSuccess) { delete pl; return hip_fail(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor"); }
    if (nb < 1) { delete pl; return fail(CMPC_E_HIP, "cmpc_plan_create: solve kernel cannot be resident"); }
#ifdef CMPC_STAMPS
    if (const char* cap = getenv("CMPC_BLOCKS_PER_CU")) {  // diagnostic build: occupancy sweep
      const int c = atoi(cap);
      if (c >= 1 && c < nb) nb = c;
    }
#endif
    pl->grid[k] = nb * cus;
    pl->slab[k] = group_slab(k);
    pl->work_off[k] = work_floats;
    work_floats += (size_t)pl->grid[k] * pl->slab[k];
  }
  {
    int nb = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, cmpc::solve_team_kernel<kTeamWaves, 2>,
                                                     64 * kTeamWaves, 0);
    if (e != hipSuccess) { delete pl; return hip_fail(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor"); }
    if (nb < 1) nb = 1;
    pl->team_grid = nb * cus;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, cmpc::solve_team_kernel<kTeamWaves, 1>,
                                                     64 * kTeamWaves, 0);
    if (e != hipSuccess) { delete pl; return hip_fail(e, "hipOccupancyMaxActiveBlocksPerMultiprocessor"); }
    // (0 if the one-per-CU image cannot be resident: team_one_per_cu then never selects it and
    // the two-per-CU image serves every team batch)
    pl->team_grid1 = nb < 1 ? 0 : cus;
    pl->team_slab = std::max({cmpc::TeamCfg<192, kTeamWaves>::SLAB, cmpc::TeamCfg<160, kTeamWaves>::SLAB,
                              cmpc::TeamCfg<128, kTeamWaves>::SLAB, cmpc::TeamCfg<96, kTeamWaves>::SLAB});
    work_floats = std::max(work_floats, (size_t)pl->team_grid * pl->team_slab);
  }
  e = hipMalloc(&pl->d_counters, 2 * cmpc::kNumBins * sizeof(int));
  if (e != hipSuccess) { delete pl; return fail(CMPC_E_NOMEM, "hipMalloc counters failed"); }
  e = hipMalloc(&pl->d_work, work_floats * sizeof(float));
  if (e != hipSuccess) {
    (void)hipFree(pl->d_counters);
    delete pl;
    return fail(CMPC_E_NOMEM, "hipMalloc workspace failed");
  }
  e = hipMalloc(&pl->d_lists, (size_t)cmpc::kNumBins * p->max_batch * sizeof(int));
  if (e != hipSuccess) {
    (void)hipFree(pl->d_counters);
    (void)hipFree(pl->d_work);
    delete pl;
    return fail(CMPC_E_NOMEM, "hipMalloc lists failed");
  }
  if ((e = hipMalloc(&pl->d_stats, CMPC_NUM_STATS * sizeof(unsigned long long))) != hipSuccess) {
    cmpc_plan_destroy(pl);
    return fail(CMPC_E_NOMEM, "hipMalloc stats failed");
  }
  // the NC 192 stream at the highest priority: its few early waves are dispatched ahead of the
  // register classes submitted right after them on the other queues (solve_impl)
  int prio_lo = 0, prio_hi = 0;
  if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) prio_hi = 0;
  if ((e = hipStreamCreateWithFlags(&pl->side, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipStreamCreateWithPriority(&pl->top, hipStreamNonBlocking, prio_hi)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&pl->fork, hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&pl->join, hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&pl->join_top, hipEventDisableTiming)) != hipSuccess) {
    cmpc_plan_destroy(pl);
    return hip_fail(e, "side stream/event creation");
  }
  // zeroed on the plan's own stream: a copy or memset on the null stream here (the caller's
  // default stream, round 6's first ABI-6 build) made the closed loop's HIP-graph replay at
  // 65,536 robots 1.3x slower than eager (profiles/r06l_*)
  if ((e = hipMemsetAsync(pl->d_stats, 0, CMPC_NUM_STATS * sizeof(unsigned long long), pl->side)) !=
          hipSuccess ||
      (e = hipStreamSynchronize(pl->side)) != hipSuccess) {
    cmpc_plan_destroy(pl);
    return hip_fail(e, "hipMemsetAsync stats");
  }
  *out = pl;
  g_err.clear();
  return CMPC_OK;
}

static int solve_impl(cmpc_plan* pl, int64_t B, const cmpc::Inputs& in, const cmpc::Outputs& out,
                      void* stream);

int cmpc_solve(cmpc_plan* pl, int64_t B, const float* Ad, const float* Bd, const float* gd,
               const float* x0, const float* xref, const uint8_t* contact, float* w_out,
               int32_t* status, int32_t* iters, void* stream) {
  if (!pl) return fail(CMPC_E_INVALID, "cmpc_solve: null plan");
  if (B < 0) return fail(CMPC_E_INVALID, "cmpc_solve: negative batch");
  if (B == 0) return CMPC_OK;
  if (B > pl->p.max_batch) return fail(CMPC_E_RANGE, "cmpc_solve: B exceeds plan max_batch");
  if (!Ad || !Bd || !gd || !x0 || !xref || !contact || !w_out || !status || !iters)
    return fail(CMPC_E_INVALID, "cmpc_solve: null array argument");
  return solve_impl(pl, B, cmpc::Inputs{Ad, Bd, gd, x0, xref, contact, nullptr, nullptr, nullptr},
                    cmpc::Outputs{w_out, status, iters, nullptr, nullptr, pl->d_stats}, stream);
}

int cmpc_solve_warm(cmpc_plan* pl, int64_t B, const float* Ad, const float* Bd,
                    const float* gd, const float* x0, const float* xref,
                    const uint8_t* contact, const float* w_init, const float* y_init,
                    float* w_out, float* y_out, int32_t* status, int32_t* iters, void* stream) {
  if (!pl) return fail(CMPC_E_INVALID, "cmpc_solve_warm: null plan");
  if (B < 0) return fail(CMPC_E_INVALID, "cmpc_solve_warm: negative batch");
  if (B == 0) return CMPC_OK;
  if (B > pl->p.max_batch) return fail(CMPC_E_RANGE, "cmpc_solve_warm: B exceeds plan max_batch");
  if (!Ad || !Bd || !gd || !x0 || !xref || !contact || !w_out || !status || !iters)
    return fail(CMPC_E_INVALID, "cmpc_solve_warm: null array argument");
  return solve_impl(pl, B, cmpc::Inputs{Ad, Bd, gd, x0, xref, contact, w_init, y_init, nullptr},
                    cmpc::Outputs{w_out, status, iters, y_out, nullptr, pl->d_stats}, stream);
}

int cmpc_solve_ref(cmpc_plan* pl, int64_t B, const float* Ad, const float* Bd, const float* gd,
                   const float* x0, const float* xref, const uint8_t* contact,
                   const float* w_init, const float* lam_init, float* w_out, float* lam_out,
                   int32_t* status, int32_t* iters, void* stream) {
  if (!pl) return fail(CMPC_E_INVALID, "cmpc_solve_ref: null plan");
  if (B < 0) return fail(CMPC_E_INVALID, "cmpc_solve_ref: negative batch");
  if (B == 0) return CMPC_OK;
  if (B > pl->p.max_batch) return fail(CMPC_E_RANGE, "cmpc_solve_ref: B exceeds plan max_batch");
  if (!Ad || !Bd || !gd || !x0 || !xref || !contact || !w_out || !status || !iters)
    return fail(CMPC_E_INVALID, "cmpc_solve_ref: null array argument");
  return solve_impl(pl, B, cmpc::Inputs{Ad, Bd, gd, x0, xref, contact, w_init, nullptr, lam_init},
                    cmpc::Outputs{w_out, status, iters, nullptr, lam_out, pl->d_stats}, stream);
}

// group k's persistent kernel with g waves whose park slabs start at wave w0 of the group's
// region (a second launch of the same group on the same queue heads takes the slabs after the
// first one's); `timed` records the launch for cmpc_plan_timing_read
static int record_launch(cmpc_plan* pl, int k, hipStream_t s, const cmpc::KParams& kp,
                         const cmpc::Inputs& in, const cmpc::Outputs& out, unsigned g,
                         unsigned w0 = 0, bool timed = true) {
  hipError_t e;
  cmpc_plan::Rec rec{nullptr, nullptr, k};
  const bool rec_this = timed && pl->timing && pl->recs.size() < 4096 * kNumGroups;
  if (rec_this) {
    if (!pl->pool.empty()) {
      rec = pl->pool.back();
      pl->pool.pop_back();
      rec.group = k;
    } else {
      if ((e = hipEventCreate(&rec.a)) != hipSuccess) return hip_fail(e, "hipEventCreate");
      if ((e = hipEventCreate(&rec.b)) != hipSuccess) return hip_fail(e, "hipEventCreate");
    }
    if ((e = hipEventRecord(rec.a, s)) != hipSuccess) return hip_fail(e, "hipEventRecord");
  }
  const int qa = group_first_bin(k);
  hipLaunchKernelGGL(group_fn(k), dim3(g), dim3(64), 0, s, kp, in, out,
                     pl->d_lists + (size_t)qa * pl->p.max_batch,
                     pl->d_lists + (size_t)(qa - 1) * pl->p.max_batch, pl->d_counters,
                     pl->d_counters + cmpc::kNumBins, qa,
                     pl->d_work + pl->work_off[k] + (size_t)w0 * pl->slab[k], pl->slab[k]);
  e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, "solve_group_kernel launch");
  if (rec_this) {
    if ((e = hipEventRecord(rec.b, s)) != hipSuccess) return hip_fail(e, "hipEventRecord");
    pl->recs.push_back(rec);
  }
  return CMPC_OK;
}

static int64_t heavy_first_batch(const cmpc_plan* pl) {
  // (0 = never: also when the horizon is too short for an NC >= 144 class to exist)
  if (!has_group(pl, 1)) return 0;
  return pl->heavy_first_min_batch >= 0 ? pl->heavy_first_min_batch : 16LL * pl->cus + 1;
}

static int64_t team_batch(const cmpc_plan* pl) {
  return pl->team_max_batch >= 0 ? pl->team_max_batch : 4LL * pl->cus;
}

// B <= CUs: every QP has a CU of its own, so the team kernel built for one workgroup per CU
// runs (CMPC_TEAM_OCC=2 forces the two-per-CU image, for A/B)
static bool team_one_per_cu(const cmpc_plan* pl, int64_t B) {
  static const int occ = [] {
    const char* v = getenv("CMPC_TEAM_OCC");
    return v ? atoi(v) : 0;
  }();
  // (experiment knob CMPC_TEAM_OCC: 2 = always the two-per-CU image, 1 = always one per CU,
  // persistent over B / CUs instances per workgroup)
  return occ != 2 && pl->team_grid1 > 0 && (occ == 1 || B <= pl->team_grid1);
}

// team mode: one launch for every bin; timed as solve kernel 0 (kernel 1 records no call)
static int record_team_launch(cmpc_plan* pl, hipStream_t s, const cmpc::KParams& kp,
                              const cmpc::Inputs& in, const cmpc::Outputs& out, int64_t B) {
  hipError_t e;
  cmpc_plan::Rec rec{nullptr, nullptr, 0};
  const bool rec_this = pl->timing && pl->recs.size() < 4096 * kNumGroups;
  if (rec_this) {
    if (!pl->pool.empty()) {
      rec = pl->pool.back();
      pl->pool.pop_back();
      rec.group = 0;
    } else {
      if ((e = hipEventCreate(&rec.a)) != hipSuccess) return hip_fail(e, "hipEventCreate");
      if ((e = hipEventCreate(&rec.b)) != hipSuccess) return hip_fail(e, "hipEventCreate");
    }
    if ((e = hipEventRecord(rec.a, s)) != hipSuccess) return hip_fail(e, "hipEventRecord");
  }
  // one QP per CU: the one-workgroup-per-CU image (512 registers per lane, no spills)
  if (team_one_per_cu(pl, B)) {
    const unsigned g = (unsigned)(pl->team_grid1 < B ? pl->team_grid1 : B);
    hipLaunchKernelGGL((cmpc::solve_team_kernel<kTeamWaves, 1>), dim3(g), dim3(64 * kTeamWaves), 0,
                       s, kp, in, out, pl->d_lists, (int64_t)pl->p.max_batch, pl->d_counters,
                       pl->d_counters + cmpc::kNumBins, pl->d_work, pl->team_slab);
  } else {
    const unsigned g = (unsigned)(pl->team_grid < B ? pl->team_grid : B);
    hipLaunchKernelGGL((cmpc::solve_team_kernel<kTeamWaves, 2>), dim3(g), dim3(64 * kTeamWaves), 0,
                       s, kp, in, out, pl->d_lists, (int64_t)pl->p.max_batch, pl->d_counters,
                       pl->d_counters + cmpc::kNumBins, pl->d_work, pl->team_slab);
  }
  e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, "solve_team_kernel launch");
  if (rec_this) {
    if ((e = hipEventRecord(rec.b, s)) != hipSuccess) return hip_fail(e, "hipEventRecord");
    pl->recs.push_back(rec);
  }
  return CMPC_OK;
}

static int solve_impl(cmpc_plan* pl, int64_t B, const cmpc::Inputs& in, const cmpc::Outputs& out,
                      void* stream) {
  int rc = check_device(pl, "cmpc_solve");
  if (rc != CMPC_OK) return rc;
  hipStream_t st = (hipStream_t)stream;
  hipError_t e;
  cmpc::KParams kp = pl->kp;
  // at most one wave per SIMD: latency-bound, the condensation with fewer MFMAs wins
  kp.latency_mode = (B <= 4LL * pl->cus) ? 1 : 0;
  if (B <= 1024) {  // one workgroup bins the batch and zeroes the queue heads (no memset)
    hipLaunchKernelGGL(cmpc::bin_small_kernel, dim3(1), dim3(1024), 0, st, pl->kp.N, (int)B,
                       in.contact, pl->d_counters, pl->d_counters + cmpc::kNumBins, pl->d_lists,
                       pl->p.max_batch);
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "bin_small_kernel launch");
  } else {
    e = hipMemsetAsync(pl->d_counters, 0, 2 * cmpc::kNumBins * sizeof(int), st);
    if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync");
    const int threads = 256;
    const unsigned blocks = (unsigned)((B + threads - 1) / threads);
    hipLaunchKernelGGL(cmpc::bin_kernel, dim3(blocks), dim3(threads), 0, st, pl->kp.N, B,
                       in.contact, pl->d_counters, pl->d_lists, pl->p.max_batch);
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "bin_kernel launch");
  }
  // small batches: a team of kTeamWaves waves per QP, all bins in one kernel on the caller's
  // stream (measured faster than one wave per QP up to B = 4 x CUs on configs 1-3, slower from
  // 2,048 up: DESIGN.md 4g)
  if (B <= team_batch(pl)) return record_team_launch(pl, st, kp, in, out, B);
  // The two classes run concurrently: the class submitted first on the caller's stream, the
  // other (the NC >= 160 class exists only when a step can hold more than 128 / 12 stance legs)
  // on the plan stream, forked after the binning and joined back.  Whichever is submitted first
  // fills the device (two NC <= 128 waves or one NC >= 160 wave per SIMD) and the other takes
  // SIMDs as they free up, so the classes run almost one after the other and the end of the
  // step is the tail of the class that runs last (tools/shard_anatomy.py timelines).  Large
  // batches put the NC >= 160 class first: its tail (one wave per SIMD, ~11 instances per wave)
  // is then filled by NC <= 128 waves, and the NC <= 128 tail (~26 cheaper instances per wave)
  // ends the step -- config 3 at 65,536 12.2 -> 11.8 ms, at 16,384 5.5 -> 4.2 ms; small ones
  // (config 2 at 4,096: 2.0 vs 2.4 ms) keep the NC <= 128 class first.  Heavy-first relies on
  // the LDS slot padding of solve_group_kernel (cmpc_wave.hip kLdsSlot): without it the
  // NC <= 128 waves that replace the NC >= 160 ones fit ~6 instead of 8 per CU.
  // The NC 192 bin (rare: one instance in config 3's 65,536, but every instance of a standing
  // batch) has its own kernel in two launches on the same queue: a few waves (one per 4 CUs)
  // on the second plan stream, submitted before the classes so that they are dispatched before
  // the classes fill the SIMDs and the bin's instances start at the beginning of the step (a
  // one-wave-per-SIMD wave could not start later, with the SIMDs held by two-wave NC <= 128
  // waves); then the rest of the grid on the caller's stream once both classes are done, to
  // drain what the few waves have not taken.  An empty bin costs one dispatch of waves that
  // exit at once on an idle device, instead of 1,024 whole-SIMD waves that trickle in as the
  // classes free their SIMDs (a 5 ms span with 0 instances, round 4).
  const bool big = has_group(pl, 1), top = has_group(pl, 2);
  if (big) {
    if ((e = hipEventRecord(pl->fork, st)) != hipSuccess) return hip_fail(e, "hipEventRecord");
    if ((e = hipStreamWaitEvent(pl->side, pl->fork, 0)) != hipSuccess)
      return hip_fail(e, "hipStreamWaitEvent");
    if (top && (e = hipStreamWaitEvent(pl->top, pl->fork, 0)) != hipSuccess)
      return hip_fail(e, "hipStreamWaitEvent");
  }
  unsigned gk[kNumGroups];
  for (int k = 0; k < kNumGroups; ++k) gk[k] = (unsigned)(pl->grid[k] < B ? pl->grid[k] : B);
  const unsigned top_early = std::min(gk[2], (unsigned)std::max(1, pl->cus / 4));
  if (top) {
    rc = record_launch(pl, 2, pl->top, kp, in, out, top_early);
    if (rc != CMPC_OK) return rc;
  }
  const int64_t hmin = heavy_first_batch(pl);
  const int first = (big && hmin > 0 && B >= hmin) ? 1 : 0;  // class submitted first
  rc = record_launch(pl, first, st, kp, in, out, gk[first]);
  if (rc != CMPC_OK) return rc;
  if (big) {
    rc = record_launch(pl, 1 - first, pl->side, kp, in, out, gk[1 - first]);
    if (rc != CMPC_OK) return rc;
    if ((e = hipEventRecord(pl->join, pl->side)) != hipSuccess) return hip_fail(e, "hipEventRecord");
    if ((e = hipStreamWaitEvent(st, pl->join, 0)) != hipSuccess)
      return hip_fail(e, "hipStreamWaitEvent");
    if (top && gk[2] > top_early) {
      rc = record_launch(pl, 2, st, kp, in, out, gk[2] - top_early, top_early, false);
      if (rc != CMPC_OK) return rc;
    }
    if (top) {
      if ((e = hipEventRecord(pl->join_top, pl->top)) != hipSuccess) return hip_fail(e, "hipEventRecord");
      if ((e = hipStreamWaitEvent(st, pl->join_top, 0)) != hipSuccess)
        return hip_fail(e, "hipStreamWaitEvent");
    }
  }
  return CMPC_OK;
}

int cmpc_build_dynamics(cmpc_plan* pl, int64_t B, float dt, const float* mass,
                        const float* inertia, const float* r_feet, const float* xref, float* Ad,
                        float* Bd, float* gd, void* stream) {
  if (!pl) return fail(CMPC_E_INVALID, "cmpc_build_dynamics: null plan");
  if (int rc = check_device(pl, "cmpc_build_dynamics")) return rc;
  if (B < 0) return fail(CMPC_E_INVALID, "cmpc_build_dynamics: negative batch");
  if (!(dt > 0.f) || !std::isfinite(dt)) return fail(CMPC_E_INVALID, "cmpc_build_dynamics: dt must be > 0");
  if (B == 0) return CMPC_OK;
  if (!mass || !inertia || !r_feet || !xref || !Ad || !Bd || !gd)
    return fail(CMPC_E_INVALID, "cmpc_build_dynamics: null array argument");
  const long long cap = 8192;
  const long long blocks = B < cap ? B : cap;  // grid-stride: ~32 resident waves per CU
  hipLaunchKernelGGL(cmpc::dynamics_kernel, dim3((unsigned)blocks), dim3(64), 0,
                     (hipStream_t)stream, pl->kp.N, (double)dt, B, mass, inertia, r_feet, xref, Ad,
                     Bd, gd);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, "dynamics_kernel launch");
  return CMPC_OK;
}

int cmpc_generate_traj(cmpc_plan* pl, int64_t B, double dt, const float* x0, double* pos_des,
                       const float* cmd, const double* t_now, const double* gait,
                       const float* foot_lever, const float* hip, float* xref, uint8_t* contact,
                       float* r_feet, void* stream) {
  if (!pl) return fail(CMPC_E_INVALID, "cmpc_generate_traj: null plan");
  if (int rc = check_device(pl, "cmpc_generate_traj")) return rc;
  if (B < 0) return fail(CMPC_E_INVALID, "cmpc_generate_traj: negative batch");
  if (!(dt > 0.0) || !std::isfinite(dt)) return fail(CMPC_E_INVALID, "cmpc_generate_traj: dt must be > 0");
  if (B == 0) return CMPC_OK;
  if (!x0 || !pos_des || !cmd || !t_now || !gait || !foot_lever || !hip || !xref || !contact ||
      !r_feet)
    return fail(CMPC_E_INVALID, "cmpc_generate_traj: null array argument");
  const long long cap = 8192;
  // one wave per group of cmpc::kTrajGroup robots (grid-stride over groups)
  const long long groups = (B + cmpc::kTrajGroup - 1) / cmpc::kTrajGroup;
  const long long blocks = groups < cap ? groups : cap;
  hipLaunchKernelGGL(cmpc::traj_group_kernel, dim3((unsigned)blocks), dim3(64), 0,
                     (hipStream_t)stream, pl->kp.N, dt, B, x0, pos_des, cmd, t_now, gait,
                     foot_lever, hip, xref, contact, r_feet);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, "traj_group_kernel launch");
  return CMPC_OK;
}

int cmpc_leg_torque(cmpc_plan* pl, int64_t B, const double* t, const double* gait,
                    const float* force, int64_t force_stride, const double* J_foot,
                    const double* J_full, const double* M, const double* C, const double* g,
                    const double* dq, const double* Jdot_dq, const double* foot_pos,
                    const double* foot_vel, const double* body, const double* hip,
                    double* state, double tau_max, double* tau, void* stream) {
  if (!pl) return fail(CMPC_E_INVALID, "cmpc_leg_torque: null plan");
  if (int rc = check_device(pl, "cmpc_leg_torque")) return rc;
  if (B < 0) return fail(CMPC_E_INVALID, "cmpc_leg_torque: negative batch");
  if (force_stride < 12) return fail(CMPC_E_INVALID, "cmpc_leg_torque: force_stride must be >= 12");
  if (!std::isfinite(tau_max)) return fail(CMPC_E_INVALID, "cmpc_leg_torque: tau_max must be finite");
  if (B == 0) return CMPC_OK;
  if (!t || !gait || !force || !J_foot || !J_full || !M || !C || !g || !dq || !Jdot_dq ||
      !foot_pos || !foot_vel || !body || !hip || !state || !tau)
    return fail(CMPC_E_INVALID, "cmpc_leg_torque: null array argument");
  cmpc::LegArgs a{t, gait, force, force_stride, J_foot, J_full, M, C, g, dq, Jdot_dq, foot_pos,
                  foot_vel, body, hip, state, tau_max, tau};
  const long long blocks = B < 16384 ? B : 16384;  // grid-stride, one wave per robot
  hipLaunchKernelGGL(cmpc::leg_kernel, dim3((unsigned)blocks), dim3(64), 0, (hipStream_t)stream,
                     B, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, "leg_kernel launch");
  return CMPC_OK;
}

int cmpc_srb_step(cmpc_plan* pl, int64_t B, int nsub, double dt, const double* t_now,
                  const double* gait, const float* mass, const float* inertia_body,
                  const float* force, int64_t force_stride, const float* hip, float* x,
                  float* feet, uint8_t* contact_state, void* stream) {
  if (!pl) return fail(CMPC_E_INVALID, "cmpc_srb_step: null plan");
  if (int rc = check_device(pl, "cmpc_srb_step")) return rc;
  if (B < 0 || nsub < 0) return fail(CMPC_E_INVALID, "cmpc_srb_step: negative batch or nsub");
  if (!(dt > 0.0) || !std::isfinite(dt)) return fail(CMPC_E_INVALID, "cmpc_srb_step: dt must be > 0");
  if (force_stride < 12) return fail(CMPC_E_INVALID, "cmpc_srb_step: force_stride must be >= 12");
  if (B == 0 || nsub == 0) return CMPC_OK;
  if (!t_now || !gait || !mass || !inertia_body || !force || !hip || !x || !feet || !contact_state)
    return fail(CMPC_E_INVALID, "cmpc_srb_step: null array argument");
  const unsigned blocks = (unsigned)((B + 255) / 256);
  hipLaunchKernelGGL(cmpc::srb_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, B, nsub,
                     dt, t_now, gait, mass, inertia_body, force, force_stride, hip, x, feet,
                     contact_state);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, "srb_kernel launch");
  return CMPC_OK;
}

int cmpc_plan_set_timing(cmpc_plan* pl, int enable) {
  if (!pl) return fail(CMPC_E_INVALID, "cmpc_plan_set_timing: null plan");
  pl->timing = enable != 0;
  return CMPC_OK;
}

int cmpc_plan_set_team(cmpc_plan* pl, int64_t max_batch) {
  if (!pl) return fail(CMPC_E_INVALID, "cmpc_plan_set_team: null plan");
  if (max_batch < -1) return fail(CMPC_E_INVALID, "cmpc_plan_set_team: max_batch must be >= -1");
  pl->team_max_batch = max_batch;
  return CMPC_OK;
}

int cmpc_plan_team_batch(const cmpc_plan* pl, int64_t* max_batch) {
  if (!pl || !max_batch) return fail(CMPC_E_INVALID, "cmpc_plan_team_batch: null argument");
  *max_batch = team_batch(pl);
  return CMPC_OK;
}

int cmpc_plan_set_heavy_first(cmpc_plan* pl, int64_t min_batch) {
  if (!pl) return fail(CMPC_E_INVALID, "cmpc_plan_set_heavy_first: null plan");
  if (min_batch < -1) return fail(CMPC_E_INVALID, "cmpc_plan_set_heavy_first: min_batch must be >= -1");
  pl->heavy_first_min_batch = min_batch;
  return CMPC_OK;
}

int cmpc_plan_heavy_first_batch(const cmpc_plan* pl, int64_t* min_batch) {
  if (!pl || !min_batch) return fail(CMPC_E_INVALID, "cmpc_plan_heavy_first_batch: null argument");
  *min_batch = heavy_first_batch(pl);
  return CMPC_OK;
}

const char* cmpc_plan_solve_kernel(const cmpc_plan* pl, int64_t B, int k) {
  if (!pl || B < 1 || k < 0 || k >= kNumGroups) return nullptr;
  if (B <= team_batch(pl))
    return k != 0 ? nullptr : team_one_per_cu(pl, B) ? "solve_team_kernel<4, 1>" : "solve_team_kernel<4, 2>";
  if (!has_group(pl, k)) return nullptr;
  return group_name(k);
}

int cmpc_plan_timing_read(cmpc_plan* pl, float* ms_per_kernel, int32_t* calls_per_kernel) {
  if (!pl || !ms_per_kernel || !calls_per_kernel)
    return fail(CMPC_E_INVALID, "cmpc_plan_timing_read: null argument");
  for (int k = 0; k < kNumGroups; ++k) { ms_per_kernel[k] = 0.f; calls_per_kernel[k] = 0; }
  for (auto& r : pl->recs) {
    hipError_t e = hipEventSynchronize(r.b);
    if (e != hipSuccess) return hip_fail(e, "hipEventSynchronize");
    float ms = 0.f;
    e = hipEventElapsedTime(&ms, r.a, r.b);
    if (e != hipSuccess) return hip_fail(e, "hipEventElapsedTime");
    ms_per_kernel[r.group] += ms;
    calls_per_kernel[r.group] += 1;
    pl->pool.push_back(r);
  }
  pl->recs.clear();
  return CMPC_OK;
}

void cmpc_plan_destroy(cmpc_plan* pl) {
  if (!pl) return;
  for (auto& r : pl->recs) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
  for (auto& r : pl->pool) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
  if (pl->side) (void)hipStreamDestroy(pl->side);
  if (pl->top) (void)hipStreamDestroy(pl->top);
  if (pl->fork) (void)hipEventDestroy(pl->fork);
  if (pl->join) (void)hipEventDestroy(pl->join);
  if (pl->join_top) (void)hipEventDestroy(pl->join_top);
  (void)hipFree(pl->d_counters);
  (void)hipFree(pl->d_lists);
  (void)hipFree(pl->d_work);
  if (pl->d_stats) (void)hipFree(pl->d_stats);
  delete pl;
}

int cmpc_plan_stats(cmpc_plan* pl, uint64_t* out, int reset) {
  if (!pl || !out) return fail(CMPC_E_INVALID, "cmpc_plan_stats: null argument");
  if (int rc = check_device(pl, "cmpc_plan_stats")) return rc;
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return hip_fail(e, "hipDeviceSynchronize");
  // (on the plan's stream, not the null stream: see cmpc_plan_create)
  unsigned long long v[CMPC_NUM_STATS];
  if ((e = hipMemcpyAsync(v, pl->d_stats, sizeof(v), hipMemcpyDeviceToHost, pl->side)) != hipSuccess ||
      (reset && (e = hipMemsetAsync(pl->d_stats, 0, sizeof(v), pl->side)) != hipSuccess) ||
      (e = hipStreamSynchronize(pl->side)) != hipSuccess)
    return hip_fail(e, "cmpc_plan_stats copy");
  for (int i = 0; i < CMPC_NUM_STATS; ++i) out[i] = (uint64_t)v[i];
  return CMPC_OK;
}

#ifdef CMPC_STAMPS
// diagnostic build only: read and clear the per-phase cycle counters
int cmpc_debug_stamps(unsigned long long* out32) {
  hipError_t e = hipMemcpyFromSymbol(out32, HIP_SYMBOL(cmpc::g_stamps), 32 * sizeof(unsigned long long));
  if (e != hipSuccess) return hip_fail(e, "hipMemcpyFromSymbol");
  unsigned long long z[32] = {0};
  e = hipMemcpyToSymbol(HIP_SYMBOL(cmpc::g_stamps), z, sizeof(z));
  if (e != hipSuccess) return hip_fail(e, "hipMemcpyToSymbol");
  return CMPC_OK;
}
#endif

const char* cmpc_last_error(void) { return g_err.c_str(); }

const char* cmpc_version(void) { return "cmpc 1 gfx950"; }

}  // extern "C"
