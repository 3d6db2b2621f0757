// cmpc_wave.hip -- batched convex-MPC contact-force QP solver for MI355X (gfx950):
// ONE WAVEFRONT PER QP INSTANCE.
//
// Each 64-lane wave solves one QP of the reference's centroidal MPC
// (convex_mpc/centroidal_mpc.py:69-359) with no workgroup barrier anywhere: the workgroup is the
// wave, all cross-lane traffic is wave-ordered LDS or DPP, and a CU keeps 8 independent QPs in
// flight (2 per SIMD) so one QP's latency is hidden behind another's MFMA/VALU work.
// Algorithm (DESIGN.md "Kernel"):
//
//   1. Condense the horizon onto the free (stance) forces straight into register tiles:
//      H = sum_t G_t' Q2 G_t + diag(R) + shift with G_t = A G_{t-1} + (step t's new columns),
//      each product three v_mfma_f32_16x16x4_f32 (K = 12 states) whose accumulator is the
//      tile itself (condense_tiles_fwd); small batches use the block-row form
//      H_ij = C_i' A^{i-j} B_j, P_i = Q2 + A'P_{i+1}A (condense_tiles_bc).  Lane (g, c) holds
//      rows 4g..4g+3, column c of every lower-triangle 16x16 tile (f4 per tile, in registers).
//   2. Invert H + diag(R) + shift in registers by the BLOCK sweep operator, four pivots at a
//      time: S <- S - P^ D^-1 P^' (P^ = the four pivot columns with the pivot block minus I),
//      then -2 on the four pivot diagonals; the rank-4 update of each tile is ONE MFMA
//      (A = -Y rows, B = diag(1/dl) Y' columns, Y = P^ L^-T from the 4x4 LDL' of the pivot
//      block, factored redundantly per lane); pivot columns go through a 4-column LDS panel.
//   3. ADMM (OSQP iteration, A = I) on the free forces, lane t owning stance triple t
//      {fz >= fz_min, |fx| <= mu fz, |fy| <= mu fz} (closed-form projection).  Defect-correction
//      x-update x~ = x + M(rho(z - x) - grad f(x) - y): M (fp32 inverse) preconditions, grad f
//      comes from the error-coordinate rollout/adjoint (e_{k+1} = A e_k + B_k u_k + d_k).
//   4. Active-set polish once the face pattern is stable: reduced basis u = T v + t0, condense
//      + invert again (the ADMM inverse is parked in a per-wave global slab), refine with the
//      exact gradient, KKT check, primal-dual repairs of the face set.
//
// Instances are binned by free-variable count (NC in {96,128,160,192}, a multiple of 16);
// each bin runs a persistent kernel whose waves pull instance ids from a device-side queue.
//
// This file is compiled as part of cmpc_host.hip (single translation unit).
#include <hip/hip_runtime.h>
#include <stdint.h>


#include "cmpc_device.h"

namespace cmpc {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

// ------------------------------------------------------------------------------------------
// wave helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float readlane_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

// wave-uniform copy of a value the compiler cannot prove uniform (keeps branches scalar)
__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float uniformf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}

// v[l] and v[l ^ 32] (resp. v[l ^ 16]) without address registers (gfx950 permlane swaps):
// after the swap the two results hold the lane's own value and its partner's in some order
__device__ __forceinline__ void pair32(float v, float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  a = __int_as_float(r[0]);
  b = __int_as_float(r[1]);
}
__device__ __forceinline__ void pair16(float v, float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  a = __int_as_float(r[0]);
  b = __int_as_float(r[1]);
}

// max over the wave, result in every lane
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp<0xB1>(v));   // quad_perm [1,0,3,2]
  v = fmaxf(v, dpp<0x4E>(v));   // quad_perm [2,3,0,1]
  v = fmaxf(v, dpp<0x141>(v));  // row_half_mirror
  v = fmaxf(v, dpp<0x140>(v));  // row_mirror
  float a, b;
  pair32(v, a, b);
  v = fmaxf(a, b);
  pair16(v, a, b);
  return fmaxf(a, b);
}

// exclusive prefix sum of small non-negative counts (< 4) across the wave
__device__ __forceinline__ int wave_excl_scan4(int v) {
  const unsigned long long b0 = __ballot(v & 1), b1 = __ballot(v & 2);
  const int c0 = __builtin_amdgcn_mbcnt_hi((unsigned)(b0 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)b0, 0));
  const int c1 = __builtin_amdgcn_mbcnt_hi((unsigned)(b1 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)b1, 0));
  return c0 + 2 * c1;
}
__device__ __forceinline__ int wave_total4(int v) {
  return __popcll(__ballot(v & 1)) + 2 * __popcll(__ballot(v & 2));
}

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

typedef double d4 __attribute__((ext_vector_type(4)));

// 64-bit DPP move (two 32-bit moves; with bound_ctrl a lane past the row reads 0.0)
template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)(b & 0xffffffffll), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// sum over the 16 lanes of a DPP row (lanes with equal lane>>4), result in every lane
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror
  return v;
}

// sum over the 4 rows (lanes c, c+16, c+32, c+48), result in every lane
__device__ __forceinline__ float col4_sum(float v) {
  float a, b;
  pair32(v, a, b);
  pair16(a + b, a, b);
  return a + b;
}

// sum over the wave, result in every lane
__device__ __forceinline__ float wave_sum(float v) { return col4_sum(row16_sum(v)); }

// Lane id the compiler cannot see as loop invariant: every phase re-derives its lane-dependent
// addresses locally instead of the persistent loops hoisting them (and spilling them) for the
// whole instance.
__device__ __forceinline__ int opaque_lane() {
  int l = threadIdx.x & 63;
  asm volatile("" : "+v"(l));
  return l;
}

// Order LDS traffic between lanes of the wave: DS instructions of one wave execute in order,
// so only the compiler must not move memory operations across this point.
#define WSYNC() asm volatile("" ::: "memory")

// ------------------------------------------------------------------------------------------
// diagnostic build only (-DCMPC_STAMPS): per-phase s_memtime cycle totals.  Phases: 0 condense
// (+tile load), 1 invert, 2 gradient, 3 symv, 4 polish (all of it), 5 instance total,
// 6 setup, 7 ADMM iteration outside gradient/symv, 14 polish setup, 15 output (+final gradient),
// 28 face downdates (their symvs included); counters: 8 condense+invert calls, 9 polish
// attempts, 10 instances, 11 ADMM iterations, 12 gradient calls, 13 symv calls, 29 downdated
// repairs, 30 downdated faces (16-27: team-mode phases, cmpc_team.hip).
// ------------------------------------------------------------------------------------------
// diagnostic build only (-DCMPC_TRACE=id, or -DCMPC_TRACE_IDS=id,id,... to trace several
// instances inside a full batch): device printf of one instance's ADMM iterations, polish
// sessions, refinements and KKT checks, every line prefixed with the instance index
#if defined(CMPC_TRACE_IDS) && !defined(CMPC_TRACE)
#define CMPC_TRACE (-1)
#endif
#ifdef CMPC_TRACE
__device__ __forceinline__ bool trace_on(int64_t b) {
#ifdef CMPC_TRACE_IDS
  constexpr int64_t ids[] = {CMPC_TRACE_IDS};
  bool on = false;
  for (int64_t i : ids) on |= (b == i);
  return on;
#else
  return b == CMPC_TRACE;
#endif
}
#endif
#ifdef CMPC_STAMPS
__device__ unsigned long long g_stamps[32];
// (fenced: outstanding memory and LDS traffic completes, no code moves across a stamp; totals
// accumulate per wave in LDS, so no contended atomic sits between two stamps)
#define CMPC_FENCE()                                            \
  do {                                                          \
    __builtin_amdgcn_sched_barrier(0);                          \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); \
    __builtin_amdgcn_sched_barrier(0);                          \
  } while (0)
#define CMPC_T0(name) \
  CMPC_FENCE();       \
  const unsigned long long name = __builtin_amdgcn_s_memtime()
#define CMPC_ACC(ph, t0)                                                              \
  do {                                                                                \
    CMPC_FENCE();                                                                     \
    const unsigned long long _t1 = __builtin_amdgcn_s_memtime();                      \
    if (threadIdx.x == 0) s.st[ph] += _t1 - (t0);                                     \
  } while (0)
#define CMPC_CNT(ph, v) \
  do { if (threadIdx.x == 0) s.st[ph] += (unsigned long long)(v); } while (0)
#else
#define CMPC_T0(name) (void)0
#define CMPC_ACC(ph, t0) (void)0
#define CMPC_CNT(ph, v) (void)0
#endif

// ------------------------------------------------------------------------------------------
// geometry and LDS image of one instance
// ------------------------------------------------------------------------------------------
constexpr int kMaxN = 16;
constexpr int kMaxP = 12 * kMaxN;   // 192
constexpr int kMaxTri = 4 * kMaxN;  // 64 = lanes: lane t owns stance triple t

template <int NC>
struct Cfg {
  static_assert(NC % 16 == 0, "bin capacity must be a multiple of 16");
  static constexpr int TT = NC / 16;             // 16x16 tile rows
  static constexpr int NTL = TT * (TT + 1) / 2;  // lower-triangle tiles (f4 per lane each)
  static constexpr int THREADS = 64;             // one wave per QP
  // per wave (floats): park slab of the register tiles (inverse or LDL' factors)
  static constexpr int SLAB = NTL * 256;
  // registers: the inverse (4 NTL) + working set; two waves per SIMD where it fits in 256
  static constexpr int WPE = (4 * NTL <= 150) ? 2 : 1;
};

// Polish sessions and their face sets.  A session starts from ADMM's face set and repairs it
// (primal-dual active-set steps, one factorization each).  Two memories cut the factorizations
// that hard instances used to spend on cycling:
//  * within a session, a repair that returns to a face set the session already tried ends the
//    session (the repair sequence has entered a cycle);
//  * a session that ends on a face set whose KKT violations are all within kLooseTol x the
//    polish tolerance is accepted: a weakly active face at a degenerate vertex can leave every
//    face set a few 1e-5 relative off in fp32 (the two sets of the cycle straddle it), and
//    5e-5 is still tighter than ADMM's own eps 1e-4 stop;
//  * the starting sets of the last kFailMem failed sessions are remembered; ADMM's face set can
//    stay "stable" while still wrong, and a session that starts from a remembered set polishes
//    it once more (it may pass now, from ADMM's better iterate) but makes no repairs.
constexpr int kRefineExtra = 4;      // polish refinements beyond polish_refine ...
constexpr float kRefineRate = 0.5f;  // ... while each step shrinks at least this much
constexpr int kBackoffCap = 3;       // polish back-off doubles per failed session, up to 8x
constexpr int kLateRepairs = 3;      // repair budget of the sessions after two failed ones
// Damped repairs (round 3).  A full primal-dual active-set step changes every violated triple
// at once; on the slow instances the polished point then violates a different handful of
// triples and the repairs wander between neighbouring face sets (traced on the NumPy model:
// 34087 made 16 repairs over four sessions, each changing 2-8 triples, maximum relative
// violation 0.02-1.0 throughout).  From the third repair of a session, and in every session
// after a failed one, a repair changes only the most violated half of the triples it would
// change (at least kRepairTop).  The first two repairs stay full steps, so an easy instance that
// misses its first polish is untouched.  A/B in one gpurun call, two alternations: the N = 8
// shard rehearsal 3.87 -> 2.99 ms, N = 4 5.18 -> 4.24 ms, config 2 at 8,192 3.72 -> 2.57 ms,
// config 3 at 8,192 +8 %, config 2 at 65,536 +2 %, config 3 at 65,536 and config 2 at 4,096
// unchanged; a fixed 2 (without the half) lost 35 % on config 2 at 4,096, a fixed 3 gained
// nothing on the shards.
constexpr int kRepairTop = 2;
// After each failed session (up to kBackoffCap) the face set must stay unchanged 3x longer
// before the next session: a hard instance's later sessions then start from a settled ADMM
// iterate instead of re-polishing a set that is still moving (ADMM iterations cost ~1/12 of a
// factorization).  NumPy model: slowest config-3 instance -21 %.  A/B in one gpurun call (two
// alternations, with the interior-point fallback off): N = 8 shard rehearsal 2.75 -> 2.43 ms,
// config 3 at 16,384 3.90 -> 3.65 ms, at 8,192 +3 %, at 65,536 +1 %, config 2 unchanged.
constexpr int kStableGrow = 3;
// The NC >= 160 bins also start at rho0 / 2 (round 3; NumPy model: -2.6 % cost in those bins).
// A/B in one gpurun call, two alternations: config 3 at 65,536 11.43 -> 11.26 ms, config 2 at
// 65,536 14.05 -> 13.67 ms, at 4,096 2.05 -> 1.95 ms, N = 8 shard rehearsal 2.51 -> 2.38 ms.
constexpr bool kRhoLowHeavy = true;
constexpr int kFailMem = 4;
constexpr int kTryMem = 8;
constexpr float kLooseTol = 5.f;
// Face multipliers in force units (polish_check, nilpotent step with the float64 rollout): a
// held face's multiplier must be >= -kFaceErr x polish_tol x us x R2 (a force error of at most
// ~5e-5 relative once released); a loose acceptance allows kLooseFace x that
constexpr float kFaceErr = 2.f;
constexpr float kLooseFace = 2.5f;
// status 1: the held faces' certified force error |c|_2 / min R2 (certified_faces) is at
// most this fraction of the force scale; with the check's primal tolerance (polish_tol, x5 for a
// loose acceptance, = 5e-5) the returned forces are within ~1e-4 of the optimum
constexpr float kCertFace = 5e-5f;
// A check decided by a face multiplier within polish_tol x gs of zero is repeated after up to
// kAmbRefine more refinement steps (unless the step is already below kAmbConverged x the
// acceptance tolerance)
constexpr int kAmbRefine = 2;
constexpr float kAmbBand = 5.f;
constexpr float kAmbConverged = 1e-2f;
// After its first failed polish session an instance continues ADMM at kFailRho x rho0.  The
// slow instances are the ones whose repairs cycle between neighbouring face sets (a degenerate
// corner of the pyramid: fz at fz_min with friction faces weakly active, coupled over steps);
// a stiffer rho settles ADMM's face set closer to the optimum's before the next session.  NumPy
// model (tests/algo_spec.py) over 8,192 config-3 / config-2 instances: mean factorizations
// unchanged, the slowest instance 30 -> 17 (config 3) and 42 -> 26 (config 2) factorizations.
constexpr float kFailRho = 4.f;

// Stride of a param's column in Smem::Bt.  (An odd stride, 13, spreads the gradient's per-step
// column reads over more LDS banks -- 12 puts the 16 steps' columns of a trot on 4 -- but it
// loses the 16-byte loads elsewhere: -1..-6 % on every workload, A/B in one gpurun call.)
constexpr int kBS = 12;

template <int NC>
struct Smem {
#ifdef CMPC_STAMPS
  unsigned long long st[32];       // per-wave stamp totals (flushed to g_stamps at exit)
#endif
  alignas(16) float Bt[NC * kBS];  // param-space input matrix, column p at Bt[kBS p .. kBS p + 11]
  alignas(16) float Rt[NC];        // param-space input weight (2R in the param basis)
  alignas(16) float x[NC];
  alignas(16) float z[NC];
  alignas(16) float y[NC];         // ADMM dual (x, z, y of triple t at 3t .. 3t+2)
  alignas(16) float v[NC];
  union {  // buffers that are dead while the matrix is condensed share the G slab
    struct {
      alignas(16) float g[NC];
      alignas(16) float r[NC];
      alignas(16) float dl[NC];
      alignas(16) float ds[NC];        // unit-diagonal scaling of the sweep
      alignas(16) float pan[NC * 4];   // sweep panel: 4 pivot columns, row-major [row][4]
      float H[kMaxP];                  // h_k = B~_k v_k + d~_k
      float E[kMaxP];                  // e_{k+1} = x_{k+1} - xref_k
      float L[kMaxP];                  // lambda_k
    };
    alignas(16) float G[NC * 12];      // condensation: G_t column p = A^{t-k_p} b_p
  };
  float D[kMaxP];                  // d_k  (error-coordinate affine term)
  float Dt[kMaxP];                 // d~_k (d_k + B_k t0_k in the polish basis)
  float A[144];
  float Q2[12];                    // KParams copies (indexed at run time -> keep out of kernarg)
  float R2[12];
  int par[NC];                     // param -> step k
  int off[kMaxN + 1];              // first param of step k
  int nil;                         // A = I + N with N^2 = 0 (nilpotent_step): closed forms apply
  int tri[kMaxTri];                // stance triple t -> 4k + leg
  int tri_of[kMaxTri];             // 4k + leg -> triple index or -1
  int8_t tcnt[kMaxTri];            // polish: params of triple t / repaired face code
  int8_t code[kMaxTri];            // face code of triple t
  int8_t pcode[kMaxTri];           // face code of the previous ADMM iteration (-1: none)
  int fpk[kMaxTri];                // polish: params of triple t, px | py << 8 | pz << 16 (255 none)
  uint8_t fpat[kFailMem][kMaxTri]; // starting face sets of failed polish sessions
  uint8_t tpat[kTryMem][kMaxTri];  // face sets tried in the current session (0 = its start)
};

__device__ __forceinline__ constexpr int tile_index(int I, int J) { return (I * (I + 1)) / 2 + J; }

// ------------------------------------------------------------------------------------------
// condensation straight into the register tiles (MFMA)
// ------------------------------------------------------------------------------------------
// H = sum_t G_t' Q2 G_t + diag(Rt) + shift, where G_t (12 x n) column p is A^{t - k_p} b_p
// for k_p <= t and 0 otherwise (the prediction-matrix row block of step t).  G_t lives in
// REGISTERS as one accumulator tile per 16-column chunk (lane (g, c): states 4g..4g+3 of
// column 16 J + c), with the state index permuted k = 4g + q across the four MFMA steps so that
// an accumulator is directly the next product's B operand: G_{t+1} = A G_t is a chain of four
// MFMAs per chunk, and every lower tile (I, J) accumulates (Q2 G_t)_I' (G_t)_J with four MFMAs
// whose accumulator IS the matrix tile.  Tile row I starts to receive terms at the step of its
// first parameter; nothing of G ever goes through memory.
// + diag(Rt) + shift, identity on padding.  Only the diagonal tiles and the tile rows that reach
// the padding (a lower tile's padded columns imply padded rows) have anything to change: the
// interior off-diagonal tiles are skipped by a uniform test instead of testing every element.
template <int NC>
__device__ __forceinline__ void condense_finish(Smem<NC>& s, f4 (&M)[Cfg<NC>::NTL], int n,
                                                float shift) {
  using C = Cfg<NC>;
  const int lane = opaque_lane();
  const int g = lane >> 4, c = lane & 15;
#pragma unroll
  for (int I = 0; I < C::TT; ++I) {
#pragma unroll
    for (int J = 0; J <= I; ++J) {
      if (J != I && 16 * I + 16 <= n) continue;  // uniform: interior off-diagonal tile
      f4 v = M[tile_index(I, J)];
      const int col = 16 * J + c;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * I + 4 * g + q;
        if (row >= n || col >= n) v[q] = (row == col) ? 1.f : 0.f;
        else if (row == col) v[q] += s.Rt[row] + shift;
      }
      M[tile_index(I, J)] = v;
    }
  }
  WSYNC();
}

template <int NC>
__device__ __forceinline__ void condense_tiles_fwd(Smem<NC>& s, const KParams& P,
                                                   f4 (&M)[Cfg<NC>::NTL], int n, float shift) {
  using C = Cfg<NC>;
  const int lane = opaque_lane();
  const int g = lane >> 4, c = lane & 15;
  const int N = P.N;
  n = uniform(n);
#pragma unroll
  for (int t = 0; t < C::NTL; ++t) M[t] = f4{0.f, 0.f, 0.f, 0.f};
  // State layout: position (g, q) of a 16-row chunk holds state 3g + q for q < 3, and q = 3 is
  // padding in every lane group, so the fourth K = 4 slice of each product is all zeros and is
  // skipped: three MFMAs per product instead of four (K = 12 exactly).
  float aA[3], q2[3];  // A operand of A G: A[state(c)][3g + q]; Q2[3g + q]
  const int sc = ((c & 3) < 3) ? 3 * (c >> 2) + (c & 3) : -1;  // state of output row c
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int r = 3 * g + q;
    aA[q] = (sc >= 0) ? s.A[sc * 12 + r] : 0.f;
    q2[q] = s.Q2[r];
  }
  int kI[C::TT];  // first step of tile row I (N: no parameters)
#pragma unroll
  for (int I = 0; I < C::TT; ++I) kI[I] = (16 * I < n) ? s.par[16 * I] : N;
  f4 Gd[C::TT];
#pragma unroll
  for (int J = 0; J < C::TT; ++J) Gd[J] = f4{0.f, 0.f, 0.f, 0.f};
  for (int t = 0; t < N; ++t) {
    if (t > 0) {  // G_t = A G_{t-1} on the chunks that already hold columns
#pragma unroll
      for (int J = 0; J < C::TT; ++J) {
        if (kI[J] >= t) continue;  // uniform
        f4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 3; ++q) d = mfma4(aA[q], Gd[J][q], d);
        Gd[J] = d;
      }
    }
    // new columns b_p of step t (params off[t] .. off[t+1]-1; at most two chunks)
    const int p0 = s.off[t], p1 = s.off[t + 1];
#pragma unroll
    for (int J = 0; J < C::TT; ++J) {
      if (16 * J + 15 < p0 || 16 * J >= p1) continue;  // uniform
      const int p = 16 * J + c;
      if (p >= p0 && p < p1) {
        const float* bp = &s.Bt[p * kBS + 3 * g];
        Gd[J] = f4{bp[0], bp[1], bp[2], 0.f};
      }
    }
#pragma unroll
    for (int I = 0; I < C::TT; ++I) {
      if (kI[I] > t) continue;  // uniform: row block I has no column yet
      float a[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) a[q] = q2[q] * Gd[I][q];
#pragma unroll
      for (int J = 0; J <= I; ++J) {
        f4 acc = M[tile_index(I, J)];
#pragma unroll
        for (int q = 0; q < 3; ++q) acc = mfma4(a[q], Gd[J][q], acc);
        M[tile_index(I, J)] = acc;
      }
    }
  }
  condense_finish<NC>(s, M, n, shift);
}

// ---- software-pipelined sweep (bins up to kSweepPipeMaxNC; measured +3-5 % on NC = 128, and
// -5 % on cfg2 when also used for the 1-wave-per-SIMD bins, whose registers it spills) ----
constexpr int kSweepPipeMaxNC = 128;
// The next 4-pivot step reads only the tiles of its pivot row/column block ("critical" tiles).
// Each step issues its MFMAs on those tiles first, publishes the next panel from them, and then
// issues the remaining MFMAs of the step in the same basic block as the next step's LDL and
// operand build, so that serial chain fills the gaps between MFMAs instead of stalling the wave.
template <int NC, int K, class SM>
__device__ __forceinline__ void sweep_publish(SM& s, const f4 (&M)[Cfg<NC>::NTL], int sub,
                                              int g, int c) {
  using C = Cfg<NC>;
  const int c0 = 4 * sub;
  const int pc = c - c0;
  const bool colw = pc >= 0 && pc < 4;
  if (colw) {
#pragma unroll
    for (int I = K; I < C::TT; ++I) {
      f4 m = M[tile_index(I, K)];
      if (I == K) {
#pragma unroll
        for (int q = 0; q < 4; ++q) m[q] -= (4 * g + q == c) ? 1.f : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) s.pan[(16 * I + 4 * g + q) * 4 + pc] = m[q];
    }
  }
  // (the factorization never reads the swept rows above the block)
  WSYNC();
}

// LDL of the 4x4 pivot block (rows k0..k0+3 of the panel) and the step's MFMA operands
template <int NC, int KMIN, class SM>
__device__ __forceinline__ void sweep_operands(SM& s, int k0, int g, int c,
                                               float (&a)[Cfg<NC>::TT], float (&b)[Cfg<NC>::TT]) {
  using C = Cfg<NC>;
  float Dm[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f4 rrow = *reinterpret_cast<const f4*>(&s.pan[(k0 + i) * 4]);
#pragma unroll
    for (int j = 0; j < 4; ++j) Dm[i * 4 + j] = (i == j) ? rrow[j] + 1.f : rrow[j];
  }
  f4 ph[C::TT];
#pragma unroll
  for (int I = KMIN; I < C::TT; ++I) ph[I] = *reinterpret_cast<const f4*>(&s.pan[(16 * I + c) * 4]);
  // (inline: factored into a helper returning a struct, the compiler spilled an operand in
  // every sweep step, 28 scratch stores and loads in the NC <= 128 kernel)
  const bool g1 = g == 1, g2 = g == 2, g3 = g == 3;
  const float i0 = __builtin_amdgcn_rcpf(Dm[0]);
  const float l10 = Dm[4] * i0, l20 = Dm[8] * i0, l30 = Dm[12] * i0;
  const float i1 = __builtin_amdgcn_rcpf(Dm[5] - l10 * Dm[4]);
  const float u21 = Dm[9] - l20 * Dm[4], u31 = Dm[13] - l30 * Dm[4];
  const float l21 = u21 * i1, l31 = u31 * i1;
  const float i2 = __builtin_amdgcn_rcpf(Dm[10] - l20 * Dm[8] - l21 * u21);
  const float u32 = Dm[14] - l30 * Dm[8] - l31 * u21;
  const float l32 = u32 * i2;
  const float i3 = __builtin_amdgcn_rcpf(Dm[15] - l30 * Dm[12] - l31 * u31 - l32 * u32);
  const float n10 = -l10, n21 = -l21, n32 = -l32;
  const float n20 = l21 * l10 - l20, n31 = l32 * l21 - l31;
  const float n30 = -l30 - l31 * n10 - l32 * n20;
  const float w0 = g3 ? n30 : g2 ? n20 : g1 ? n10 : 1.f;
  const float w1 = g3 ? n31 : g2 ? n21 : g1 ? 1.f : 0.f;
  const float w2 = g3 ? n32 : g2 ? 1.f : 0.f;
  const float w3 = g3 ? 1.f : 0.f;
  const float ig = g3 ? i3 : g2 ? i2 : g1 ? i1 : i0;
#pragma unroll
  for (int I = KMIN; I < C::TT; ++I) {
    const float yg = fmaf(w3, ph[I][3], fmaf(w2, ph[I][2], fmaf(w1, ph[I][1], w0 * ph[I][0])));
    a[I] = -yg;
    b[I] = yg * ig;
  }
}

// rank-4 update of the tiles whose criticality for pivot block Kc is CRIT
template <int NC, int Kc, bool CRIT, int KMIN>
__device__ __forceinline__ void sweep_mfma(f4 (&M)[Cfg<NC>::NTL], const float (&a)[Cfg<NC>::TT],
                                           const float (&b)[Cfg<NC>::TT], int TA) {
  using C = Cfg<NC>;
#pragma unroll
  for (int I = KMIN; I < C::TT; ++I) {
    if (I >= TA) continue;  // uniform
#pragma unroll
    for (int J = KMIN; J <= I; ++J) {
      const bool crit = J == Kc && I >= Kc;
      if (crit != CRIT) continue;  // compile-time after unrolling
      const int t = tile_index(I, J);
      M[t] = mfma4(a[I], b[J], M[t]);
    }
  }
}

template <int NC, int K>
__device__ __forceinline__ void sweep_diagfix(f4 (&M)[Cfg<NC>::NTL], int sub, int g, int c) {
  const int pc = c - 4 * sub;
  const bool roww = g == sub;
  f4& m = M[tile_index(K, K)];
#pragma unroll
  for (int q = 0; q < 4; ++q) m[q] -= (roww && pc == q) ? 2.f : 0.f;
}

template <int NC, int K, class SM>
__device__ __forceinline__ void sweep_block(SM& s, f4 (&M)[Cfg<NC>::NTL], int ng, int TA,
                                            int g, int c, float (&a)[Cfg<NC>::TT],
                                            float (&b)[Cfg<NC>::TT]) {
  using C = Cfg<NC>;
  constexpr int KM = K;  // first tile column the block's steps update
  if constexpr (K < C::TT) {
    if (4 * K < ng) {  // uniform
      const int subs = (ng - 4 * K) < 4 ? (ng - 4 * K) : 4;
      for (int sub = 0; sub < subs - 1; ++sub) {  // next step in the same pivot block
        sweep_mfma<NC, K, true, KM>(M, a, b, TA);
        sweep_diagfix<NC, K>(M, sub, g, c);
        sweep_publish<NC, K>(s, M, sub + 1, g, c);
        sweep_mfma<NC, K, false, KM>(M, a, b, TA);
        sweep_operands<NC, KM>(s, 16 * K + 4 * (sub + 1), g, c, a, b);
      }
      {  // last step of the block: the next step opens block K + 1
        const int sub = subs - 1;
        const bool has_next = 4 * (K + 1) < ng;
        sweep_mfma<NC, K + 1, true, KM>(M, a, b, TA);
        if constexpr (K + 1 < C::TT) {
          if (has_next) sweep_publish<NC, K + 1>(s, M, 0, g, c);
        }
        sweep_mfma<NC, K + 1, false, KM>(M, a, b, TA);
        sweep_diagfix<NC, K>(M, sub, g, c);
        if constexpr (K + 1 < C::TT) {
          if (has_next) sweep_operands<NC, K + 1>(s, 16 * (K + 1), g, c, a, b);
        }
      }
    }
    sweep_block<NC, K + 1>(s, M, ng, TA, g, c, a, b);
  }
}

// Block-row condensation: the lower blocks of the same H are
//   H[rows of step i, cols of step j <= i] = C_i' A^{i-j} B_j,   C_i = P_i B_i,
//   P_i = sum_{t >= i} (A^{t-i})' Q2 A^{t-i} = Q2 + A' P_{i+1} A,
// so step i only adds its own 1-2 tile rows (C_i' G_i, G_i = [A^{i-j} B_j]_{j <= i} as above)
// instead of every active tile: ~25 % fewer MFMAs at n = 120.  A backward pass builds P_i in one
// accumulator tile (A' P A: eight MFMAs; P is symmetric, so its accumulator layout is also its
// A-operand layout) and stores C_i, param-major, in the G slab.  Diagonal tiles then receive
// only the entries whose column step <= row step; the others are mirrored across.
template <int NC>
__device__ __forceinline__ void condense_tiles_bc(Smem<NC>& s, const KParams& P,
                                                  f4 (&M)[Cfg<NC>::NTL], int n, float shift) {
  using C = Cfg<NC>;
  const int lane = opaque_lane();
  const int g = lane >> 4, c = lane & 15;
  const int N = P.N;
  n = uniform(n);
#pragma unroll
  for (int t = 0; t < C::NTL; ++t) M[t] = f4{0.f, 0.f, 0.f, 0.f};
  // K = 12 state layout (as condense_tiles_fwd): accumulator position 4g + q holds state 3g + q
  // for q < 3 and is padding for q = 3, so every product over the states is three MFMAs
  const int sc = ((c & 3) < 3) ? 3 * (c >> 2) + (c & 3) : -1;
  float aA[3], aT[3];  // A[sc][3g + q] (A operand of A X), A[3g + q][sc] (of A' X)
  f4 q2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int r = 3 * g + q;
    aA[q] = (sc >= 0) ? s.A[sc * 12 + r] : 0.f;
    aT[q] = (sc >= 0) ? s.A[r * 12 + sc] : 0.f;
    q2[q] = (r == sc) ? s.Q2[r] : 0.f;
  }
  float* Cs = s.G;  // C_i columns, param-major [p][12] (the G slab is free while condensing)
  // ---- backward: P_i and C_i = P_i B_i for i = N-1 .. 0 ----
  f4 Pt = q2;  // P_{N-1} = Q2 (diagonal)
  WSYNC();
  for (int i = N - 1; i >= 0; --i) {
    const int p0 = s.off[i], p1 = s.off[i + 1];
#pragma unroll
    for (int J = 0; J < C::TT; ++J) {
      if (16 * J + 15 < p0 || 16 * J >= p1) continue;  // uniform: chunks holding step i's params
      const int p = 16 * J + c;
      float bt[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) bt[q] = (p < n) ? s.Bt[p * kBS + 3 * g + q] : 0.f;
      f4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 3; ++q) d = mfma4(Pt[q], bt[q], d);  // C = P B (P symmetric)
      if (p >= p0 && p < p1) {
#pragma unroll
        for (int q = 0; q < 3; ++q) Cs[p * 12 + 3 * g + q] = d[q];
      }
    }
    if (i > 0) {  // P_{i-1} = Q2 + A' P_i A
      f4 y = {0.f, 0.f, 0.f, 0.f}, z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 3; ++q) y = mfma4(Pt[q], aT[q], y);   // Y = P A
#pragma unroll
      for (int q = 0; q < 3; ++q) z = mfma4(aT[q], y[q], z);    // Z = A' Y
#pragma unroll
      for (int q = 0; q < 4; ++q) Pt[q] = z[q] + q2[q];
    }
  }
  WSYNC();
  // ---- forward: G_t = A G_{t-1} + new columns; rows of step t += C_t' G_t ----
  int kI[C::TT];
#pragma unroll
  for (int I = 0; I < C::TT; ++I) kI[I] = (16 * I < n) ? s.par[16 * I] : N;
  f4 Gd[C::TT];
#pragma unroll
  for (int J = 0; J < C::TT; ++J) Gd[J] = f4{0.f, 0.f, 0.f, 0.f};
  for (int t = 0; t < N; ++t) {
    if (t > 0) {
#pragma unroll
      for (int J = 0; J < C::TT; ++J) {
        if (kI[J] >= t) continue;  // uniform
        f4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 3; ++q) d = mfma4(aA[q], Gd[J][q], d);
        Gd[J] = d;
      }
    }
    const int p0 = s.off[t], p1 = s.off[t + 1];
#pragma unroll
    for (int J = 0; J < C::TT; ++J) {
      if (16 * J + 15 < p0 || 16 * J >= p1) continue;  // uniform
      const int p = 16 * J + c;
      if (p >= p0 && p < p1) {
        const float* bp = &s.Bt[p * kBS + 3 * g];
        Gd[J] = f4{bp[0], bp[1], bp[2], 0.f};
      }
    }
#pragma unroll
    for (int I = 0; I < C::TT; ++I) {
      if (16 * I + 15 < p0 || 16 * I >= p1) continue;  // uniform: tile rows holding step t
      const int p = 16 * I + c;
      float a[3] = {0.f, 0.f, 0.f};
      if (p >= p0 && p < p1) {
#pragma unroll
        for (int q = 0; q < 3; ++q) a[q] = Cs[p * 12 + 3 * g + q];
      }
#pragma unroll
      for (int J = 0; J <= I; ++J) {
        f4 acc = M[tile_index(I, J)];
#pragma unroll
        for (int q = 0; q < 3; ++q) acc = mfma4(a[q], Gd[J][q], acc);
        M[tile_index(I, J)] = acc;
      }
    }
  }
  // ---- diagonal tiles: entry (r, c) with step(c) > step(r) is the mirror of (c, r) ----
  WSYNC();
  float* T = s.G;  // 16 x 16 scratch per tile
#pragma unroll
  for (int I = 0; I < C::TT; ++I) {
    if (16 * I >= n) continue;  // uniform
    f4 v = M[tile_index(I, I)];
#pragma unroll
    for (int q = 0; q < 4; ++q) T[(4 * g + q) * 16 + c] = v[q];
    WSYNC();
    const int pc = 16 * I + c;
    const int kc = (pc < n) ? s.par[pc] : N;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int pr = 16 * I + 4 * g + q;
      const int kr = (pr < n) ? s.par[pr] : N;
      if (kc > kr) v[q] = T[c * 16 + 4 * g + q];
    }
    M[tile_index(I, I)] = v;
    WSYNC();
  }
  condense_finish<NC>(s, M, n, shift);
}

// Closed-form condensation for a nilpotent step matrix (round 4).  The reference discretises a
// nilpotent Ac (Ac^2 = 0: its only blocks map velocity to position and omega to the Euler
// rates), so its zero-order hold is exactly A = I + N with N = Ac dt and N^2 = 0
// (com_trajectory.py:272-286; cmpc_build_dynamics).  Then A^j = I + j N and the
// prediction column of param p (step k_p) at step t >= k_p is affine in t:
//     A^{t - k_p} b_p = U_p + t V_p,   V_p = N b_p,   U_p = b_p - k_p V_p,
// so  H[p][p'] = sum_{t >= m} (U_p + t V_p)' Q2 (U_p' + t V_p'),  m = max(k_p, k_p'),
//              = X_p' U_p' + Y_p' V_p'   with   X_p = Q2 (S0 U_p + S1 V_p),
//                                               Y_p = Q2 (S1 U_p + S2 V_p),
// S_i = sum_{t=m}^{N-1} t^i, whenever m = k_p (the row param's step).  Params are ordered by
// step, so that holds for every entry of an off-diagonal tile (rows later than columns) and for
// the lower part of a diagonal tile; the rest of a diagonal tile is mirrored, as in the
// block-row form.  Every tile is then SIX MFMAs (two K = 12 products, 3 each) instead of the
// three per active step of the forward form: ~240 MFMAs for n = 120 instead of 1,248 (936 in
// the block-row form), with V = N b three MFMAs per 16-param chunk, parked in the G slab.  fp32
// error on the fixture matrices (unit-diagonal scaled, vs float64): 2.6e-7 against 4.1e-7 for
// the step-by-step products.  The solve checks N^2 = 0 exactly per instance (nilpotent_step);
// any other A takes the general forms above.
// Sums over the horizon's remaining steps t = k .. N-1 of 1, t and t^2 (condense_tiles_nil), as
// exact integers
__device__ __forceinline__ void step_sums(int k, int N, float& S0, float& S1, float& S2) {
  S0 = (float)(N - k);
  S1 = (float)((N * (N - 1) - k * (k - 1)) >> 1);
  S2 = (float)(((N - 1) * N * (2 * N - 1) - (k - 1) * k * (2 * k - 1)) / 6);
}

template <int NC>
__device__ __forceinline__ void condense_tiles_nil(Smem<NC>& s, const KParams& P,
                                                   f4 (&M)[Cfg<NC>::NTL], int n, float shift) {
  using C = Cfg<NC>;
  const int lane = opaque_lane();
  const int g = lane >> 4, c = lane & 15;
  const int N = P.N;
  n = uniform(n);
  const int TA = (n + 15) >> 4;
#pragma unroll
  for (int t = 0; t < C::NTL; ++t) M[t] = f4{0.f, 0.f, 0.f, 0.f};
  float* Vs = s.G;  // V = N b, param-major [p][12] (the G slab is free while condensing)
  {
    // K = 12 state layout (as condense_tiles_fwd): accumulator position 4g + q holds state 3g + q
    const int sc = ((c & 3) < 3) ? 3 * (c >> 2) + (c & 3) : -1;
    float aN[3];  // A operand of N X: N[sc][3g + q]
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int r = 3 * g + q;
      aN[q] = (sc >= 0) ? s.A[sc * 12 + r] - ((sc == r) ? 1.f : 0.f) : 0.f;
    }
    WSYNC();
#pragma unroll
    for (int J = 0; J < C::TT; ++J) {
      if (J >= TA) continue;  // uniform
      const int p = 16 * J + c;
      float bt[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) bt[q] = (p < n) ? s.Bt[p * kBS + 3 * g + q] : 0.f;
      f4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 3; ++q) d = mfma4(aN[q], bt[q], d);
#pragma unroll
      for (int q = 0; q < 3; ++q) Vs[p * 12 + 3 * g + q] = d[q];
    }
  }
  WSYNC();
  float q2[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) q2[q] = s.Q2[3 * g + q];
  // the column operands (u, v) of every chunk, once: each is reused by every tile row below it
  // (loaded per tile instead: 7 LDS reads between every tile's MFMAs; caching them took config 3
  // 9.09 -> 8.60 ms, config 2 at 65,536 10.55 -> 9.99 ms, A/B in one gpurun call)
  float uc[C::TT][3], vc[C::TT][3];
#pragma unroll
  for (int J = 0; J < C::TT; ++J) {
    const int p = 16 * J + c;
    const bool ok = J < TA && p < n;
    const float kf = ok ? (float)s.par[p] : 0.f;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      vc[J][q] = ok ? Vs[p * 12 + 3 * g + q] : 0.f;
      uc[J][q] = ok ? fmaf(-kf, vc[J][q], s.Bt[p * kBS + 3 * g + q]) : 0.f;
    }
  }
#pragma unroll
  for (int I = 0; I < C::TT; ++I) {
    if (I >= TA) continue;  // uniform
    float x[3], y[3];
    {
      const int p = 16 * I + c;
      const bool ok = p < n;
      const int k = ok ? s.par[p] : 0;
      const float kf = (float)k;
      float S0, S1, S2;  // sum_{t=k}^{N-1} 1, t, t^2
      step_sums(k, N, S0, S1, S2);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const float v = ok ? Vs[p * 12 + 3 * g + q] : 0.f;
        const float u = ok ? fmaf(-kf, v, s.Bt[p * kBS + 3 * g + q]) : 0.f;
        x[q] = q2[q] * fmaf(S0, u, S1 * v);
        y[q] = q2[q] * fmaf(S1, u, S2 * v);
      }
    }
#pragma unroll
    for (int J = 0; J <= I; ++J) {
      float u[3], v[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        u[q] = uc[J][q];
        v[q] = vc[J][q];
      }
      f4 acc = M[tile_index(I, J)];
#pragma unroll
      for (int q = 0; q < 3; ++q) acc = mfma4(x[q], u[q], acc);
#pragma unroll
      for (int q = 0; q < 3; ++q) acc = mfma4(y[q], v[q], acc);
      M[tile_index(I, J)] = acc;
    }
  }
  // diagonal tiles: entry (r, c) with step(c) > step(r) is the mirror of (c, r)
  WSYNC();
  float* T = s.G;  // 16 x 16 scratch per tile (V is dead)
#pragma unroll
  for (int I = 0; I < C::TT; ++I) {
    if (I >= TA) continue;  // uniform
    f4 v = M[tile_index(I, I)];
#pragma unroll
    for (int q = 0; q < 4; ++q) T[(4 * g + q) * 16 + c] = v[q];
    WSYNC();
    const int pc = 16 * I + c;
    const int kc = (pc < n) ? s.par[pc] : N;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int pr = 16 * I + 4 * g + q;
      const int kr = (pr < n) ? s.par[pr] : N;
      if (kc > kr) v[q] = T[c * 16 + 4 * g + q];
    }
    M[tile_index(I, I)] = v;
    WSYNC();
  }
  condense_finish<NC>(s, M, n, shift);
}

// Is the step matrix A = I + N with N^2 = 0 exactly (the reference's discretisation)?  Then
// condense_tiles_nil applies.  Uniform.
template <class SM>
__device__ __forceinline__ bool nilpotent_step(SM& s) {
  const int lane = opaque_lane();
  WSYNC();
  bool nz = false;
#pragma unroll
  for (int e0 = 0; e0 < 144; e0 += 64) {
    const int e = e0 + lane;
    if (e < 144) {
      const int i = e / 12, j = e % 12;
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 12; ++k) {
        const float nik = s.A[i * 12 + k] - ((i == k) ? 1.f : 0.f);
        const float nkj = s.A[k * 12 + j] - ((k == j) ? 1.f : 0.f);
        acc = fmaf(nik, nkj, acc);
      }
      nz |= acc != 0.f;
    }
  }
  return __any(nz) == 0;
}

// Which condensation: the closed form for a nilpotent step (nil); otherwise the block-row form
// has ~25 % fewer MFMAs but longer dependency chains.  With one wave per SIMD (small batches,
// latency) the chains are what a wave waits on either way and the fewer MFMAs win (B = 256:
// 0.61 -> 0.48 ms); with two busy waves per SIMD the forward form keeps the matrix pipe ~80 %
// busy and is ~5 % faster (tools/phase_bench.hip).
template <int NC>
__device__ __forceinline__ void condense_tiles(Smem<NC>& s, const KParams& P,
                                               f4 (&M)[Cfg<NC>::NTL], int n, float shift,
                                               bool nil = false) {
  if (nil) {  // uniform
    condense_tiles_nil<NC>(s, P, M, n, shift);
    return;
  }
  if constexpr (NC <= 128) {  // the 1-wave-per-SIMD bins would spill the second form
    if (P.latency_mode) {  // uniform
      condense_tiles_bc<NC>(s, P, M, n, shift);
      return;
    }
  }
  condense_tiles_fwd<NC>(s, P, M, n, shift);
}

// ------------------------------------------------------------------------------------------
// block LDL' factorization by the sweep operator (4 pivots per step, MFMA rank-4 updates)
// ------------------------------------------------------------------------------------------
// The symmetric sweep restricted to the tiles right of the swept pivots (round 5; rounds 1-4
// swept every tile into the explicit inverse): a block LDL' factorization with 16-pivot blocks,
// 4 T(TT - K) MFMAs per block K instead of 4 NTL (T(m) = m (m + 1) / 2: 480 instead of 1,152 for
// NC = 128).  Sweeping block K on rows / columns >= 16 K leaves -D_K^-1 in tile (K, K) (D_K the
// Schur-complemented pivot block), L_IK = H_IK D_K^-1 in the tiles below it, and the Schur
// complement to its right; unscaled, tile (K, K) holds D_K^-1 and tiles (I > J) the unit
// block-lower L of H = L D L' (applied by ldl_apply).
template <int NC, class SM>
__device__ __forceinline__ void ldl_tiles(SM& s, f4 (&M)[Cfg<NC>::NTL], int n) {
  using C = Cfg<NC>;
  const int lane = opaque_lane();
  const int g = lane >> 4, c = lane & 15;
  n = uniform(n);
  const int TA = (n + 15) >> 4;
  // unit-diagonal scaling (padding: 1)
#pragma unroll
  for (int I = 0; I < C::TT; ++I) {
    const f4 d = M[tile_index(I, I)];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int p = 16 * I + c;
      if (4 * g + q == c) s.ds[p] = (p < n && d[q] > 0.f) ? rsqrtf(d[q]) : 1.f;
    }
  }
  WSYNC();
#pragma unroll
  for (int I = 0; I < C::TT; ++I) {
    const f4 ri = *reinterpret_cast<const f4*>(&s.ds[16 * I + 4 * g]);
#pragma unroll
    for (int J = 0; J <= I; ++J) {
      const float cj = s.ds[16 * J + c];
      f4& m = M[tile_index(I, J)];
#pragma unroll
      for (int q = 0; q < 4; ++q) m[q] *= ri[q] * cj;
    }
  }
  const int ng = (n + 3) >> 2;
  if constexpr (NC <= kSweepPipeMaxNC) {
    if (ng > 0) {
      float a[C::TT], b[C::TT];
      sweep_publish<NC, 0>(s, M, 0, g, c);
      sweep_operands<NC, 0>(s, 0, g, c, a, b);
      sweep_block<NC, 0>(s, M, ng, TA, g, c, a, b);
    }
  } else {
  const bool g1 = g == 1, g2 = g == 2, g3 = g == 3;
  // The pivot-block column K is a compile-time constant of the outer (unrolled) loop, so the
  // panel publish, the P^ identity and the diagonal fix address their tiles directly (no
  // runtime dispatch over register tiles); the four 4-pivot steps inside a tile column are a
  // runtime loop.
#pragma unroll
  for (int K = 0; K < C::TT; ++K) {
    if (4 * K >= ng) continue;  // uniform; `continue` keeps the unrolled loop's tiles static
    const int subs = (ng - 4 * K) < 4 ? (ng - 4 * K) : 4;
    for (int sub = 0; sub < subs; ++sub) {
      const int c0 = 4 * sub, k0 = 16 * K + c0;
      const int pc = c - c0;
      const bool colw = pc >= 0 && pc < 4, roww = g == sub;
      // publish the 4 pivot columns (P^ = P - I on the pivot rows) as panel rows [row][0..3]
      // from tiles (I >= K, K) (the factorization never reads the swept rows above the block)
      if (colw) {
#pragma unroll
        for (int I = K; I < C::TT; ++I) {
          f4 m = M[tile_index(I, K)];
          if (I == K) {
#pragma unroll
            for (int q = 0; q < 4; ++q) m[q] -= (4 * g + q == c) ? 1.f : 0.f;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) s.pan[(16 * I + 4 * g + q) * 4 + pc] = m[q];
        }
      }
      WSYNC();
      // D = L diag(dl) L' (unit lower L), so P^ D^-1 P^' = Y diag(1/dl) Y' with Y = P^ L^-T: the
      // columns of Y are the pivot columns as the scalar sweep would see them (each already
      // eliminated by the earlier pivots of the step), which keeps the scalar sweep's accuracy.
      float Dm[16];  // the panel holds P^ = P - I: add the identity back for D
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f4 rrow = *reinterpret_cast<const f4*>(&s.pan[(k0 + i) * 4]);
#pragma unroll
        for (int j = 0; j < 4; ++j) Dm[i * 4 + j] = (i == j) ? rrow[j] + 1.f : rrow[j];
      }
      const float i0 = __builtin_amdgcn_rcpf(Dm[0]);
      const float l10 = Dm[4] * i0, l20 = Dm[8] * i0, l30 = Dm[12] * i0;
      const float i1 = __builtin_amdgcn_rcpf(Dm[5] - l10 * Dm[4]);
      const float u21 = Dm[9] - l20 * Dm[4], u31 = Dm[13] - l30 * Dm[4];
      const float l21 = u21 * i1, l31 = u31 * i1;
      const float i2 = __builtin_amdgcn_rcpf(Dm[10] - l20 * Dm[8] - l21 * u21);
      const float u32 = Dm[14] - l30 * Dm[8] - l31 * u21;
      const float l32 = u32 * i2;
      const float i3 = __builtin_amdgcn_rcpf(Dm[15] - l30 * Dm[12] - l31 * u31 - l32 * u32);
      // y_g = (P^ L^-T)_g = sum_m L^-1[g][m] P^_m: this lane's row of L^-1 (unit lower) and
      // 1/dl_g, selected once per step, so each panel row costs four FMAs and no branches
      const float n10 = -l10, n21 = -l21, n32 = -l32;
      const float n20 = l21 * l10 - l20, n31 = l32 * l21 - l31;
      const float n30 = -l30 - l31 * n10 - l32 * n20;
      const float w0 = g3 ? n30 : g2 ? n20 : g1 ? n10 : 1.f;
      const float w1 = g3 ? n31 : g2 ? n21 : g1 ? 1.f : 0.f;
      const float w2 = g3 ? n32 : g2 ? 1.f : 0.f;
      const float w3 = g3 ? 1.f : 0.f;
      const float ig = g3 ? i3 : g2 ? i2 : g1 ? i1 : i0;
      const int KM = K;  // (a constant once the K loop is unrolled)
      float a[C::TT], b[C::TT];
#pragma unroll
      for (int I = KM; I < C::TT; ++I) {
        const f4 ph = *reinterpret_cast<const f4*>(&s.pan[(16 * I + c) * 4]);
        const float yg = fmaf(w3, ph[3], fmaf(w2, ph[2], fmaf(w1, ph[1], w0 * ph[0])));
        a[I] = -yg;
        b[I] = yg * ig;
      }
#pragma unroll
      for (int I = KM; I < C::TT; ++I) {
        if (I >= TA) continue;  // uniform
#pragma unroll
        for (int J = KM; J <= I; ++J) {
          const int t = tile_index(I, J);
          M[t] = mfma4(a[I], b[J], M[t]);
        }
      }
      {  // -2 on the 4 pivot diagonals
        f4& m = M[tile_index(K, K)];
#pragma unroll
        for (int q = 0; q < 4; ++q) m[q] -= (roww && pc == q) ? 2.f : 0.f;
      }
    }
  }
  }
  // undo the scaling: the diagonal tiles hold -(scaled D_K^-1), the tiles below them the
  // scaled L~ = S^-1 L S
#pragma unroll
  for (int I = 0; I < C::TT; ++I) {
    const f4 ri = *reinterpret_cast<const f4*>(&s.ds[16 * I + 4 * g]);
    f4 rinv;
#pragma unroll
    for (int q = 0; q < 4; ++q) rinv[q] = 1.f / ri[q];
#pragma unroll
    for (int J = 0; J <= I; ++J) {
      const float cj = s.ds[16 * J + c];
      f4& m = M[tile_index(I, J)];
#pragma unroll
      for (int q = 0; q < 4; ++q) m[q] *= (J < I) ? rinv[q] * cj : -(ri[q] * cj);
    }
  }
}

// out = (L D L')^-1 in over the first n params (factors from ldl_tiles; out is
// zero beyond n): z = L^-1 in block row by block row (row sums over the block's columns), then
// x = L'^-1 D^-1 z from the last block row up (column sums over the row's 4-lane groups); each
// block's result turns layout (rows <-> columns) through `out`, which holds z, then x.
template <int NC, class SM>
__device__ __forceinline__ void ldl_apply(SM& s, const f4 (&M)[Cfg<NC>::NTL], int n,
                                          const float* in, float* out) {
  using C = Cfg<NC>;
  CMPC_T0(t_sv);
  const int lane = opaque_lane();
  const int g = lane >> 4, c = lane & 15;
  n = uniform(n);
  const int TA = (n + 15) >> 4;
  WSYNC();
  float zc[C::TT];  // z by block, column layout (lane c: z[16 J + c])
  // backward accumulators (column layout, per lane before the 4-group sum): sum_J L_JI' x_J
  // as each x_J is known
  float bc[C::TT];
#pragma unroll
  for (int I = 0; I < C::TT; ++I) bc[I] = 0.f;
#pragma unroll
  for (int I = 0; I < C::TT; ++I) {
    if (I >= TA) {  // padding rows: zero (uniform branch)
      if (c == 0) *reinterpret_cast<f4*>(&out[16 * I + 4 * g]) = f4{0.f, 0.f, 0.f, 0.f};
      continue;
    }
    f4 zr = *reinterpret_cast<const f4*>(&in[16 * I + 4 * g]);
    if (I > 0) {
      f2 r01 = {0.f, 0.f}, r23 = {0.f, 0.f};
#pragma unroll
      for (int J = 0; J < I; ++J) {
        const f4 m = M[tile_index(I, J)];
        const f2 zj = {zc[J], zc[J]};
        r01 = __builtin_elementwise_fma(f2{m[0], m[1]}, zj, r01);
        r23 = __builtin_elementwise_fma(f2{m[2], m[3]}, zj, r23);
      }
      zr[0] -= row16_sum(r01[0]);
      zr[1] -= row16_sum(r01[1]);
      zr[2] -= row16_sum(r23[0]);
      zr[3] -= row16_sum(r23[1]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) zr[q] = (16 * I + 4 * g + q < n) ? zr[q] : 0.f;
    // the block turns from rows to columns through `out` (a register turn -- DPP / permlane
    // swaps -- measured 1.3 % slower with this arithmetic, round 5)
    if (c == 0) *reinterpret_cast<f4*>(&out[16 * I + 4 * g]) = zr;
    WSYNC();
    zc[I] = out[16 * I + c];
  }
  // backward: x_I = D_I^-1 z_I - sum_{J > I} L_JI' x_J
#pragma unroll
  for (int I = C::TT - 1; I >= 0; --I) {
    if (I >= TA) continue;  // uniform
    const f4 zr = *reinterpret_cast<const f4*>(&out[16 * I + 4 * g]);
    const f4 d = M[tile_index(I, I)];
    const float t =
        fmaf(d[3], zr[3], fmaf(d[2], zr[2], fmaf(d[1], zr[1], fmaf(d[0], zr[0], -bc[I]))));
    float xc = col4_sum(t);
    xc = (16 * I + c < n) ? xc : 0.f;
    WSYNC();
    if (g == 0) out[16 * I + c] = xc;
    if (I == 0) break;
    WSYNC();
    const f4 xr = *reinterpret_cast<const f4*>(&out[16 * I + 4 * g]);
#pragma unroll
    for (int J = 0; J < I; ++J) {
      const f4 m = M[tile_index(I, J)];
      bc[J] = fmaf(m[3], xr[3], fmaf(m[2], xr[2], fmaf(m[1], xr[1], fmaf(m[0], xr[0], bc[J]))));
    }
  }
  WSYNC();
  CMPC_ACC(3, t_sv);
  CMPC_CNT(13, 1);
}

// Gradient of sum_k e_{k+1}'(Q2/2)e_{k+1} + v'(Rt/2)v in the current param basis
// (e by the error-coordinate rollout).  Leaves E (e_{k+1}) and L (lambda_k) in LDS.
//
// Both recursions run as log-depth scans on the matrix cores, the 12 x N state trajectory
// held as ONE accumulator tile (lane (g, c): states 4g..4g+3 of step c):
//   forward  e_{k+1} = sum_j A^{k-j} h_j :   E <- E + A^d shift_d(E),      d = 1, 2, 4, 8
//   adjoint  lambda_k = sum_j (A')^{j-k} Q2 e_{j+1} : L <- L + (A')^d shift_-d(L)
// (Hillis-Steele; the step shift is a DPP row shift, the product three MFMAs whose accumulator
// is the trajectory itself).  A^d and (A')^d come from repeated squaring in the same layout.
// powers A^d and (A')^d, d = 1, 2, 4, 8, in accumulator layout over state positions
// (pw[l][q] = A^(2^l)[state 3g+q][state of position c]); the gradient's scans use them
// (nilpotent step, s.nil: A^d = I + d N exactly, no squaring)
template <class SM>
__device__ __forceinline__ void gradient_powers(SM& s, f4 (&pw)[4], f4 (&tw)[4]) {
  const int lane = opaque_lane();
  const int g = lane >> 4, c = lane & 15;
  const int sc = ((c & 3) < 3) ? 3 * (c >> 2) + (c & 3) : -1;
  f4 Pd = {0.f, 0.f, 0.f, 0.f}, Td = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int r = 3 * g + q;
    Pd[q] = (sc >= 0) ? s.A[r * 12 + sc] : 0.f;
    Td[q] = (sc >= 0) ? s.A[sc * 12 + r] : 0.f;
  }
  pw[0] = Pd;
  tw[0] = Td;
  if (uniform(s.nil)) {
#pragma unroll
    for (int l = 1; l < 4; ++l) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float dl = (sc == 3 * g + q && q < 3) ? 1.f : 0.f;
        pw[l][q] = fmaf((float)(1 << l), Pd[q] - dl, dl);
        tw[l][q] = fmaf((float)(1 << l), Td[q] - dl, dl);
      }
    }
    return;
  }
#pragma unroll
  for (int l = 1; l < 4; ++l) {
    f4 pn = {0.f, 0.f, 0.f, 0.f}, tn = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      pn = mfma4(tw[l - 1][q], pw[l - 1][q], pn);  // A^2d  = A^d A^d   (A operand = (A^d)')
      tn = mfma4(pw[l - 1][q], tw[l - 1][q], tn);  // A'^2d = A'^d A'^d
    }
    pw[l] = pn;
    tw[l] = tn;
  }
}

// LAT (team / latency mode): the powers come precomputed (one set per instance, `pwc`/`twc`),
// and the per-step B~ v sum is unrolled to the 12 params a step can hold so that its LDS reads
// issue together (with two busy waves per SIMD the rolled loop measured faster: issue-bound)
//
// PREC (the polish: refinement and KKT check): the rollout e_{k+1} in float64.  Its inputs are
// B_k u_k + d_k, where the legs' torques on the body (~8 rad/s per step at 200 N) cancel to a
// small e: rounded in fp32 they leave ~4e-7 of noise in the gradient, as large as the
// multiplier of a face whose release moves a force by 1e-4 relative (the direction is weighed
// only by R = 1e-5: instance 3458 of test_warm_next_tick's batch held fy at mu fz = 8 N with
// a true multiplier of -8.3e-7, optimum 7.97 N).  In float64 (products of fp32 operands are
// exact) the noise is ~5e-9; e is rounded to fp32 once and the adjoint stays fp32 (NumPy
// study: only the rollout needs the precision).  Nilpotent step only; the general A keeps the
// fp32 rollout and the relative multiplier tolerance (polish_check).
template <int NC, bool LAT = false, bool PREC = false>
__device__ __forceinline__ void gradient(Smem<NC>& s, const KParams& P, int n, const float* vin,
                                         float* gout, const f4* pwc = nullptr,
                                         const f4* twc = nullptr) {
  CMPC_T0(t_gr);
  const int lane = opaque_lane();
  const int g = lane >> 4, c = lane & 15;
  const int N = P.N;
  n = uniform(n);
  WSYNC();
  // State positions (as in condense_tiles_fwd): register q of lane group g holds state 3g + q
  // (q < 3), q = 3 is padding, so every K = 16 product over states is three MFMAs (K = 12).
  // h_k = B~_k v_k + d~_k for states 3g..3g+2 of step c
  f4 Et = {0.f, 0.f, 0.f, 0.f};
  double Eh[3] = {0.0, 0.0, 0.0};  // PREC: h in float64
  if constexpr (LAT) {
    const int cc = (c < N) ? c : 0;
    const int p0 = s.off[cc], p1 = s.off[cc + 1];
    float dt[3], bv[12][3], vv[12];
#pragma unroll
    for (int q = 0; q < 3; ++q) dt[q] = s.Dt[12 * cc + 3 * g + q];
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const int p = min(p0 + i, NC - 1);
#pragma unroll
      for (int q = 0; q < 3; ++q) bv[i][q] = s.Bt[p * kBS + 3 * g + q];
      vv[i] = vin[p];
    }
    if constexpr (PREC) {
#pragma unroll
      for (int q = 0; q < 3; ++q) Eh[q] = (double)dt[q];
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        const bool ok = p0 + i < p1;
#pragma unroll
        for (int q = 0; q < 3; ++q) Eh[q] = ok ? fma((double)bv[i][q], (double)vv[i], Eh[q]) : Eh[q];
      }
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        if (c >= N) Eh[q] = 0.0;
        Et[q] = (float)Eh[q];
      }
    } else {
#pragma unroll
      for (int q = 0; q < 3; ++q) Et[q] = dt[q];
#pragma unroll
      for (int i = 0; i < 12; ++i) {  // (params past the step may hold anything, even NaN: select)
        const bool ok = p0 + i < p1;
#pragma unroll
        for (int q = 0; q < 3; ++q) Et[q] = ok ? fmaf(bv[i][q], vv[i], Et[q]) : Et[q];
      }
      if (c >= N) Et = f4{0.f, 0.f, 0.f, 0.f};
    }
  } else if (c < N) {
    const int p1 = s.off[c + 1];
    if constexpr (PREC) {
#pragma unroll
      for (int q = 0; q < 3; ++q) Eh[q] = (double)s.Dt[12 * c + 3 * g + q];
      for (int p = s.off[c]; p < p1; ++p) {
        const float* bt = &s.Bt[p * kBS + 3 * g];
        const double vp = (double)vin[p];
#pragma unroll
        for (int q = 0; q < 3; ++q) Eh[q] = fma((double)bt[q], vp, Eh[q]);
      }
#pragma unroll
      for (int q = 0; q < 3; ++q) Et[q] = (float)Eh[q];
    } else {
#pragma unroll
      for (int q = 0; q < 3; ++q) Et[q] = s.Dt[12 * c + 3 * g + q];
      for (int p = s.off[c]; p < p1; ++p) {
        const float* bt = &s.Bt[p * kBS + 3 * g];
        const float vp = vin[p];
#pragma unroll
        for (int q = 0; q < 3; ++q) Et[q] = fmaf(bt[q], vp, Et[q]);
      }
    }
  }
  if (uniform(s.nil)) {
    // Nilpotent step (A = I + N, N^2 = 0, condense_tiles_nil): A^m = I + m N, so
    //   e_{k+1} = sum_{j<=k} A^{k-j} h_j = S_k + N u_k,   S_k = sum_{j<=k} h_j,
    //                                                      u_k = sum_{j<=k} (k-j) h_j = sum_{i<k} S_i,
    //   lambda_k = R_k + N' v_k,   R_k = sum_{j>=k} w_j,   v_k = sum_{i>k} R_i,   w_j = Q2 e_{j+1}:
    // four DPP prefix / suffix scans (row_shr / row_shl, zero past the row) and three MFMAs per
    // recursion instead of twelve in a dependent chain (and no powers of A); u and v are sums of
    // sums, so nothing cancels.
    const int sc = ((c & 3) < 3) ? 3 * (c >> 2) + (c & 3) : -1;
    float aN[3], aNt[3];  // A operands of N X and N' X
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int r = 3 * g + q;
      const float dl = (sc == r) ? 1.f : 0.f;
      aN[q] = (sc >= 0) ? s.A[sc * 12 + r] - dl : 0.f;
      aNt[q] = (sc >= 0) ? s.A[r * 12 + sc] - dl : 0.f;
    }
    if constexpr (PREC) {
      // the same scans in float64; N u on the f64 matrix cores, whose D layout (row = g + 4 reg)
      // puts state 3g + reg of step c in register reg of lane (g, c), as above
      double u64[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        double x = Eh[q];
        x += dpp64<0x111>(x);
        x += dpp64<0x112>(x);
        x += dpp64<0x114>(x);
        x += dpp64<0x118>(x);
        Eh[q] = x;
        double y = dpp64<0x111>(x);
        y += dpp64<0x111>(y);
        y += dpp64<0x112>(y);
        y += dpp64<0x114>(y);
        y += dpp64<0x118>(y);
        u64[q] = y;
      }
      const int sr = ((c >> 2) < 3) ? 3 * (c & 3) + (c >> 2) : -1;  // state of A-operand row c
      d4 acc = {Eh[0], Eh[1], Eh[2], 0.0};
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int r = 3 * g + q;
        const double a = (sr >= 0) ? (double)(s.A[sr * 12 + r] - ((sr == r) ? 1.f : 0.f)) : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, u64[q], acc, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 3; ++q) Et[q] = (float)acc[q];
    } else {
    f4 u = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      float x = Et[q];  // S: inclusive prefix sum over the steps (lanes c of the DPP row)
      x += dpp<0x111>(x);
      x += dpp<0x112>(x);
      x += dpp<0x114>(x);
      x += dpp<0x118>(x);
      Et[q] = x;
      float y = dpp<0x111>(x);  // u: exclusive prefix sum of S
      y += dpp<0x111>(y);
      y += dpp<0x112>(y);
      y += dpp<0x114>(y);
      y += dpp<0x118>(y);
      u[q] = y;
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) Et = mfma4(aN[q], u[q], Et);
    }
    if (c < N) {
#pragma unroll
      for (int q = 0; q < 3; ++q) s.E[12 * c + 3 * g + q] = Et[q];
    }
    f4 Lt = {0.f, 0.f, 0.f, 0.f}, v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      float x = (c < N) ? s.Q2[3 * g + q] * Et[q] : 0.f;  // R: inclusive suffix sum
      x += dpp<0x101>(x);
      x += dpp<0x102>(x);
      x += dpp<0x104>(x);
      x += dpp<0x108>(x);
      Lt[q] = x;
      float y = dpp<0x101>(x);  // v: exclusive suffix sum of R
      y += dpp<0x101>(y);
      y += dpp<0x102>(y);
      y += dpp<0x104>(y);
      y += dpp<0x108>(y);
      v[q] = y;
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) Lt = mfma4(aNt[q], v[q], Lt);
    if (c < N) {
#pragma unroll
      for (int q = 0; q < 3; ++q) s.L[12 * c + 3 * g + q] = Lt[q];
    }
  } else {
  f4 pw[4], tw[4];  // d = 1, 2, 4, 8
  if (pwc != nullptr) {  // (a compile-time constant at every call site)
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      pw[l] = pwc[l];
      tw[l] = twc[l];
    }
  } else {
    gradient_powers(s, pw, tw);
  }
  // forward scan: E[:, k] += A^d E[:, k - d]  (A operand = (A^d)' = tw)
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    if ((1 << l) >= N) break;  // uniform
    f4 sh = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      switch (l) {
        case 0: sh[q] = dpp<0x111>(Et[q]); break;  // row_shr:1
        case 1: sh[q] = dpp<0x112>(Et[q]); break;  // row_shr:2
        case 2: sh[q] = dpp<0x114>(Et[q]); break;  // row_shr:4
        default: sh[q] = dpp<0x118>(Et[q]); break; // row_shr:8
      }
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) Et = mfma4(tw[l][q], sh[q], Et);
  }
  if (c < N) {
#pragma unroll
    for (int q = 0; q < 3; ++q) s.E[12 * c + 3 * g + q] = Et[q];
  }
  // adjoint: L0 = Q2 e_{k+1} (zero past the horizon), L[:, k] += (A')^d L[:, k + d]
  f4 Lt = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 3; ++q) Lt[q] = (c < N) ? s.Q2[3 * g + q] * Et[q] : 0.f;
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    if ((1 << l) >= N) break;
    f4 sh = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      switch (l) {
        case 0: sh[q] = dpp<0x101>(Lt[q]); break;  // row_shl:1
        case 1: sh[q] = dpp<0x102>(Lt[q]); break;  // row_shl:2
        case 2: sh[q] = dpp<0x104>(Lt[q]); break;  // row_shl:4
        default: sh[q] = dpp<0x108>(Lt[q]); break; // row_shl:8
      }
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) Lt = mfma4(pw[l][q], sh[q], Lt);  // A operand = A^d = ((A')^d)'
  }
  if (c < N) {
#pragma unroll
    for (int q = 0; q < 3; ++q) s.L[12 * c + 3 * g + q] = Lt[q];
  }
  }  // (general A)
  WSYNC();
  for (int p = lane; p < n; p += 64) {  // g = B~' lambda + Rt v
    const int k = s.par[p];
    const f4* l = reinterpret_cast<const f4*>(&s.L[12 * k]);
    f2 a2 = {s.Rt[p] * vin[p], 0.f};  // packed: even and odd states in the two halves
    const f4* bt = reinterpret_cast<const f4*>(&s.Bt[p * kBS]);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const f4 lv = l[j], bv = bt[j];
      a2 = __builtin_elementwise_fma(f2{bv[0], bv[1]}, f2{lv[0], lv[1]}, a2);
      a2 = __builtin_elementwise_fma(f2{bv[2], bv[3]}, f2{lv[2], lv[3]}, a2);
    }
    gout[p] = a2[0] + a2[1];
  }
  WSYNC();
  CMPC_ACC(2, t_gr);
  CMPC_CNT(12, 1);
}

// (H + shift)^-1 applied to a param vector: the LDL' solve on the register tiles
template <int NC, int NT>
__device__ __forceinline__ void minv_apply(Smem<NC>& s, const KParams& P, const f4 (&M)[NT], int n,
                                           const float* in, float* out) {
  ldl_apply<NC>(s, M, n, in, out);
}

// Euclidean projection of (a, b, c) onto {|x| <= mu z, |y| <= mu z, z >= fz_min}.
// Face code bits: 1 fz at fz_min, 2/4 fx at +/-mu fz, 8/16 fy at +/-mu fz.
__device__ __forceinline__ int project(float a, float b, float c, float mu, float fzmin,
                                       float& px, float& py, float& pz) {
  const float Aa = fabsf(a), Bb = fabsf(b);
  const float lo = fminf(Aa, Bb), hi = fmaxf(Aa, Bb);
  const float z1 = (c + mu * (Aa + Bb)) / (1.f + 2.f * mu * mu);
  const float z2 = (c + mu * hi) / (1.f + mu * mu);
  float zz = (mu * z1 < lo) ? z1 : ((mu * z2 < hi) ? z2 : c);
  int code = 0;
  if (zz < fzmin) { zz = fzmin; code |= 1; }
  const float lim = mu * zz;
  if (a > lim) { px = lim; code |= 2; } else if (a < -lim) { px = -lim; code |= 4; } else px = a;
  if (b > lim) { py = lim; code |= 8; } else if (b < -lim) { py = -lim; code |= 16; } else py = b;
  pz = zz;
  return code;
}

// ADMM basis: every stance triple contributes (fx, fy, fz) as params 3t, 3t+1, 3t+2
template <int NC>
__device__ __forceinline__ void build_admm_basis(Smem<NC>& s, const KParams& P,
                                                 const float* __restrict__ Bg, int ntri) {
  const int lane = opaque_lane();
  const int N = P.N;
  const int n = 3 * ntri;
  WSYNC();
  if (lane < ntri) {  // lane t copies the 12x3 block of its triple (all loads in flight at once)
    const int kl = s.tri[lane];
    const float* src = Bg + (kl >> 2) * 144 + 3 * (kl & 3);
    float bv[36];
#pragma unroll
    for (int r = 0; r < 12; ++r) {
#pragma unroll
      for (int a = 0; a < 3; ++a) bv[3 * r + a] = src[r * 12 + a];
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
#pragma unroll
      for (int r = 0; r < 12; ++r) s.Bt[(3 * lane + a) * kBS + r] = bv[3 * r + a];
    }
  }
  for (int p = lane; p < NC; p += 64) {
    if (p < n) {
      const int t = p / 3, a = p % 3;
      const int kl = s.tri[t];
      s.Rt[p] = s.R2[3 * (kl & 3) + a];
      s.par[p] = kl >> 2;
    } else {
      s.Rt[p] = 0.f;
      s.par[p] = 0;
      s.x[p] = 0.f; s.z[p] = 0.f; s.g[p] = 0.f; s.r[p] = 0.f;
      s.v[p] = 0.f; s.dl[p] = 0.f;
    }
  }
  {  // off[k] = 3 x (stance (step, leg) pairs before step k): popcount of the stance mask
    const unsigned long long sm = __ballot(lane < 4 * N && s.tri_of[lane] >= 0);
    if (lane <= N) {
      const unsigned long long below = (lane >= 16) ? ~0ull : ((1ull << (4 * lane)) - 1ull);
      s.off[lane] = 3 * __popcll(sm & below);
    }
  }
  for (int o = lane; o < 12 * N; o += 64) s.Dt[o] = s.D[o];
  WSYNC();
}

// Polish setup: the reduced basis of the faces in s.code (lane t owns triple t),
// u = T v + t0 with t0 = locked components, v initialised from the triple forces in `vsrc`
// (ADMM's z, or the candidate forces a polish check left in s.dl; read before anything is
// written, since s.dl shares the G slab).  Returns nr; the param indices of each triple are
// left packed in s.fpk for the KKT check.
template <int NC>
__device__ __forceinline__ int polish_setup(Smem<NC>& s, const KParams& P,
                                            const float* __restrict__ Bg, int ntri,
                                            const float* vsrc) {
  const int lane = opaque_lane();
  const int N = P.N;
  const float mu = P.mu, fzmin = P.fz_min;
  WSYNC();
  const bool owns = lane < ntri;
  float vs[3] = {0.f, 0.f, 0.f};
  if (owns) {
#pragma unroll
    for (int a = 0; a < 3; ++a) vs[a] = vsrc[3 * lane + a];
  }
  WSYNC();
  const int code = owns ? s.code[lane] : 0;
  const int kl = owns ? s.tri[lane] : 0;
  const int k = kl >> 2, leg = kl & 3;
  const int sx = (code & 2) ? 1 : ((code & 4) ? -1 : 0);
  const int sy = (code & 8) ? 1 : ((code & 16) ? -1 : 0);
  const bool zl = (code & 1) != 0;
  const int cnt = owns ? ((sx == 0) + (sy == 0) + (!zl)) : 0;
  const int base = wave_excl_scan4(cnt);
  const int nr = wave_total4(cnt);
  if (owns) {
    float bx[12], by[12], bz[12];  // columns fx, fy, fz of B_k for this leg (loads in flight together)
    {
      const float* src = Bg + k * 144 + 3 * leg;
#pragma unroll
      for (int r = 0; r < 12; ++r) {
        bx[r] = src[r * 12];
        by[r] = src[r * 12 + 1];
        bz[r] = src[r * 12 + 2];
      }
    }
    s.tcnt[lane] = cnt;
    int p = base;
    int px = 255, py = 255, pz = 255;
    if (sx == 0) {
      px = p++;
#pragma unroll
      for (int r = 0; r < 12; ++r) s.Bt[px * kBS + r] = bx[r];
      s.Rt[px] = s.R2[3 * leg];
      s.par[px] = k;
      s.v[px] = vs[0];
    }
    if (sy == 0) {
      py = p++;
#pragma unroll
      for (int r = 0; r < 12; ++r) s.Bt[py * kBS + r] = by[r];
      s.Rt[py] = s.R2[3 * leg + 1];
      s.par[py] = k;
      s.v[py] = vs[1];
    }
    if (!zl) {
      pz = p++;
      const float cx = sx * mu, cy = sy * mu;
#pragma unroll
      for (int r = 0; r < 12; ++r) s.Bt[pz * kBS + r] = bz[r] + cx * bx[r] + cy * by[r];
      s.Rt[pz] = s.R2[3 * leg + 2] + mu * mu * ((sx != 0 ? s.R2[3 * leg] : 0.f) +
                                                (sy != 0 ? s.R2[3 * leg + 1] : 0.f));
      s.par[pz] = k;
      s.v[pz] = vs[2];
    } else {  // fz locked at fz_min: the triple's constant force t0 enters d~ through B_k t0
      const float tx = sx * mu * fzmin, ty = sy * mu * fzmin;
#pragma unroll
      for (int r = 0; r < 12; ++r) s.G[lane * 12 + r] = fmaf(bz[r], fzmin, fmaf(by[r], ty, bx[r] * tx));
    }
    s.fpk[lane] = px | (py << 8) | (pz << 16);
  }
  WSYNC();
  {  // off[kk] = params of the triples before step kk = the scan base of the first triple of
     // step >= kk (its index: popcount of the stance mask below step kk), nr past the last
    const unsigned long long sm = __ballot(lane < 4 * N && s.tri_of[lane] >= 0);
    const unsigned long long below = (lane >= 16) ? ~0ull : ((1ull << (4 * lane)) - 1ull);
    const int tstar = __popcll(sm & below);
    const int bt = __shfl(base, tstar < 64 ? tstar : 63, 64);
    if (lane <= N) s.off[lane] = (tstar < ntri) ? bt : nr;
  }
  for (int o = lane; o < 12 * N; o += 64) {  // d~ = d + B t0 (LDS only)
    const int kk = o / 12, r = o % 12;
    float acc = s.D[o];
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      const int t = s.tri_of[4 * kk + l];
      if (t >= 0 && (s.code[t] & 1)) acc += s.G[t * 12 + r];
    }
    s.Dt[o] = acc;
  }
  for (int p = lane; p < NC; p += 64)
    if (p >= nr) s.v[p] = 0.f;
  WSYNC();
  return nr;
}

// Polish check after refinement (E, L at the final v in LDS): KKT conditions per triple
// (lane t = triple t, its params from s.fpk).  On success the triple's force is written over
// its ADMM primal s.x[3t .. 3t+2]; the repaired face code of a failing triple is left in
// s.tcnt and `changed` says whether any face changed.  `loose` says whether every relative KKT
// violation (multipliers against the gradient scale, forces against the force scale) is within
// kLooseTol x polish_tol; the candidate forces are left in s.dl[3t .. 3t+2] for that case.
// top > 0: the repair changes only the `top` triples with the largest relative violation (the
// others keep their faces).
template <int NC>
__device__ __forceinline__ bool polish_check(Smem<NC>& s, const KParams& P,
                                             const float* __restrict__ Bg, int ntri, float step,
                                             bool& changed, bool& loose, bool& converged,
                                             bool& amb, bool& decisive, float& vworst,
                                             int top = 0, int tr = -1) {
  const int lane = opaque_lane();
  const float mu = P.mu, fzmin = P.fz_min;
  float fx = 0.f, fy = 0.f, fz = 0.f;
  float gx = 0.f, gy = 0.f, gz = 0.f;
  bool lok = true;
  WSYNC();
  const bool owns = lane < ntri;
  const int code = owns ? s.code[lane] : 0;
  const int kl = owns ? s.tri[lane] : 0;
  const int k = kl >> 2, leg = kl & 3;
  const int sx = (code & 2) ? 1 : ((code & 4) ? -1 : 0);
  const int sy = (code & 8) ? 1 : ((code & 16) ? -1 : 0);
  const bool zl = (code & 1) != 0;
  if (owns) {
    // the forces on the current faces exactly (a face added by a downdate keeps its basis
    // param, which the refinement holds on the face only to rounding -- up to 1e-2 N off in
    // fp32 -- so the face's own value is taken, as for a face of the basis)
    const int pk = s.fpk[lane];
    const int px = pk & 255, py = (pk >> 8) & 255, pz = (pk >> 16) & 255;
    fz = zl ? fzmin : s.v[pz];
    fx = (sx == 0) ? s.v[px] : sx * mu * fz;
    fy = (sy == 0) ? s.v[py] : sy * mu * fz;
    const float* Bk = Bg + k * 144 + 3 * leg;
    float ax = 0.f, ay = 0.f, az = 0.f;
#pragma unroll
    for (int r = 0; r < 12; ++r) {
      const float lr = s.L[12 * k + r];
      ax = fmaf(Bk[r * 12], lr, ax);
      ay = fmaf(Bk[r * 12 + 1], lr, ay);
      az = fmaf(Bk[r * 12 + 2], lr, az);
    }
    gx = ax + s.R2[3 * leg] * fx;
    gy = ay + s.R2[3 * leg + 1] * fy;
    gz = az + s.R2[3 * leg + 2] * fz;
  }
  const float gs = wave_max(fmaxf(fabsf(gx), fmaxf(fabsf(gy), fabsf(gz))));
  const float us = wave_max(fmaxf(1.f, fmaxf(fabsf(fx), fmaxf(fabsf(fy), fabsf(fz)))));
  const float tol_d = P.polish_tol * gs, tol_p = P.polish_tol * us;
  // Face multipliers.  A face held with multiplier -l moves the forces, once released, by up
  // to ~2.6 l / R2 (strong convexity: the condensed Hessian is >= diag(R2), and |a_f| <= 1.28
  // for a pyramid face), so with the float64 rollout (gradient<PREC>, nilpotent step) the
  // tolerance of each face is also bounded by kFaceErr x polish_tol x the force scale in those
  // units: 8e-8 at 200 N against ~5e-9 of gradient noise, where polish_tol x gs (the relative
  // test, ~5e-7) admitted 3458's -8.3e-7 (a 1.48e-4 error).  The general A keeps the fp32
  // rollout and the relative test.
  const bool prec = uniform(s.nil) != 0;
  float tfx = tol_d, tfy = tol_d, tfz = tol_d;
  if (prec && owns) {
    const float fe = kFaceErr * P.polish_tol * us;
    tfx = fminf(tol_d, fe * s.R2[3 * leg]);
    tfy = fminf(tol_d, fe * s.R2[3 * leg + 1]);
    tfz = fminf(tol_d, fe * s.R2[3 * leg + 2]);
  }
  bool ok = true, am = false, dec = false;
  int nc = 0;
  float v = 0.f, csq = 0.f;
  if (owns) {
    // KKT per triple; on a violation also derive the repaired face set (primal-dual
    // active-set step): drop faces with a negative multiplier, add violated faces
    const float lx = sx ? -sx * gx : 0.f;
    const float ly = sy ? -sy * gy : 0.f;
    const float l0 = gz - mu * (lx + ly);
    // (precise: a multiplier within kAmbBand x the relative band of zero is ambiguous at this
    // point -- the point's remaining error moves it by up to ~|H| x (step / 30))
    const float ta = kAmbBand * tol_d;
    am = prec && ((sx && lx < ta) || (sy && ly < ta) || (zl && l0 < ta));
    nc = code;
    if (sx && lx < -tfx) { ok = false; nc &= ~6; dec = dec || lx < -ta; }
    if (sy && ly < -tfy) { ok = false; nc &= ~24; dec = dec || ly < -ta; }
    if (zl && l0 < -tfz) { ok = false; nc &= ~1; dec = dec || l0 < -ta; }
    if (!sx && fabsf(fx) > mu * fz + tol_p) { ok = false; nc |= (fx > 0.f) ? 2 : 4; dec = true; }
    if (!sy && fabsf(fy) > mu * fz + tol_p) { ok = false; nc |= (fy > 0.f) ? 8 : 16; dec = true; }
    if (!zl && fz < fzmin - tol_p) { ok = false; nc |= 1; dec = true; }
    if (!(isfinite(fx) && isfinite(fy) && isfinite(fz))) { ok = false; dec = true; }
    const float ig = 1.f / fmaxf(gs, 1e-30f), iu = 1.f / us;
    v = fmaxf(fmaxf(sx ? -lx * ig : 0.f, sy ? -ly * ig : 0.f), zl ? -l0 * ig : 0.f);
    v = fmaxf(v, fmaxf(sx ? 0.f : (fabsf(fx) - mu * fz) * iu, sy ? 0.f : (fabsf(fy) - mu * fz) * iu));
    v = fmaxf(v, zl ? 0.f : (fzmin - fz) * iu);
    const bool fin = isfinite(fx) && isfinite(fy) && isfinite(fz);
#ifdef CMPC_TRACE
    if (tr >= 0 && (v > 0.f || (sx && lx < tfx) || (sy && ly < tfy) || (zl && l0 < tfz)))
      printf("[%d]       tri %d k %d leg %d code %d f %g %g %g  l %g %g %g  tol %g %g %g  v %g\n", tr,
             lane, k, leg, code, fx, fy, fz, lx, ly, l0, tfx, tfy, tfz, v);
#endif
    lok = fin && v <= kLooseTol * P.polish_tol;
    // (precise: a loose acceptance also bounds the force error of every face it holds)
    if (prec)
      lok = lok && !(sx && lx < -kLooseFace * tfx) && !(sy && ly < -kLooseFace * tfy) &&
            !(zl && l0 < -kLooseFace * tfz);
    s.dl[3 * lane] = fx;  // the candidate, for a loose acceptance by the caller
    s.dl[3 * lane + 1] = fy;
    s.dl[3 * lane + 2] = fz;
    // certified force error of the held faces (status 1 contract): the point is the exact
    // optimum of the problem tilted by c = sum_f min(l_f, 0) a_f over the faces it holds
    // (a = (sx, 0, -mu), (0, sy, -mu), (0, 0, -1)), so |u - u*|_2 <= |c|_2 / min R2 (strong
    // convexity of the condensed objective, Hessian >= diag(R2))
    const float nx = sx ? fminf(lx, 0.f) : 0.f, ny = sy ? fminf(ly, 0.f) : 0.f;
    const float nz = zl ? fminf(l0, 0.f) : 0.f;
    const float cx = nx * sx, cy = ny * sy, cz = -mu * (nx + ny) - nz;
    csq = fmaf(cx, cx, fmaf(cy, cy, cz * cz));
    if (!isfinite(csq)) csq = INFINITY;
  }
  // (parked in the ADMM scratch s.r, which nothing reads before the next ADMM iteration or
  // face downdate rewrites it: certified_faces reduces it only for an accepted point)
  s.r[lane] = owns ? csq : 0.f;
  if (lane == 0) s.r[64] = us;
  if (top > 0) {  // uniform: keep the faces of all but the `top` most violated triples
    const bool cand = owns && nc != code;
    float key = cand ? (isfinite(v) ? v : INFINITY) : -1.f;  // a changed triple has v > 0
    bool sel = false;
    const int ncand = __popcll(__ballot(cand));
    const int kk = max(top, (ncand + 1) >> 1);  // (uniform)
    for (int r = 0; r < kk; ++r) {
      const float m = wave_max(key);
      if (!(m > 0.f)) break;  // uniform: no candidate left
      const unsigned long long bal = __ballot(key == m);
      if (lane == __builtin_ctzll(bal)) {
        sel = true;
        key = -1.f;
      }
    }
    if (cand && !sel) nc = code;
  }
  if (owns) s.tcnt[lane] = nc;  // repaired code (copied into s.code by the caller if used)
  changed = __any(owns && nc != code) != 0;
  amb = __any(am) != 0;
  // (only multipliers within the ambiguity band fail: the decision rests on the point's accuracy)
  decisive = __any(dec) != 0;
  vworst = wave_max((owns && isfinite(v)) ? v : (owns ? 1e30f : 0.f));
  const bool step_ok = step <= P.polish_tol * us;
  converged = step_ok;
  loose = (__all(lok) != 0) && step_ok;
  const bool all_ok = (__all(ok) != 0) && step_ok;
  if (all_ok && owns) {
    // onto the pyramid exactly: the check admits violations up to polish_tol x the force scale
    // (~2e-3 N), the reference's bounds take none (a move of at most that, far inside the 1e-4
    // parity bar)
    float px, py, pz;
    project(fx, fy, fz, mu, fzmin, px, py, pz);
    s.x[3 * lane] = px;
    s.x[3 * lane + 1] = py;
    s.x[3 * lane + 2] = pz;
  }
  return all_ok;
}

// ------------------------------------------------------------------------------------------
// The certified force error of the held faces at the point polish_check accepted (its per-triple
// |c_t|^2 and the force scale are in s.r): within kCertFace of the force scale?  Uniform.
template <int NC>
__device__ __forceinline__ bool certified_faces(Smem<NC>& s, const KParams& P) {
  const int lane = opaque_lane();
  WSYNC();
  const float c2 = wave_sum(s.r[lane]);
  return uniformf(sqrtf(c2)) <= kCertFace * P.r2_min * uniformf(s.r[64]);
}

#ifdef CMPC_DIAG_GRES
// diagnostic build: at an accepted point, |grad|_2 (the gradient at the final refinement point,
// s.g over the nact params) and |c|_2, both over min 2R x the force scale (force-error units)
template <int NC>
__device__ __forceinline__ void diag_gres(Smem<NC>& s, const KParams& P, int nact, float& gm,
                                          float& cm, float& us) {
  const int lane = opaque_lane();
  WSYNC();
  float g2 = 0.f;
  for (int p = lane; p < nact; p += 64) g2 = fmaf(s.g[p], s.g[p], g2);
  g2 = wave_sum(g2);
  const float c2 = wave_sum(s.r[lane]);
  us = uniformf(s.r[64]);
  gm = uniformf(sqrtf(g2)) / (P.r2_min * us);
  cm = uniformf(sqrtf(c2)) / (P.r2_min * us);
}
#endif

// Face downdates (round 4).  A repair that only ADDS faces to the current face set keeps the
// basis and the inverse M of the last factorization: each added face is an equality a'v = c on
// the basis params (fz at fz_min: v_pz = fz_min; fx on the face of sign s: v_px - s mu v_pz = 0,
// or v_px = s mu fz_min where the basis locks fz; fy alike), and the inverse on the constrained
// set is the sequence of rank-1 downdates
//     M_j = M_{j-1} - w_j w_j' / d_j,   w_j = M_{j-1} a_j,   d_j = a_j' w_j,
// kept ASIDE: M stays in the register tiles untouched, the w_j are vectors in the polish
// session's free LDS (the sweep scaling / panel / H slab), and every refinement step applies
//     M_F g = M g - sum_j w_j (w_j' g) / d_j
// after its symv (dd_apply: one wave reduction per face).  w_j is one symv with the sparse a_j
// (two params at most) minus the earlier faces' terms, whose w_i' a_j are two LDS reads.  v is
// projected onto each new equality in the M_{j-1} metric, v -= w_j (a_j' v - c_j) / d_j, which
// keeps the earlier ones (a_i' w_j = 0, i < j).  Cost: a symv per added face instead of a
// condensation + inversion (~150 k cycles).  (Rank-4 MFMA updates of the tiles themselves do the
// same arithmetic, but writing the tiles in the polish branch kept them live across the KKT
// check and the register allocator spilled 600-1,100 VGPRs in every variant tried.)  NumPy model
// (tests/algo_spec.py downdate=True, the fp32 sweep inverse): unchanged refinement counts, half of
// all repairs are pure additions, and 6 faces per factorization keep almost all of the gain
// (config 3: 2.37 -> 2.19 factorizations per instance, the slowest instances -20 %).
// (diagnostic override only: -DCMPC_DD_CAP=3 exercises the refactor-on-cap path far more often;
// round 5 recorded its build as run-to-run non-deterministic, round 6's determinism records
// cover it)
#ifndef CMPC_DD_CAP
#define CMPC_DD_CAP 6
#endif
// faces per factorization: the w_j fill the ds / pan / H slab (5 NC + kMaxP floats) but its
// last 32 floats, which hold the faces' 1 / d_j, params, coefficients and right-hand sides
__host__ __device__ constexpr int dd_max(int NC) {
  return (5 * NC + kMaxP - 32) / NC < CMPC_DD_CAP ? (5 * NC + kMaxP - 32) / NC : CMPC_DD_CAP;
}
template <int NC>
__device__ __forceinline__ float* dd_w(Smem<NC>& s, int j) { return s.ds + j * NC; }
template <int NC>
__device__ __forceinline__ float* dd_meta(Smem<NC>& s) { return s.H + kMaxP - 32; }

// Append the faces added by the repair (s.code -> s.tcnt, no drops) as downdates; nadd counts
// the faces held so far.  False if they do not fit or a d_j is not positive (rounding after
// many downdates): the caller refactors.
template <int NC, class MT>
__device__ __forceinline__ bool face_downdate(Smem<NC>& s, const KParams& P, const MT& M, int n,
                                              int ntri, int& nadd) {
  static_assert(dd_max(NC) >= 1 && dd_max(NC) <= 8, "the meta block holds 8 faces");
  static_assert(offsetof(Smem<NC>, H) == offsetof(Smem<NC>, ds) + 5 * NC * sizeof(float),
                "ds, pan and H are one slab");
  const int lane = opaque_lane();
  n = uniform(n);
  float* meta = dd_meta(s);  // [0, 8) 1 / d_j, [8, 16) p1 | p2 << 8, [16, 24) coefficient, [24, 32) c
  WSYNC();
  int F;
  {
    const bool owns = lane < ntri;
    const int oc = owns ? s.code[lane] : 0, nc = owns ? s.tcnt[lane] : 0;
    const int add = nc & ~oc;
    const int cnt = (add & 1) + ((add & 6) != 0) + ((add & 24) != 0);
    int j = nadd + wave_excl_scan4(cnt);
    F = uniform(wave_total4(cnt));
    if (nadd + F > dd_max(NC)) return false;  // (uniform)
    if (owns && add) {
      // a face with no second param has p2 = p1 and coefficient 0
      const float mu = P.mu, fzmin = P.fz_min;
      const int pk = s.fpk[lane];
      const int px = pk & 255, py = (pk >> 8) & 255, pz = (pk >> 16) & 255;
      if (add & 1) {  // (first: a friction face added with it then reads fz = fz_min)
        meta[8 + j] = __int_as_float(pz | (pz << 8)); meta[16 + j] = 0.f; meta[24 + j] = fzmin; ++j;
      }
#pragma unroll
      for (int ax = 0; ax < 2; ++ax) {
        const int bits = ax ? (add & 24) : (add & 6);
        if (!bits) continue;
        const int pa = ax ? py : px;
        const float sg = (bits & (ax ? 8 : 2)) ? 1.f : -1.f;
        if (pz != 255) {
          meta[8 + j] = __int_as_float(pa | (pz << 8)); meta[16 + j] = -sg * mu; meta[24 + j] = 0.f;
        } else {
          meta[8 + j] = __int_as_float(pa | (pa << 8)); meta[16 + j] = 0.f; meta[24 + j] = sg * mu * fzmin;
        }
        ++j;
      }
    }
  }
  WSYNC();
  const int j1 = nadd + F;
  for (int j = nadd; j < j1; ++j) {  // uniform
    const int q = __float_as_int(meta[8 + j]);
    const int p1 = q & 255, p2 = (q >> 8) & 255;
    const float cf = meta[16 + j], cv = meta[24 + j];
    for (int p = lane; p < NC; p += 64) s.r[p] = (p == p1) ? 1.f : (p == p2) ? cf : 0.f;
    float* w = dd_w(s, j);
    minv_apply<NC>(s, P, M, n, s.r, w);  // w = M a_j
    for (int i = 0; i < j; ++i) {  // w -= w_i (w_i' a_j) / d_i  (uniform trip count)
      const float* wi = dd_w(s, i);
      const float t = fmaf(cf, wi[p2], wi[p1]) * meta[i];
      for (int p = lane; p < n; p += 64) w[p] = fmaf(-t, wi[p], w[p]);
      WSYNC();
    }
    const float d = fmaf(cf, w[p2], w[p1]);
    if (!(d > 0.f) || !isfinite(d)) return false;  // (the same value in every lane)
    const float id = 1.f / d;
    const float res = (fmaf(cf, s.v[p2], s.v[p1]) - cv) * id;
    WSYNC();
    for (int p = lane; p < n; p += 64) s.v[p] = fmaf(-res, w[p], s.v[p]);  // v onto a_j' v = c_j
    if (lane == 0) meta[j] = id;
    WSYNC();
  }
  nadd = j1;
  return true;
}

// dl = M_F g from dl = M g: dl -= sum_j w_j (w_j' g) / d_j over the nadd faces held
template <int NC>
__device__ __forceinline__ void dd_apply(Smem<NC>& s, int n, int nadd, const float* gin,
                                         float* dl) {
  const int lane = opaque_lane();
  const float* meta = dd_meta(s);
  n = uniform(n);
  WSYNC();
  float sj[dd_max(NC)];
#pragma unroll
  for (int j = 0; j < dd_max(NC); ++j) {
    if (j >= nadd) break;  // uniform
    const float* w = dd_w(s, j);
    float part = 0.f;
    for (int p = lane; p < n; p += 64) part = fmaf(w[p], gin[p], part);
    sj[j] = wave_sum(part) * meta[j];
  }
  for (int p = lane; p < n; p += 64) {
    float acc = dl[p];
#pragma unroll
    for (int j = 0; j < dd_max(NC); ++j) {
      if (j >= nadd) break;
      acc = fmaf(-sj[j], dd_w(s, j)[p], acc);
    }
    dl[p] = acc;
  }
  WSYNC();
}

// park / restore the register-resident inverse in the wave's global slab (uniform base,
// 32-bit lane offset: no per-tile 64-bit address registers)
template <int NC>
__device__ __forceinline__ void park_store(float* __restrict__ park, const f4 (&M)[Cfg<NC>::NTL]) {
  const int lane = opaque_lane();
#pragma unroll
  for (int t = 0; t < Cfg<NC>::NTL; ++t)
    *reinterpret_cast<f4*>(&park[t * 256 + lane * 4]) = M[t];
}

template <int NC>
__device__ __forceinline__ void park_load(const float* __restrict__ park, f4 (&M)[Cfg<NC>::NTL]) {
  const int lane = opaque_lane();
  asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc1" ::: "memory");
#pragma unroll
  for (int t = 0; t < Cfg<NC>::NTL; ++t)
    M[t] = *reinterpret_cast<const f4*>(&park[t * 256 + lane * 4]);
}

#include "cmpc_team.hip"  // W waves per QP for small batches (leader + helpers)

// ------------------------------------------------------------------------------------------
// one QP instance on one wave (W = 1) or led by wave 0 of a W-wave team (cmpc_team.hip)
// A polish session starts from the face set in s.code: record it as the session's first tried
// set and look it up among the starting sets of failed sessions.  Returns the session's repair
// budget (none for a remembered set).
template <int NC>
__device__ __forceinline__ int session_start(Smem<NC>& s, const KParams& P, int ntri, int nfail,
                                             int& ntried, bool& seen) {
  const int l = opaque_lane();
  WSYNC();
  uint8_t c = 0;
  if (l < ntri) {
    c = (uint8_t)s.code[l];
    s.tpat[0][l] = c;
  }
  ntried = 1;
  seen = false;
#pragma unroll
  for (int k = 0; k < kFailMem; ++k) {
    if (k >= nfail) break;  // uniform: only this instance's failed sessions
    const bool diff = (l < ntri) && (s.fpat[k][l] != c);
    seen |= (__any(diff) == 0);
  }
  if (seen) return 0;  // a remembered set is polished once more, without repairs
  // after two failed sessions the repair budget shrinks: a wandering repair sequence costs a
  // factorization per step (cfg1 +1 %, cfg2 +1-2 %)
  return (nfail >= 2) ? min(P.polish_repairs, kLateRepairs) : P.polish_repairs;
}

// Has the current session already tried the repaired face set in s.tcnt?
template <int NC>
__device__ __forceinline__ bool tried_before(Smem<NC>& s, int ntri, int ntried) {
  const int l = opaque_lane();
  WSYNC();
  const uint8_t c = (l < ntri) ? (uint8_t)s.tcnt[l] : 0;
  bool hit = false;
  for (int k = 0; k < ntried; ++k) {  // uniform trip count
    const bool diff = (l < ntri) && (s.tpat[k][l] != c);
    hit |= (__any(diff) == 0);
  }
  return hit;
}

template <int NC, int W>
__device__ __forceinline__ void solve_instance(Smem<NC>& s, const KParams& P, int64_t b,
                                               const Inputs& in, const Outputs& out,
                                               float* __restrict__ park, TeamSmem<NC, W>* ts,
                                               int* seq) {
  // W = 1: the whole lower triangle in this wave's registers; W > 1: this wave's team slots
  f4 M[TeamCfg<NC, W>::SLOTS];
  static_assert(W > 1 || TeamCfg<NC, W>::SLOTS == Cfg<NC>::NTL, "W = 1 holds every tile");
  const int lane = opaque_lane();
  const int N = P.N;
  const int NP = 12 * N;
#if defined(CMPC_POISON_LDS)  // diagnostic: NaN into the float scratch before every instance
  if constexpr (W == 1) {
    const float qn = __int_as_float(0x7fc00000);
    for (int i = lane; i < 12 * NC; i += 64) s.G[i] = qn;
    for (int i = lane; i < NC; i += 64) s.v[i] = qn;
    WSYNC();
  }
#endif
#if defined(CMPC_POISON_PARK)  // diagnostic: NaN into the wave's park slab before every instance
  if constexpr (W == 1) {
    const float qn = __int_as_float(0x7fc00000);
    for (int i = lane; i < Cfg<NC>::SLAB; i += 64) park[i] = qn;
  }
#endif
  const float* Ab = in.Ad + b * 144;
  const float* Bg = in.Bd + b * (int64_t)N * 144;
  const float* gdb = in.gd + b * 12;
  const float* x0b = in.x0 + b * 12;
  const float* xrb = in.xref + b * (int64_t)N * 12;
  const uint8_t* ctb = in.contact + b * (int64_t)4 * N;
  CMPC_T0(t_inst);
  CMPC_CNT(10, 1);

  WSYNC();
  {  // one round of global loads: A, r_0..r_N (= x0, xref), gd; staged in LDS (G is free here)
    float av[3], rv[4];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int e = lane + 64 * i;
      av[i] = (e < 144) ? Ab[e] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = lane + 64 * i;
      rv[i] = (e < 12) ? x0b[e] : (e < 12 * (N + 1)) ? xrb[e - 12] : 0.f;
    }
    const float gv = (lane < 12) ? gdb[lane] : 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int e = lane + 64 * i;
      if (e < 144) s.A[e] = av[i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) s.G[lane + 64 * i] = rv[i];
    if (lane < 12) s.G[256 + lane] = gv;
  }
  // stance triples in (k, leg) order; lane = 4k + leg
  const bool stc = (lane < 4 * N) ? (ctb[(lane & 3) * N + (lane >> 2)] != 0) : false;
  const int pos = wave_excl_scan4(stc ? 1 : 0);
  const int ntri = wave_total4(stc ? 1 : 0);
  if (stc) s.tri[pos] = lane;
  if (lane < 4 * N) s.tri_of[lane] = stc ? pos : -1;
  WSYNC();
  {
    for (int o = lane; o < NP; o += 64) {  // d_k = A r_k + gd - r_{k+1}, r_0 = x0
      const int k = o / 12, r = o % 12;
      const float* rk = &s.G[12 * k];
      float acc = s.G[256 + r] - rk[12 + r];
#pragma unroll
      for (int j = 0; j < 12; ++j) acc = fmaf(s.A[r * 12 + j], rk[j], acc);
      s.D[o] = acc;
    }
    build_admm_basis<NC>(s, P, Bg, ntri);
  }
  const int n = 3 * ntri;
  const bool nil = nilpotent_step(s);  // A = I + N, N^2 = 0: the closed-form condensation
  if (lane == 0) s.nil = nil ? 1 : 0;   // (and the gradient's powers of A)
  WSYNC();
  // team mode: the gradient's powers of A once per instance (registers to spare: the tiles are
  // split over the team)
  // (NC <= 128 only: the larger bins need those registers for their tiles)
  constexpr bool kPow = W > 1 && NC <= 128;
  f4 pw_c[4], tw_c[4];
  if constexpr (kPow) gradient_powers(s, pw_c, tw_c);
  const f4* pwc = kPow ? pw_c : nullptr;
  const f4* twc = kPow ? tw_c : nullptr;
  // initial rho per bin: the NC >= 128 bins (33-64 stance triples) converge in fewer iterations
  // from rho0 / 2; their hard instances (a failed polish session) go back to rho0, where they
  // converge as before (NC = 128: cfg1 +6-10 %, cfg2 +1 %; NC >= 160: kRhoLowHeavy; rho0 / 2
  // for the NC = 96 bin too loses 7 % on cfg2)
  constexpr bool kLow = (NC == 128) || (kRhoLowHeavy && NC > 128);
  float rho = kLow ? 0.5f * P.rho0 : P.rho0;
  bool rho_low = kLow;  // still at the bin's reduced initial rho
  s.pcode[lane] = -1;
  if (in.w_init == nullptr && in.y_init == nullptr && in.lam_init == nullptr) {
    for (int p = lane; p < n; p += 64) { s.x[p] = 0.f; s.z[p] = 0.f; s.y[p] = 0.f; }
  } else if (lane < ntri) {
    // warm start (the reference's x0 / lam_x0 of centroidal_mpc.py:91-95): triple `lane`
    // (step k, leg l) starts at x = z = Pi_K(u_init), y = y_init; its face code seeds the
    // polish trigger with the projection of u + y / rho, the first z-update's argument
    const int kl = s.tri[lane];
    const int fo = 12 * (kl >> 2) + 3 * (kl & 3);
    float u[3] = {0.f, 0.f, 0.f}, yv[3] = {0.f, 0.f, 0.f};
    if (in.w_init) {
      const float* wi = in.w_init + b * (int64_t)(24 * N) + NP + fo;
#pragma unroll
      for (int a = 0; a < 3; ++a) u[a] = wi[a];
    }
    if (in.y_init) {
      const float* yi = in.y_init + b * (int64_t)NP + fo;
#pragma unroll
      for (int a = 0; a < 3; ++a) yv[a] = yi[a];
    } else if (in.lam_init) {
      // the reference's multipliers (centroidal_mpc.py:91-95 lam_x0 / lam_a0) -> this solver's
      // dual of the force: y = F' lam_fric + lam_x[u] (stationarity of the input rows:
      // 2R u - Bd' lam_eq + F' lam_fric + lam_x = 0 and y = -(2R u - Bd' lam_eq))
      const float* li = in.lam_init + b * (int64_t)(52 * N);
      const float* lf = li + 24 * N + NP + 16 * (kl >> 2) + 4 * (kl & 3);  // lam_a friction rows
      const float* lx = li + NP + fo;                                        // lam_x of the force
      const float f0 = lf[0], f1 = lf[1], f2 = lf[2], f3 = lf[3];
      yv[0] = f0 - f1 + lx[0];
      yv[1] = f2 - f3 + lx[1];
      yv[2] = -P.mu * (f0 + f1 + f2 + f3) + lx[2];
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {  // non-finite warm data falls back to a cold start
      if (!isfinite(u[a])) u[a] = 0.f;
      if (!isfinite(yv[a])) yv[a] = 0.f;
    }
    float pv[3], qv[3];
    project(u[0], u[1], u[2], P.mu, P.fz_min, pv[0], pv[1], pv[2]);
    int code;
    if (in.y_init || in.lam_init) {  // the dual pushes the faces it holds outward (at the bin's initial rho)
      const float ir = 1.f / rho;
      code = project(pv[0] + yv[0] * ir, pv[1] + yv[1] * ir, pv[2] + yv[2] * ir, P.mu, P.fz_min,
                     qv[0], qv[1], qv[2]);
    } else {          // primal only: the faces the warm point lies on, to fp32 rounding
      const float tz = 1e-5f * fmaxf(pv[2], 1.f), lim = P.mu * pv[2] - 1e-5f * pv[2];
      code = (pv[2] <= P.fz_min + tz) ? 1 : 0;
      code |= (pv[0] >= lim) ? 2 : (pv[0] <= -lim) ? 4 : 0;
      code |= (pv[1] >= lim) ? 8 : (pv[1] <= -lim) ? 16 : 0;
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      s.x[3 * lane + a] = pv[a];
      s.z[3 * lane + a] = pv[a];
      s.y[3 * lane + a] = yv[a];
    }
    s.pcode[lane] = code;
  }

  CMPC_ACC(6, t_inst);
  // ADMM state (x, z, y of triple t at 3t .. 3t+2) lives in LDS, not in registers

  int status = -2, iters = 0;
#ifdef CMPC_DIAG_GRES
  float dg_gm = -1.f, dg_cm = -1.f, dg_us = 0.f;  // (-1: not a polished point)
#endif
#ifdef CMPC_DIAG_COUNTS
  int dg_fact = 0, dg_pol = 0, dg_flags = 0;
  unsigned long long dg_t0 = __builtin_amdgcn_s_memtime();
  float dg_fail_t[4] = {0.f, 0.f, 0.f, 0.f};  // cycles at the end of failed sessions 1..4
  int dg_fail_f[4] = {0, 0, 0, 0};            // factorizations by then
  int dg_nf = 0;
#endif
#ifdef CMPC_DIAG_TIMES  // diagnostic build: start / end on the 100 MHz constant clock
  unsigned long long dt_t0 = __builtin_amdgcn_s_memrealtime();
#endif
  bool polished = false;
  float rp = 0.f, rd = 0.f, np_ = 0.f, nd = 0.f;
  int stable = 0;
  bool refactor = n > 0;  // (re)build + invert the matrix for the current basis
  bool in_polish = false;
  int nact = n;           // params of the current basis
  float shift = uniformf(P.sigma + rho);
  int it = 0;
  int repairs_left = 0;
  int nadd = 0;           // faces added by downdates since the last factorization
  bool from_cand = false; // the polish refactored from a candidate that passed its check
  bool parked = false;    // the ADMM inverse is in the park slab
  int nfail = 0;          // failed sessions so far (the memory holds the last kFailMem)
  int ntried = 0;         // face sets tried in the current session
  bool seen_start = false;  // the current session started from a remembered failed set
  int last_pol = 0;       // iteration of the last polish session
  bool fail_rho_done = false;  // rho moved to kFailRho x rho0 after the first failed session
  const float alpha = P.alpha;
  if (n == 0) status = 1;
  bool warm_session = false;  // the current polish session is the warm start's
  if (n > 0 && in.w_init != nullptr) {
    // warm active set: the face set of the warm point goes straight to the polish (one
    // reduced factorization instead of the ADMM one + the polish one); if its KKT check and
    // repairs fail, the instance restarts as a cold solve (below)
    warm_session = true;
    WSYNC();
    if (lane < ntri) s.code[lane] = s.pcode[lane];
    repairs_left = session_start<NC>(s, P, ntri, nfail, ntried, seen_start);
    nact = polish_setup<NC>(s, P, Bg, ntri, s.z);
    shift = P.sigma;
    in_polish = true;
  }
  while (n > 0) {
    if (refactor) {  // the only condense + invert call site
      CMPC_CNT(8, 1);
#ifdef CMPC_TRACE
      if (trace_on(b) && lane == 0)
        printf("[%d] it %d FACTOR polish %d nact %d shift %g\n", (int)b, it, (int)in_polish, nact, shift);
#endif
#ifdef CMPC_DIAG_COUNTS
      ++dg_fact;
#endif
      if constexpr (W == 1) {
        CMPC_T0(t_c);
        condense_tiles<NC>(s, P, M, nact, uniformf(shift), nil);
        CMPC_ACC(0, t_c);
        CMPC_T0(t_i);
        ldl_tiles<NC>(s, M, nact);
        CMPC_ACC(1, t_i);
      } else {
        CMPC_T0(t_c);
        team_factor_lead<NC, W>(s, *ts, *seq, P, M, nact, uniformf(shift));
        CMPC_ACC(0, t_c);
      }
      refactor = false;
    }
    if (in_polish) {
      CMPC_T0(t_pol);
      // iterative refinement v -= M (grad): polish_refine steps, then more (up to
      // kRefineExtra) while the step still contracts and is above the acceptance tolerance --
      // an ill-conditioned face set (internal foot forces weigh only R) contracts slowly
      float step = 3.0e38f, prev = 3.0e38f, vscale = 1.f;
      bool ok = false, changed = false, loose = false, converged = false, stalled = false;
      bool decisive = true;
      bool amb_last = false;  // (trace)
      float vworst = 0.f;
      // refinement steps before the convergence test may stop them: polish_refine from ADMM's
      // rough point; one from a candidate that already passed the check (a stall re-check)
      const int qmin = from_cand ? 1 : P.polish_refine;
      from_cand = false;
      for (int pass = 0;; ++pass) {
        // (an extra pass -- ambiguous face multipliers, below -- is one more refinement step)
        for (int q = pass == 0 ? 0 : P.polish_refine + kRefineExtra - 1;
             q < P.polish_refine + kRefineExtra; ++q) {
          gradient<NC, (W > 1), true>(s, P, nact, s.v, s.g, pwc, twc);
          if constexpr (W == 1) {
            minv_apply<NC>(s, P, M, nact, s.g, s.dl);
            if (nadd > 0) dd_apply<NC>(s, nact, nadd, s.g, s.dl);  // (uniform)
          } else {
            team_symv_lead<NC, W>(s, *ts, *seq, M, nact, s.g, s.dl);
          }
          float m = 0.f, mv = 1.f;
          for (int p = lane; p < nact; p += 64) {
            const float vn = s.v[p] - s.dl[p];
            s.v[p] = vn;
            m = fmaxf(m, fabsf(s.dl[p]));
            mv = fmaxf(mv, fabsf(vn));
          }
          step = wave_max(m);
          vscale = wave_max(mv);
  #ifdef CMPC_TRACE
          if (trace_on(b) && lane == 0) printf("[%d]     refine %d step %g\n", (int)b, q, step);
  #endif
          stalled = step > kRefineRate * prev;
          if (q + 1 >= qmin && (step <= P.polish_tol * wave_max(mv) || stalled)) break;
          prev = step;
        }
        gradient<NC, (W > 1), true>(s, P, nact, s.v, s.g, pwc, twc);  // E, L at the final point
        // a hard instance's later repairs move only the worst triples: full primal-dual
        // active-set steps swap several faces at a time and can wander between neighbouring sets
        const int top = (kRepairTop > 0 && (nfail > 0 || ntried >= 3)) ? kRepairTop : 0;
        bool amb = false;
  #ifdef CMPC_TRACE
        ok = polish_check<NC>(s, P, Bg, ntri, step, changed, loose, converged, amb, decisive,
                              vworst, top, trace_on(b) ? (int)b : -1);
  #else
        ok = polish_check<NC>(s, P, Bg, ntri, step, changed, loose, converged, amb, decisive,
                              vworst, top);
  #endif
        amb_last = amb;
        // A face multiplier near zero decides the check but moves by ~|H| x the point's remaining
        // error (a step accepted at polish_tol x the force scale leaves ~1e-5 N, i.e. ~1e-7 in a
        // multiplier -- the force-unit tolerance's size: config-3 instance 54289 passed with fz
        // held at fz_min, multiplier -3e-8 at its point, -1.3e-6 at the converged one, a
        // 1.2e-4 error; next-tick 55062 warm held fy at mu fz with +2.5e-7 at its point,
        // -3.2e-7 converged, 1.06e-4).  Such a check is repeated after further refinement steps.
        if (!(amb && (ok || loose)) || pass >= kAmbRefine ||
            step <= kAmbConverged * P.polish_tol * vscale)
          break;
      }
#ifdef CMPC_TRACE
      if (trace_on(b) && lane == 0)
        printf("[%d] it %d polish nact %d nadd %d ok %d loose %d changed %d amb %d dec %d step %g "
               "stalled %d repairs_left %d ntried %d nfail %d\n", (int)b, it, nact, nadd, (int)ok,
               (int)loose, (int)changed, (int)amb_last, (int)decisive, step, (int)stalled,
               repairs_left, ntried, nfail);
#endif
      CMPC_ACC(4, t_pol);
      // A refinement on a downdated inverse that stopped contracting above the tight level
      // (fp32 downdates of an ill-conditioned face set: steps 1e-4, 3.1e-5, 2.9e-5) leaves
      // multipliers near zero unreliable -- config-3 instance 31861 held a degenerate friction
      // face at -1.6e-7, released it, found it violated, and cycled through 5 sessions and 130
      // ADMM iterations.  When only such multipliers fail the check, the face set is refactored
      // exactly before the check decides.  (Refactoring every stalled downdate also fixed 31861
      // but cost 6-10 % more factorizations on configs 2-3: most stalls sit at the fp32 floor
      // of checks that large violations decide anyway.)
      // Nor is a point accepted while a downdated refinement stopped contracting above the
      // fp32 floor: the step is then no bound on the point's error (config-3 instance 39503:
      // three downdates, steps 2.2e-4, 5.7e-4, 5.0e-4 against a tolerance of 9.7e-4, accepted
      // 0.037 N = 3.8e-4 off; 25651: one downdate, steps 6.8e-5, 4.3e-5, 1.0e-4, 2.0e-4 off).
      // The face set is refactored and refined afresh first (round 6: the guard is the product
      // rule -- 9.5 % of config-3 instances, 18 % of config 2's, pass a check on such a
      // refinement, so answering them as status 2 instead was no option; profiles/r06a_*)
      const bool dd_stalled = nadd > 0 && stalled && step > kAmbConverged * P.polish_tol * vscale;
      const bool dd_stall = dd_stalled && (ok || loose || !decisive);
      if (dd_stall) {
        converged = false;
        if (out.stats != nullptr && lane == 0) atomicAdd(&out.stats[2], 1ull);  // (rare)
#ifdef CMPC_DIAG_COUNTS
        dg_flags |= 4;
#endif
      }
      // status 1 contract (include/cmpc.h): the check passed on a refinement that converged
      // (and, after downdates, still contracted), and the held faces' certified force error is
      // within kCertFace of the force scale (nilpotent step: the float64 rollout's
      // multipliers); a point that misses the bound is returned as status 2
      if (ok && !dd_stall) {
#ifdef CMPC_DIAG_GRES
        diag_gres<NC>(s, P, nact, dg_gm, dg_cm, dg_us);
#endif
        const bool cert = !uniform(s.nil) || certified_faces<NC>(s, P);
        if (!cert && out.stats != nullptr && lane == 0) atomicAdd(&out.stats[1], 1ull);
#ifdef CMPC_DIAG_COUNTS
        if (!cert) dg_flags |= 2;
#endif
        polished = true;
        status = cert ? 1 : 2;
        break;
      }
      if (nadd > 0 && !converged) {
        // the downdated inverse stopped contracting: refactor the current face set, from the
        // candidate forces (not a repair)
#ifdef CMPC_TRACE
        if (trace_on(b) && lane == 0) printf("[%d] it %d STALL-REFACTOR dd_stall %d\n", (int)b, it, (int)dd_stall);
#endif
        nact = polish_setup<NC>(s, P, Bg, ntri, s.dl);
        nadd = 0;
        shift = P.sigma;
        refactor = true;
        from_cand = ok || loose;  // (the guard: the candidate passed; its error is what is checked)
        continue;
      }
      if (repairs_left > 0 && changed && !tried_before<NC>(s, ntri, ntried)) {
        // re-polish on the repaired face set
        --repairs_left;
        bool dd = false;
        if constexpr (W == 1) {
          // only added faces: downdate the inverse in the current basis (no refactorization)
          const int l = opaque_lane();
          WSYNC();
          const int oc = (l < ntri) ? s.code[l] : 0, nc = (l < ntri) ? s.tcnt[l] : 0;
          const int add = nc & ~oc;
          const int nf = wave_total4((add & 1) + ((add & 6) != 0) + ((add & 24) != 0));
#ifdef CMPC_TRACE
          {
            const bool drop = __any((nc & oc) != oc), freed = __any(((nc ^ oc) & oc & 1) != 0);
            if (trace_on(b) && lane == 0)
              printf("[%d] it %d repair drop %d (fz face freed %d) nf %d nadd %d cap %d\n", (int)b,
                     it, (int)drop, (int)freed, nf, nadd, dd_max(NC));
          }
#endif
          if (__any((nc & oc) != oc) == 0 && nadd + nf <= dd_max(NC)) {  // (uniform)
            CMPC_T0(t_dd);
            dd = face_downdate<NC>(s, P, M, nact, ntri, nadd);
#ifdef CMPC_TRACE
            if (trace_on(b) && lane == 0)
              printf("[%d] it %d downdate nf %d -> %d nadd %d\n", (int)b, it, nf, (int)dd, nadd);
#endif
            CMPC_ACC(28, t_dd);
            CMPC_CNT(29, 1);
            CMPC_CNT(30, nf);
          }
        }
        if (lane < ntri) {
          s.code[lane] = s.tcnt[lane];
          if (ntried < kTryMem) s.tpat[ntried][lane] = (uint8_t)s.tcnt[lane];
        }
        if (ntried < kTryMem) ++ntried;
        if (dd) continue;  // refine on the downdated inverse
        nact = polish_setup<NC>(s, P, Bg, ntri, s.z);
        nadd = 0;
        shift = P.sigma;
        refactor = true;
        continue;
      }
      if (loose) {  // the session ends on a set within the loose tolerance: accept it
#ifdef CMPC_DIAG_GRES
        diag_gres<NC>(s, P, nact, dg_gm, dg_cm, dg_us);
#endif
        const bool certok = certified_faces<NC>(s, P);
        const int l = opaque_lane();
        WSYNC();
        if (l < ntri) {  // (projected onto the pyramid: the loose check admits 5x polish_tol)
          float px, py, pz;
          project(s.dl[3 * l], s.dl[3 * l + 1], s.dl[3 * l + 2], P.mu, P.fz_min, px, py, pz);
          s.x[3 * l] = px;
          s.x[3 * l + 1] = py;
          s.x[3 * l + 2] = pz;
        }
        polished = true;
        // KKT-verified within the loose bounds only with the float64 rollout (polish_check) and
        // the certified face bound; a general A's loose acceptance is reported as not verified
        status = (uniform(s.nil) && certok) ? 1 : 2;
        if (out.stats != nullptr && lane == 0) {
          atomicAdd(&out.stats[0], 1ull);
          if (!certok) atomicAdd(&out.stats[1], 1ull);
        }
#ifdef CMPC_DIAG_COUNTS
        dg_flags |= 1 | (certok ? 0 : 2);
#endif
        break;
      }
      if (warm_session) {
        // The warm face set failed (the state moved across a face change): restart exactly as
        // the cold solve of this problem -- x = z = y = 0, the bin's initial rho, no failed
        // session on record -- so a warm start never takes more ADMM iterations than cold.
        // (Continuing ADMM from the warm (x, z, y) counted the warm set as a failed session:
        // 4 x rho0, 3x the stable run, the back-off -- the hard-instance schedule -- and the
        // round-4 bench's warm maximum was 253 iterations against 107 cold.)
        warm_session = false;
        build_admm_basis<NC>(s, P, Bg, ntri);  // (zeroes x, z, y past n)
        {
          const int l = opaque_lane();
          for (int p = l; p < n; p += 64) { s.x[p] = 0.f; s.z[p] = 0.f; s.y[p] = 0.f; }
          s.pcode[l] = -1;
        }
        WSYNC();
        in_polish = false;
        nact = n;
        nadd = 0;
        rho = kLow ? 0.5f * P.rho0 : P.rho0;
        rho_low = kLow;
        shift = uniformf(P.sigma + rho);
        refactor = true;
        stable = 0;
        last_pol = 0;
        ntried = 0;
        seen_start = false;
        parked = false;
        continue;
      }
      warm_session = false;
#ifdef CMPC_TRACE
      if (trace_on(b) && lane == 0)
        printf("[%d] it %d SESSION-FAIL nfail %d seen %d parked %d rho_low %d fail_rho_done %d nadd %d\n",
               (int)b, it, nfail, (int)seen_start, (int)parked, (int)rho_low, (int)fail_rho_done, nadd);
#endif
#ifdef CMPC_DIAG_COUNTS
      if (dg_nf < 4) {
        dg_fail_t[dg_nf] = (float)(__builtin_amdgcn_s_memtime() - dg_t0);
        dg_fail_f[dg_nf] = dg_fact;
      }
      ++dg_nf;
#endif
      // the session failed: remember its starting face set (unless it came from the memory)
      if (!seen_start) {
        const int l = opaque_lane();
        if (l < ntri) s.fpat[nfail % kFailMem][l] = s.tpat[0][l];
        ++nfail;
      }
      // restore the basis and the parked ADMM inverse (or rebuild it first), continue ADMM
      build_admm_basis<NC>(s, P, Bg, ntri);
      in_polish = false;
      nact = n;
      if (nfail == 1 && !seen_start && kFailRho != 1.f && !fail_rho_done) {
        // the first failed session: a hard instance continues at kFailRho x rho0 (one refactor;
        // nothing is parked before the second session, so it would refactor anyway)
        fail_rho_done = true;
        rho_low = false;
        rho = uniformf(kFailRho * P.rho0);
        shift = uniformf(P.sigma + rho);
        refactor = true;
        continue;
      }
      if (rho_low) {  // a hard instance: back to the standard rho0 (one refactor)
        rho_low = false;
        rho = uniformf(P.rho0);
        shift = uniformf(P.sigma + rho);
        refactor = true;
        continue;
      }
      shift = uniformf(P.sigma + rho);
      if (parked) {
        if constexpr (W == 1) {
          park_load<NC>(park, M);
        } else {
          team_issue<NC, W>(*ts, *seq, kOpParkLoad, 0, 0, 0);
          team_park_load<NC, W, 0>(park, M, 0);
        }
      } else {
        refactor = true;  // M holds the polish inverse: refactor before the next iteration
        continue;
      }
    }
    if (it >= P.max_iter) break;
    ++it;
    iters = it;
    // ---- one ADMM iteration ----
    gradient<NC, (W > 1)>(s, P, n, s.x, s.g, pwc, twc);
    {
      const int l = opaque_lane();
      if (l < ntri) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          const int p = 3 * l + a;
          s.r[p] = rho * (s.z[p] - s.x[p]) - s.g[p] - s.y[p];
        }
      }
    }
    if constexpr (W == 1) {
      minv_apply<NC>(s, P, M, n, s.r, s.dl);
    } else {
      team_symv_lead<NC, W>(s, *ts, *seq, M, n, s.r, s.dl);
    }
    CMPC_T0(t_rest);
    const bool last = (it == P.max_iter);
    const bool adapt = P.adaptive_interval > 0 && (it % P.adaptive_interval) == 0;
    const float inv_rho = 1.f / rho;
    float lrp = 0.f, lrd = 0.f, lnp = 0.f, lnd = 0.f;
    bool changed = false;
    {
      const int l = opaque_lane();
      if (l < ntri) {
        float w[3], xr[3], xs[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          const int p = 3 * l + a;
          const float x = s.x[p], z = s.z[p];
          const float xt = x + s.dl[p];
          xr[a] = alpha * xt + (1.f - alpha) * z;
          xs[a] = alpha * xt + (1.f - alpha) * x;
          w[a] = xr[a] + s.y[p] * inv_rho;
        }
        float pv[3];
        const int code = project(w[0], w[1], w[2], P.mu, P.fz_min, pv[0], pv[1], pv[2]);
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          const int p = 3 * l + a;
          const float zn = pv[a];
          const float yn = s.y[p] + rho * (xr[a] - zn);
          s.x[p] = xs[a];
          s.z[p] = zn;
          s.y[p] = yn;
          const float gp = s.g[p];
          lrp = fmaxf(lrp, fabsf(xs[a] - zn));
          lrd = fmaxf(lrd, fabsf(gp + yn));
          lnp = fmaxf(lnp, fmaxf(fabsf(xs[a]), fabsf(zn)));
          lnd = fmaxf(lnd, fmaxf(fabsf(gp), fabsf(yn)));
        }
        changed = code != s.pcode[l];
        s.pcode[l] = code;
        s.code[l] = code;
      }
    }
#ifdef CMPC_TRACE
    if (trace_on(b)) {
      const float trp = wave_max(lrp), trd = wave_max(lrd);
      if (lane == 0)
        printf("[%d] it %d rho %g rp %g rd %g stable %d\n", (int)b, it, rho, trp, trd, stable);
    }
#endif
    stable = (__any(changed) != 0) ? 0 : stable + 1;
    bool do_pol = false;
    // back off before a further attempt, longer after failed sessions: both the stable run and
    // the distance to the last session grow as polish_stable x 2^min(nfail, kBackoffCap)
    const int pstable = P.polish_stable;
    const int backoff = pstable << min(nfail, kBackoffCap);
    int need = pstable;  // (kStableGrow: the stable run required grows per failed session)
    for (int f = 0; f < min(nfail, kBackoffCap); ++f) need *= kStableGrow;
    if (stable >= need && !last && it - last_pol >= backoff &&
        (P.check_every == 1 || it % P.check_every == 0)) {  // (OPTS check_termination)
      do_pol = true;
      last_pol = it;
      stable = -backoff;
    }
    if (adapt || last) {
      rp = wave_max(lrp); rd = wave_max(lrd); np_ = wave_max(lnp); nd = wave_max(lnd);
    }
    if (adapt && !last) {
      float q = rho * sqrtf((rp / fmaxf(np_, 1e-30f)) / (rd / fmaxf(nd, 1e-30f) + 1e-30f));
      q = fminf(fmaxf(q, 1e-6f), 1e6f);
      if (q > 5.f * rho || q < 0.2f * rho) {
        rho = uniformf(q);
        rho_low = false;
        shift = uniformf(P.sigma + rho);
        refactor = true;
      }
    }
    CMPC_ACC(7, t_rest);
    if (do_pol) {
      CMPC_CNT(9, 1);
#ifdef CMPC_DIAG_COUNTS
      ++dg_pol;
#endif
      CMPC_T0(t_ps);
      // Park (write the 36-108 KB inverse to the wave's slab) only where a failed session will
      // restore it: not when a refactor is pending (rho changed: the inverse is stale), not at
      // the NC = 128 bin's reduced rho (a failure refactors at rho0), and not in the first
      // session (most instances pass it; the few that fail refactor once).  HBM writes of a
      // config-3 step drop from ~36 KB to a few hundred bytes per instance at unchanged speed.
      parked = !refactor && !rho_low && nfail > 0;
      if (parked) {  // restored if the polish fails
        if constexpr (W == 1) {
          park_store<NC>(park, M);
        } else {
          team_issue<NC, W>(*ts, *seq, kOpParkStore, 0, 0, 0);
          team_park_store<NC, W, 0>(park, M, 0);
        }
      }
      repairs_left = session_start<NC>(s, P, ntri, nfail, ntried, seen_start);
      nact = polish_setup<NC>(s, P, Bg, ntri, s.z);
      nadd = 0;
#ifdef CMPC_TRACE
      if (trace_on(b) && lane == 0)
        printf("[%d] it %d SESSION nfail %d parked %d rho %g refactor_pending %d seen %d repairs %d nact %d\n",
               (int)b, it, nfail, (int)parked, rho, (int)refactor, (int)seen_start, repairs_left, nact);
#endif
      CMPC_ACC(14, t_ps);
      shift = P.sigma;
      refactor = true;
      in_polish = true;
    }
  }
  if (!polished) {
    if (n > 0) {
      const bool conv = rp <= P.eps_abs + P.eps_rel * np_ && rd <= P.eps_abs + P.eps_rel * nd;
      status = conv ? 2 : -2;
    }
    gradient<NC, (W > 1)>(s, P, n, s.z, s.g, pwc, twc);  // E at u = z (the pure rollout when every leg swings)
  }
#ifdef CMPC_TRACE
  if (trace_on(b) && lane == 0) printf("[%d] END status %d iters %d\n", (int)b, status, iters);
#endif
  CMPC_T0(t_out);
  // ---- outputs: x_{k+1} = e_{k+1} + xref_k, u from the triples (zero on swing legs) ----
  WSYNC();
  float* wb = out.w + b * (int64_t)(24 * N);
  const float* uf = polished ? s.x : s.z;  // polished forces overwrote x; else u = z
  int bad = 0;
  for (int o = lane; o < NP; o += 64) {
    const float xv = s.E[o] + xrb[o];
    const int k = o / 12, l = (o % 12) / 3, a = o % 3;
    const int t = s.tri_of[4 * k + l];
    const float uv = (t >= 0) ? uf[3 * t + a] : 0.f;
    bad |= !(isfinite(xv) && isfinite(uv));
    wb[o] = xv;
    wb[NP + o] = uv;
  }
  if (__any(bad)) status = -10;
#ifdef CMPC_DIAG_COUNTS  // diagnostic build: w[0..7] = cycles and factorizations at failed sessions 1..4
  if (lane < 4) wb[lane] = dg_fail_t[lane];
  else if (lane < 8) wb[lane] = (float)dg_fail_f[lane - 4];
#endif
#ifdef CMPC_DIAG_GRES  // diagnostic build: w[0..2] = the gradient and face metrics, the force scale
  if (lane == 0) { wb[0] = dg_gm; wb[1] = dg_cm; wb[2] = dg_us; }
#endif
  if (out.y) {  // dual at the returned forces, in the force layout (zero on swing legs)
    if (polished && n > 0) {  // y = -grad f(u*) (the ADMM fixed point); s.g is the reduced one
      build_admm_basis<NC>(s, P, Bg, ntri);
      gradient<NC, (W > 1)>(s, P, n, s.x, s.g, pwc, twc);
    }
    const float* yf = polished ? s.g : s.y;
    const float sg = polished ? -1.f : 1.f;
    float* yb = out.y + b * (int64_t)NP;
    for (int o = lane; o < NP; o += 64) {
      const int k = o / 12, l = (o % 12) / 3, a = o % 3;
      const int t = s.tri_of[4 * k + l];
      yb[o] = (t >= 0) ? sg * yf[3 * t + a] : 0.f;
    }
  }
  if (out.lam) {  // the reference's multipliers at the returned point (CasADi convention)
    // L holds lambda_k = the adjoint at the returned forces (the last gradient call), and
    // lam_eq[k] = -lambda_k (stationarity of x_{k+1}).  Lane 4k + leg: s = 2R u + Bd_k' lambda_k
    // on its three forces, then the friction-row / bound multipliers of its faces.
    WSYNC();
    float* lb = out.lam + b * (int64_t)(52 * N);
    for (int o = lane; o < NP; o += 64) {
      lb[o] = 0.f;                 // lam_x of the states (free)
      lb[24 * N + o] = -s.L[o];    // lam_a of the dynamics rows
    }
    if (lane < 4 * N) {
      const int k = lane >> 2, leg = lane & 3;
      const int t = s.tri_of[lane];
      const float* Bk = Bg + k * 144 + 3 * leg;
      float sv[3], u[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        u[a] = (t >= 0) ? uf[3 * t + a] : 0.f;
        float acc = s.R2[3 * leg + a] * u[a];
#pragma unroll
        for (int r = 0; r < 12; ++r) acc = fmaf(Bk[r * 12 + a], s.L[12 * k + r], acc);
        sv[a] = acc;
      }
      float lf[4] = {0.f, 0.f, 0.f, 0.f}, lxv[3] = {0.f, 0.f, 0.f};
      if (t < 0) {  // swing: f = 0 by equal bounds, lam_x = -s
#pragma unroll
        for (int a = 0; a < 3; ++a) lxv[a] = -sv[a];
      } else {
        int code;
        if (polished) {
          code = s.code[t];
        } else {  // faces the forces lie on, to fp32 rounding
          const float tz = 1e-5f * fmaxf(u[2], 1.f), lim = P.mu * u[2] - 1e-5f * fmaxf(u[2], 1.f);
          code = (u[2] <= P.fz_min + tz) ? 1 : 0;
          code |= (u[0] >= lim) ? 2 : (u[0] <= -lim) ? 4 : 0;
          code |= (u[1] >= lim) ? 8 : (u[1] <= -lim) ? 16 : 0;
        }
        // rows: fx - mu fz, -fx - mu fz, fy - mu fz, -fy - mu fz  (centroidal_mpc.py:332-355)
        if (code & 2) lf[0] = fmaxf(-sv[0], 0.f);
        if (code & 4) lf[1] = fmaxf(sv[0], 0.f);
        if (code & 8) lf[2] = fmaxf(-sv[1], 0.f);
        if (code & 16) lf[3] = fmaxf(sv[1], 0.f);
        if (code & 1) lxv[2] = fminf(-(sv[2] - P.mu * (lf[0] + lf[1] + lf[2] + lf[3])), 0.f);
      }
      float* lxo = lb + NP + 12 * k + 3 * leg;
#pragma unroll
      for (int a = 0; a < 3; ++a) lxo[a] = lxv[a];
      float* lfo = lb + 24 * N + NP + 16 * k + 4 * leg;
#pragma unroll
      for (int f = 0; f < 4; ++f) lfo[f] = lf[f];
    }
  }
  if (lane == 0) {
#if defined(CMPC_DIAG_COUNTS)  // diagnostic build: iters | attempts | factorizations, cycles / 16
    out.status[b] = (int)((__builtin_amdgcn_s_memtime() - dg_t0) >> 4);
    // (flags: 1 loose acceptance, 2 certified face bound missed, 4 a check on a stalled
    // downdated refinement redone on a fresh factorization)
    out.iters[b] = iters + 1000 * (dg_pol + 100 * dg_flags) + 1000000 * dg_fact;
#elif defined(CMPC_DIAG_TIMES)  // start (10 ns ticks, low 31 bits) | duration + 1e9 if teamed
    out.status[b] = (int)(dt_t0 & 0x7fffffffull);
    out.iters[b] = (int)(__builtin_amdgcn_s_memrealtime() - dt_t0) ;
#else
    out.status[b] = status;
    out.iters[b] = iters;
#endif
  }
  CMPC_CNT(11, iters);
  CMPC_ACC(15, t_out);
  CMPC_ACC(5, t_inst);
}

// Drain one bin's queue with this wave (persistent: instance ids come from a device counter).
// (W > 1: the leader's loop; the helpers leave their command loop at the closing kOpExit)
template <int NC, int W>
__device__ __forceinline__ void drain_bin(Smem<NC>& s, const KParams& P, const Inputs& in,
                                          const Outputs& out, const int* __restrict__ list,
                                          const int* __restrict__ count, int* __restrict__ head,
                                          float* __restrict__ park, TeamSmem<NC, W>* ts = nullptr,
                                          int* seq = nullptr) {
  const int lane = opaque_lane();
  WSYNC();
  if (lane < 12) {  // KParams copies (each bin's Smem layout places them differently)
    s.Q2[lane] = P.Q2[lane];
    s.R2[lane] = P.R2[lane];
  }
  const int total = *count;
  for (;;) {
    int idx = 0;
    if (lane == 0) idx = atomicAdd(head, 1);
    idx = __builtin_amdgcn_readfirstlane(idx);
    if (idx >= total) break;
    const int64_t b = list[idx];
    solve_instance<NC, W>(s, P, b, in, out, park, ts, seq);
  }
  if constexpr (W > 1) team_issue<NC, W>(*ts, *seq, kOpExit, 0, 0, 0);
}

// LDS slot: each class kernel's allocation is padded to a multiple of kLdsSlot, so that an
// NC >= 160 wave's block (2 slots, 39,936 B) is exactly two NC <= 128 blocks (1 slot; 19,632 B
// used) and the 160 KiB of a CU hold 8 of one or 4 of the other (every power-of-two allocation
// granule up to 4 KiB rounds both alike).  When the NC >= 160 class runs first and its waves
// exit one by one, the two NC <= 128 waves that take over each freed SIMD then also fit into
// the LDS it freed: unpadded (27,056 B), the CU's LDS fragmented and the NC <= 128 kernel ran
// with ~1,550 of its 2,048 waves resident for the rest of the step (tools/shard_anatomy.py).
constexpr size_t kLdsSlot = 19968;

// LDS image of a group kernel's bins (NCB = 0: a single-bin kernel)
template <int NC>
constexpr size_t smem_size() {
  if constexpr (NC == 0) return 0;
  else return sizeof(Smem<NC>);
}

// One persistent kernel per register class: bins NCA and NCB share the occupancy (two waves per
// SIMD for NC <= 128, one for NC >= 144), so one kernel serves both, draining the larger bin
// first (its instances are the slower ones: hardest first shortens the batch tail).  NCB = 0:
// one bin (the NC = 192 kernel).  Kernels submitted concurrently on their own streams (the
// caller's + two plan streams) stay within the device's hardware queues, so the classes really
// overlap.
template <int NCA, int NCB>
__global__ void __launch_bounds__(64, Cfg<NCA>::WPE)
    solve_group_kernel(KParams P, Inputs in, Outputs out, const int* __restrict__ list_a,
                       const int* __restrict__ list_b, const int* __restrict__ counts,
                       int* __restrict__ heads, int qa, float* __restrict__ work,
                       size_t slab) {
  static_assert(NCB == 0 || Cfg<NCA>::WPE == Cfg<NCB>::WPE, "a group shares one occupancy class");
  constexpr size_t kImg = smem_size<NCA>() > smem_size<NCB>() ? smem_size<NCA>() : smem_size<NCB>();
  constexpr size_t kBytes = kLdsSlot ? (kImg + kLdsSlot - 1) / kLdsSlot * kLdsSlot : kImg;
  static_assert(!kLdsSlot || 4 * kBytes <= 160 * 1024, "one wave per SIMD must fit the CU's LDS");
  // the two-wave class must stay within ONE slot: a layout change that rounds it up to two
  // would halve its waves per CU (and break the heavy-first hand-over of freed LDS)
  static_assert(!kLdsSlot || Cfg<NCA>::WPE == 1 || kImg <= kLdsSlot, "NC <= 128 image exceeds the LDS slot");
  static_assert(Cfg<NCA>::WPE * 4 * kBytes <= 160 * 1024, "the class's waves per CU must fit the LDS");
  __shared__ __attribute__((aligned(16))) unsigned char raw[kBytes];
  float* park = work + (size_t)blockIdx.x * slab;
#ifdef CMPC_STAMPS
  // st[] is the first member of every Smem<NC>: one set of totals for the wave
  Smem<NCA>& s0 = *reinterpret_cast<Smem<NCA>*>(raw);
  if (threadIdx.x < 32) s0.st[threadIdx.x] = 0;
#endif
  drain_bin<NCA, 1>(*reinterpret_cast<Smem<NCA>*>(raw), P, in, out, list_a, counts + qa,
                         heads + qa, park);
  if constexpr (NCB > 0) {
    drain_bin<NCB, 1>(*reinterpret_cast<Smem<NCB>*>(raw), P, in, out, list_b,
                           counts + qa - 1, heads + qa - 1, park);
  }
#ifdef CMPC_STAMPS
  WSYNC();
  if (threadIdx.x < 32) atomicAdd(&g_stamps[threadIdx.x], s0.st[threadIdx.x]);
#endif
}

// Team mode (cmpc_team.hip): one workgroup of W waves per QP, one kernel for all five bins
// (heaviest first: the slow instances start first).  Wave 0 leads (drain loop +
// solve_instance), waves 1..W-1 serve its matrix commands; the tiles are split W ways, so
// every bin fits the same register class and a small batch needs one launch on the caller's
// stream, no fork/join.  OCC = workgroups per CU: 2 (<= 256 registers per lane) for B > CUs,
// 1 (<= 512: no spills) when every QP has a CU of its own.
template <int W, int OCC>
__global__ void __launch_bounds__(64 * W, OCC)
    solve_team_kernel(KParams P, Inputs in, Outputs out, const int* __restrict__ lists,
                      int64_t stride, const int* __restrict__ counts, int* __restrict__ heads,
                      float* __restrict__ work, size_t slab) {
  constexpr size_t kS0 = sizeof(Smem<192>);
  static_assert(sizeof(Smem<192>) >= sizeof(Smem<160>) && sizeof(Smem<160>) >= sizeof(Smem<128>) &&
                    sizeof(Smem<128>) >= sizeof(Smem<96>), "Smem grows with NC");
  constexpr size_t kS = (kS0 + 15) & ~size_t(15);
  constexpr size_t kT = sizeof(TeamSmem<192, W>);
  static_assert(sizeof(TeamSmem<192, W>) >= sizeof(TeamSmem<160, W>) &&
                    sizeof(TeamSmem<160, W>) >= sizeof(TeamSmem<128, W>) &&
                    sizeof(TeamSmem<128, W>) >= sizeof(TeamSmem<96, W>), "TeamSmem grows with NC");
  __shared__ __attribute__((aligned(16))) unsigned char raw[kS + kT];
  float* park = work + (size_t)blockIdx.x * slab;
  Smem<192>& s3 = *reinterpret_cast<Smem<192>*>(raw);
  Smem<160>& s2 = *reinterpret_cast<Smem<160>*>(raw);
  Smem<128>& s1 = *reinterpret_cast<Smem<128>*>(raw);
  Smem<96>& s0 = *reinterpret_cast<Smem<96>*>(raw);
  TeamSmem<192, W>& t3 = *reinterpret_cast<TeamSmem<192, W>*>(raw + kS);
  TeamSmem<160, W>& t2 = *reinterpret_cast<TeamSmem<160, W>*>(raw + kS);
  TeamSmem<128, W>& t1 = *reinterpret_cast<TeamSmem<128, W>*>(raw + kS);
  TeamSmem<96, W>& t0 = *reinterpret_cast<TeamSmem<96, W>*>(raw + kS);
  const int w = uniform((int)(threadIdx.x >> 6));
  int seq = 0;
#ifdef CMPC_STAMPS
  if (threadIdx.x < 32) s1.st[threadIdx.x] = 0;
#endif
  if (w == 0) {
    drain_bin<192, W>(s3, P, in, out, lists + 4 * stride, counts + 4, heads + 4, park, &t3, &seq);
    // bins 3 (NC 160) and 2 (NC 144) in the NC = 160 image (team mode pairs tile columns, so
    // TT must be even); one copy of the code
#pragma unroll 1
    for (int q = 3; q >= 2; --q)
      drain_bin<160, W>(s2, P, in, out, lists + q * stride, counts + q, heads + q, park, &t2, &seq);
    drain_bin<128, W>(s1, P, in, out, lists + stride, counts + 1, heads + 1, park, &t1, &seq);
    drain_bin<96, W>(s0, P, in, out, lists, counts, heads, park, &t0, &seq);
  } else {
    team_helpers<W, 1>(s3, t3, s2, t2, s1, t1, s0, t0, P, park, w, seq);
  }
#ifdef CMPC_STAMPS
  __syncthreads();
  if (threadIdx.x < 32) atomicAdd(&g_stamps[threadIdx.x], s1.st[threadIdx.x]);
#endif
}

// Binning of a small batch (B <= 1024) in one workgroup: counts are written, not accumulated,
// and the queue heads are zeroed here, so no memset precedes it (one launch less per solve).
__global__ void __launch_bounds__(1024) bin_small_kernel(int N, int B,
                                                         const uint8_t* __restrict__ contact,
                                                         int* __restrict__ counts,
                                                         int* __restrict__ heads,
                                                         int* __restrict__ lists, int64_t stride) {
  __shared__ int wcnt[16][kNumBins];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  int bin = -1;
  if (t < B) {
    const uint8_t* c = contact + (int64_t)t * 4 * N;
    int cnt = 0;
    for (int i = 0; i < 4 * N; ++i) cnt += c[i] != 0;
    const int nf = 3 * cnt;
    bin = kNumBins - 1;
    for (int q = 0; q < kNumBins; ++q)
      if (nf <= kBinCap[q]) { bin = q; break; }
  }
  unsigned long long mine = 0;
#pragma unroll
  for (int q = 0; q < kNumBins; ++q) {
    const unsigned long long m = __ballot(bin == q);
    if (bin == q) mine = m;
    if (lane == 0) wcnt[wv][q] = __popcll(m);
  }
  __syncthreads();
  if (bin >= 0) {
    int base = 0;
    for (int v = 0; v < wv; ++v) base += wcnt[v][bin];
    const int rank = __popcll(mine & ((1ull << lane) - 1ull));
    lists[(int64_t)bin * stride + base + rank] = t;
  }
  if (t < kNumBins) {
    int total = 0;
    for (int v = 0; v < 16; ++v) total += wcnt[v][t];
    counts[t] = total;
    heads[t] = 0;
  }
}

__global__ void __launch_bounds__(256) bin_kernel(int N, int64_t B,
                                                  const uint8_t* __restrict__ contact,
                                                  int* __restrict__ counts,
                                                  int* __restrict__ lists, int64_t stride) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  int bin = -1;
  if (b < B) {
    const uint8_t* c = contact + b * 4 * N;
    int cnt = 0;
    if ((N & 3) == 0) {  // 4N bytes = N words
      const uint32_t* c4 = reinterpret_cast<const uint32_t*>(c);
      for (int i = 0; i < N; ++i) {
        const uint32_t v = c4[i];
        cnt += ((v & 0xffu) != 0) + ((v & 0xff00u) != 0) + ((v & 0xff0000u) != 0) +
               ((v >> 24) != 0);
      }
    } else {
      for (int i = 0; i < 4 * N; ++i) cnt += c[i] != 0;
    }
    const int nf = 3 * cnt;
    bin = kNumBins - 1;
    for (int q = 0; q < kNumBins; ++q)
      if (nf <= kBinCap[q]) { bin = q; break; }
  }
  // one atomic per (wave, bin)
#pragma unroll
  for (int q = 0; q < kNumBins; ++q) {
    const unsigned long long m = __ballot(bin == q);
    if (m == 0) continue;
    const int leader = __ffsll((long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(&counts[q], __popcll(m));
    base = __shfl(base, leader, 64);
    if (bin == q) {
      const int rank = __popcll(m & ((1ull << lane) - 1ull));
      lists[(int64_t)q * stride + base + rank] = (int)b;
    }
  }
}

}  // namespace cmpc
