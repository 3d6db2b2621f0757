// cmpc_kernels.hip -- batched convex-MPC contact-force QP solver for MI355X (gfx950).
//
// One workgroup solves one QP instance of the reference's centroidal MPC
// (convex_mpc/centroidal_mpc.py:69-359).  Algorithm (DESIGN.md "Kernel"):
//
//   1. Condense the horizon onto the free forces only (stance legs; swing forces are fixed at
//      0 by the reference's bounds, centroidal_mpc.py:150-161): H = 2 G'QG + 2R over the
//      free columns via the backward recursion S_j = Q2 + A'S_{j+1}A, W_jj = S_j B_j,
//      W_ij = A'W_{i+1,j}, H_ij = B_i'W_ij.  Every 12x12 product is a chain of four
//      v_mfma_f32_16x16x4_f32 (12 padded to 16) whose accumulator feeds the next MFMA as its
//      B operand without leaving registers (k is permuted as k = 4*(lane>>4) + step).  The
//      waves of the workgroup split the j loop; H is staged in LDS in tile layout.
//   2. The symmetric H + diag(R) + shift is held in REGISTERS as 8x8 tiles of its lower
//      triangle, one tile per lane (workgroup = ceil(tiles/64) waves), and inverted in place
//      by the symmetric sweep operator (Gauss-Jordan on the unit-diagonal-scaled matrix):
//      one barrier per pivot, pivot column exchanged through a double-buffered LDS vector.
//   3. ADMM (OSQP iteration with A = I) on the free forces with the per-(step, leg) set
//      {fz >= fz_min, |fx| <= mu fz, |fy| <= mu fz} projected in closed form.  The x-update
//      is x~ = x + M(rho(z - x) - grad f(x) - y): M (the fp32 inverse) is only a
//      preconditioner; grad f comes from an error-coordinate rollout/adjoint recursion
//      (e_{k+1} = A e_k + B_k u_k + d_k, d_k = A r_k + g - r_{k+1}), so the fixed point is as
//      accurate as that gradient, not eps32 x cond(H).
//   4. Active-set polish once the face pattern of z is stable: condense + invert the
//      equality-constrained reduced problem (u = T v + t0), refine with the accurate gradient,
//      accept only if the KKT conditions hold -> status 1.  The ADMM inverse is parked in a
//      per-workgroup global slab (L2-resident) during the attempt and restored if it fails.
//
// Instances are binned by free-variable count (capacity NC in {96,128,160,192}); each bin
// runs a persistent kernel pulling instance ids from a device-side queue.
//
// This file is compiled as part of cmpc_host.hip (single translation unit).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cmpc_device.h"

namespace cmpc {

typedef float f4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------
// wave / block helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float readlane_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
  return v;
}

// exclusive prefix sum across the 64 lanes of a wave
__device__ __forceinline__ int wave_excl_scan(int v, int lane) {
  int incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(incl, d, 64);
    if (lane >= d) incl += t;
  }
  return incl - v;
}

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------------------------------
// diagnostic build only (-DCMPC_STAMPS): per-phase s_memtime cycle totals, never in the
// product library.  Phases: 0 condense, 1 invert, 2 gradient, 3 symv, 4 polish (all of it),
// 5 instance total; counters: 8 condense+invert calls, 9 polish attempts, 10 instances,
// 11 ADMM iterations.
// ------------------------------------------------------------------------------------------
#ifdef CMPC_STAMPS
__device__ unsigned long long g_stamps[16];
#define CMPC_T0(name) const unsigned long long name = __builtin_amdgcn_s_memtime()
#define CMPC_ACC(ph, t0)                                                              \
  do {                                                                                \
    const unsigned long long _t1 = __builtin_amdgcn_s_memtime();                      \
    if (threadIdx.x == 0) atomicAdd(&g_stamps[ph], _t1 - (t0));                       \
  } while (0)
#define CMPC_CNT(ph, v) \
  do { if (threadIdx.x == 0) atomicAdd(&g_stamps[ph], (unsigned long long)(v)); } while (0)
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
constexpr int kMaxTri = 4 * kMaxN;  // 64 (= lanes of wave 0: lane t owns stance triple t)

template <int NC>
struct Cfg {
  static constexpr int TT = NC / 8;                      // tile rows
  static constexpr int NT = TT * (TT + 1) / 2;           // lower-triangle tiles
  static constexpr int THREADS = ((NT + 63) / 64) * 64;  // one tile per lane
  static constexpr int WAVES = THREADS / 64;
  static constexpr int SLAB = NT * 64;                   // floats per park slab (global)
  static constexpr int TS = 68;                          // LDS staging tile stride (floats):
  // a lane reading its own tile then hits bank (4t + c) mod 64 -> conflict-free 16-B reads
};

template <int NC>
struct Smem {
  alignas(16) float Bt[NC * 12];   // param-space input matrix, column p at Bt[12p .. 12p+11]
  alignas(16) float Rt[NC];        // param-space input weight (2R in the param basis)
  alignas(16) float x[NC];
  alignas(16) float z[NC];
  alignas(16) float y[NC];
  alignas(16) float g[NC];
  alignas(16) float r[NC];
  alignas(16) float xr[NC];
  alignas(16) float w[NC];
  alignas(16) float v[NC];
  alignas(16) float dl[NC];
  alignas(16) float av[2][NC];     // sweep pivot column (double buffered)
  alignas(16) float ds[NC];        // unit-diagonal scaling
  alignas(16) float part[Cfg<NC>::NT * 16];  // symv partial sums per tile (rows | cols)
  alignas(16) float stg[Cfg<NC>::NT * Cfg<NC>::TS];  // condensation output, tile layout
  float D[kMaxP];                  // d_k  (error-coordinate affine term)
  float Dt[kMaxP];                 // d~_k (d_k + B_k t0_k in the polish basis)
  float H[kMaxP];                  // h_k = B~_k v_k + d~_k
  float E[kMaxP];                  // e_{k+1} = x_{k+1} - xref_k
  float L[kMaxP];                  // lambda_k
  float U[kMaxP];                  // final full u
  float A[144];
  float Q2[12];                    // KParams copies (indexed at run time -> keep out of kernarg)
  float R2[12];
  float red[16];
  int par[NC];                     // param -> step k
  int off[kMaxN + 1];              // first param of step k
  int tri[kMaxTri];                // stance triple t -> 4k + leg
  int tri_of[kMaxTri];             // 4k + leg -> triple index or -1
  int tcnt[kMaxTri];               // polish: params of triple t
  int code[kMaxTri];               // face code of triple t
  float fctl[8];                   // wave-0 -> block broadcasts
  int ctl[8];
};

__device__ __forceinline__ int tile_index(int I, int J) { return (I * (I + 1)) / 2 + J; }

template <int W>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float m = red[0];
#pragma unroll
  for (int i = 1; i < W; ++i) m = fmaxf(m, red[i]);
  return m;
}

// ------------------------------------------------------------------------------------------
// condensation (MFMA) -> staging slab (global, tile layout, lower triangle)
// ------------------------------------------------------------------------------------------
template <int NC>
__device__ __forceinline__ f4 load_bcol(const Smem<NC>& s, int p0, int m, int g, int c) {
  f4 v = {0.f, 0.f, 0.f, 0.f};
  if (c < m && g < 3) v = *reinterpret_cast<const f4*>(&s.Bt[(p0 + c) * 12 + 4 * g]);
  return v;
}

template <int TS>
__device__ __forceinline__ void stage_store(float* stg, int p, int q, float val) {
  // p >= q; diagonal tiles keep both halves
  const int t = tile_index(p >> 3, q >> 3);
  stg[t * TS + (p & 7) * 8 + (q & 7)] = val;
  if ((p >> 3) == (q >> 3) && p != q) stg[t * TS + (q & 7) * 8 + (p & 7)] = val;
}

template <int NC>
__device__ __forceinline__ void condense_stage(Smem<NC>& s, const KParams& P) {
  using C = Cfg<NC>;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int N = P.N;
  float Ar[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = 4 * g + q;
    Ar[q] = (row < 12 && c < 12) ? s.A[row * 12 + c] : 0.f;
  }
  f4 S;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = 4 * g + q;
    S[q] = (row < 12 && row == c) ? s.Q2[row] : 0.f;
  }
  // boustrophedon split of the j loop over the waves (step j costs j+1 blocks)
  unsigned mine = 0;
  for (int j = N - 1; j >= 0; --j) {
    const int m = N - 1 - j, cyc = m / C::WAVES, r = m % C::WAVES;
    const int w = (cyc & 1) ? (C::WAVES - 1 - r) : r;
    if (w == wv) mine |= 1u << j;
  }
  for (int j = N - 1; j >= 0; --j) {
    if (j < N - 1) {  // S_j = Q2 + A' (S_{j+1} A)
      f4 T1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q) T1 = mfma4(S[q], Ar[q], T1);
      f4 Sn = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q) Sn = mfma4(Ar[q], T1[q], Sn);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 4 * g + q;
        if (row < 12 && row == c) Sn[q] += s.Q2[row];
      }
      S = Sn;
    }
    if (!((mine >> j) & 1u)) continue;
    const int pj0 = s.off[j], mj = s.off[j + 1] - pj0;
    if (mj == 0) continue;
    const f4 bj = load_bcol(s, pj0, mj, g, c);
    f4 W = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 4; ++q) W = mfma4(S[q], bj[q], W);
    for (int i = j; i >= 0; --i) {
      if (i < j) {  // W <- A' W
        f4 Wn = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 4; ++q) Wn = mfma4(Ar[q], W[q], Wn);
        W = Wn;
      }
      const int pi0 = s.off[i], mi = s.off[i + 1] - pi0;
      if (mi == 0) continue;
      const f4 bi = load_bcol(s, pi0, mi, g, c);
      f4 Hb = {0.f, 0.f, 0.f, 0.f};  // Hb[q] = H[pi0 + 4g+q][pj0 + c]
#pragma unroll
      for (int q = 0; q < 4; ++q) Hb = mfma4(bi[q], W[q], Hb);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int qq = 4 * g + q;
        if (qq < mi && c < mj && (i != j || c >= qq))
          stage_store<C::TS>(s.stg, pj0 + c, pi0 + qq, Hb[q]);
      }
    }
  }
}

// register tile <- LDS staging, + diag(Rt) + shift, identity on padding
template <int NC>
__device__ __forceinline__ void load_tile(float (&T)[64], const Smem<NC>& s, int I, int J,
                                          bool own, int n, float shift) {
  if (!own) {
#pragma unroll
    for (int q = 0; q < 64; ++q) T[q] = 0.f;
    return;
  }
  const f4* src = reinterpret_cast<const f4*>(&s.stg[tile_index(I, J) * Cfg<NC>::TS]);
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const f4 v = src[q];
    T[4 * q] = v[0]; T[4 * q + 1] = v[1]; T[4 * q + 2] = v[2]; T[4 * q + 3] = v[3];
  }
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int p = 8 * I + a, q = 8 * J + b;
      if (p >= n || q >= n) T[a * 8 + b] = (p == q) ? 1.f : 0.f;
      else if (p == q) T[a * 8 + b] += s.Rt[p] + shift;
    }
}

// symmetric sweep (Gauss-Jordan) inversion of the register-tiled matrix
template <int NC>
__device__ __forceinline__ void invert_tile(Smem<NC>& s, float (&T)[64], int I, int J, bool own,
                                            int n) {
  const int TA = (n + 7) >> 3;
  const bool act = own && I < TA;
  if (act && I == J) {
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      const int p = 8 * I + a;
      const float dg = T[a * 9];
      s.ds[p] = (p < n && dg > 0.f) ? rsqrtf(dg) : 1.f;
    }
  }
  __syncthreads();
  if (act) {
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      const float ra = s.ds[8 * I + a];
#pragma unroll
      for (int b = 0; b < 8; ++b) T[a * 8 + b] *= ra * s.ds[8 * J + b];
    }
  }
  // pivot k: M_ij -= a_i a_j / d with a = column k except a_k = d - 1, then M_kk -= 2
  // (= M_ij - c_i c_j / d, M_ik = c_i / d, M_kk = -1/d: the sweep operator)
  for (int K = 0; K < TA; ++K) {
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int k = 8 * K + kk;
      if (k >= n) continue;  // uniform; no `break` so the loop fully unrolls (T stays in VGPRs)
      float* av = s.av[k & 1];
      if (act) {
        if (J == K) {
#pragma unroll
          for (int a = 0; a < 8; ++a) av[8 * I + a] = T[a * 8 + kk];
        } else if (I == K) {
#pragma unroll
          for (int b = 0; b < 8; ++b) av[8 * J + b] = T[kk * 8 + b];
        }
      }
      __syncthreads();
      if (act) {
        const float d = av[k];
        const float invd = 1.f / d;
        float ci[8], cj[8];
        const f4 r0 = *reinterpret_cast<const f4*>(&av[8 * I]);
        const f4 r1 = *reinterpret_cast<const f4*>(&av[8 * I + 4]);
        const f4 c0 = *reinterpret_cast<const f4*>(&av[8 * J]);
        const f4 c1 = *reinterpret_cast<const f4*>(&av[8 * J + 4]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          ci[q] = r0[q]; ci[q + 4] = r1[q];
          cj[q] = c0[q]; cj[q + 4] = c1[q];
        }
        if (I == K) ci[kk] = d - 1.f;
        if (J == K) cj[kk] = d - 1.f;
#pragma unroll
        for (int a = 0; a < 8; ++a) {
          const float nb = -ci[a] * invd;
#pragma unroll
          for (int b = 0; b < 8; ++b) T[a * 8 + b] = fmaf(nb, cj[b], T[a * 8 + b]);
        }
        if (I == K && J == K) T[kk * 9] -= 2.f;
      }
    }
  }
  if (act) {  // T holds -(scaled inverse): undo sign and scaling (ds is unchanged)
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      const float ra = -s.ds[8 * I + a];
#pragma unroll
      for (int b = 0; b < 8; ++b) T[a * 8 + b] *= ra * s.ds[8 * J + b];
    }
  }
}

// out = M in over n params (M in register tiles); `in` read only for indices < n
template <int NC>
__device__ __forceinline__ void symv(Smem<NC>& s, const float (&T)[64], int I, int J, bool own,
                                     int n, const float* in, float* out) {
  using C = Cfg<NC>;
  CMPC_T0(t_sv);
  const int TA = (n + 7) >> 3;
  const int tid = threadIdx.x;
  __syncthreads();
  if (own && I < TA) {
    float rj[8], ri[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      rj[b] = (8 * J + b < n) ? in[8 * J + b] : 0.f;
      ri[b] = (8 * I + b < n) ? in[8 * I + b] : 0.f;
    }
    float pr[8], pc[8];
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      float acc = 0.f;
#pragma unroll
      for (int b = 0; b < 8; ++b) acc = fmaf(T[a * 8 + b], rj[b], acc);
      pr[a] = acc;
    }
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      float acc = 0.f;
#pragma unroll
      for (int a = 0; a < 8; ++a) acc = fmaf(T[a * 8 + b], ri[a], acc);
      pc[b] = (I != J) ? acc : 0.f;
    }
    f4* dst = reinterpret_cast<f4*>(&s.part[tid * 16]);
    dst[0] = f4{pr[0], pr[1], pr[2], pr[3]};
    dst[1] = f4{pr[4], pr[5], pr[6], pr[7]};
    dst[2] = f4{pc[0], pc[1], pc[2], pc[3]};
    dst[3] = f4{pc[4], pc[5], pc[6], pc[7]};
  }
  __syncthreads();
  for (int p = tid; p < n; p += C::THREADS) {
    const int Ip = p >> 3, pp = p & 7;
    float acc = 0.f;
    for (int Jb = 0; Jb <= Ip; ++Jb) acc += s.part[tile_index(Ip, Jb) * 16 + pp];
    for (int Ib = Ip + 1; Ib < TA; ++Ib) acc += s.part[tile_index(Ib, Ip) * 16 + 8 + pp];
    out[p] = acc;
  }
  __syncthreads();
  CMPC_ACC(3, t_sv);
}

// Gradient of sum_k e_{k+1}'(Q2/2)e_{k+1} + v'(Rt/2)v in the current param basis
// (e by the error-coordinate rollout).  Leaves E (e_{k+1}) and L (lambda_k) in LDS.
template <int NC>
__device__ __forceinline__ void gradient(Smem<NC>& s, const KParams& P, int n, const float* vin, float* gout) {
  using C = Cfg<NC>;
  CMPC_T0(t_gr);
  const int tid = threadIdx.x;
  const int N = P.N;
  const int NP = 12 * N;
  __syncthreads();
  for (int o = tid; o < NP; o += C::THREADS) {  // h_k = B~_k v_k + d~_k
    const int k = o / 12, r = o % 12;
    float acc = s.Dt[o];
    for (int p = s.off[k]; p < s.off[k + 1]; ++p) acc = fmaf(s.Bt[p * 12 + r], vin[p], acc);
    s.H[o] = acc;
  }
  __syncthreads();
  if (tid < 64) {  // sequential recursions on wave 0 (lanes 0..11 carry the state)
    const int lane = tid;
    const int i = lane % 12;
    float Arow[12], Acol[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      Arow[j] = s.A[i * 12 + j];
      Acol[j] = s.A[j * 12 + i];
    }
    float e = 0.f;
    for (int k = 0; k < N; ++k) {  // e_{k+1} = A e_k + h_k
      float acc = s.H[12 * k + i];
#pragma unroll
      for (int j = 0; j < 12; ++j) acc = fmaf(Arow[j], readlane_f(e, j), acc);
      e = acc;
      if (lane < 12) s.E[12 * k + i] = e;
    }
    float lam = 0.f;
    const float q2 = s.Q2[i];
    for (int k = N - 1; k >= 0; --k) {  // lambda_k = Q2 e_{k+1} + A' lambda_{k+1}
      float acc = q2 * s.E[12 * k + i];
#pragma unroll
      for (int j = 0; j < 12; ++j) acc = fmaf(Acol[j], readlane_f(lam, j), acc);
      lam = acc;
      if (lane < 12) s.L[12 * k + i] = lam;
    }
  }
  __syncthreads();
  for (int p = tid; p < n; p += C::THREADS) {  // g = B~' lambda + Rt v
    const int k = s.par[p];
    float acc = s.Rt[p] * vin[p];
#pragma unroll
    for (int r = 0; r < 12; ++r) acc = fmaf(s.Bt[p * 12 + r], s.L[12 * k + r], acc);
    gout[p] = acc;
  }
  __syncthreads();
  CMPC_ACC(2, t_gr);
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
__device__ __forceinline__ void build_admm_basis(Smem<NC>& s, const KParams& P, const float* __restrict__ Bg,
                                 int ntri) {
  using C = Cfg<NC>;
  const int tid = threadIdx.x;
  const int N = P.N;
  const int n = 3 * ntri;
  __syncthreads();
  for (int e = tid; e < n * 12; e += C::THREADS) {
    const int p = e / 12, r = e % 12;
    const int t = p / 3, a = p % 3;
    const int kl = s.tri[t];
    const int k = kl >> 2, leg = kl & 3;
    s.Bt[e] = Bg[(k * 12 + r) * 12 + 3 * leg + a];
  }
  for (int p = tid; p < NC; p += C::THREADS) {
    if (p < n) {
      const int t = p / 3, a = p % 3;
      const int kl = s.tri[t];
      s.Rt[p] = s.R2[3 * (kl & 3) + a];
      s.par[p] = kl >> 2;
    } else {
      s.Rt[p] = 0.f;
      s.par[p] = 0;
      s.x[p] = 0.f; s.z[p] = 0.f; s.y[p] = 0.f; s.g[p] = 0.f; s.r[p] = 0.f;
      s.xr[p] = 0.f; s.w[p] = 0.f; s.v[p] = 0.f; s.dl[p] = 0.f;
    }
  }
  for (int k = tid; k <= N; k += C::THREADS) {
    int c = 0;
    for (int t = 0; t < ntri; ++t) c += ((s.tri[t] >> 2) < k) ? 1 : 0;
    s.off[k] = 3 * c;
  }
  for (int o = tid; o < 12 * N; o += C::THREADS) s.Dt[o] = s.D[o];
  __syncthreads();
}

// Polish setup: the reduced basis of the faces in s.code (wave-0 lane t owns triple t),
// u = T v + t0 with t0 = locked components, v initialised from z.  Returns nr.  The per-triple
// face data of wave-0 lanes is returned in `tf` for the KKT check.
struct TripleFaces {
  int k, leg, sx, sy, px, py, pz;
  bool zl, owns;
};

template <int NC>
__device__ __forceinline__ int polish_setup(Smem<NC>& s, const KParams& P, const float* __restrict__ Bg,
                            int ntri, TripleFaces& tf) {
  using C = Cfg<NC>;
  const int tid = threadIdx.x;
  const int N = P.N;
  const float mu = P.mu, fzmin = P.fz_min;
  tf = TripleFaces{0, 0, 0, 0, -1, -1, -1, false, false};
  __syncthreads();
  if (tid < 64) {
    const int lane = tid;
    tf.owns = lane < ntri;
    const int code = tf.owns ? s.code[lane] : 0;
    const int kl = tf.owns ? s.tri[lane] : 0;
    const int k = kl >> 2, leg = kl & 3;
    const int sx = (code & 2) ? 1 : ((code & 4) ? -1 : 0);
    const int sy = (code & 8) ? 1 : ((code & 16) ? -1 : 0);
    const bool zl = (code & 1) != 0;
    tf.k = k; tf.leg = leg; tf.sx = sx; tf.sy = sy; tf.zl = zl;
    const int cnt = tf.owns ? ((sx == 0) + (sy == 0) + (!zl)) : 0;
    const int base = wave_excl_scan(cnt, lane);
    const int nr = __shfl(base + cnt, 63, 64);
    const float* Bk = Bg + k * 144;
    if (tf.owns) {
      s.tcnt[lane] = cnt;
      int p = base;
      if (sx == 0) {
        tf.px = p++;
        for (int r = 0; r < 12; ++r) s.Bt[tf.px * 12 + r] = Bk[r * 12 + 3 * leg];
        s.Rt[tf.px] = s.R2[3 * leg];
        s.par[tf.px] = k;
        s.v[tf.px] = s.z[3 * lane];
      }
      if (sy == 0) {
        tf.py = p++;
        for (int r = 0; r < 12; ++r) s.Bt[tf.py * 12 + r] = Bk[r * 12 + 3 * leg + 1];
        s.Rt[tf.py] = s.R2[3 * leg + 1];
        s.par[tf.py] = k;
        s.v[tf.py] = s.z[3 * lane + 1];
      }
      if (!zl) {
        tf.pz = p++;
        const float cx = sx * mu, cy = sy * mu;
        for (int r = 0; r < 12; ++r)
          s.Bt[tf.pz * 12 + r] = Bk[r * 12 + 3 * leg + 2] + cx * Bk[r * 12 + 3 * leg] +
                                 cy * Bk[r * 12 + 3 * leg + 1];
        s.Rt[tf.pz] = s.R2[3 * leg + 2] + mu * mu * ((sx != 0 ? s.R2[3 * leg] : 0.f) +
                                                     (sy != 0 ? s.R2[3 * leg + 1] : 0.f));
        s.par[tf.pz] = k;
        s.v[tf.pz] = s.z[3 * lane + 2];
      }
    }
    if (lane == 0) s.ctl[1] = nr;
  }
  __syncthreads();
  const int nr = s.ctl[1];
  for (int kk = tid; kk <= N; kk += C::THREADS) {
    int c = 0;
    for (int t = 0; t < ntri; ++t) c += ((s.tri[t] >> 2) < kk) ? s.tcnt[t] : 0;
    s.off[kk] = c;
  }
  for (int o = tid; o < 12 * N; o += C::THREADS) {  // d~ = d + B t0 (fz locked at fz_min)
    const int kk = o / 12, r = o % 12;
    float acc = s.D[o];
    for (int l = 0; l < 4; ++l) {
      const int t = s.tri_of[4 * kk + l];
      if (t < 0) continue;
      const int c = s.code[t];
      if (!(c & 1)) continue;
      const float tx = (c & 2) ? mu * fzmin : ((c & 4) ? -mu * fzmin : 0.f);
      const float ty = (c & 8) ? mu * fzmin : ((c & 16) ? -mu * fzmin : 0.f);
      const float* Bkk = Bg + kk * 144 + r * 12 + 3 * l;
      acc = fmaf(Bkk[0], tx, acc);
      acc = fmaf(Bkk[1], ty, acc);
      acc = fmaf(Bkk[2], fzmin, acc);
    }
    s.Dt[o] = acc;
  }
  for (int p = tid; p < NC; p += C::THREADS)
    if (p >= nr) { s.v[p] = 0.f; s.g[p] = 0.f; s.dl[p] = 0.f; }
  __syncthreads();
  return nr;
}

// Polish check after refinement (E, L at the final v in LDS): KKT conditions per triple on
// wave 0.  On success writes the full u into s.U.
template <int NC>
__device__ __forceinline__ bool polish_check(Smem<NC>& s, const KParams& P, const float* __restrict__ Bg,
                             const TripleFaces& tf, float step) {
  using C = Cfg<NC>;
  const int tid = threadIdx.x;
  const float mu = P.mu, fzmin = P.fz_min;
  for (int o = tid; o < 12 * P.N; o += C::THREADS) s.U[o] = 0.f;
  __syncthreads();
  if (tid < 64) {
    float fx = 0.f, fy = 0.f, fz = 0.f, gx = 0.f, gy = 0.f, gz = 0.f;
    const int k = tf.k, leg = tf.leg, sx = tf.sx, sy = tf.sy;
    if (tf.owns) {
      fz = tf.zl ? fzmin : s.v[tf.pz];
      fx = (sx == 0) ? s.v[tf.px] : sx * mu * fz;
      fy = (sy == 0) ? s.v[tf.py] : sy * mu * fz;
      const float* Bk = Bg + k * 144;
      float ax = 0.f, ay = 0.f, az = 0.f;
      for (int r = 0; r < 12; ++r) {
        const float lr = s.L[12 * k + r];
        ax = fmaf(Bk[r * 12 + 3 * leg], lr, ax);
        ay = fmaf(Bk[r * 12 + 3 * leg + 1], lr, ay);
        az = fmaf(Bk[r * 12 + 3 * leg + 2], lr, az);
      }
      gx = ax + s.R2[3 * leg] * fx;
      gy = ay + s.R2[3 * leg + 1] * fy;
      gz = az + s.R2[3 * leg + 2] * fz;
    }
    const float gs = wave_max(fmaxf(fabsf(gx), fmaxf(fabsf(gy), fabsf(gz))));
    const float us = wave_max(fmaxf(1.f, fmaxf(fabsf(fx), fmaxf(fabsf(fy), fabsf(fz)))));
    const float tol_d = P.polish_tol * gs, tol_p = P.polish_tol * us;
    bool ok = true;
    if (tf.owns) {
      // KKT per triple; on a violation also derive the repaired face set (primal-dual
      // active-set step): drop faces with a negative multiplier, add violated faces
      const float lx = sx ? -sx * gx : 0.f;
      const float ly = sy ? -sy * gy : 0.f;
      const float l0 = gz - mu * (lx + ly);
      int nc = s.code[tid];
      if (sx && lx < -tol_d) { ok = false; nc &= ~6; }
      if (sy && ly < -tol_d) { ok = false; nc &= ~24; }
      if (tf.zl && l0 < -tol_d) { ok = false; nc &= ~1; }
      if (!sx && fabsf(fx) > mu * fz + tol_p) { ok = false; nc |= (fx > 0.f) ? 2 : 4; }
      if (!sy && fabsf(fy) > mu * fz + tol_p) { ok = false; nc |= (fy > 0.f) ? 8 : 16; }
      if (!tf.zl && fz < fzmin - tol_p) { ok = false; nc |= 1; }
      if (!(isfinite(fx) && isfinite(fy) && isfinite(fz))) ok = false;
      s.tcnt[tid] = nc;  // repaired code (copied into s.code by the caller if used)
    }
    const bool all_ok = (__all(ok) != 0) && (step <= P.polish_tol * us);
    if (all_ok && tf.owns) {
      s.U[12 * k + 3 * leg] = fx;
      s.U[12 * k + 3 * leg + 1] = fy;
      s.U[12 * k + 3 * leg + 2] = fz;
    }
    const bool changed = tf.owns && (s.tcnt[tid] != s.code[tid]);
    const bool any_changed = __any(changed) != 0;
    if (tid == 0) {
      s.ctl[2] = all_ok ? 1 : 0;
      s.ctl[4] = any_changed ? 1 : 0;
    }
  }
  __syncthreads();
  return s.ctl[2] != 0;
}

// One instance.  A small state machine keeps a single call site of the (inlined) condense +
// invert and of each symv, so the register tile T never leaves VGPRs.
template <int NC>
__device__ __forceinline__ void solve_instance(Smem<NC>& s, const KParams& P, int64_t b,
                                               const Inputs& in, const Outputs& out,
                                               float* __restrict__ park,
                                               float (&T)[64], int I, int J, bool own) {
  using C = Cfg<NC>;
  const int tid = threadIdx.x;
  const int N = P.N;
  const int NP = 12 * N;
  const float* Ab = in.Ad + b * 144;
  const float* Bg = in.Bd + b * (int64_t)N * 144;
  const float* gdb = in.gd + b * 12;
  const float* x0b = in.x0 + b * 12;
  const float* xrb = in.xref + b * (int64_t)N * 12;
  const uint8_t* ctb = in.contact + b * (int64_t)4 * N;
  CMPC_T0(t_inst);
  CMPC_CNT(10, 1);

  for (int e = tid; e < 144; e += C::THREADS) s.A[e] = Ab[e];
  if (tid < 64) {  // stance triples in (k, leg) order; lane = 4k + leg
    const int lane = tid;
    const bool st = (lane < 4 * N) ? (ctb[(lane & 3) * N + (lane >> 2)] != 0) : false;
    const int pos = wave_excl_scan(st ? 1 : 0, lane);
    const int nt = __shfl(pos + (st ? 1 : 0), 63, 64);
    if (st) s.tri[pos] = lane;
    if (lane < 4 * N) s.tri_of[lane] = st ? pos : -1;
    if (lane == 0) s.ctl[0] = nt;
  }
  __syncthreads();
  const int ntri = s.ctl[0];
  for (int o = tid; o < NP; o += C::THREADS) {  // d_k = A r_k + gd - r_{k+1}, r_0 = x0
    const int k = o / 12, r = o % 12;
    const float* rk = (k == 0) ? x0b : (xrb + (k - 1) * 12);
    float acc = gdb[r] - xrb[k * 12 + r];
#pragma unroll
    for (int j = 0; j < 12; ++j) acc = fmaf(s.A[r * 12 + j], rk[j], acc);
    s.D[o] = acc;
  }
  build_admm_basis<NC>(s, P, Bg, ntri);
  const int n = 3 * ntri;
  for (int p = tid; p < n; p += C::THREADS) { s.x[p] = 0.f; s.z[p] = 0.f; s.y[p] = 0.f; }

  int status = -2, iters = 0;
  bool polished = false;
  float rho = P.rho0;
  float rp = 0.f, rd = 0.f, np_ = 0.f, nd = 0.f;
  int prev_code = -1, stable = 0;  // wave-0 state
  bool refactor = n > 0;           // (re)build + invert the matrix for the current basis
  bool in_polish = false;
  int nact = n;                    // params of the current basis
  float shift = P.sigma + rho;
  TripleFaces tf;
  int it = 0;
  int repairs_left = 0;
  float nq = 0.f;                  // |q| of the condensed QP (= |grad f(0)|, iteration 1)
  const float alpha = P.alpha;
  if (n == 0) status = 1;
  while (n > 0) {
    if (refactor) {  // the only condense + invert call site
      CMPC_CNT(8, 1);
      CMPC_T0(t_c);
      __syncthreads();
      condense_stage<NC>(s, P);
      __syncthreads();
      load_tile<NC>(T, s, I, J, own, nact, shift);
      CMPC_ACC(0, t_c);
      CMPC_T0(t_i);
      invert_tile<NC>(s, T, I, J, own, nact);
      CMPC_ACC(1, t_i);
      refactor = false;
    }
    if (in_polish) {
      CMPC_T0(t_pol);
      float step = 3.0e38f;
      for (int q = 0; q < P.polish_refine; ++q) {
        gradient<NC>(s, P, nact, s.v, s.g);
        symv<NC>(s, T, I, J, own, nact, s.g, s.dl);
        float m = 0.f;
        for (int p = tid; p < nact; p += C::THREADS) {
          s.v[p] -= s.dl[p];
          m = fmaxf(m, fabsf(s.dl[p]));
        }
        step = block_max<C::WAVES>(m, s.red);
      }
      gradient<NC>(s, P, nact, s.v, s.g);  // E, L at the final point
      const bool ok = polish_check<NC>(s, P, Bg, tf, step);
      CMPC_ACC(4, t_pol);
      if (ok) {
        polished = true;
        status = 1;
        break;
      }
      if (repairs_left > 0 && s.ctl[4]) {  // re-polish on the repaired face set
        --repairs_left;
        for (int t = tid; t < ntri; t += C::THREADS) s.code[t] = s.tcnt[t];
        nact = polish_setup<NC>(s, P, Bg, ntri, tf);
        shift = P.sigma;
        refactor = true;
        continue;
      }
      // restore the parked ADMM inverse and basis, continue ADMM
      if (own) {
        const f4* src = reinterpret_cast<const f4*>(park + tid * 64);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const f4 v = src[q];
          T[4 * q] = v[0]; T[4 * q + 1] = v[1]; T[4 * q + 2] = v[2]; T[4 * q + 3] = v[3];
        }
      }
      build_admm_basis<NC>(s, P, Bg, ntri);
      in_polish = false;
      nact = n;
      shift = P.sigma + rho;
    }
    if (it >= P.max_iter) break;
    ++it;
    iters = it;
    // ---- one ADMM iteration ----
    gradient<NC>(s, P, n, s.x, s.g);
    for (int p = tid; p < n; p += C::THREADS) s.r[p] = rho * (s.z[p] - s.x[p]) - s.g[p] - s.y[p];
    symv<NC>(s, T, I, J, own, n, s.r, s.dl);
    const float inv_rho = 1.f / rho;
    for (int p = tid; p < n; p += C::THREADS) {
      const float xt = s.x[p] + s.dl[p];
      const float xr = alpha * xt + (1.f - alpha) * s.z[p];
      s.x[p] = alpha * xt + (1.f - alpha) * s.x[p];
      s.xr[p] = xr;
      s.w[p] = xr + s.y[p] * inv_rho;
    }
    __syncthreads();
    const bool last = (it == P.max_iter);
    const bool adapt = P.adaptive_interval > 0 && (it % P.adaptive_interval) == 0;
    if (tid < 64) {  // projection, residuals and the polish trigger on wave 0
      const int lane = tid;
      int code = 0;
      float lrp = 0.f, lrd = 0.f, lnp = 0.f, lnd = 0.f;
      if (lane < ntri) {
        float pv[3];
        code = project(s.w[3 * lane], s.w[3 * lane + 1], s.w[3 * lane + 2], P.mu, P.fz_min,
                       pv[0], pv[1], pv[2]);
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          const int p = 3 * lane + a;
          const float zn = pv[a];
          const float yn = s.y[p] + rho * (s.xr[p] - zn);
          s.z[p] = zn;
          s.y[p] = yn;
          const float xp = s.x[p], gp = s.g[p];
          lrp = fmaxf(lrp, fabsf(xp - zn));
          lrd = fmaxf(lrd, fabsf(gp + yn));
          lnp = fmaxf(lnp, fmaxf(fabsf(xp), fabsf(zn)));
          lnd = fmaxf(lnd, fmaxf(fabsf(gp), fabsf(yn)));
        }
        s.code[lane] = code;
      }
      const bool changed = (lane < ntri) && (code != prev_code);
      prev_code = code;
      stable = (__any(changed) != 0) ? 0 : stable + 1;
      int do_pol = 0;
      if (stable >= P.polish_stable && !last) {
        do_pol = 1;
        stable = -P.polish_stable;  // back off before a further attempt
      }
      if (adapt || last) {
        rp = wave_max(lrp); rd = wave_max(lrd); np_ = wave_max(lnp); nd = wave_max(lnd);
      }
      float nrho = rho;
      if (adapt && !last) {
        float q = rho * sqrtf((rp / fmaxf(np_, 1e-30f)) / (rd / fmaxf(nd, 1e-30f) + 1e-30f));
        q = fminf(fmaxf(q, 1e-6f), 1e6f);
        if (q > 5.f * rho || q < 0.2f * rho) nrho = q;
      }
      if (lane == 0) {
        s.ctl[3] = do_pol;
        s.fctl[0] = nrho;
        s.fctl[1] = rp; s.fctl[2] = rd; s.fctl[3] = np_; s.fctl[4] = nd;
      }
    }
    __syncthreads();
    const int do_pol = s.ctl[3];
    const float nrho = s.fctl[0];
    rp = s.fctl[1]; rd = s.fctl[2]; np_ = s.fctl[3]; nd = s.fctl[4];
    if (nrho != rho) {
      rho = nrho;
      shift = P.sigma + rho;
      refactor = true;
    }
    if (do_pol) {
      CMPC_CNT(9, 1);
      if (!refactor && own) {  // park the ADMM inverse (restored if the polish fails)
        f4* dst = reinterpret_cast<f4*>(park + tid * 64);
#pragma unroll
        for (int q = 0; q < 16; ++q)
          dst[q] = f4{T[4 * q], T[4 * q + 1], T[4 * q + 2], T[4 * q + 3]};
      }
      nact = polish_setup<NC>(s, P, Bg, ntri, tf);
      shift = P.sigma;
      refactor = true;
      in_polish = true;
      repairs_left = P.polish_repairs;
    }
  }
  if (n > 0 && !polished) {
    const bool conv = rp <= P.eps_abs + P.eps_rel * np_ && rd <= P.eps_abs + P.eps_rel * nd;
    status = conv ? 2 : -2;
  }
  if (!polished) {  // u from z (ADMM basis), E at that u
    gradient<NC>(s, P, n, s.z, s.g);
    for (int o = tid; o < NP; o += C::THREADS) s.U[o] = 0.f;
    __syncthreads();
    for (int p = tid; p < n; p += C::THREADS) {
      const int kl = s.tri[p / 3];
      s.U[12 * (kl >> 2) + 3 * (kl & 3) + (p % 3)] = s.z[p];
    }
  }
  __syncthreads();
  float* wb = out.w + b * (int64_t)(24 * N);
  int bad = 0;
  for (int o = tid; o < NP; o += C::THREADS) {
    const float xv = s.E[o] + xrb[o];
    const float uv = s.U[o];
    bad |= !(isfinite(xv) && isfinite(uv));
    wb[o] = xv;
    wb[NP + o] = uv;
  }
  bad = __syncthreads_or(bad);
  if (bad) status = -10;
  if (tid == 0) {
    out.status[b] = status;
    out.iters[b] = iters;
  }
  CMPC_CNT(11, iters);
  CMPC_ACC(5, t_inst);
}

template <int NC>
__global__ void __launch_bounds__(Cfg<NC>::THREADS, 2)
    solve_bin_kernel(KParams P, Inputs in, Outputs out, const int* __restrict__ list,
                     const int* __restrict__ count, int* __restrict__ head,
                     float* __restrict__ work) {
  using C = Cfg<NC>;
  __shared__ Smem<NC> s;
  const int tid = threadIdx.x;
  const bool own = tid < C::NT;
  int I = 0;
  while ((I + 1) * (I + 2) / 2 <= tid) ++I;
  const int J = tid - I * (I + 1) / 2;
  if (!own) I = 1 << 20;
  float* park = work + (size_t)blockIdx.x * C::SLAB;
  float T[64];
#pragma unroll
  for (int q = 0; q < 64; ++q) T[q] = 0.f;
  if (tid < 12) {
    s.Q2[tid] = P.Q2[tid];
    s.R2[tid] = P.R2[tid];
  }
  const int total = *count;
  for (;;) {
    if (tid == 0) s.ctl[7] = atomicAdd(head, 1);
    __syncthreads();
    const int idx = s.ctl[7];
    __syncthreads();
    if (idx >= total) break;
    solve_instance<NC>(s, P, (int64_t)list[idx], in, out, park, T, I, J, own);
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
      lists[q * stride + base + rank] = (int)b;
    }
  }
}

}  // namespace cmpc
