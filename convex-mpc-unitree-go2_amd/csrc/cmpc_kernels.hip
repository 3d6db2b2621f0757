// cmpc_kernels.hip -- batched convex-MPC contact-force QP solver for MI355X (gfx950).
//
// One wavefront (64 lanes) solves one QP instance of the reference's centroidal MPC
// (convex_mpc/centroidal_mpc.py:69-359).  Algorithm (DESIGN.md "Kernel"):
//
//   1. Condense the horizon onto the free forces only (stance legs; swing forces are fixed at
//      0 by the reference's bounds, centroidal_mpc.py:150-161): H = 2 G'QG + 2R over the
//      free columns, built with the backward recursion S_j = Q2 + A'S_{j+1}A,
//      W_jj = S_j B_j, W_ij = A'W_{i+1,j}, H_ij = B_i'W_ij.  H lives in LDS as 8x8 tiles of
//      the lower triangle and is inverted in place by the symmetric sweep operator
//      (Gauss-Jordan) after unit-diagonal scaling.
//   2. ADMM (OSQP iteration with A = I) on the free forces with the per-(step, leg) set
//      {fz >= fz_min, |fx| <= mu fz, |fy| <= mu fz} projected in closed form.  The x-update
//      is written in defect-correction form x~ = x + M(rho(z - x) - grad f(x) - y): M is the
//      fp32 inverse (a preconditioner only) and grad f is evaluated by an error-coordinate
//      rollout/adjoint recursion (e_{k+1} = A e_k + B_k u_k + d_k, d_k = A r_k + g - r_{k+1}),
//      so the fixed point is accurate to the gradient's precision, not to eps32 x cond(H).
//   3. Active-set polish: once the face pattern of z is stable, solve the equality-constrained
//      QP on the identified faces (reduced basis u = T v + t0, condensed + inverted the same
//      way), refine with the accurate gradient, and accept only if the KKT conditions hold
//      (primal feasibility, multiplier signs, converged refinement) -> status 1.
//
// Instances are binned by free-variable count (capacity NC in {96,128,160,192}) so the LDS
// footprint of a wave matches its instance; each bin runs a persistent kernel that pulls
// instance ids from a device-side queue.
//
// This file is compiled as part of cmpc_host.hip (single translation unit).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cmpc_device.h"

namespace cmpc {

// ------------------------------------------------------------------------------------------
// wave helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float readlane_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
  return v;
}

// exclusive prefix sum across the 64 lanes
__device__ __forceinline__ int wave_excl_scan(int v, int lane) {
  int incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int t = __shfl_up(incl, d, 64);
    if (lane >= d) incl += t;
  }
  return incl - v;
}

// ------------------------------------------------------------------------------------------
// LDS image of one instance
// ------------------------------------------------------------------------------------------
constexpr int kMaxN = 16;
constexpr int kMaxP = 12 * kMaxN;   // 192
constexpr int kMaxTri = 4 * kMaxN;  // 64 (= lanes: lane t owns stance triple t)

template <int NC>
struct Smem {
  static constexpr int TT = NC / 8;
  static constexpr int NT = TT * (TT + 1) / 2;
  float M[NT * 64];           // lower-triangle 8x8 tiles (diagonal tiles stored full)
  float Bt[NC * 12];          // param-space input matrix, column p at Bt[12p .. 12p+11]
  float Rt[NC];               // param-space input weight (2R in the param basis)
  float x[NC], z[NC], y[NC], g[NC], r[NC], w[NC], xr[NC], v[NC], dl[NC];
  float av[NC], bv[NC], ds[NC];
  float D[kMaxP];             // d_k  (error-coordinate affine term)
  float Dt[kMaxP];            // d~_k (d_k + B_k t0_k in the polish basis)
  float H[kMaxP];             // h_k = B~_k v_k + d~_k
  float E[kMaxP];             // e_{k+1} = x_{k+1} - xref_k
  float L[kMaxP];             // lambda_k
  float U[kMaxP];             // final full u
  float A[144];
  float S[144], T1[144], W0[144], W1[144];
  int par[NC];                // param descriptor (pack_par)
  int off[kMaxN + 1];         // first param of step k
  int tri[kMaxTri];           // stance triple t -> 4k + leg
  int tri_of[kMaxTri];        // 4k + leg -> triple index or -1
  int tcnt[kMaxTri];          // polish: params of triple t
  int code[kMaxTri];          // face code of triple t
};

// param descriptor: k (5 bits) | leg (2) | axis (2) | sx+1 (2) | sy+1 (2)
__device__ __forceinline__ int pack_par(int k, int leg, int axis, int sx, int sy) {
  return k | (leg << 5) | (axis << 7) | ((sx + 1) << 9) | ((sy + 1) << 11);
}
__device__ __forceinline__ int par_k(int d) { return d & 31; }

__device__ __forceinline__ int tile_index(int I, int J) { return (I * (I + 1)) / 2 + J; }

// address of element (i, j) of the symmetric matrix in tile storage (either order)
__device__ __forceinline__ int sym_addr(int i, int j) {
  int I = i >> 3, J = j >> 3;
  if (I < J) {
    int t = i; i = j; j = t;
    t = I; I = J; J = t;
  }
  return tile_index(I, J) * 64 + (i & 7) * 8 + (j & 7);
}

template <int NC>
__device__ __forceinline__ void sym_store(Smem<NC>& s, int i, int j, float v) {
  s.M[sym_addr(i, j)] = v;
  if ((i >> 3) == (j >> 3) && i != j) s.M[sym_addr(j, i)] = v;  // diagonal tiles: both halves
}

// per-lane tile ownership: tile t = lane + 64 u  ->  (I, J)
template <int NC>
struct TileMap {
  static constexpr int NT = Smem<NC>::NT;
  static constexpr int TPL = (NT + 63) / 64;
  int I[TPL], J[TPL];
  __device__ void init(int lane) {
#pragma unroll
    for (int u = 0; u < TPL; ++u) {
      int t = lane + 64 * u;
      int Ii = 0;
      while ((Ii + 1) * (Ii + 2) / 2 <= t) ++Ii;
      I[u] = (t < NT) ? Ii : 1 << 20;
      J[u] = (t < NT) ? t - Ii * (Ii + 1) / 2 : 0;
    }
  }
};

// ------------------------------------------------------------------------------------------
// condensation + inversion:  M <- (2 G~'Q G~ + diag(Rt) + shift I)^-1 over n params
// ------------------------------------------------------------------------------------------
template <int NC>
__device__ void condense_invert(Smem<NC>& s, const KParams& P, const TileMap<NC>& tm, int n,
                                float shift, int lane) {
  constexpr int NT = Smem<NC>::NT;
  constexpr int TPL = TileMap<NC>::TPL;
  const int N = P.N;
  for (int e = lane; e < NT * 64; e += 64) s.M[e] = 0.f;
  for (int e = lane; e < 144; e += 64) s.S[e] = ((e / 12) == (e % 12)) ? P.Q2[e / 12] : 0.f;
  __syncthreads();
  for (int j = N - 1; j >= 0; --j) {
    if (j < N - 1) {  // S_j = Q2 + A' S_{j+1} A
      for (int e = lane; e < 144; e += 64) {
        const int r = e / 12, c = e % 12;
        float acc = 0.f;
#pragma unroll
        for (int q = 0; q < 12; ++q) acc = fmaf(s.S[r * 12 + q], s.A[q * 12 + c], acc);
        s.T1[e] = acc;
      }
      __syncthreads();
      for (int e = lane; e < 144; e += 64) {
        const int r = e / 12, c = e % 12;
        float acc = (r == c) ? P.Q2[r] : 0.f;
#pragma unroll
        for (int q = 0; q < 12; ++q) acc = fmaf(s.A[q * 12 + r], s.T1[q * 12 + c], acc);
        s.S[e] = acc;
      }
      __syncthreads();
    }
    const int pj0 = s.off[j], mj = s.off[j + 1] - pj0;
    if (mj == 0) continue;
    float* W = s.W0;
    float* Wn = s.W1;
    for (int e = lane; e < 12 * mj; e += 64) {  // W = S_j B~_j
      const int r = e / mj, c = e % mj;
      float acc = 0.f;
#pragma unroll
      for (int q = 0; q < 12; ++q) acc = fmaf(s.S[r * 12 + q], s.Bt[(pj0 + c) * 12 + q], acc);
      W[r * 12 + c] = acc;
    }
    __syncthreads();
    for (int i = j; i >= 0; --i) {
      if (i < j) {  // W <- A' W
        for (int e = lane; e < 12 * mj; e += 64) {
          const int r = e / mj, c = e % mj;
          float acc = 0.f;
#pragma unroll
          for (int q = 0; q < 12; ++q) acc = fmaf(s.A[q * 12 + r], W[q * 12 + c], acc);
          Wn[r * 12 + c] = acc;
        }
        __syncthreads();
        float* t = W; W = Wn; Wn = t;
      }
      const int pi0 = s.off[i], mi = s.off[i + 1] - pi0;
      // rows = params of step j (p), cols = params of step i (q): H[p][q] = B~_i[:,q]' W[:,p]
      for (int e = lane; e < mi * mj; e += 64) {
        const int pc = e / mi, qc = e % mi;
        if (i == j && pc < qc) continue;
        float acc = 0.f;
#pragma unroll
        for (int q = 0; q < 12; ++q) acc = fmaf(s.Bt[(pi0 + qc) * 12 + q], W[q * 12 + pc], acc);
        sym_store<NC>(s, pj0 + pc, pi0 + qc, acc);
      }
      // The next i only writes Wn before its barrier; W stays valid until the swap.
    }
    __syncthreads();
  }
  for (int p = lane; p < NC; p += 64) {  // + diag(Rt) + shift; padding -> identity
    const int a = sym_addr(p, p);
    if (p < n) s.M[a] += s.Rt[p] + shift;
    else s.M[a] = 1.f;
  }
  __syncthreads();

  // ---- symmetric sweep (Gauss-Jordan) inversion of the unit-diagonal-scaled matrix ----
  for (int p = lane; p < NC; p += 64) {
    const float dg = s.M[sym_addr(p, p)];
    s.ds[p] = (p < n && dg > 0.f) ? rsqrtf(dg) : 1.f;
  }
  __syncthreads();
  const int TA = (n + 7) >> 3;  // active tile rows
#pragma unroll
  for (int u = 0; u < TPL; ++u) {
    if (tm.I[u] < TA) {
      float* T = &s.M[(lane + 64 * u) * 64];
      const int I = tm.I[u], J = tm.J[u];
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) T[a * 8 + b] *= s.ds[I * 8 + a] * s.ds[J * 8 + b];
    }
  }
  __syncthreads();
  // Sweep pivot k: M_ij -= a_i a_j / d with a = column k except a_k = d - 1, then M_kk -= 2.
  // (gives M_ij - c_i c_j/d, M_ik = c_i/d, M_kk = -1/d: the sweep operator.)
  for (int k = 0; k < n; ++k) {
    const float d = s.M[sym_addr(k, k)];
    const float invd = 1.f / d;
    for (int i = lane; i < NC; i += 64) {
      const float c = (i < n) ? s.M[sym_addr(i, k)] : 0.f;
      const float a = (i == k) ? (d - 1.f) : c;
      s.av[i] = a;
      s.bv[i] = a * invd;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < TPL; ++u) {
      if (tm.I[u] < TA) {
        const int I = tm.I[u], J = tm.J[u];
        float bi[8], aj[8];
#pragma unroll
        for (int a = 0; a < 8; ++a) { bi[a] = s.bv[I * 8 + a]; aj[a] = s.av[J * 8 + a]; }
        float* T = &s.M[(lane + 64 * u) * 64];
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
          for (int b = 0; b < 8; ++b) T[a * 8 + b] = fmaf(-bi[a], aj[b], T[a * 8 + b]);
        if (I == J && (k >> 3) == I) T[(k & 7) * 9] -= 2.f;
      }
    }
    __syncthreads();
  }
  // M holds -(scaled inverse): undo the sign and the scaling
#pragma unroll
  for (int u = 0; u < TPL; ++u) {
    if (tm.I[u] < TA) {
      float* T = &s.M[(lane + 64 * u) * 64];
      const int I = tm.I[u], J = tm.J[u];
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) T[a * 8 + b] *= -s.ds[I * 8 + a] * s.ds[J * 8 + b];
    }
  }
  __syncthreads();
}

// out = M in  (n x n symmetric, tile storage)
template <int NC>
__device__ void symv(Smem<NC>& s, int n, const float* in, float* out, int lane) {
  for (int p = lane; p < n; p += 64) {
    const int Ip = p >> 3, pi = p & 7;
    float acc = 0.f;
    for (int J = 0; J * 8 < n; ++J) {
      const bool lower = Ip >= J;
      const int base = lower ? tile_index(Ip, J) * 64 + pi * 8 : tile_index(J, Ip) * 64 + pi;
      const int stride = lower ? 1 : 8;
      const int qe = min(8, n - J * 8);
      for (int b = 0; b < qe; ++b) acc = fmaf(s.M[base + b * stride], in[J * 8 + b], acc);
    }
    out[p] = acc;
  }
  __syncthreads();
}

// Gradient of  sum_k e_{k+1}'(Q2/2)e_{k+1} + v'(Rt/2)v  in the current param basis
// (e by the error-coordinate rollout).  Leaves E (e_{k+1}) and L (lambda_k) in LDS.
template <int NC>
__device__ void gradient(Smem<NC>& s, const KParams& P, int n, const float* vin, float* gout,
                         const float (&Arow)[12], const float (&Acol)[12], int lane) {
  const int N = P.N;
  const int NP = 12 * N;
  for (int o = lane; o < NP; o += 64) {  // h_k = B~_k v_k + d~_k
    const int k = o / 12, r = o % 12;
    float acc = s.Dt[o];
    for (int p = s.off[k]; p < s.off[k + 1]; ++p) acc = fmaf(s.Bt[p * 12 + r], vin[p], acc);
    s.H[o] = acc;
  }
  __syncthreads();
  const int i = lane % 12;
  float e = 0.f;
  for (int k = 0; k < N; ++k) {  // e_{k+1} = A e_k + h_k
    float acc = s.H[12 * k + i];
#pragma unroll
    for (int j = 0; j < 12; ++j) acc = fmaf(Arow[j], readlane_f(e, j), acc);
    e = acc;
    if (lane < 12) s.E[12 * k + i] = e;
  }
  float lam = 0.f;
  const float q2 = P.Q2[i];
  for (int k = N - 1; k >= 0; --k) {  // lambda_k = Q2 e_{k+1} + A' lambda_{k+1}
    float acc = q2 * s.E[12 * k + i];
#pragma unroll
    for (int j = 0; j < 12; ++j) acc = fmaf(Acol[j], readlane_f(lam, j), acc);
    lam = acc;
    if (lane < 12) s.L[12 * k + i] = lam;
  }
  __syncthreads();
  for (int p = lane; p < n; p += 64) {  // g = B~' lambda + Rt v
    const int k = par_k(s.par[p]);
    float acc = s.Rt[p] * vin[p];
#pragma unroll
    for (int r = 0; r < 12; ++r) acc = fmaf(s.Bt[p * 12 + r], s.L[12 * k + r], acc);
    gout[p] = acc;
  }
  __syncthreads();
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
__device__ void build_admm_basis(Smem<NC>& s, const KParams& P, const float* __restrict__ Bg,
                                 int ntri, int lane) {
  const int N = P.N;
  for (int e = lane; e < 3 * ntri * 12; e += 64) {
    const int p = e / 12, r = e % 12;
    const int t = p / 3, a = p % 3;
    const int kl = s.tri[t];
    const int k = kl >> 2, leg = kl & 3;
    s.Bt[e] = Bg[(k * 12 + r) * 12 + 3 * leg + a];
  }
  for (int p = lane; p < 3 * ntri; p += 64) {
    const int t = p / 3, a = p % 3;
    const int kl = s.tri[t];
    const int leg = kl & 3;
    s.Rt[p] = P.R2[3 * leg + a];
    s.par[p] = pack_par(kl >> 2, leg, a, 0, 0);
  }
  for (int k = lane; k <= N; k += 64) {
    int c = 0;
    for (int t = 0; t < ntri; ++t) c += ((s.tri[t] >> 2) < k) ? 1 : 0;
    s.off[k] = 3 * c;
  }
  for (int o = lane; o < 12 * N; o += 64) s.Dt[o] = s.D[o];
  __syncthreads();
}

// Active-set polish on the faces of z (lane t owns triple t and its face code).
// On success s.U holds the full u (12N) and s.E the state errors at that u.
template <int NC>
__device__ bool polish(Smem<NC>& s, const KParams& P, const TileMap<NC>& tm,
                       const float* __restrict__ Bg, int ntri, int code, const float (&Arow)[12],
                       const float (&Acol)[12], int lane) {
  const int N = P.N;
  const float mu = P.mu, fzmin = P.fz_min;
  const bool own = lane < ntri;
  const int kl = own ? s.tri[lane] : 0;
  const int k = kl >> 2, leg = kl & 3;
  const int sx = (code & 2) ? 1 : ((code & 4) ? -1 : 0);
  const int sy = (code & 8) ? 1 : ((code & 16) ? -1 : 0);
  const bool zl = (code & 1) != 0;
  const int cnt = own ? ((sx == 0) + (sy == 0) + (!zl)) : 0;
  const int base = wave_excl_scan(cnt, lane);
  const int nr = __shfl(base + cnt, 63, 64);
  const float* Bk = Bg + k * 144;
  int px = -1, py = -1, pz = -1;
  if (own) {
    s.tcnt[lane] = cnt;
    s.code[lane] = code;
    int p = base;
    if (sx == 0) {
      px = p++;
      for (int r = 0; r < 12; ++r) s.Bt[px * 12 + r] = Bk[r * 12 + 3 * leg];
      s.Rt[px] = P.R2[3 * leg];
      s.par[px] = pack_par(k, leg, 0, sx, sy);
      s.v[px] = s.z[3 * lane];
    }
    if (sy == 0) {
      py = p++;
      for (int r = 0; r < 12; ++r) s.Bt[py * 12 + r] = Bk[r * 12 + 3 * leg + 1];
      s.Rt[py] = P.R2[3 * leg + 1];
      s.par[py] = pack_par(k, leg, 1, sx, sy);
      s.v[py] = s.z[3 * lane + 1];
    }
    if (!zl) {
      pz = p++;
      const float cx = sx * mu, cy = sy * mu;
      for (int r = 0; r < 12; ++r)
        s.Bt[pz * 12 + r] = Bk[r * 12 + 3 * leg + 2] + cx * Bk[r * 12 + 3 * leg] +
                            cy * Bk[r * 12 + 3 * leg + 1];
      s.Rt[pz] = P.R2[3 * leg + 2] +
                 mu * mu * ((sx != 0 ? P.R2[3 * leg] : 0.f) + (sy != 0 ? P.R2[3 * leg + 1] : 0.f));
      s.par[pz] = pack_par(k, leg, 2, sx, sy);
      s.v[pz] = s.z[3 * lane + 2];
    }
  }
  __syncthreads();
  for (int kk = lane; kk <= N; kk += 64) {
    int c = 0;
    for (int t = 0; t < ntri; ++t) c += ((s.tri[t] >> 2) < kk) ? s.tcnt[t] : 0;
    s.off[kk] = c;
  }
  for (int o = lane; o < 12 * N; o += 64) {  // d~ = d + B t0 (fz locked at fz_min)
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
  __syncthreads();
  condense_invert<NC>(s, P, tm, nr, P.sigma, lane);
  float step = 3.0e38f;
  for (int it = 0; it < P.polish_refine; ++it) {
    gradient<NC>(s, P, nr, s.v, s.g, Arow, Acol, lane);
    symv<NC>(s, nr, s.g, s.dl, lane);
    float m = 0.f;
    for (int p = lane; p < nr; p += 64) {
      s.v[p] -= s.dl[p];
      m = fmaxf(m, fabsf(s.dl[p]));
    }
    step = wave_max(m);
    __syncthreads();
  }
  gradient<NC>(s, P, nr, s.v, s.g, Arow, Acol, lane);  // E, L at the final point
  // KKT checks per triple
  float fx = 0.f, fy = 0.f, fz = 0.f, gx = 0.f, gy = 0.f, gz = 0.f;
  if (own) {
    fz = zl ? fzmin : s.v[pz];
    fx = (sx == 0) ? s.v[px] : sx * mu * fz;
    fy = (sy == 0) ? s.v[py] : sy * mu * fz;
    float ax = 0.f, ay = 0.f, az = 0.f;
    for (int r = 0; r < 12; ++r) {
      const float lr = s.L[12 * k + r];
      ax = fmaf(Bk[r * 12 + 3 * leg], lr, ax);
      ay = fmaf(Bk[r * 12 + 3 * leg + 1], lr, ay);
      az = fmaf(Bk[r * 12 + 3 * leg + 2], lr, az);
    }
    gx = ax + P.R2[3 * leg] * fx;
    gy = ay + P.R2[3 * leg + 1] * fy;
    gz = az + P.R2[3 * leg + 2] * fz;
  }
  const float gs = wave_max(fmaxf(fabsf(gx), fmaxf(fabsf(gy), fabsf(gz))));
  const float us = wave_max(fmaxf(1.f, fmaxf(fabsf(fx), fmaxf(fabsf(fy), fabsf(fz)))));
  const float tol_d = P.polish_tol * gs, tol_p = P.polish_tol * us;
  bool ok = true;
  if (own) {
    const float lx = sx ? -sx * gx : 0.f;
    const float ly = sy ? -sy * gy : 0.f;
    const float l0 = gz - mu * (lx + ly);
    if (sx && lx < -tol_d) ok = false;
    if (sy && ly < -tol_d) ok = false;
    if (zl && l0 < -tol_d) ok = false;
    if (!sx && fabsf(fx) > mu * fz + tol_p) ok = false;
    if (!sy && fabsf(fy) > mu * fz + tol_p) ok = false;
    if (!zl && fz < fzmin - tol_p) ok = false;
    if (!(isfinite(fx) && isfinite(fy) && isfinite(fz))) ok = false;
  }
  const bool all_ok = (__all(ok) != 0) && (step <= P.polish_tol * us);
  if (all_ok) {
    for (int o = lane; o < 12 * N; o += 64) s.U[o] = 0.f;
    __syncthreads();
    if (own) {
      s.U[12 * k + 3 * leg] = fx;
      s.U[12 * k + 3 * leg + 1] = fy;
      s.U[12 * k + 3 * leg + 2] = fz;
    }
    __syncthreads();
  }
  return all_ok;
}

template <int NC>
__device__ void solve_instance(Smem<NC>& s, const KParams& P, const TileMap<NC>& tm, int64_t b,
                               const Inputs& in, const Outputs& out, int lane) {
  const int N = P.N;
  const int NP = 12 * N;
  const float* Ab = in.Ad + b * 144;
  const float* Bg = in.Bd + b * (int64_t)N * 144;
  const float* gdb = in.gd + b * 12;
  const float* x0b = in.x0 + b * 12;
  const float* xrb = in.xref + b * (int64_t)N * 12;
  const uint8_t* ctb = in.contact + b * (int64_t)4 * N;

  for (int e = lane; e < 144; e += 64) s.A[e] = Ab[e];
  // stance triples in (k, leg) order; lane = 4k + leg
  const bool st = (lane < 4 * N) ? (ctb[(lane & 3) * N + (lane >> 2)] != 0) : false;
  const int pos = wave_excl_scan(st ? 1 : 0, lane);
  const int ntri = __shfl(pos + (st ? 1 : 0), 63, 64);
  if (st) s.tri[pos] = lane;
  if (lane < 4 * N) s.tri_of[lane] = st ? pos : -1;
  __syncthreads();
  const int i12 = lane % 12;
  float Arow[12], Acol[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    Arow[j] = s.A[i12 * 12 + j];
    Acol[j] = s.A[j * 12 + i12];
  }
  // d_k = A r_k + gd - r_{k+1},  r_0 = x0, r_{k+1} = xref[k]
  for (int o = lane; o < NP; o += 64) {
    const int k = o / 12, r = o % 12;
    const float* rk = (k == 0) ? x0b : (xrb + (k - 1) * 12);
    float acc = gdb[r] - xrb[k * 12 + r];
#pragma unroll
    for (int j = 0; j < 12; ++j) acc = fmaf(s.A[r * 12 + j], rk[j], acc);
    s.D[o] = acc;
  }
  __syncthreads();
  build_admm_basis<NC>(s, P, Bg, ntri, lane);
  const int n = 3 * ntri;

  int status = -2, iters = 0;
  bool polished = false;
  if (n == 0) {
    status = 1;
  } else {
    float rho = P.rho0;
    condense_invert<NC>(s, P, tm, n, P.sigma + rho, lane);
    for (int p = lane; p < n; p += 64) { s.x[p] = 0.f; s.z[p] = 0.f; s.y[p] = 0.f; }
    __syncthreads();
    int prev_code = -1, stable = 0;
    const float alpha = P.alpha;
    float rp = 0.f, rd = 0.f, np_ = 0.f, nd = 0.f;
    for (int it = 1; it <= P.max_iter; ++it) {
      iters = it;
      gradient<NC>(s, P, n, s.x, s.g, Arow, Acol, lane);
      for (int p = lane; p < n; p += 64) s.r[p] = rho * (s.z[p] - s.x[p]) - s.g[p] - s.y[p];
      __syncthreads();
      symv<NC>(s, n, s.r, s.dl, lane);
      const float inv_rho = 1.f / rho;
      for (int p = lane; p < n; p += 64) {
        const float xt = s.x[p] + s.dl[p];
        const float xr = alpha * xt + (1.f - alpha) * s.z[p];
        s.x[p] = alpha * xt + (1.f - alpha) * s.x[p];
        s.xr[p] = xr;
        s.w[p] = xr + s.y[p] * inv_rho;
      }
      __syncthreads();
      int code = 0;
      float lrp = 0.f, lrd = 0.f, lnp = 0.f, lnd = 0.f;
      if (lane < ntri) {
        float pxv, pyv, pzv;
        code = project(s.w[3 * lane], s.w[3 * lane + 1], s.w[3 * lane + 2], P.mu, P.fz_min,
                       pxv, pyv, pzv);
        const float pr[3] = {pxv, pyv, pzv};
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          const int p = 3 * lane + a;
          const float zn = pr[a];
          const float yn = s.y[p] + rho * (s.xr[p] - zn);
          s.z[p] = zn;
          s.y[p] = yn;
          const float xp = s.x[p], gp = s.g[p];
          lrp = fmaxf(lrp, fabsf(xp - zn));
          lrd = fmaxf(lrd, fabsf(gp + yn));
          lnp = fmaxf(lnp, fmaxf(fabsf(xp), fabsf(zn)));
          lnd = fmaxf(lnd, fmaxf(fabsf(gp), fabsf(yn)));
        }
      }
      __syncthreads();
      const bool changed = (lane < ntri) && (code != prev_code);
      prev_code = code;
      stable = (__any(changed) != 0) ? 0 : stable + 1;
      if (stable >= P.polish_stable) {
        if (polish<NC>(s, P, tm, Bg, ntri, code, Arow, Acol, lane)) {
          polished = true;
          status = 1;
          break;
        }
        stable = -P.polish_stable;  // back off before the next attempt
        build_admm_basis<NC>(s, P, Bg, ntri, lane);
        condense_invert<NC>(s, P, tm, n, P.sigma + rho, lane);
      }
      const bool last = (it == P.max_iter);
      const bool adapt = P.adaptive_interval > 0 && (it % P.adaptive_interval) == 0;
      if (adapt || last) {
        rp = wave_max(lrp); rd = wave_max(lrd); np_ = wave_max(lnp); nd = wave_max(lnd);
      }
      if (adapt && !last) {
        float nr = rho * sqrtf((rp / fmaxf(np_, 1e-30f)) / (rd / fmaxf(nd, 1e-30f) + 1e-30f));
        nr = fminf(fmaxf(nr, 1e-6f), 1e6f);
        if (nr > 5.f * rho || nr < 0.2f * rho) {
          rho = nr;
          condense_invert<NC>(s, P, tm, n, P.sigma + rho, lane);
        }
      }
    }
    if (!polished) {
      const bool conv = rp <= P.eps_abs + P.eps_rel * np_ && rd <= P.eps_abs + P.eps_rel * nd;
      status = conv ? 2 : -2;
    }
  }
  if (!polished) {
    // u from z (ADMM basis), E at that u
    gradient<NC>(s, P, n, s.z, s.g, Arow, Acol, lane);
    for (int o = lane; o < NP; o += 64) s.U[o] = 0.f;
    __syncthreads();
    for (int p = lane; p < n; p += 64) {
      const int kl = s.tri[p / 3];
      s.U[12 * (kl >> 2) + 3 * (kl & 3) + (p % 3)] = s.z[p];
    }
    __syncthreads();
  }
  float* wb = out.w + b * (int64_t)(24 * N);
  bool finite = true;
  for (int o = lane; o < NP; o += 64) {
    const float xv = s.E[o] + xrb[o];
    const float uv = s.U[o];
    finite = finite && isfinite(xv) && isfinite(uv);
    wb[o] = xv;
    wb[NP + o] = uv;
  }
  if (__all(finite) == 0) status = -10;
  if (lane == 0) {
    out.status[b] = status;
    out.iters[b] = iters;
  }
  __syncthreads();
}

template <int NC>
__global__ void __launch_bounds__(64) solve_bin_kernel(KParams P, Inputs in, Outputs out,
                                                      const int* __restrict__ list,
                                                      const int* __restrict__ count,
                                                      int* __restrict__ head) {
  __shared__ Smem<NC> s;
  const int lane = threadIdx.x;
  TileMap<NC> tm;
  tm.init(lane);
  const int total = *count;
  for (;;) {
    int idx = 0;
    if (lane == 0) idx = atomicAdd(head, 1);
    idx = __shfl(idx, 0, 64);
    if (idx >= total) break;
    solve_instance<NC>(s, P, tm, (int64_t)list[idx], in, out, lane);
  }
}

__global__ void bin_kernel(int N, int64_t B, const uint8_t* __restrict__ contact,
                           int* __restrict__ counts, int* __restrict__ lists, int64_t stride) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint8_t* c = contact + b * 4 * N;
  int cnt = 0;
  for (int i = 0; i < 4 * N; ++i) cnt += c[i] != 0;
  const int nf = 3 * cnt;
  int bin = kNumBins - 1;
  for (int q = 0; q < kNumBins; ++q)
    if (nf <= kBinCap[q]) { bin = q; break; }
  const int pos = atomicAdd(&counts[bin], 1);
  lists[bin * stride + pos] = (int)b;
}

}  // namespace cmpc
