// cmpc_wspace.hip -- the WRENCH-SPACE factorization: one kernel for every instance of a large
// batch, whatever its number of free forces.
//
// The reference's discrete input matrices have the centroidal structure (com_trajectory.py:
// 221-286): Bd_k = (I dt + Ac dt^2 / 2) Bc_k with Bc_k = [0; E_k] (forces enter only the
// velocity and angular-velocity rows), so rows 0-5 of every force column b are
//     b[0:6] = K b[6:12],   K = 1/2 (Ad - I)[0:6, 6:12]  (= 1/2 Ad[0:6, 6:12]).
// Every column of the condensed problem is therefore b_p = Mb e_p with Mb = [K; I6] (12 x 6, one
// per instance) and e_p = b_p[6:12], the column's 6-dim "wrench" (its share of the step's net
// force and torque).  The condensed Hessian of any basis (ADMM: every stance force; polish: a
// face set) is
//     H + shift = D + V' Pw V,    D = diag(Rt) + shift (n x n),
//                                 V = the e_p placed in their step's 6 rows (6N x n),
//     Pw = sum_t Gw_t' Q2 Gw_t    (6N x 6N: the condensation over wrenches, Gw_t block k = A^{t-k} Mb),
// and by Woodbury
//     (H + shift)^-1 = D^-1 - D^-1 V' W V D^-1,     W = (Pw^-1 + S)^-1,  S = V D^-1 V'
// with S block diagonal (one 6 x 6 block per step).  Pw depends only on (A, Q): it is condensed and
// inverted ONCE per instance (96 x 96 for N = 16) and parked in the wave's slab; every
// factorization (ADMM rho, each polish face set and repair) then loads Pw^-1, adds S and inverts
// 96 x 96 -- for any number n of free forces (up to 192), in 21 register tiles.  The old path
// condensed and inverted n x n per factorization (36 tiles at n <= 128, 55-78 above, one wave
// alone on a SIMD): here every instance is one register class, two waves per SIMD.
//
// The inverse is only the preconditioner of the defect-correction iterations (cmpc_wave.hip 3):
// the gradient stays the exact error-coordinate rollout, so the fixed points -- the solutions --
// are unchanged.  Woodbury's fp32 cancellation makes it a looser preconditioner than the n x n
// inverse (NumPy model, tests/algo_spec.py with this factorization: spectral radius of I - M H
// 1e-3 (ADMM) / 1e-2 (face sets) against 4e-4 / 2e-3, with the same iterations, polish sessions
// and refinement counts on the cfg1 / cfg2 / hard fixtures).
//
// An instance whose Bd is not of this form (not produced by the reference's discretisation) is
// handed to the n-space kernels (cmpc_wave.hip solve_group_kernel) through their bin queues.
//
// This file is compiled as part of cmpc_wave.hip (single translation unit).

constexpr int kWN = 6 * kMaxN;  // wrench coordinates (96 at N = 16)
using CW = Cfg<kWN>;            // W in 6 x 6 / 2 = 21 lower-triangle register tiles

struct SmemW {
#ifdef CMPC_STAMPS
  unsigned long long st[32];
#endif
  alignas(16) float Et[kMaxP * 6];  // e_p of param p at Et[6p .. 6p+5]
  alignas(16) float Rt[kMaxP];      // param weight (2R in the param basis)
  alignas(16) float x[kMaxP];
  alignas(16) float z[kMaxP];
  alignas(16) float y[kMaxP];       // ADMM dual (x, z, y of triple t at 3t .. 3t+2)
  alignas(16) float v[kMaxP];
  union {
    struct {
      alignas(16) float g[kMaxP];
      alignas(16) float r[kMaxP];
      alignas(16) float dl[kMaxP];
    };
    alignas(16) float T0w[kMaxTri * 6];  // polish setup: wrench of each triple's locked forces
    alignas(16) float Sb[kMaxN * 36];    // factorization: the 6 x 6 blocks S_k
  };
  union {
    struct {  // factorization: the sweep's scaling and panel
      alignas(16) float ds[kWN];
      alignas(16) float pan[kWN * 4];
    };
    struct {  // apply: t = V D^-1 in, then W t
      alignas(16) float tw[kWN];
      alignas(16) float zw[kWN];
    };
  };
  float E[kMaxP];   // e_{k+1} = x_{k+1} - xref_k
  float L[kMaxP];   // lambda_k
  float Mu[kWN];    // Mb' lambda_k
  float D[kMaxP];   // d_k  (error-coordinate affine term)
  float Dt[kMaxP];  // d~_k (d_k + B_k t0_k in the polish basis)
  float A[144];
  float Mb[72];     // [12][6]
  float Q2[12];
  float R2[12];
  int par[kMaxP];   // param -> step k
  int off[kMaxN + 1];
  int tri[kMaxTri];
  int tri_of[kMaxTri];
  int tcnt[kMaxTri];
  int code[kMaxTri];
  int pcode[kMaxTri];
  int fpk[kMaxTri];
  uint8_t fpat[kFailMem][kMaxTri];
  uint8_t tpat[kTryMem][kMaxTri];
};
#ifndef CMPC_STAMPS
static_assert(sizeof(SmemW) <= 20480, "eight one-wave workgroups per CU");
#endif
static_assert(offsetof(SmemW, v) == offsetof(SmemW, y) + kMaxP * sizeof(float),
              "y and v are one free 2 kMaxP block during the interior-point steps");

// per-wave slab (floats): Pw^-1, the parked ADMM W, the ADMM state kept aside during the
// interior-point steps (x, z, y), the interior-point state (z, s, ds_aff, dz_aff x 5 rows x 64)
constexpr size_t kWsSlab = 2 * CW::NTL * 256 + 3 * kMaxP + kIpmKeep;

// ------------------------------------------------------------------------------------------
// structure matrix, basis, wrench condensation
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void ws_setup_mb(SmemW& s) {
  const int l = opaque_lane();
  WSYNC();
  for (int e = l; e < 72; e += 64) {
    const int r = e / 6, j = e % 6;
    s.Mb[e] = (r < 6) ? 0.5f * s.A[r * 12 + 6 + j] : ((r - 6 == j) ? 1.f : 0.f);
  }
  WSYNC();
}

// ADMM basis: every stance triple contributes (fx, fy, fz) as params 3t, 3t+1, 3t+2, e_p = rows
// 6-11 of its Bd column.  Returns false (wave-uniform) if some column is not Mb e_p (to fp32
// rounding): that instance goes to the n-space kernels.
__device__ __forceinline__ bool ws_admm_basis(SmemW& s, const KParams& P,
                                              const float* __restrict__ Bg, int ntri, bool check) {
  const int lane = opaque_lane();
  const int N = P.N;
  const int n = 3 * ntri;
  WSYNC();
  bool bad = false;
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
      for (int i = 0; i < 6; ++i) s.Et[(3 * lane + a) * 6 + i] = bv[3 * (6 + i) + a];
    }
    if (check) {
#pragma unroll
      for (int a = 0; a < 3; ++a) {
#pragma unroll
        for (int r = 0; r < 6; ++r) {
          float pr = 0.f, pa = 0.f;
#pragma unroll
          for (int j = 0; j < 6; ++j) {
            const float t = s.Mb[r * 6 + j] * bv[3 * (6 + j) + a];
            pr += t;
            pa += fabsf(t);
          }
          const float b0 = bv[3 * r + a];
          // (a NaN fails the test too)
          if (!(fabsf(b0 - pr) <= 4e-6f * (fabsf(b0) + pa) + 1e-30f)) bad = true;
        }
      }
    }
  }
  for (int p = lane; p < kMaxP; p += 64) {
    if (p < n) {
      const int t = p / 3, a = p % 3;
      const int kl = s.tri[t];
      s.Rt[p] = s.R2[3 * (kl & 3) + a];
      s.par[p] = kl >> 2;
    } else {
      s.Rt[p] = 0.f;
      s.par[p] = 0;
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
  return __any(bad) == 0;
}

// Pw = sum_t Gw_t' Q2 Gw_t straight into the register tiles (as condense_tiles_fwd, with six
// params per step whose columns are Mb's), identity on padding, then inverted in place.
__device__ __forceinline__ void ws_condense_pw(SmemW& s, const KParams& P, f4 (&M)[CW::NTL]) {
  const int lane = opaque_lane();
  const int g = lane >> 4, c = lane & 15;
  const int N = P.N;
  const int nw = 6 * N;
#pragma unroll
  for (int t = 0; t < CW::NTL; ++t) M[t] = f4{0.f, 0.f, 0.f, 0.f};
  const int sc = ((c & 3) < 3) ? 3 * (c >> 2) + (c & 3) : -1;
  float aA[3], q2[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int r = 3 * g + q;
    aA[q] = (sc >= 0) ? s.A[sc * 12 + r] : 0.f;
    q2[q] = s.Q2[r];
  }
  int kI[CW::TT];  // first step of tile row I
#pragma unroll
  for (int I = 0; I < CW::TT; ++I) kI[I] = (16 * I < nw) ? (16 * I) / 6 : N;
  f4 Gd[CW::TT];
#pragma unroll
  for (int J = 0; J < CW::TT; ++J) Gd[J] = f4{0.f, 0.f, 0.f, 0.f};
  for (int t = 0; t < N; ++t) {
    if (t > 0) {  // Gw_t = A Gw_{t-1} on the chunks that already hold columns
#pragma unroll
      for (int J = 0; J < CW::TT; ++J) {
        if (kI[J] >= t) continue;  // uniform
        f4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 3; ++q) d = mfma4(aA[q], Gd[J][q], d);
        Gd[J] = d;
      }
    }
    const int p0 = 6 * t;  // the six new columns of step t: Mb's
#pragma unroll
    for (int J = 0; J < CW::TT; ++J) {
      if (16 * J + 15 < p0 || 16 * J >= p0 + 6) continue;  // uniform
      const int p = 16 * J + c;
      if (p >= p0 && p < p0 + 6) {
        const int j = p - p0;
        Gd[J] = f4{s.Mb[(3 * g) * 6 + j], s.Mb[(3 * g + 1) * 6 + j], s.Mb[(3 * g + 2) * 6 + j], 0.f};
      }
    }
#pragma unroll
    for (int I = 0; I < CW::TT; ++I) {
      if (kI[I] > t) continue;  // uniform
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
#pragma unroll
  for (int I = 0; I < CW::TT; ++I) {
#pragma unroll
    for (int J = 0; J <= I; ++J) {
      f4 v = M[tile_index(I, J)];
      const int col = 16 * J + c;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * I + 4 * g + q;
        if (row >= nw || col >= nw) v[q] = (row == col) ? 1.f : 0.f;
        else if (row == col) v[q] *= 1.f + 1e-7f;  // (keeps a Q with zeros from a singular Pw)
      }
      M[tile_index(I, J)] = v;
    }
  }
  WSYNC();
  invert_tiles<kWN>(s, M, nw);
}

// W = (Pw^-1 + S)^-1 for the basis in Et / Rt and this shift: the tiles get the parked Pw^-1 plus
// the blocks S_k = sum_{p in step k} e_p e_p' / (Rt_p + shift), then the block sweep.
__device__ __forceinline__ void ws_factor(SmemW& s, const KParams& P, f4 (&M)[CW::NTL], int n,
                                          float shift, const float* __restrict__ park_pw) {
  const int lane = opaque_lane();
  const int g = lane >> 4, c = lane & 15;
  const int N = P.N;
  const int nw = 6 * N;
  n = uniform(n);
  WSYNC();
  for (int e = lane; e < 36 * N; e += 64) {
    const int k = e / 36, ij = e % 36, i = ij / 6, j = ij % 6;
    const int p1 = s.off[k + 1];
    float acc = 0.f;
    for (int p = s.off[k]; p < p1; ++p)
      acc = fmaf(s.Et[6 * p + i] * s.Et[6 * p + j], __builtin_amdgcn_rcpf(s.Rt[p] + shift), acc);
    s.Sb[e] = acc;
  }
  park_load<kWN>(park_pw, M);
  WSYNC();
  // a step's 6 x 6 block spans at most two tile rows / columns: only tiles (I, I) and (I, I-1)
#pragma unroll
  for (int I = 0; I < CW::TT; ++I) {
#pragma unroll
    for (int J = (I > 0 ? I - 1 : 0); J <= I; ++J) {
      f4 m = M[tile_index(I, J)];
      const int col = 16 * J + c;
      const int kc = col / 6;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * I + 4 * g + q;
        const int kr = row / 6;
        if (row < nw && col < nw && kr == kc) m[q] += s.Sb[kc * 36 + (row - 6 * kr) * 6 + (col - 6 * kc)];
      }
      M[tile_index(I, J)] = m;
    }
  }
  WSYNC();
  invert_tiles<kWN>(s, M, nw);
}

// out = (H + shift)^-1 in over the first n params: y = D^-1 in, t = V y, z = W t,
// out = y - D^-1 V' z.  (in and out distinct; both read as zero past n.)
__device__ __forceinline__ void ws_apply(SmemW& s, const KParams& P, const f4 (&M)[CW::NTL],
                                         int n, float shift, const float* in, float* out) {
  const int lane = opaque_lane();
  const int N = P.N;
  const int nw = 6 * N;
  n = uniform(n);
  WSYNC();
  for (int p = lane; p < n; p += 64) out[p] = in[p] * __builtin_amdgcn_rcpf(s.Rt[p] + shift);
  WSYNC();
  for (int w = lane; w < nw; w += 64) {
    const int k = w / 6, i = w % 6;
    const int p1 = s.off[k + 1];
    float acc = 0.f;
    for (int p = s.off[k]; p < p1; ++p) acc = fmaf(s.Et[6 * p + i], out[p], acc);
    s.tw[w] = acc;
  }
  symv<kWN>(s, M, nw, s.tw, s.zw);
  for (int p = lane; p < n; p += 64) {
    const int k = s.par[p];
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 6; ++i) acc = fmaf(s.Et[6 * p + i], s.zw[6 * k + i], acc);
    out[p] = fmaf(-acc, __builtin_amdgcn_rcpf(s.Rt[p] + shift), out[p]);
  }
  WSYNC();
}

// Gradient of sum_k e_{k+1}'(Q2/2)e_{k+1} + v'(Rt/2)v in the current param basis (exact
// error-coordinate rollout and adjoint as cmpc_wave.hip gradient, with b_p = Mb e_p): h_k =
// Mb (sum_{p in k} e_p v_p) + d~_k, then the MFMA scans; g_p = e_p' (Mb' lambda_k) + Rt_p v_p.
// Leaves E, L and Mu in LDS.
__device__ __forceinline__ void ws_gradient(SmemW& s, const KParams& P, int n, const float* vin,
                                            float* gout) {
  CMPC_T0(t_gr);
  const int lane = opaque_lane();
  const int g = lane >> 4, c = lane & 15;
  const int N = P.N;
  n = uniform(n);
  WSYNC();
  f4 Et4 = {0.f, 0.f, 0.f, 0.f};
  if (c < N) {
    float w6[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int p1 = s.off[c + 1];
    for (int p = s.off[c]; p < p1; ++p) {
      const float vp = vin[p];
#pragma unroll
      for (int i = 0; i < 6; ++i) w6[i] = fmaf(s.Et[6 * p + i], vp, w6[i]);
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int r = 3 * g + q;
      float h = s.Dt[12 * c + r];
#pragma unroll
      for (int i = 0; i < 6; ++i) h = fmaf(s.Mb[r * 6 + i], w6[i], h);
      Et4[q] = h;
    }
  }
  f4 pw[4], tw[4];  // d = 1, 2, 4, 8
  gradient_powers(s, pw, tw);
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    if ((1 << l) >= N) break;  // uniform
    f4 sh = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      switch (l) {
        case 0: sh[q] = dpp<0x111>(Et4[q]); break;  // row_shr:1
        case 1: sh[q] = dpp<0x112>(Et4[q]); break;  // row_shr:2
        case 2: sh[q] = dpp<0x114>(Et4[q]); break;  // row_shr:4
        default: sh[q] = dpp<0x118>(Et4[q]); break; // row_shr:8
      }
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) Et4 = mfma4(tw[l][q], sh[q], Et4);
  }
  if (c < N) {
#pragma unroll
    for (int q = 0; q < 3; ++q) s.E[12 * c + 3 * g + q] = Et4[q];
  }
  f4 Lt = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 3; ++q) Lt[q] = (c < N) ? s.Q2[3 * g + q] * Et4[q] : 0.f;
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
    for (int q = 0; q < 3; ++q) Lt = mfma4(pw[l][q], sh[q], Lt);
  }
  if (c < N) {
#pragma unroll
    for (int q = 0; q < 3; ++q) s.L[12 * c + 3 * g + q] = Lt[q];
  }
  WSYNC();
  for (int w = lane; w < 6 * N; w += 64) {  // Mu_k = Mb' lambda_k
    const int k = w / 6, i = w % 6;
    float acc = 0.f;
#pragma unroll
    for (int r = 0; r < 12; ++r) acc = fmaf(s.Mb[r * 6 + i], s.L[12 * k + r], acc);
    s.Mu[w] = acc;
  }
  WSYNC();
  for (int p = lane; p < n; p += 64) {
    const int k = s.par[p];
    float acc = s.Rt[p] * vin[p];
#pragma unroll
    for (int i = 0; i < 6; ++i) acc = fmaf(s.Et[6 * p + i], s.Mu[6 * k + i], acc);
    gout[p] = acc;
  }
  WSYNC();
  CMPC_ACC(2, t_gr);
  CMPC_CNT(12, 1);
}

// Polish setup in the wrench space: the reduced basis of the faces in s.code (cmpc_wave.hip
// polish_setup), e_p of each reduced column, and d~ = d + Mb (the locked forces' wrench).
__device__ __forceinline__ int ws_polish_setup(SmemW& s, const KParams& P,
                                               const float* __restrict__ Bg, int ntri) {
  const int lane = opaque_lane();
  const int N = P.N;
  const float mu = P.mu, fzmin = P.fz_min;
  WSYNC();
  const bool owns = lane < ntri;
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
    float ex[6], ey[6], ez[6];  // wrench rows of the leg's fx, fy, fz columns
    {
      const float* src = Bg + k * 144 + 6 * 12 + 3 * leg;
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        ex[i] = src[i * 12];
        ey[i] = src[i * 12 + 1];
        ez[i] = src[i * 12 + 2];
      }
    }
    s.tcnt[lane] = cnt;
    int p = base;
    int px = 255, py = 255, pz = 255;
    if (sx == 0) {
      px = p++;
#pragma unroll
      for (int i = 0; i < 6; ++i) s.Et[px * 6 + i] = ex[i];
      s.Rt[px] = s.R2[3 * leg];
      s.par[px] = k;
      s.v[px] = s.z[3 * lane];
    }
    if (sy == 0) {
      py = p++;
#pragma unroll
      for (int i = 0; i < 6; ++i) s.Et[py * 6 + i] = ey[i];
      s.Rt[py] = s.R2[3 * leg + 1];
      s.par[py] = k;
      s.v[py] = s.z[3 * lane + 1];
    }
    if (!zl) {
      pz = p++;
      const float cx = sx * mu, cy = sy * mu;
#pragma unroll
      for (int i = 0; i < 6; ++i) s.Et[pz * 6 + i] = ez[i] + cx * ex[i] + cy * ey[i];
      s.Rt[pz] = s.R2[3 * leg + 2] + mu * mu * ((sx != 0 ? s.R2[3 * leg] : 0.f) +
                                                (sy != 0 ? s.R2[3 * leg + 1] : 0.f));
      s.par[pz] = k;
      s.v[pz] = s.z[3 * lane + 2];
    } else {  // fz locked at fz_min: the triple's constant force enters d~ through Mb (its wrench)
      const float tx = sx * mu * fzmin, ty = sy * mu * fzmin;
#pragma unroll
      for (int i = 0; i < 6; ++i) s.T0w[lane * 6 + i] = fmaf(ez[i], fzmin, fmaf(ey[i], ty, ex[i] * tx));
    }
    s.fpk[lane] = px | (py << 8) | (pz << 16);
  }
  WSYNC();
  {  // off[kk] = params of the triples before step kk (cmpc_wave.hip polish_setup)
    const unsigned long long sm = __ballot(lane < 4 * N && s.tri_of[lane] >= 0);
    const unsigned long long below = (lane >= 16) ? ~0ull : ((1ull << (4 * lane)) - 1ull);
    const int tstar = __popcll(sm & below);
    const int bt = __shfl(base, tstar < 64 ? tstar : 63, 64);
    if (lane <= N) s.off[lane] = (tstar < ntri) ? bt : nr;
  }
  for (int o = lane; o < 12 * N; o += 64) {  // d~ = d + Mb w0 (LDS only)
    const int kk = o / 12, r = o % 12;
    float w0[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      const int t = s.tri_of[4 * kk + l];
      if (t >= 0 && (s.code[t] & 1)) {
#pragma unroll
        for (int i = 0; i < 6; ++i) w0[i] += s.T0w[t * 6 + i];
      }
    }
    float acc = s.D[o];
#pragma unroll
    for (int i = 0; i < 6; ++i) acc = fmaf(s.Mb[r * 6 + i], w0[i], acc);
    s.Dt[o] = acc;
  }
  for (int p = lane; p < kMaxP; p += 64)
    if (p >= nr) s.v[p] = 0.f;
  WSYNC();
  return nr;
}

// Polish check (cmpc_wave.hip polish_check) with B_k' lambda_k = E_k' Mu_k (Mu from the last
// gradient call, at the final point).
__device__ __forceinline__ bool ws_polish_check(SmemW& s, const KParams& P,
                                                const float* __restrict__ Bg, int ntri, float step,
                                                bool& changed, bool& loose) {
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
    const int pk = s.fpk[lane];
    const int px = pk & 255, py = (pk >> 8) & 255, pz = (pk >> 16) & 255;
    fz = zl ? fzmin : s.v[pz];
    fx = (sx == 0) ? s.v[px] : sx * mu * fz;
    fy = (sy == 0) ? s.v[py] : sy * mu * fz;
    const float* Bk = Bg + k * 144 + 6 * 12 + 3 * leg;
    float ax = 0.f, ay = 0.f, az = 0.f;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const float m = s.Mu[6 * k + i];
      ax = fmaf(Bk[i * 12], m, ax);
      ay = fmaf(Bk[i * 12 + 1], m, ay);
      az = fmaf(Bk[i * 12 + 2], m, az);
    }
    gx = ax + s.R2[3 * leg] * fx;
    gy = ay + s.R2[3 * leg + 1] * fy;
    gz = az + s.R2[3 * leg + 2] * fz;
  }
  const float gs = wave_max(fmaxf(fabsf(gx), fmaxf(fabsf(gy), fabsf(gz))));
  const float us = wave_max(fmaxf(1.f, fmaxf(fabsf(fx), fmaxf(fabsf(fy), fabsf(fz)))));
  const float tol_d = P.polish_tol * gs, tol_p = P.polish_tol * us;
  bool ok = true;
  int nc = 0;
  if (owns) {
    const float lx = sx ? -sx * gx : 0.f;
    const float ly = sy ? -sy * gy : 0.f;
    const float l0 = gz - mu * (lx + ly);
    nc = code;
    if (sx && lx < -tol_d) { ok = false; nc &= ~6; }
    if (sy && ly < -tol_d) { ok = false; nc &= ~24; }
    if (zl && l0 < -tol_d) { ok = false; nc &= ~1; }
    if (!sx && fabsf(fx) > mu * fz + tol_p) { ok = false; nc |= (fx > 0.f) ? 2 : 4; }
    if (!sy && fabsf(fy) > mu * fz + tol_p) { ok = false; nc |= (fy > 0.f) ? 8 : 16; }
    if (!zl && fz < fzmin - tol_p) { ok = false; nc |= 1; }
    if (!(isfinite(fx) && isfinite(fy) && isfinite(fz))) ok = false;
    s.tcnt[lane] = nc;
    const float ig = 1.f / fmaxf(gs, 1e-30f), iu = 1.f / us;
    float v = fmaxf(fmaxf(sx ? -lx * ig : 0.f, sy ? -ly * ig : 0.f), zl ? -l0 * ig : 0.f);
    v = fmaxf(v, fmaxf(sx ? 0.f : (fabsf(fx) - mu * fz) * iu, sy ? 0.f : (fabsf(fy) - mu * fz) * iu));
    v = fmaxf(v, zl ? 0.f : (fzmin - fz) * iu);
    const bool fin = isfinite(fx) && isfinite(fy) && isfinite(fz);
    lok = fin && v <= kLooseTol * P.polish_tol;
    s.dl[3 * lane] = fx;  // the candidate, for a loose acceptance by the caller
    s.dl[3 * lane + 1] = fy;
    s.dl[3 * lane + 2] = fz;
  }
  changed = __any(owns && nc != code) != 0;
  const bool step_ok = step <= P.polish_tol * us;
  loose = (__all(lok) != 0) && step_ok;
  const bool all_ok = (__all(ok) != 0) && step_ok;
  if (all_ok && owns) {
    s.x[3 * lane] = fx;
    s.x[3 * lane + 1] = fy;
    s.x[3 * lane + 2] = fz;
  }
  return all_ok;
}

// the starting face set of a polish session (cmpc_wave.hip session_start / tried_before)
__device__ __forceinline__ int ws_session_start(SmemW& s, const KParams& P, int ntri, int nfail,
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
    if (k >= nfail) break;
    const bool diff = (l < ntri) && (s.fpat[k][l] != c);
    seen |= (__any(diff) == 0);
  }
  if (seen) return 0;
  return (nfail >= 2) ? min(P.polish_repairs, kLateRepairs) : P.polish_repairs;
}

__device__ __forceinline__ bool ws_tried_before(SmemW& s, int ntri, int ntried) {
  const int l = opaque_lane();
  WSYNC();
  const uint8_t c = (l < ntri) ? (uint8_t)s.tcnt[l] : 0;
  bool hit = false;
  for (int k = 0; k < ntried; ++k) {
    const bool diff = (l < ntri) && (s.tpat[k][l] != c);
    hit |= (__any(diff) == 0);
  }
  return hit;
}

// ------------------------------------------------------------------------------------------
// Interior-point identification of the face set (cmpc_wave.hip ipm_identify) in the wrench
// space.  The Newton matrix P + sigma I + G' diag(z/s) G only changes the block diagonal: each
// stance triple's 3 x 3 block D_t = diag(Rt + sigma) + G_t' diag(d) G_t (d = z/s of its five
// pyramid rows), so Woodbury still holds with D block diagonal.  D_t has the arrow form
// [[a, 0, b], [0, c, e], [b, e, f]]; its LDL' (l31 = b/a, l32 = e/c) has the Schur complement
//   f - b^2/a - e^2/c = d0 + rz + mu^2 (4 d1 d2 + (d1 + d2) rx) / a + mu^2 (4 d3 d4 + (d3 + d4) ry) / c,
// a sum of positive terms (no cancellation, however large the barrier weights grow).
// ------------------------------------------------------------------------------------------
struct WsTri {
  float ia, ic, is, l31, l32;  // 1/a, 1/c, 1/Schur, L entries
};

__device__ __forceinline__ WsTri ws_ipm_block(const SmemW& s, const KParams& P, int t, int ntri,
                                              float sig) {
  const float* dd = s.y;  // z/s of row i of triple t at dd[i * ntri + t]
  const float d0 = dd[t], d1 = dd[ntri + t], d2 = dd[2 * ntri + t], d3 = dd[3 * ntri + t],
              d4 = dd[4 * ntri + t];
  const float mu = P.mu, mu2 = P.mu * P.mu;
  const float rx = s.Rt[3 * t] + sig, ry = s.Rt[3 * t + 1] + sig, rz = s.Rt[3 * t + 2] + sig;
  const float a = d1 + d2 + rx, c = d3 + d4 + ry;
  const float ia = 1.f / a, ic = 1.f / c;
  const float sch = d0 + rz + mu2 * (4.f * d1 * d2 + (d1 + d2) * rx) * ia +
                    mu2 * (4.f * d3 * d4 + (d3 + d4) * ry) * ic;
  return WsTri{ia, ic, 1.f / sch, -mu * (d1 - d2) * ia, -mu * (d3 - d4) * ic};
}

// v <- D_t^-1 v = L^-T diag(ia, ic, is) L^-1 v
__device__ __forceinline__ void ws_tri_solve(const WsTri& T, float& v0, float& v1, float& v2) {
  const float w2 = (v2 - T.l31 * v0 - T.l32 * v1) * T.is;
  const float w0 = v0 * T.ia, w1 = v1 * T.ic;
  v0 = w0 - T.l31 * w2;
  v1 = w1 - T.l32 * w2;
  v2 = w2;
}

// W = (Pw^-1 + sum_t E_t D_t^-1 E_t')^-1 in the ADMM basis (params 3t .. 3t+2 of triple t):
// E_t D_t^-1 E_t' = E0 E0' ia + E1 E1' ic + F F' is with F = E2 - l31 E0 - l32 E1.
__device__ __forceinline__ void ws_factor_ipm(SmemW& s, const KParams& P, f4 (&M)[CW::NTL],
                                              int ntri, float sig, const float* __restrict__ park_pw) {
  const int lane = opaque_lane();
  const int g = lane >> 4, c = lane & 15;
  const int N = P.N;
  const int nw = 6 * N;
  WSYNC();
  for (int e = lane; e < 36 * N; e += 64) {
    const int k = e / 36, ij = e % 36, i = ij / 6, j = ij % 6;
    float acc = 0.f;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      const int t = s.tri_of[4 * k + l];
      if (t < 0) continue;
      const WsTri T = ws_ipm_block(s, P, t, ntri, sig);
      const float* E = &s.Et[(3 * t) * 6];
      const float fi = E[12 + i] - T.l31 * E[i] - T.l32 * E[6 + i];
      const float fj = E[12 + j] - T.l31 * E[j] - T.l32 * E[6 + j];
      acc = fmaf(E[i] * E[j], T.ia, acc);
      acc = fmaf(E[6 + i] * E[6 + j], T.ic, acc);
      acc = fmaf(fi * fj, T.is, acc);
    }
    s.Sb[e] = acc;
  }
  park_load<kWN>(park_pw, M);
  WSYNC();
#pragma unroll
  for (int I = 0; I < CW::TT; ++I) {
#pragma unroll
    for (int J = (I > 0 ? I - 1 : 0); J <= I; ++J) {
      f4 m = M[tile_index(I, J)];
      const int col = 16 * J + c;
      const int kc = col / 6;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * I + 4 * g + q;
        const int kr = row / 6;
        if (row < nw && col < nw && kr == kc) m[q] += s.Sb[kc * 36 + (row - 6 * kr) * 6 + (col - 6 * kc)];
      }
      M[tile_index(I, J)] = m;
    }
  }
  WSYNC();
  invert_tiles<kWN>(s, M, nw);
}

// out = (P + sigma I + G' diag(z/s) G)^-1 in (ADMM basis; lane t owns triple t's three params)
__device__ __forceinline__ void ws_apply_ipm(SmemW& s, const KParams& P, const f4 (&M)[CW::NTL],
                                             int ntri, float sig, const float* in, float* out) {
  const int lane = opaque_lane();
  const int N = P.N;
  const int nw = 6 * N;
  WSYNC();
  WsTri T{0.f, 0.f, 0.f, 0.f, 0.f};
  if (lane < ntri) {
    T = ws_ipm_block(s, P, lane, ntri, sig);
    float v0 = in[3 * lane], v1 = in[3 * lane + 1], v2 = in[3 * lane + 2];
    ws_tri_solve(T, v0, v1, v2);
    out[3 * lane] = v0;
    out[3 * lane + 1] = v1;
    out[3 * lane + 2] = v2;
  }
  WSYNC();
  for (int w = lane; w < nw; w += 64) {
    const int k = w / 6, i = w % 6;
    const int p1 = s.off[k + 1];
    float acc = 0.f;
    for (int p = s.off[k]; p < p1; ++p) acc = fmaf(s.Et[6 * p + i], out[p], acc);
    s.tw[w] = acc;
  }
  symv<kWN>(s, M, nw, s.tw, s.zw);
  if (lane < ntri) {
    const int k = s.par[3 * lane];
    float cr[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < 6; ++i) acc = fmaf(s.Et[6 * (3 * lane + a) + i], s.zw[6 * k + i], acc);
      cr[a] = acc;
    }
    ws_tri_solve(T, cr[0], cr[1], cr[2]);
#pragma unroll
    for (int a = 0; a < 3; ++a) out[3 * lane + a] -= cr[a];
  }
  WSYNC();
}

// cmpc_wave.hip ipm_identify with the wrench-space Newton solves: leaves the face set in
// s.code, u in s.x and s.z, the multiplier y = G' z in s.y; clobbers M and the parked ADMM W.
// Returns false if a step went non-finite.
__device__ __forceinline__ bool ws_ipm_identify(SmemW& s, const KParams& P, f4 (&M)[CW::NTL],
                                                const float* __restrict__ park_pw,
                                                float* __restrict__ st, int n, int ntri) {
  const float mu = P.mu, fzm = P.fz_min, sig = P.sigma;
  n = uniform(n);
  ntri = uniform(ntri);
  float* dd = s.y;  // z / s of row i of triple t at dd[i * ntri + t] (5 ntri <= y and v)
  {
    const int l = opaque_lane();
    WSYNC();
    if (l < ntri) {
      s.x[3 * l] = 0.f;
      s.x[3 * l + 1] = 0.f;
      s.x[3 * l + 2] = 2.f * fzm;
    }
    float gu[5], zc[5], sl[5];
    ipm_rows(0.f, 0.f, 2.f * fzm, mu, fzm, gu);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      zc[i] = (l < ntri) ? 1.f : 0.f;
      sl[i] = (l < ntri) ? -gu[i] : 1.f;
    }
    ipm_st(st, 0, l, zc);
    ipm_st(st, 1, l, sl);
  }
  const float m_inv = 1.f / (5.f * (float)max(ntri, 1));
  for (int it = 0; it < kIpmIters; ++it) {
    {  // d = z / s, then the Newton matrix (needs only d)
      const int l = opaque_lane();
      ipm_sync();
      float zc[5], sl[5];
      ipm_ld(st, 0, l, zc);
      ipm_ld(st, 1, l, sl);
      WSYNC();
#pragma unroll
      for (int i = 0; i < 5; ++i)
        if (l < ntri) dd[i * ntri + l] = zc[i] / sl[i];
    }
    ws_factor_ipm(s, P, M, ntri, sig, park_pw);
    ws_gradient(s, P, n, s.x, s.g);  // grad f(u)
    float mu_c;
    {
      const int l = opaque_lane();
      float zc[5], sl[5];
      ipm_ld(st, 0, l, zc);
      ipm_ld(st, 1, l, sl);
      float sz = 0.f;
#pragma unroll
      for (int i = 0; i < 5; ++i) sz += sl[i] * zc[i];
      mu_c = uniformf(wave_sum(sz) * m_inv);
    }
    // predictor: rhs = -grad f (the slacks are exact, so the primal residual is zero)
    for (int p = opaque_lane(); p < n; p += 64) s.r[p] = -s.g[p];
    ws_apply_ipm(s, P, M, ntri, sig, s.r, s.dl);
    float smu;
    {
      const int l = opaque_lane();
      const bool own = l < ntri;
      float zc[5], sl[5], dsa[5], dza[5], gd[5];
      ipm_ld(st, 0, l, zc);
      ipm_ld(st, 1, l, sl);
      WSYNC();
      ipm_gdir(own ? s.dl[3 * l] : 0.f, own ? s.dl[3 * l + 1] : 0.f, own ? s.dl[3 * l + 2] : 0.f,
               mu, gd);
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        dsa[i] = own ? -gd[i] : 0.f;
        dza[i] = own ? -zc[i] - zc[i] * dsa[i] / sl[i] : 0.f;
      }
      const float apa = wave_min(ipm_maxstep(sl, dsa)), ada = wave_min(ipm_maxstep(zc, dza));
      float sza = 0.f;
#pragma unroll
      for (int i = 0; i < 5; ++i) sza += (sl[i] + apa * dsa[i]) * (zc[i] + ada * dza[i]);
      const float mu_a = wave_sum(own ? sza : 0.f) * m_inv;
      const float rat = mu_a / fmaxf(mu_c, 1e-30f);
      smu = uniformf(rat * rat * rat * mu_c);
      float wv[5];
#pragma unroll
      for (int i = 0; i < 5; ++i) wv[i] = (dsa[i] * dza[i] - smu) / sl[i];
      if (own) {
        s.r[3 * l] = -s.g[3 * l] + (wv[1] - wv[2]);
        s.r[3 * l + 1] = -s.g[3 * l + 1] + (wv[3] - wv[4]);
        s.r[3 * l + 2] = -s.g[3 * l + 2] - wv[0] - mu * (wv[1] + wv[2] + wv[3] + wv[4]);
      }
      ipm_st(st, 2, l, dsa);
      ipm_st(st, 3, l, dza);
    }
    ws_apply_ipm(s, P, M, ntri, sig, s.r, s.dl);
    bool stop;
    {
      const int l = opaque_lane();
      const bool own = l < ntri;
      ipm_sync();
      float zc[5], sl[5], dsa[5], dza[5], du[3], ds[5], dz[5], gd[5];
      ipm_ld(st, 0, l, zc);
      ipm_ld(st, 1, l, sl);
      ipm_ld(st, 2, l, dsa);
      ipm_ld(st, 3, l, dza);
      WSYNC();
#pragma unroll
      for (int a = 0; a < 3; ++a) du[a] = own ? s.dl[3 * l + a] : 0.f;
      ipm_gdir(du[0], du[1], du[2], mu, gd);
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        ds[i] = own ? -gd[i] : 0.f;
        const float rc = sl[i] * zc[i] + dsa[i] * dza[i] - smu;
        dz[i] = own ? (-zc[i] * ds[i] - rc) / sl[i] : 0.f;
      }
      const float ap = 0.99f * wave_min(ipm_maxstep(sl, ds)), ad = 0.99f * wave_min(ipm_maxstep(zc, dz));
      stop = it > 0 && ap < 0.1f;  // a collapsed step: fp32 running out, keep the last iterate
      if (!stop) {
        if (own) {
#pragma unroll
          for (int a = 0; a < 3; ++a) s.x[3 * l + a] += ap * du[a];
        }
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          zc[i] += ad * dz[i];
          sl[i] += ap * ds[i];
        }
        ipm_st(st, 0, l, zc);
        ipm_st(st, 1, l, sl);
      }
    }
    if (stop) break;  // (uniform)
  }
  const int l = opaque_lane();
  ipm_sync();
  float zc[5], sl[5];
  ipm_ld(st, 0, l, zc);
  ipm_ld(st, 1, l, sl);
  WSYNC();
  bool bad = false;
  if (l < ntri) {
    const float ux = s.x[3 * l], uy = s.x[3 * l + 1], uz = s.x[3 * l + 2];
    bool act[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) act[i] = zc[i] > sl[i];
    int code = act[0] ? 1 : 0;
    if (act[1] && (!act[2] || zc[1] >= zc[2])) code |= 2;
    else if (act[2]) code |= 4;
    if (act[3] && (!act[4] || zc[3] >= zc[4])) code |= 8;
    else if (act[4]) code |= 16;
    s.code[l] = code;
    s.z[3 * l] = ux;
    s.z[3 * l + 1] = uy;
    s.z[3 * l + 2] = uz;
  }
  WSYNC();
  if (l < ntri) {  // (y holds d until here)
    s.y[3 * l] = zc[1] - zc[2];
    s.y[3 * l + 1] = zc[3] - zc[4];
    s.y[3 * l + 2] = -zc[0] - mu * (zc[1] + zc[2] + zc[3] + zc[4]);
    bad = !(isfinite(s.x[3 * l]) && isfinite(s.x[3 * l + 1]) && isfinite(s.x[3 * l + 2]) &&
            isfinite(s.y[3 * l]) && isfinite(s.y[3 * l + 1]) && isfinite(s.y[3 * l + 2]));
  }
  WSYNC();
  return __any(bad) == 0;
}

// the ADMM state (x, z, y) kept aside in the slab while the interior-point steps run
__device__ __forceinline__ void ws_ipm_save(SmemW& s, float* __restrict__ keep, int n) {
  WSYNC();
  for (int p = opaque_lane(); p < n; p += 64) {
    keep[p] = s.x[p];
    keep[kMaxP + p] = s.z[p];
    keep[2 * kMaxP + p] = s.y[p];
  }
}
__device__ __forceinline__ void ws_ipm_restore(SmemW& s, const float* __restrict__ keep, int n) {
  asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc1" ::: "memory");
  for (int p = opaque_lane(); p < n; p += 64) {
    const float xv = keep[p], zv = keep[kMaxP + p], yv = keep[2 * kMaxP + p];
    s.x[p] = xv;
    s.z[p] = zv;
    s.y[p] = yv;
  }
  WSYNC();
}

// Where an instance whose Bd is not of the centroidal form goes: the n-space kernels' bin of its
// free-force count (cmpc_wave.hip bin_kernel), drained after this kernel.
struct Fallback {
  int* counts;   // counts[kNumBins] of the n-space bins
  int* lists;    // lists[bin * stride + i]
  int64_t stride;
};

// ------------------------------------------------------------------------------------------
// one QP instance on one wave, wrench-space factorization (control flow as cmpc_wave.hip
// solve_instance: ADMM, polish sessions with repairs and the anti-cycling memories, warm start)
// ------------------------------------------------------------------------------------------
template <bool IPM>
__device__ __forceinline__ void ws_solve_instance(SmemW& s, const KParams& P, int64_t b,
                                                  const Inputs& in, const Outputs& out,
                                                  float* __restrict__ park_pw,
                                                  float* __restrict__ park_w, const Fallback& fb) {
  f4 M[CW::NTL];
  const int lane = opaque_lane();
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

  WSYNC();
  {  // one round of global loads: A, r_0..r_N (= x0, xref), gd; staged in LDS (E, L are free)
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
    // r_0 .. r_N at E[0 .. 12N) + L[0 .. 12), gd at L[12 .. 24)
    float* rs = s.E;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = lane + 64 * i;
      if (e < 12 * (N + 1)) {
        if (e < kMaxP) rs[e] = rv[i];
        else s.L[e - kMaxP] = rv[i];
      }
    }
    if (lane < 12) s.L[12 + lane] = gv;
  }
  const bool stc = (lane < 4 * N) ? (ctb[(lane & 3) * N + (lane >> 2)] != 0) : false;
  const int pos = wave_excl_scan4(stc ? 1 : 0);
  const int ntri = wave_total4(stc ? 1 : 0);
  if (stc) s.tri[pos] = lane;
  if (lane < 4 * N) s.tri_of[lane] = stc ? pos : -1;
  WSYNC();
  for (int o = lane; o < NP; o += 64) {  // d_k = A r_k + gd - r_{k+1}, r_0 = x0
    const int k = o / 12, r = o % 12;
    auto rr = [&](int e) { return (e < kMaxP) ? s.E[e] : s.L[e - kMaxP]; };
    float acc = s.L[12 + r] - rr(12 * (k + 1) + r);
#pragma unroll
    for (int j = 0; j < 12; ++j) acc = fmaf(s.A[r * 12 + j], rr(12 * k + j), acc);
    s.D[o] = acc;
  }
  ws_setup_mb(s);
  if (!ws_admm_basis(s, P, Bg, ntri, true)) {
    // not of the centroidal form: the n-space kernels solve it (their bin of its free forces)
    if (lane == 0) {
      const int nf = 3 * ntri;
      int q = kNumBins - 1;
      for (int i = 0; i < kNumBins; ++i)
        if (nf <= kBinCap[i]) { q = i; break; }
      const int at = atomicAdd(&fb.counts[q], 1);
      fb.lists[(int64_t)q * fb.stride + at] = (int)b;
    }
    return;
  }
  const int n = 3 * ntri;
  float rho = P.rho0;
  s.pcode[lane] = -1;
  if (in.w_init == nullptr && in.y_init == nullptr && in.lam_init == nullptr) {
    for (int p = lane; p < n; p += 64) { s.x[p] = 0.f; s.z[p] = 0.f; s.y[p] = 0.f; }
  } else if (lane < ntri) {
    // warm start (centroidal_mpc.py:91-95), as cmpc_wave.hip solve_instance
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
      const float* li = in.lam_init + b * (int64_t)(52 * N);
      const float* lf = li + 24 * N + NP + 16 * (kl >> 2) + 4 * (kl & 3);
      const float* lx = li + NP + fo;
      const float f0 = lf[0], f1 = lf[1], f2 = lf[2], f3 = lf[3];
      yv[0] = f0 - f1 + lx[0];
      yv[1] = f2 - f3 + lx[1];
      yv[2] = -P.mu * (f0 + f1 + f2 + f3) + lx[2];
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      if (!isfinite(u[a])) u[a] = 0.f;
      if (!isfinite(yv[a])) yv[a] = 0.f;
    }
    float pv[3], qv[3];
    project(u[0], u[1], u[2], P.mu, P.fz_min, pv[0], pv[1], pv[2]);
    int code;
    if (in.y_init || in.lam_init) {
      const float ir = 1.f / rho;
      code = project(pv[0] + yv[0] * ir, pv[1] + yv[1] * ir, pv[2] + yv[2] * ir, P.mu, P.fz_min,
                     qv[0], qv[1], qv[2]);
    } else {
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
  if (n > 0) {  // Pw^-1 of this instance, parked for every factorization
    CMPC_T0(t_pw);
    ws_condense_pw(s, P, M);
    park_store<kWN>(park_pw, M);
    CMPC_ACC(0, t_pw);
  }
  CMPC_ACC(6, t_inst);

  int status = -2, iters = 0;
#ifdef CMPC_DIAG_COUNTS
  int dg_fact = 0, dg_pol = 0;
  const unsigned long long dg_t0 = __builtin_amdgcn_s_memtime();
#endif
#ifdef CMPC_DIAG_TIMES
  const unsigned long long dt_t0 = __builtin_amdgcn_s_memrealtime();
#endif
  bool polished = false;
  float rp = 0.f, rd = 0.f, np_ = 0.f, nd = 0.f;
  int stable = 0;
  bool refactor = n > 0;
  bool in_polish = false;
  int nact = n;
  float shift = uniformf(P.sigma + rho);
  int it = 0;
  int repairs_left = 0;
  bool parked = false;
  int nfail = 0;
  int ntried = 0;
  bool seen_start = false;
  int last_pol = 0;
  bool ipm_done = false;     // the interior-point fallback ran (at most once per instance)
  int nsfail = 0;            // failed sessions, remembered starts included
  int nfact = 0;             // factorizations so far
  bool ipm_session = false;  // the current polish session started from its face set
  float* keep = park_w + CW::NTL * 256;  // ADMM state during the interior-point steps
  const float alpha = P.alpha;
  if (n == 0) status = 1;
  if (n > 0 && in.w_init != nullptr) {  // warm active set straight to the polish
    WSYNC();
    if (lane < ntri) s.code[lane] = s.pcode[lane];
    repairs_left = ws_session_start(s, P, ntri, nfail, ntried, seen_start);
    nact = ws_polish_setup(s, P, Bg, ntri);
    shift = P.sigma;
    in_polish = true;
  }
  while (n > 0) {
    if (refactor) {
      CMPC_CNT(8, 1);
      ++nfact;
#ifdef CMPC_DIAG_COUNTS
      ++dg_fact;
#endif
      CMPC_T0(t_i);
      ws_factor(s, P, M, nact, uniformf(shift), park_pw);
      CMPC_ACC(1, t_i);
      refactor = false;
    }
    if (in_polish) {
      CMPC_T0(t_pol);
      float step = 3.0e38f, prev = 3.0e38f;
      for (int q = 0; q < CMPC_REFINE_N + kRefineExtra; ++q) {
        ws_gradient(s, P, nact, s.v, s.g);
        ws_apply(s, P, M, nact, shift, s.g, s.dl);
        float m = 0.f, mv = 1.f;
        for (int p = lane; p < nact; p += 64) {
          const float vn = s.v[p] - s.dl[p];
          s.v[p] = vn;
          m = fmaxf(m, fabsf(s.dl[p]));
          mv = fmaxf(mv, fabsf(vn));
        }
        step = wave_max(m);
        if (q + 1 >= CMPC_REFINE_N &&
            (step <= P.polish_tol * wave_max(mv) || step > kRefineRate * prev))
          break;
        prev = step;
      }
      ws_gradient(s, P, nact, s.v, s.g);  // E, L, Mu at the final point
      bool changed = false, loose = false;
      const bool ok = ws_polish_check(s, P, Bg, ntri, step, changed, loose);
      CMPC_ACC(4, t_pol);
      if (ok) {
        polished = true;
        status = 1;
        break;
      }
      if (repairs_left > 0 && changed && !ws_tried_before(s, ntri, ntried)) {
        --repairs_left;
        if (lane < ntri) {
          s.code[lane] = s.tcnt[lane];
          if (ntried < kTryMem) s.tpat[ntried][lane] = (uint8_t)s.tcnt[lane];
        }
        if (ntried < kTryMem) ++ntried;
        nact = ws_polish_setup(s, P, Bg, ntri);
        shift = P.sigma;
        refactor = true;
        continue;
      }
      if (loose) {
        const int l = opaque_lane();
        WSYNC();
        if (l < ntri) {
#pragma unroll
          for (int a = 0; a < 3; ++a) s.x[3 * l + a] = s.dl[3 * l + a];
        }
        polished = true;
        status = 1;
        break;
      }
      ++nsfail;
      if (!seen_start) {
        const int l = opaque_lane();
        if (l < ntri) s.fpat[nfail % kFailMem][l] = s.tpat[0][l];
        ++nfail;
      }
      ws_admm_basis(s, P, Bg, ntri, false);
      in_polish = false;
      nact = n;
      shift = uniformf(P.sigma + rho);
      if (ipm_session) {  // ADMM resumes from where it was before the interior-point steps
        ipm_session = false;
        ws_ipm_restore(s, keep, n);
      }
      if constexpr (IPM && kIpmAfter > 0) {
        if (!ipm_done && P.ipm_facts > 0 && nsfail >= kIpmAfter && nfact >= P.ipm_facts) {
          // a hard instance: identify the face set by interior-point steps, then polish it with
          // the full repair budget (ADMM resumes where it was if that session fails too)
          ipm_done = true;
#ifdef CMPC_DIAG_COUNTS
          dg_pol += 100;
#endif
          ws_ipm_save(s, keep, n);
          const bool ok_ipm = ws_ipm_identify(s, P, M, park_pw, keep + 3 * kMaxP, n, ntri);
          parked = false;
          if (!ok_ipm) {  // (non-finite steps) back to ADMM as it was, refactoring first
            ws_ipm_restore(s, keep, n);
            refactor = true;
            continue;
          }
          ipm_session = true;
          ws_session_start(s, P, ntri, nfail, ntried, seen_start);
          seen_start = false;
          repairs_left = P.polish_repairs;
          nact = ws_polish_setup(s, P, Bg, ntri);
          shift = P.sigma;
          refactor = true;
          in_polish = true;
          last_pol = it;
          stable = -(P.polish_stable << min(nfail, kBackoffCap));
          continue;
        }
      }
      if (parked) {
        park_load<kWN>(park_w, M);
      } else {
        refactor = true;
        continue;
      }
    }
    if (it >= P.max_iter) break;
    ++it;
    iters = it;
    // ---- one ADMM iteration ----
    ws_gradient(s, P, n, s.x, s.g);
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
    ws_apply(s, P, M, n, shift, s.r, s.dl);
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
    stable = (__any(changed) != 0) ? 0 : stable + 1;
    bool do_pol = false;
    const int backoff = P.polish_stable << min(nfail, kBackoffCap);
    if (stable >= P.polish_stable && !last && it - last_pol >= backoff &&
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
      // park the ADMM W where a failed session will restore it (not when a refactor is pending,
      // not in the first session: most instances pass it, the few that fail refactor once)
      parked = !refactor && nfail > 0;
      if (parked) park_store<kWN>(park_w, M);
      repairs_left = ws_session_start(s, P, ntri, nfail, ntried, seen_start);
      nact = ws_polish_setup(s, P, Bg, ntri);
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
    ws_gradient(s, P, n, s.z, s.g);  // E at u = z (the pure rollout when every leg swings)
  }
  CMPC_T0(t_out);
  WSYNC();
  float* wb = out.w + b * (int64_t)(24 * N);
  const float* uf = polished ? s.x : s.z;
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
  if (out.y) {  // dual at the returned forces (force layout, zero on swing legs)
    if (polished && n > 0) {
      ws_admm_basis(s, P, Bg, ntri, false);
      ws_gradient(s, P, n, s.x, s.g);
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
  if (out.lam) {  // the reference's multipliers at the returned point (cmpc_wave.hip)
    WSYNC();
    float* lb = out.lam + b * (int64_t)(52 * N);
    for (int o = lane; o < NP; o += 64) {
      lb[o] = 0.f;
      lb[24 * N + o] = -s.L[o];
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
      if (t < 0) {
#pragma unroll
        for (int a = 0; a < 3; ++a) lxv[a] = -sv[a];
      } else {
        int code;
        if (polished) {
          code = s.code[t];
        } else {
          const float tz = 1e-5f * fmaxf(u[2], 1.f), lim = P.mu * u[2] - 1e-5f * fmaxf(u[2], 1.f);
          code = (u[2] <= P.fz_min + tz) ? 1 : 0;
          code |= (u[0] >= lim) ? 2 : (u[0] <= -lim) ? 4 : 0;
          code |= (u[1] >= lim) ? 8 : (u[1] <= -lim) ? 16 : 0;
        }
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
#if defined(CMPC_DIAG_COUNTS)
    out.status[b] = (int)((__builtin_amdgcn_s_memtime() - dg_t0) >> 4);
    out.iters[b] = iters + 1000 * dg_pol + 1000000 * dg_fact;
#elif defined(CMPC_DIAG_TIMES)
    out.status[b] = (int)(dt_t0 & 0x7fffffffull);
    out.iters[b] = (int)(__builtin_amdgcn_s_memrealtime() - dt_t0);
#else
    out.status[b] = status;
    out.iters[b] = iters;
#endif
  }
  CMPC_CNT(11, iters);
  CMPC_ACC(15, t_out);
  CMPC_ACC(5, t_inst);
}

// Large batches: every instance through the wrench-space path, one wave per QP, two waves per
// SIMD, one persistent kernel on the caller's stream; the queue is the batch in index order.
template <bool IPM>
__global__ void __launch_bounds__(64, 2)
    solve_ws_kernel(KParams P, Inputs in, Outputs out, int64_t B, int* __restrict__ head,
                    Fallback fb, float* __restrict__ work) {
  __shared__ SmemW s;
  float* park_pw = work + (size_t)blockIdx.x * kWsSlab;
  float* park_w = park_pw + CW::NTL * 256;
  const int lane = opaque_lane();
#ifdef CMPC_STAMPS
  if (lane < 32) s.st[lane] = 0;
#endif
  if (lane < 12) {
    s.Q2[lane] = P.Q2[lane];
    s.R2[lane] = P.R2[lane];
  }
  for (;;) {
    int idx = 0;
    if (lane == 0) idx = atomicAdd(head, 1);
    idx = __builtin_amdgcn_readfirstlane(idx);
    if (idx >= B) break;
    ws_solve_instance<IPM>(s, P, (int64_t)idx, in, out, park_pw, park_w, fb);
  }
#ifdef CMPC_STAMPS
  WSYNC();
  if (lane < 32) atomicAdd(&g_stamps[lane], s.st[lane]);
#endif
}
