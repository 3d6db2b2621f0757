// cmpc_riccati.hip -- the ADMM / polish matrix (H + shift I)^-1 of one instance as a Riccati
// factorization of the horizon instead of an explicit inverse (included by cmpc_wave.hip).
//
// H is the condensed Hessian of the reference QP in the current param basis (centroidal_mpc.py:
// 178-201, 287-303: min sum_k e_{k+1}' (Q2/2) e_{k+1} + v' (Rt/2) v, e_{k+1} = A e_k + B~_k v_k).
// Solving (H + shift I) v = r is the LQR problem with stage weight Rt + shift and a linear term
// r on the params, so the backward Riccati recursion factors it in O(N 12^3):
//     W = P_{k+1};  T = W B~;  S = B~' T + diag(Rt_k + shift);  G = T' A;  K = S^-1 G
//     Phi = A - B~ K;  P_k = Q2 + A' W A - G' K
// and an apply is a backward and a forward sweep of 12-vectors:
//     p_k = Phi' p_{k+1} + K' r_k,  b_k = B~' p_{k+1} - r_k,  q_k = S^-1 b_k      (k = N-1 .. 0)
//     e_{k+1} = Phi e_k - B~ q_k,   v_k = -K e_k - q_k                           (k = 0 .. N-1)
// The condensation + block sweep cost ~1,300 MFMAs at n = 120 (the explicit inverse of the
// condensed matrix); the recursion ~30 per step, whatever the number of free forces.
//
// Layout.  A 12 x 12 block (states or a step's params) lives in ONE 16 x 16 MFMA tile in the
// "D layout": lane (g, c) holds rows 3g..3g+2 (registers q = 0..2) of column rho(c), where
// rho(c) = 3 (c >> 2) + (c & 3) for (c & 3) < 3 (lanes c = 3, 7, 11, 15 are padding).  Then an
// accumulator is directly the B operand of the next v_mfma_f32_16x16x4_f32 (K = 12: three
// MFMAs, slice q = state 3g + q), the A operand of a symmetric block is its own D layout, and
// the A operand of X' is the D layout of X -- every product of the recursion chains through
// registers.  A step's params are numbered in the same 12-slot layout (padding params carry
// zero columns and a unit diagonal).  Vectors are either R (lane (g, *) register q holds entry
// 3g + q) or C (lane (*, c) holds entry rho(c)); a block in D layout maps R -> C as Y' x (sum
// over the lane groups: two permlane swaps) and C -> R as Y x (sum over the 16 lanes of a row:
// DPP).  The sweeps alternate R and C every step, so the factorization stores per step k the
// forms its parity needs: Y_k = Phi_k (even k) or Phi_k' (odd), Z_k = K_k (even) or K_k'
// (odd), and S_k^-1 -- 9 registers per step, 144 for N = 16.

__device__ __forceinline__ int ric_rho(int c) { return ((c & 3) < 3) ? 3 * (c >> 2) + (c & 3) : -1; }

// the value of v at lane (b, c) in every lane (g, c) (b uniform): lane-group broadcast with the
// gfx950 permlane swaps
__device__ __forceinline__ float rowgroup_bcast(float v, int b, int g) {
  const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  const float p16 = __int_as_float((g & 1) ? r16[0] : r16[1]);  // lane (g ^ 1, c)
  const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  const float p32 = __int_as_float((g & 2) ? r32[0] : r32[1]);  // lane (g ^ 2, c)
  const auto r48 = __builtin_amdgcn_permlane32_swap(__float_as_int(p16), __float_as_int(p16), false, false);
  const float p48 = __int_as_float((g & 2) ? r48[0] : r48[1]);  // lane (g ^ 3, c)
  const int x = g ^ b;
  return x == 0 ? v : (x == 1 ? p16 : (x == 2 ? p32 : p48));
}

struct RicRegs {
  float y[kMaxN][3];   // Phi_k (k even) / Phi_k' (k odd), D layout
  float z[kMaxN][3];   // K_k (k even) / K_k' (k odd)
  float si[kMaxN][3];  // S_k^-1
};

// S (D layout, registers 0..2; m real params, the rest padding with a unit diagonal) ->
// S^-1, by the symmetric sweep three pivots at a time (the pivot rows of block b are lane group
// b's registers): S <- S - C^ D^-1 C^' with C^ = the pivot columns, the pivot block minus I,
// then -2 on the pivot diagonal; after every block -S^-1.  D = L diag(d) L' is factored
// redundantly per lane and the rank-3 update is ONE MFMA (A = -C^ L^-T, B = diag(1/d) (C^ L^-T)').
template <int bk>
__device__ __forceinline__ void ric_tile_block(f4& X, int nb, int g, int rc) {
  if (bk < nb) {  // uniform
    float pv[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) pv[j] = rowgroup_bcast(X[j], bk, g);  // X[3bk + j][rc]
    constexpr int base = 20 * bk;  // lane (bk, 4bk + j) holds X[3bk + i][3bk + j] in register i
    const float d00 = readlane_f(X[0], base), d01 = readlane_f(X[0], base + 1),
                d02 = readlane_f(X[0], base + 2), d11 = readlane_f(X[1], base + 1),
                d12 = readlane_f(X[1], base + 2), d22 = readlane_f(X[2], base + 2);
    const float i0 = __builtin_amdgcn_rcpf(d00);
    const float l10 = d01 * i0, l20 = d02 * i0;
    const float i1 = __builtin_amdgcn_rcpf(d11 - l10 * d01);
    const float u21 = d12 - l20 * d01;
    const float l21 = u21 * i1;
    const float i2 = __builtin_amdgcn_rcpf(d22 - l20 * d02 - l21 * u21);
    float ph[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) ph[j] = pv[j] - ((rc == 3 * bk + j) ? 1.f : 0.f);
    // row g of L^-1 against the pivot row: this lane's K index is pivot g of the block
    float yg;
    if (g == 0) yg = ph[0];
    else if (g == 1) yg = fmaf(-l10, ph[0], ph[1]);
    else if (g == 2) yg = fmaf(fmaf(l10, l21, -l20), ph[0], fmaf(-l21, ph[1], ph[2]));
    else yg = 0.f;
    const float ig = (g == 0) ? i0 : ((g == 1) ? i1 : i2);
    X = mfma4(-yg, yg * ig, X);
#pragma unroll
    for (int q = 0; q < 3; ++q) X[q] -= (g == bk && 3 * g + q == rc) ? 2.f : 0.f;
  }
  if constexpr (bk < 3) ric_tile_block<bk + 1>(X, nb, g, rc);
}

__device__ __forceinline__ f4 ric_tile_inverse(f4 X, int m, int g, int rc) {
  const int nb = uniform((m + 2) / 3);
  ric_tile_block<0>(X, nb, g, rc);
#pragma unroll
  for (int q = 0; q < 3; ++q) X[q] = (3 * g + q < 3 * nb) ? -X[q] : X[q];
  return X;
}

// one step k of the backward recursion (compile-time k: the factors stay in registers)
template <int NC, int k>
__device__ __forceinline__ void ric_factor_step(Smem<NC>& s, RicRegs& F, f4& W, int N, float shift,
                                                const float (&adB)[3], const float (&adA)[3],
                                                const float (&q2d)[3], int g, int rc) {
  {
    const bool act = k < N;  // uniform (a step past the horizon: m = 0, W kept)
    const int p0 = act ? s.off[k] : 0, m = act ? s.off[k + 1] - p0 : 0;
    const bool cv = rc >= 0 && rc < m;
    float bq[3], ba[3];  // B~[3g+q][rc] (D layout of B~), B~[rc][3g+q] (of B~')
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int j = 3 * g + q;
      bq[q] = cv ? s.Bt[(p0 + rc) * kBS + j] : 0.f;
      ba[q] = (rc >= 0 && j < m) ? s.Bt[(p0 + j) * kBS + rc] : 0.f;
    }
    f4 T = {0.f, 0.f, 0.f, 0.f}, U0 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 3; ++q) T = mfma4(W[q], bq[q], T);     // W B~
#pragma unroll
    for (int q = 0; q < 3; ++q) U0 = mfma4(W[q], adB[q], U0);  // W A
    f4 S = {0.f, 0.f, 0.f, 0.f}, V0 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 3; ++q) S = mfma4(bq[q], T[q], S);     // B~' W B~
#pragma unroll
    for (int q = 0; q < 3; ++q) V0 = mfma4(adB[q], U0[q], V0); // A' W A
    const float rt = cv ? s.Rt[p0 + rc] + shift : 1.f;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      if (3 * g + q == rc) S[q] = cv ? S[q] + rt : 1.f;
    }
    const f4 Si = ric_tile_inverse(S, m, g, rc);
    f4 G = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 3; ++q) G = mfma4(T[q], adB[q], G);    // T' A = B~' W A
    f4 K = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 3; ++q) K = mfma4(Si[q], G[q], K);     // S^-1 G
    f4 GK = {0.f, 0.f, 0.f, 0.f}, BK = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 3; ++q) GK = mfma4(G[q], K[q], GK);    // G' K
#pragma unroll
    for (int q = 0; q < 3; ++q) BK = mfma4(ba[q], K[q], BK);   // B~ K
#pragma unroll
    for (int q = 0; q < 3; ++q) F.si[k][q] = Si[q];
    if constexpr ((k & 1) == 0) {
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        F.y[k][q] = adB[q] - BK[q];  // Phi
        F.z[k][q] = K[q];
      }
    } else {
      f4 Kt = {0.f, 0.f, 0.f, 0.f}, KB = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 3; ++q) Kt = mfma4(G[q], Si[q], Kt);   // K' = G' S^-1
#pragma unroll
      for (int q = 0; q < 3; ++q) KB = mfma4(K[q], ba[q], KB);   // K' B~'
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        F.y[k][q] = adA[q] - KB[q];  // Phi'
        F.z[k][q] = Kt[q];
      }
    }
    if constexpr (k > 0) {
#pragma unroll
      for (int q = 0; q < 3; ++q) W[q] = act ? V0[q] - GK[q] + q2d[q] : W[q];
    }
  }
  if constexpr (k > 0) ric_factor_step<NC, k - 1>(s, F, W, N, shift, adB, adA, q2d, g, rc);
}

// Backward Riccati recursion of (H + shift I) in the param basis of s (Bt, Rt, off; the first
// n params); the step matrix A and Q2 from LDS.
template <int NC>
__device__ __forceinline__ void ric_factor(Smem<NC>& s, const KParams& P, RicRegs& F, int n,
                                           float shift) {
  const int lane = opaque_lane();
  const int g = lane >> 4, c = lane & 15;
  const int rc = ric_rho(c);
  WSYNC();
  float adB[3], adA[3], q2d[3];  // A[3g+q][rc] (D layout of A), A[rc][3g+q] (of A'), Q2 diagonal
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int r = 3 * g + q;
    adB[q] = (rc >= 0) ? s.A[r * 12 + rc] : 0.f;
    adA[q] = (rc >= 0) ? s.A[rc * 12 + r] : 0.f;
    q2d[q] = (rc == r) ? s.Q2[r] : 0.f;
  }
  f4 W = {q2d[0], q2d[1], q2d[2], 0.f};  // P_N = Q2 (the stage weight of e_N)
  ric_factor_step<NC, kMaxN - 1>(s, F, W, uniform(P.N), shift, adB, adA, q2d, g, rc);
}

// backward sweep step k: p_k = Phi_k' p_{k+1} + K_k' r_k; q_k = S_k^-1 (B~_k' p_{k+1} - r_k)
// -> qv.  The step's loads do not depend on the chain and no step is a branch of its own (a
// step past the horizon has m = 0 and keeps p), so the compiler can issue them early.
template <int NC, int k>
__device__ __forceinline__ void ric_bwd(Smem<NC>& s, int N, const RicRegs& F,
                                        const float* __restrict__ in, float* __restrict__ qv,
                                        float& pC, float (&pR)[3], int g, int c, int rc) {
  const bool act = k < N;  // uniform
  const int p0 = act ? s.off[k] : 0, m = act ? s.off[k + 1] - p0 : 0;
  const bool cv = rc >= 0 && rc < m;
  float rR[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) rR[q] = (3 * g + q < m) ? in[p0 + 3 * g + q] : 0.f;
  const float rC = cv ? in[p0 + rc] : 0.f;
  if constexpr ((k & 1) == 0) {  // p_{k+1} R -> p_k C
    float bq[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) bq[q] = cv ? s.Bt[(p0 + rc) * kBS + 3 * g + q] : 0.f;
    float t = 0.f, tb = 0.f;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      t = fmaf(F.y[k][q], pR[q], fmaf(F.z[k][q], rR[q], t));
      tb = fmaf(bq[q], pR[q], tb);
    }
    const float bC = col4_sum(tb) - rC;
    const float pn = col4_sum(t);
    pC = act ? pn : pC;
    float qR[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) qR[q] = row16_sum(F.si[k][q] * bC);
    if (c == 0) {
#pragma unroll
      for (int q = 0; q < 3; ++q)
        if (3 * g + q < m) qv[p0 + 3 * g + q] = qR[q];
    }
  } else {  // p_{k+1} C -> p_k R
    float ba[3];
#pragma unroll
    for (int q = 0; q < 3; ++q)
      ba[q] = (rc >= 0 && 3 * g + q < m) ? s.Bt[(p0 + 3 * g + q) * kBS + rc] : 0.f;
    float bR[3], pn[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      pn[q] = row16_sum(fmaf(F.y[k][q], pC, F.z[k][q] * rC));
      bR[q] = row16_sum(ba[q] * pC) - rR[q];
    }
    float tq = 0.f;
#pragma unroll
    for (int q = 0; q < 3; ++q) tq = fmaf(F.si[k][q], bR[q], tq);
    const float qC = col4_sum(tq);
    if (g == 0 && cv) qv[p0 + rc] = qC;
#pragma unroll
    for (int q = 0; q < 3; ++q) pR[q] = act ? pn[q] : pR[q];
  }
  if constexpr (k > 0) ric_bwd<NC, k - 1>(s, N, F, in, qv, pC, pR, g, c, rc);
}

// forward sweep step k: e_{k+1} = Phi_k e_k - B~_k q_k,  v_k = -K_k e_k - q_k -> vv
template <int NC, int k>
__device__ __forceinline__ void ric_fwd(Smem<NC>& s, int N, const RicRegs& F,
                                        const float* __restrict__ qv, float* __restrict__ vv,
                                        float& eC, float (&eR)[3], int g, int c, int rc) {
  const bool act = k < N;  // uniform
  const int p0 = act ? s.off[k] : 0, m = act ? s.off[k + 1] - p0 : 0;
  const bool cv = rc >= 0 && rc < m;
  float qR[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) qR[q] = (3 * g + q < m) ? qv[p0 + 3 * g + q] : 0.f;
  const float qC = cv ? qv[p0 + rc] : 0.f;
  if constexpr ((k & 1) == 0) {  // e_k C -> e_{k+1} R
    float bq[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) bq[q] = cv ? s.Bt[(p0 + rc) * kBS + 3 * g + q] : 0.f;
    float en[3], vR[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      en[q] = row16_sum(fmaf(F.y[k][q], eC, -bq[q] * qC));
      vR[q] = -row16_sum(F.z[k][q] * eC) - qR[q];
    }
    if (c == 0) {
#pragma unroll
      for (int q = 0; q < 3; ++q)
        if (3 * g + q < m) vv[p0 + 3 * g + q] = vR[q];
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) eR[q] = act ? en[q] : eR[q];
  } else {  // e_k R -> e_{k+1} C
    float ba[3];
#pragma unroll
    for (int q = 0; q < 3; ++q)
      ba[q] = (rc >= 0 && 3 * g + q < m) ? s.Bt[(p0 + 3 * g + q) * kBS + rc] : 0.f;
    float te = 0.f, tk = 0.f;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      te = fmaf(F.y[k][q], eR[q], fmaf(-ba[q], qR[q], te));
      tk = fmaf(F.z[k][q], eR[q], tk);
    }
    const float vC = -col4_sum(tk) - qC;
    const float en = col4_sum(te);
    eC = act ? en : eC;
    if (g == 0 && cv) vv[p0 + rc] = vC;
  }
  if constexpr (k + 1 < kMaxN) ric_fwd<NC, k + 1>(s, N, F, qv, vv, eC, eR, g, c, rc);
}

// out = (H + shift I)^-1 in over the first n params (out is zero beyond n).  in must not alias
// out and is CLOBBERED (the forward sweep writes v there, then v is copied to out: the two
// sweeps read one buffer and write the other, so their loads issue early).
template <int NC>
__device__ __forceinline__ void ric_apply(Smem<NC>& s, int N, const RicRegs& F, int n,
                                          float* __restrict__ in, float* __restrict__ out) {
  CMPC_T0(t_sv);
  const int lane = opaque_lane();
  const int g = lane >> 4, c = lane & 15;
  const int rc = ric_rho(c);
  n = uniform(n);
  N = uniform(N);
  WSYNC();
  float pC = 0.f, pR[3] = {0.f, 0.f, 0.f};  // p_N = 0
  ric_bwd<NC, kMaxN - 1>(s, N, F, in, out, pC, pR, g, c, rc);   // q -> out
  WSYNC();
  float eC = 0.f, eR[3] = {0.f, 0.f, 0.f};  // e_0 = 0
  ric_fwd<NC, 0>(s, N, F, out, in, eC, eR, g, c, rc);           // v -> in
  WSYNC();
  for (int p = lane; p < NC; p += 64) out[p] = (p < n) ? in[p] : 0.f;
  WSYNC();
  CMPC_ACC(3, t_sv);
  CMPC_CNT(13, 1);
}

// park / restore the factors in the wave's global slab (144 floats per lane)
__device__ __forceinline__ void ric_park_store(float* __restrict__ park, const RicRegs& F) {
  const int lane = opaque_lane();
#pragma unroll
  for (int k = 0; k < kMaxN; ++k)
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      park[((k * 3 + q) * 3 + 0) * 64 + lane] = F.y[k][q];
      park[((k * 3 + q) * 3 + 1) * 64 + lane] = F.z[k][q];
      park[((k * 3 + q) * 3 + 2) * 64 + lane] = F.si[k][q];
    }
}

__device__ __forceinline__ void ric_park_load(const float* __restrict__ park, RicRegs& F) {
  const int lane = opaque_lane();
  asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc1" ::: "memory");
#pragma unroll
  for (int k = 0; k < kMaxN; ++k)
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      F.y[k][q] = park[((k * 3 + q) * 3 + 0) * 64 + lane];
      F.z[k][q] = park[((k * 3 + q) * 3 + 1) * 64 + lane];
      F.si[k][q] = park[((k * 3 + q) * 3 + 2) * 64 + lane];
    }
}
