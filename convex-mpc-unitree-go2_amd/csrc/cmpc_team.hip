// cmpc_team.hip -- W WAVES PER QP ("team" mode) for small batches.
//
// With one wave per QP a batch of B <= 1,024 instances leaves most of the 1,024 SIMDs idle and
// every instance's latency is its wave's serial chain (BASELINE config 1: B = 256 on 256 CUs).
// Team mode gives each QP a workgroup of W waves on W SIMDs of one CU.  Wave 0 (the leader)
// runs solve_instance's control flow unchanged; waves 1..W-1 (helpers) sit in a command loop and
// join the leader in the matrix phases, which hold ~70 % of a wave's time:
//   FACTOR  block-row condensation + 4-pivot block sweep inversion (cmpc_wave.hip 1-2),
//   SYMV    out = M in,
//   PSTORE / PLOAD  park / restore the inverse,
// each wave on its own share of the lower-triangle tiles, held in its registers.
//
// Tile ownership: the tile COLUMNS J and TT-1-J form a pair of exactly TT+1 tiles; pair pr goes
// to wave pr % W as its local pair pr / W.  Local slot l of a pair is tile
//   (pr + l, pr)              for l <  TT - pr   (column pr, rows pr .. TT-1)
//   (l - 1, TT - 1 - pr)      for l >= TT - pr   (column TT-1-pr, rows TT-1-pr .. TT-1),
// so the register array is indexed at compile time and (I, J) are uniform scalars.  Owning
// whole columns keeps the condensation's G_t chunks (the MFMA B operand of column J) local to
// the wave: only C_t (the A operand, one row chunk per step) and the sweep's pivot panel go
// through LDS.
//
// Synchronisation: a command is published by the leader in a double-buffered slot and starts at
// a workgroup barrier; the barriers inside a command depend only on its arguments, so every wave
// passes the same number of them (no data-dependent barrier counts).  Helpers write only the
// team block (panel, partial sums, scratch); the leader mutates the instance's LDS image only
// between commands, while the helpers wait at the next command's barrier.
//
// This file is compiled as part of cmpc_wave.hip (single translation unit).

template <int NC, int W>
struct TeamCfg {
  static constexpr int TT = NC / 16;
  static constexpr int NPAIR = TT / 2;
  static constexpr int PPW = (NPAIR + W - 1) / W;  // column pairs per wave
  // register tiles per wave (W = 1: the one-wave kernels, every lower tile)
  static constexpr int SLOTS = W == 1 ? TT * (TT + 1) / 2 : PPW * (TT + 1);
  static constexpr int SLAB = W * SLOTS * 256;     // park slab of the team (floats)
  static_assert(W == 1 || TT % 2 == 0, "team mode pairs tile columns");
};

enum : int { kOpExit = 0, kOpFactor = 1, kOpSymv = 2, kOpParkStore = 3, kOpParkLoad = 4 };

// The phase buffers share one region: the diagonal mirror's scratch is dead once the factor's
// scaling barrier has passed (the sweep's panel is written after it), and a SYMV command starts
// at a barrier that every wave reaches only after the previous command's last panel read.
template <int NC, int W>
struct TeamSmem {
  int cmd[2][4];                           // op, n, arg1, arg2 (double-buffered by sequence)
  alignas(16) float ds[NC];                // unit-diagonal scaling of the sweep
  union {
    alignas(16) float pan[2][NC * 4];      // FACTOR sweep: panel, double-buffered by pivot step
    struct {
      alignas(16) float partR[NC / 32][NC];  // SYMV: row sums of column pair pr's tiles
      alignas(16) float partC[NC];           // SYMV: column sums (J < I tiles) landing in chunk J
    };
    alignas(16) float scr[W][512];         // FACTOR diagonal mirror: per-wave 2 x 16 x 16 scratch
  };
};

// slot geometry: local pair j of wave w, slot l -> tile (I, J); valid iff the pair exists
template <int NC, int W>
__device__ __forceinline__ bool team_slot(int w, int j, int l, int& I, int& J) {
  using T = TeamCfg<NC, W>;
  const int pr = w + j * W;
  if (l < T::TT - pr) {
    I = pr + l;
    J = pr;
  } else {
    I = l - 1;
    J = T::TT - 1 - pr;
  }
  return pr < T::NPAIR;
}

__device__ __forceinline__ void team_barrier() { __syncthreads(); }

// Pin a loaded value at this point: the LDS reads issued before it complete under ONE wait
// instead of the scheduler sinking each read to its use, where every read would wait for its
// own latency (~100 cycles) in a dependent chain.
__device__ __forceinline__ void pin(f4& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void pin(float& v) { asm volatile("" : "+v"(v)); }

// One 4-pivot step of the block sweep (pivots 16 K + 4 sub .. +3): publish the pivot columns
// from the owned tiles, one barrier, then every wave updates its tiles with one MFMA each.
template <int NC, int W, int WV>
__device__ __forceinline__ void team_sweep_step(Smem<NC>& s, TeamSmem<NC, W>& ts,
                                                f4 (&M)[TeamCfg<NC, W>::SLOTS], int w, int K,
                                                int sub, int g, int c) {
  using T = TeamCfg<NC, W>;
  constexpr int TT = T::TT;
  const bool g1 = g == 1, g2 = g == 2, g3 = g == 3;
  const int c0 = 4 * sub, k0 = 16 * K + c0;
  const int pc = c - c0;
  const bool colw = pc >= 0 && pc < 4, roww = g == sub;
  float* pb = ts.pan[sub & 1];  // = (4 K + sub) & 1
  // publish the 4 pivot columns (P^ = P - I on the pivot rows) from the tiles of column K and
  // (transposed) of row K
#pragma unroll
  for (int j = 0; j < T::PPW; ++j) {
#pragma unroll
    for (int l = 0; l <= TT; ++l) {
      int I, J;
      if (!team_slot<NC, W>(w, j, l, I, J)) continue;
      const f4 mm = M[j * (TT + 1) + l];
      if (J == K) {
        if (colw) {
          f4 m = mm;
          if (I == K) {
#pragma unroll
            for (int q = 0; q < 4; ++q) m[q] -= (4 * g + q == c) ? 1.f : 0.f;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) pb[(16 * I + 4 * g + q) * 4 + pc] = m[q];
        }
      } else if (I == K) {  // J < K
        if (roww) *reinterpret_cast<f4*>(&pb[(16 * J + c) * 4]) = mm;
      }
    }
  }
  team_barrier();
  // the LDS reads of the step are issued together ahead of the LDL chain (no branch between
  // them: a read inside a per-tile branch would wait for its own latency): the pivot block and
  // the first pair's panel rows; a further pair (PPW > 1) reads its rows when its turn comes,
  // so only one pair's rows are live at a time
  f4 rr[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) rr[i] = *reinterpret_cast<const f4*>(&pb[(k0 + i) * 4]);
  f4 phs[TT + 1], phj[2];
  auto read_pair = [&](int j) {
    const int pr = w + j * W;
    const bool ok = pr < T::NPAIR;  // (a missing pair reads row 0 and is skipped below)
#pragma unroll
    for (int l = 0; l <= TT; ++l) {
      int I, J;
      team_slot<NC, W>(w, j, l, I, J);
      phs[l] = *reinterpret_cast<const f4*>(&pb[(16 * (ok ? I : 0) + c) * 4]);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int J = ok ? (h ? TT - 1 - pr : pr) : 0;
      phj[h] = *reinterpret_cast<const f4*>(&pb[(16 * J + c) * 4]);
    }
#pragma unroll
    for (int l = 0; l <= TT; ++l) pin(phs[l]);
    pin(phj[0]);
    pin(phj[1]);
  };
  read_pair(0);
#pragma unroll
  for (int i = 0; i < 4; ++i) pin(rr[i]);
  float Dm[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) Dm[i * 4 + jj] = (i == jj) ? rr[i][jj] + 1.f : rr[i][jj];
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
  const float n10 = -l10, n21 = -l21, n32 = -l32;
  const float n20 = l21 * l10 - l20, n31 = l32 * l21 - l31;
  const float n30 = -l30 - l31 * n10 - l32 * n20;
  const float w0 = g3 ? n30 : g2 ? n20 : g1 ? n10 : 1.f;
  const float w1 = g3 ? n31 : g2 ? n21 : g1 ? 1.f : 0.f;
  const float w2 = g3 ? n32 : g2 ? 1.f : 0.f;
  const float w3 = g3 ? 1.f : 0.f;
  const float ig = g3 ? i3 : g2 ? i2 : g1 ? i1 : i0;
#pragma unroll
  for (int j = 0; j < T::PPW; ++j) {
    const int pr = w + j * W;
    if (pr >= T::NPAIR) continue;
    if (j > 0) read_pair(j);
    float bj[2];  // b = diag(1/dl) Y' operand of the pair's two columns
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f4 ph = phj[h];
      bj[h] = fmaf(w3, ph[3], fmaf(w2, ph[2], fmaf(w1, ph[1], w0 * ph[0]))) * ig;
    }
    // padding tiles (I >= TA) are updated too: their panel rows are zero, so is the update
#pragma unroll
    for (int l = 0; l <= TT; ++l) {
      const f4 ph = phs[l];
      const float a = -fmaf(w3, ph[3], fmaf(w2, ph[2], fmaf(w1, ph[1], w0 * ph[0])));
      const float b = (l < TT - pr) ? bj[0] : bj[1];
      M[j * (TT + 1) + l] = mfma4(a, b, M[j * (TT + 1) + l]);
    }
    // -2 on the 4 pivot diagonals (tile (K, K): slot 0 when K == pr, slot TT - pr when
    // K == TT - 1 - pr)
#pragma unroll
    for (int l = 0; l <= TT; ++l) {
      int I, J;
      team_slot<NC, W>(w, j, l, I, J);
      if (I != K || J != K) continue;
      f4& m = M[j * (TT + 1) + l];
#pragma unroll
      for (int q = 0; q < 4; ++q) m[q] -= (roww && pc == q) ? 2.f : 0.f;
    }
  }
}

// M_IJ *= sgn diag(ds_I) M_IJ diag(ds_J) on every owned tile (all reads issued first)
template <int NC, int W>
__device__ __forceinline__ void team_scale(TeamSmem<NC, W>& ts, f4 (&M)[TeamCfg<NC, W>::SLOTS],
                                           int w, int g, int c, float sgn) {
  using T = TeamCfg<NC, W>;
  constexpr int TT = T::TT;
#pragma unroll
  for (int j = 0; j < T::PPW; ++j) {
    const int pr = w + j * W;
    if (pr >= T::NPAIR) continue;  // uniform
    f4 ri[TT];  // rows pr .. TT-1 (index I - pr)
#pragma unroll
    for (int r = 0; r < TT; ++r) {
      const int I = min(pr + r, TT - 1);
      ri[r] = *reinterpret_cast<const f4*>(&ts.ds[16 * I + 4 * g]);
    }
    float c0 = ts.ds[16 * pr + c], c1 = ts.ds[16 * (TT - 1 - pr) + c];
#pragma unroll
    for (int r = 0; r < TT; ++r) pin(ri[r]);
    pin(c0);
    pin(c1);
    c0 *= sgn;
    c1 *= sgn;
#pragma unroll
    for (int l = 0; l <= TT; ++l) {
      int I, J;
      team_slot<NC, W>(w, j, l, I, J);
      const f4 rv = ri[I - pr];
      const float cj = (l < TT - pr) ? c0 : c1;
      f4& m = M[j * (TT + 1) + l];
#pragma unroll
      for (int q = 0; q < 4; ++q) m[q] *= rv[q] * cj;
    }
  }
}

// ------------------------------------------------------------------------------------------
// FACTOR: M <- -(H + diag(Rt) + shift)^-1 share of this wave (block-row condensation, then the
// 4-pivot block sweep; cmpc_wave.hip condense_tiles_bc / invert_tiles restated per slot)
// ------------------------------------------------------------------------------------------
template <int NC, int W, int WV>
__device__ __forceinline__ void team_factor(Smem<NC>& s, TeamSmem<NC, W>& ts, const KParams& P,
                                            f4 (&M)[TeamCfg<NC, W>::SLOTS], int n, float shift,
                                            int w_rt) {
  using T = TeamCfg<NC, W>;
  // WV >= 0: the wave index is a compile-time constant, so every slot's tile (I, J) is too and
  // the per-tile tests below fold away (straight-line code per wave)
  const int w = (WV >= 0) ? WV : uniform(w_rt);
  constexpr int TT = T::TT;
  const int lane = opaque_lane();
  const int g = lane >> 4, c = lane & 15;
  const int N = P.N;
  n = uniform(n);
#pragma unroll
  for (int t = 0; t < T::SLOTS; ++t) M[t] = f4{0.f, 0.f, 0.f, 0.f};
  // State layout (as condense_tiles_fwd and the gradient): accumulator position 4g + q holds
  // state 3g + q for q < 3 and is padding for q = 3, so every product over the 12 states is
  // three v_mfma_f32_16x16x4_f32 (K = 12), not four.  Lane column c holds state sc (or none).
  const int sc = ((c & 3) < 3) ? 3 * (c >> 2) + (c & 3) : -1;
  float aA[3], aT[3];  // A[sc][3g + q] (A operand of A X), A[3g + q][sc] (of A' X)
  f4 q2 = {0.f, 0.f, 0.f, 0.f};  // Q2 in accumulator layout
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int r = 3 * g + q;
    aA[q] = (sc >= 0) ? s.A[sc * 12 + r] : 0.f;
    aT[q] = (sc >= 0) ? s.A[r * 12 + sc] : 0.f;
    q2[q] = (r == sc) ? s.Q2[r] : 0.f;
  }
  float* Cs = s.G;  // C_i columns (or V = N b: the closed form), param-major [p][12]
  CMPC_T0(t_f0);
  if (uniform(s.nil)) {
    // ---- closed form for a nilpotent step (cmpc_wave.hip condense_tiles_nil): V = N b by the
    // chunk's wave (J % W), one barrier, then every owned tile is six MFMAs
    {
      float aN[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int r = 3 * g + q;
        aN[q] = (sc >= 0) ? s.A[sc * 12 + r] - ((sc == r) ? 1.f : 0.f) : 0.f;
      }
#pragma unroll
      for (int J = 0; J < TT; ++J) {
        if (J % W != w) continue;  // uniform
        if (16 * J >= n) continue;  // uniform
        const int p = 16 * J + c;
        float bt[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) bt[q] = (p < n) ? s.Bt[p * kBS + 3 * g + q] : 0.f;
        f4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 3; ++q) d = mfma4(aN[q], bt[q], d);
#pragma unroll
        for (int q = 0; q < 3; ++q) Cs[p * 12 + 3 * g + q] = d[q];
      }
    }
    team_barrier();  // every V chunk in LDS
    CMPC_ACC(16, t_f0);
    CMPC_T0(t_f1);
    float qd[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) qd[q] = s.Q2[3 * g + q];
#pragma unroll
    for (int j = 0; j < T::PPW; ++j) {
      const int pr = w + j * W;
      if (pr >= T::NPAIR) continue;  // uniform
      // the pair's two columns' operands, once (every slot of the pair reuses one of them)
      float uc[2][3], vc[2][3];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int p = 16 * (h ? TT - 1 - pr : pr) + c;
        const bool ok = p < n;
        const float kf = ok ? (float)s.par[p] : 0.f;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          vc[h][q] = ok ? Cs[p * 12 + 3 * g + q] : 0.f;
          uc[h][q] = ok ? fmaf(-kf, vc[h][q], s.Bt[p * kBS + 3 * g + q]) : 0.f;
        }
      }
#pragma unroll
      for (int l = 0; l <= TT; ++l) {
        int I, J;
        team_slot<NC, W>(w, j, l, I, J);
        if (16 * I >= n) continue;  // uniform: padding rows stay zero
        float x[3], y[3], u[3], v[3];
        {
          const int p = 16 * I + c;
          const bool ok = p < n;
          const int k = ok ? s.par[p] : 0;
          const float kf = (float)k;
          float S0, S1, S2;
          step_sums(k, N, S0, S1, S2);
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            const float vv = ok ? Cs[p * 12 + 3 * g + q] : 0.f;
            const float uu = ok ? fmaf(-kf, vv, s.Bt[p * kBS + 3 * g + q]) : 0.f;
            x[q] = qd[q] * fmaf(S0, uu, S1 * vv);
            y[q] = qd[q] * fmaf(S1, uu, S2 * vv);
          }
        }
        {
          const int h = (l < TT - pr) ? 0 : 1;  // (compile-time after unrolling)
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            v[q] = vc[h][q];
            u[q] = uc[h][q];
          }
        }
        f4 acc = M[j * (TT + 1) + l];
#pragma unroll
        for (int q = 0; q < 3; ++q) acc = mfma4(x[q], u[q], acc);
#pragma unroll
        for (int q = 0; q < 3; ++q) acc = mfma4(y[q], v[q], acc);
        M[j * (TT + 1) + l] = acc;
      }
    }
    CMPC_ACC(17, t_f1);
  } else {
  // ---- backward: P_i (every wave, registers) and C_i = P_i B_i (chunk J written by wave J % W)
  {
    f4 Pt = q2;
    for (int i = N - 1; i >= 0; --i) {
      const int p0 = s.off[i], p1 = s.off[i + 1];
#pragma unroll
      for (int J = 0; J < TT; ++J) {
        if (J % W != w) continue;                        // uniform
        if (16 * J + 15 < p0 || 16 * J >= p1) continue;  // uniform
        const int p = 16 * J + c;
        float bt[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) bt[q] = s.Bt[p * kBS + 3 * g + q];
        f4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 3; ++q) d = mfma4(Pt[q], (p < n) ? bt[q] : 0.f, d);
        if (p >= p0 && p < p1) {
#pragma unroll
          for (int q = 0; q < 3; ++q) Cs[p * 12 + 3 * g + q] = d[q];
        }
      }
      if (i > 0) {
        f4 y = {0.f, 0.f, 0.f, 0.f}, z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 3; ++q) y = mfma4(Pt[q], aT[q], y);
#pragma unroll
        for (int q = 0; q < 3; ++q) z = mfma4(aT[q], y[q], z);
#pragma unroll
        for (int q = 0; q < 4; ++q) Pt[q] = z[q] + q2[q];
      }
    }
  }
  team_barrier();  // every C_i in LDS
  CMPC_ACC(16, t_f0);
  CMPC_T0(t_f1);
  // ---- forward: owned column chunks G_t = A G_{t-1} + new columns; rows of step t += C_t' G_t
  {
    f4 Gd[T::PPW][2];
    int kJ[T::PPW][2];
#pragma unroll
    for (int j = 0; j < T::PPW; ++j) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int pr = w + j * W;
        const int J = h ? TT - 1 - pr : pr;
        Gd[j][h] = f4{0.f, 0.f, 0.f, 0.f};
        kJ[j][h] = (pr < T::NPAIR && 16 * J < n) ? uniform(s.par[16 * J]) : N;
      }
    }
    for (int t = 0; t < N; ++t) {
      const int p0 = uniform(s.off[t]), p1 = uniform(s.off[t + 1]);
      // step t's params lie in at most two row chunks, Ia and Ib; their C rows and the new
      // B columns of the owned chunks are read together, before any MFMA of the step
      const int Ia = min(p0 >> 4, TT - 1), Ib = (p1 > p0) ? (p1 - 1) >> 4 : Ia;
      f4 alo = {0.f, 0.f, 0.f, 0.f}, ahi = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        alo[q] = Cs[(16 * Ia + c) * 12 + 3 * g + q];
        ahi[q] = Cs[(16 * Ib + c) * 12 + 3 * g + q];
      }
      f4 bn[T::PPW][2];
#pragma unroll
      for (int j = 0; j < T::PPW; ++j) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int pr = w + j * W;
          const int J = (pr < T::NPAIR) ? (h ? TT - 1 - pr : pr) : 0;
          bn[j][h] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int q = 0; q < 3; ++q) bn[j][h][q] = s.Bt[(16 * J + c) * kBS + 3 * g + q];
        }
      }
      pin(alo);
      pin(ahi);
#pragma unroll
      for (int j = 0; j < T::PPW; ++j) {
        pin(bn[j][0]);
        pin(bn[j][1]);
      }
      {
        const int pa = 16 * Ia + c, pb_ = 16 * Ib + c;
        const bool ma = pa >= p0 && pa < p1, mb = pb_ >= p0 && pb_ < p1;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          alo[q] = ma ? alo[q] : 0.f;
          ahi[q] = mb ? ahi[q] : 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < T::PPW; ++j) {
        const int pr = w + j * W;
        if (pr >= T::NPAIR) continue;  // uniform
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int J = h ? TT - 1 - pr : pr;
          if (t > 0 && kJ[j][h] < t) {
            f4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int q = 0; q < 3; ++q) d = mfma4(aA[q], Gd[j][h][q], d);
            Gd[j][h] = d;
          }
          const int p = 16 * J + c;
          if (p >= p0 && p < p1) Gd[j][h] = bn[j][h];
        }
#pragma unroll
        for (int l = 0; l <= TT; ++l) {
          int I, J;
          team_slot<NC, W>(w, j, l, I, J);
          if (I != Ia && I != Ib) continue;  // uniform: rows of step t (none if p1 == p0)
          if (p1 == p0) continue;
          const f4 a = (I == Ia) ? alo : ahi;
          const f4 gj = (l < TT - pr) ? Gd[j][0] : Gd[j][1];
          f4 acc = M[j * (TT + 1) + l];
#pragma unroll
          for (int q = 0; q < 3; ++q) acc = mfma4(a[q], gj[q], acc);
          M[j * (TT + 1) + l] = acc;
        }
      }
    }
  }
  CMPC_ACC(17, t_f1);
  }  // (general A)
  CMPC_T0(t_f2);
  // ---- diagonal tiles: entry (r, c) with step(c) > step(r) is the mirror of (c, r); then
  // + diag(Rt) + shift, identity on padding; the sweep's scaling from the diagonals.  A pair's
  // two diagonal tiles are slots 0 and TT - pr; their transposes go through the wave's scratch,
  // and every LDS read of the phase is issued before its first use.
  float* scr = ts.scr[w];
#pragma unroll
  for (int j = 0; j < T::PPW; ++j) {
    const int pr = w + j * W;
    if (pr >= T::NPAIR) continue;  // uniform
    const int base = j * (TT + 1);
    const int Jd[2] = {pr, TT - 1 - pr};
    const int ld[2] = {0, TT - pr};
    f4 v[2], tr[2];
    int kc[2], kr[2][4];
    float rt[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) v[h] = M[base + ld[h]];
    WSYNC();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int q = 0; q < 4; ++q) scr[256 * h + (4 * g + q) * 16 + c] = v[h][q];
    }
    WSYNC();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int I = Jd[h];
#pragma unroll
      for (int q = 0; q < 4; ++q) tr[h][q] = scr[256 * h + c * 16 + 4 * g + q];
      kc[h] = s.par[16 * I + c];
#pragma unroll
      for (int q = 0; q < 4; ++q) kr[h][q] = s.par[16 * I + 4 * g + q];
      rt[h] = s.Rt[16 * I + c];
    }
    WSYNC();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int I = Jd[h];
      const int pc = 16 * I + c;
      const int kcv = (pc < n) ? kc[h] : N;
      f4 m = v[h];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * I + 4 * g + q;
        const int krv = (row < n) ? kr[h][q] : N;
        if (16 * I < n && kcv > krv) m[q] = tr[h][q];
        if (row >= n || pc >= n) m[q] = (row == pc) ? 1.f : 0.f;
        else if (row == pc) m[q] += rt[h] + shift;
        if (4 * g + q == c) ts.ds[pc] = (pc < n && m[q] > 0.f) ? rsqrtf(m[q]) : 1.f;
      }
      M[base + ld[h]] = m;
    }
    // off-diagonal tiles: zero where the row or the column is padding
#pragma unroll
    for (int l = 0; l <= TT; ++l) {
      int I, J;
      team_slot<NC, W>(w, j, l, I, J);
      if (I == J) continue;
      f4& m = M[base + l];
      const int col = 16 * J + c;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * I + 4 * g + q;
        if (row >= n || col >= n) m[q] = 0.f;
      }
    }
  }
  team_barrier();  // scaling complete
  CMPC_ACC(18, t_f2);
  CMPC_T0(t_f3);
  team_scale<NC, W>(ts, M, w, g, c, 1.f);
  // ---- block sweep, four pivots per step, one barrier per step (double-buffered panel)
  const int ng = (n + 3) >> 2;
  if constexpr (WV >= 0) {  // K unrolled: the owned tiles of column K / row K are known
#pragma unroll
    for (int K = 0; K < TT; ++K) {
      if (4 * K >= ng) continue;  // uniform
      const int subs = (ng - 4 * K) < 4 ? (ng - 4 * K) : 4;
      for (int sub = 0; sub < subs; ++sub) team_sweep_step<NC, W, WV>(s, ts, M, w, K, sub, g, c);
    }
  } else {
    for (int kk = 0; kk < ng; ++kk) team_sweep_step<NC, W, WV>(s, ts, M, w, kk >> 2, kk & 3, g, c);
  }
  CMPC_ACC(19, t_f3);
  // M holds -(scaled inverse): undo sign and scaling
  team_scale<NC, W>(ts, M, w, g, c, -1.f);
}

// ------------------------------------------------------------------------------------------
// SYMV: this wave's partial sums of out = M in (M symmetric, lower tiles stored).  Row sums of
// tile (I, J) go to partR[J][rows of chunk I] (each written by the column's owner exactly once),
// the transposed contributions of the J < I tiles to partC[chunk J].  The leader adds them up
// after the command's barrier in a fixed order (deterministic).
// ------------------------------------------------------------------------------------------
// SYMV: this wave's partial sums of out = M in (M symmetric, lower tiles stored).  Row sums of
// column pair pr's tiles in row chunk I (both columns' tiles of a row summed before the one
// 16-lane reduction) go to partR[pr][rows of chunk I], written once by the pair's owner; the
// transposed contributions of the J < I tiles go to partC[chunk J].  The leader adds them up
// after the command's barrier in a fixed order (deterministic).
template <int NC, int W, int WV>
__device__ __forceinline__ void team_symv_part(TeamSmem<NC, W>& ts,
                                               const f4 (&M)[TeamCfg<NC, W>::SLOTS], int n,
                                               const float* in, int w_rt) {
  using T = TeamCfg<NC, W>;
  const int w = (WV >= 0) ? WV : uniform(w_rt);
  constexpr int TT = T::TT;
  const int lane = opaque_lane();
  const int g = lane >> 4, c = lane & 15;
  n = uniform(n);
#pragma unroll
  for (int j = 0; j < T::PPW; ++j) {
    const int pr = w + j * W;
    if (pr >= T::NPAIR) continue;
    const int J0 = pr, J1 = TT - 1 - pr;
    // all reads first (in[] has NC entries; entries at or past n count as zero).  Padding
    // tiles (rows >= n) are included: their products are zero, and the leader ignores them.
    float xc0, xc1;
    f4 xr[TT];  // rows pr .. TT-1 (index I - pr)
    {
      const float v0 = in[16 * J0 + c], v1 = in[16 * J1 + c];
      xc0 = (16 * J0 + c < n) ? v0 : 0.f;
      xc1 = (16 * J1 + c < n) ? v1 : 0.f;
    }
#pragma unroll
    for (int r = 0; r < TT; ++r) {
      const int I = min(pr + r, TT - 1);
      xr[r] = *reinterpret_cast<const f4*>(&in[16 * I + 4 * g]);
#pragma unroll
      for (int q = 0; q < 4; ++q) xr[r][q] = (16 * I + 4 * g + q < n) ? xr[r][q] : 0.f;
    }
    pin(xc0);
    pin(xc1);
#pragma unroll
    for (int r = 0; r < TT; ++r) pin(xr[r]);
    float cacc0 = 0.f, cacc1 = 0.f;
#pragma unroll
    for (int r = 0; r < TT; ++r) {
      const int I = pr + r;
      if (I >= TT) break;
      const f4 m0 = M[j * (TT + 1) + r];  // tile (I, J0): slot I - pr
      f4 racc;
#pragma unroll
      for (int q = 0; q < 4; ++q) racc[q] = m0[q] * xc0;
      if (I > J0) {
        float cp = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) cp = fmaf(m0[q], xr[r][q], cp);
        cacc0 += cp;
      }
      if (I >= J1) {  // tile (I, J1): slot I + 1
        const f4 m1 = M[j * (TT + 1) + I + 1];
#pragma unroll
        for (int q = 0; q < 4; ++q) racc[q] = fmaf(m1[q], xc1, racc[q]);
        if (I > J1) {
          float cp = 0.f;
#pragma unroll
          for (int q = 0; q < 4; ++q) cp = fmaf(m1[q], xr[r][q], cp);
          cacc1 += cp;
        }
      }
      f4 rs;
#pragma unroll
      for (int q = 0; q < 4; ++q) rs[q] = row16_sum(racc[q]);
      if (c == 0) *reinterpret_cast<f4*>(&ts.partR[pr][16 * I + 4 * g]) = rs;
    }
    const float cs0 = col4_sum(cacc0), cs1 = col4_sum(cacc1);
    if (g == 0) {
      ts.partC[16 * J0 + c] = cs0;
      ts.partC[16 * J1 + c] = cs1;
    }
  }
}

// leader side: out[p] = partC[p] + sum_{pr <= p/16} partR[pr][p] over the first TA chunks, 0
// beyond
template <int NC, int W>
__device__ __forceinline__ void team_symv_reduce(TeamSmem<NC, W>& ts, int n, float* out) {
  constexpr int NPAIR = NC / 32;
  const int lane = opaque_lane();
  n = uniform(n);
  const int TA = (n + 15) >> 4;
  for (int p = lane; p < NC; p += 64) {
    const int I = p >> 4;
    float acc = ts.partC[p];
#pragma unroll
    for (int pr = 0; pr < NPAIR; ++pr) {
      const float v = ts.partR[pr][p];
      acc += (pr <= I) ? v : 0.f;
    }
    out[p] = (I < TA) ? acc : 0.f;
  }
  WSYNC();
}

template <int NC, int W, int WV>
__device__ __forceinline__ void team_park_store(float* __restrict__ park,
                                                const f4 (&M)[TeamCfg<NC, W>::SLOTS], int w_rt) {
  const int w = (WV >= 0) ? WV : uniform(w_rt);
  const int lane = opaque_lane();
  float* base = park + (size_t)w * TeamCfg<NC, W>::SLOTS * 256;
#pragma unroll
  for (int t = 0; t < TeamCfg<NC, W>::SLOTS; ++t)
    *reinterpret_cast<f4*>(&base[t * 256 + lane * 4]) = M[t];
}

template <int NC, int W, int WV>
__device__ __forceinline__ void team_park_load(const float* __restrict__ park,
                                               f4 (&M)[TeamCfg<NC, W>::SLOTS], int w_rt) {
  const int w = (WV >= 0) ? WV : uniform(w_rt);
  const int lane = opaque_lane();
  const float* base = park + (size_t)w * TeamCfg<NC, W>::SLOTS * 256;
  asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc1" ::: "memory");
#pragma unroll
  for (int t = 0; t < TeamCfg<NC, W>::SLOTS; ++t)
    M[t] = *reinterpret_cast<const f4*>(&base[t * 256 + lane * 4]);
}

// ------------------------------------------------------------------------------------------
// leader: publish a command (wave 0, lane 0) and start it at the barrier
// ------------------------------------------------------------------------------------------
template <int NC, int W>
__device__ __forceinline__ void team_issue(TeamSmem<NC, W>& ts, int& seq, int op, int a0, int a1,
                                           int a2) {
  const int lane = opaque_lane();
  WSYNC();
  if (lane == 0) {
    int* cm = ts.cmd[seq & 1];
    cm[0] = op;
    cm[1] = a0;
    cm[2] = a1;
    cm[3] = a2;
  }
  ++seq;
  team_barrier();
}

// helpers: execute the leader's commands until kOpExit (one bin's drain loop)
template <int NC, int W, int WV>
__device__ __forceinline__ void team_helper(Smem<NC>& s, TeamSmem<NC, W>& ts, const KParams& P,
                                            float* __restrict__ park, int& seq) {
  constexpr int w = WV;
  f4 M[TeamCfg<NC, W>::SLOTS];
#pragma unroll
  for (int t = 0; t < TeamCfg<NC, W>::SLOTS; ++t) M[t] = f4{0.f, 0.f, 0.f, 0.f};
  for (;;) {
    team_barrier();
    const int* cm = ts.cmd[seq & 1];
    const int op = uniform(cm[0]), a0 = uniform(cm[1]), a1 = uniform(cm[2]);
    ++seq;
    if (op == kOpExit) break;
    if (op == kOpFactor) {
      team_factor<NC, W, WV>(s, ts, P, M, a0, __int_as_float(a1), w);
    } else if (op == kOpSymv) {
      const float* in = reinterpret_cast<const float*>(reinterpret_cast<const char*>(&s) + a1);
      team_symv_part<NC, W, WV>(ts, M, a0, in, w);
      team_barrier();  // partial sums complete (the leader reduces)
    } else if (op == kOpParkStore) {
      team_park_store<NC, W, WV>(park, M, w);
    } else if (op == kOpParkLoad) {
      team_park_load<NC, W, WV>(park, M, w);
    }
  }
}

// leader wrappers used by solve_instance
template <int NC, int W>
__device__ __forceinline__ void team_factor_lead(Smem<NC>& s, TeamSmem<NC, W>& ts, int& seq,
                                                 const KParams& P,
                                                 f4 (&M)[TeamCfg<NC, W>::SLOTS], int n,
                                                 float shift) {
  team_issue<NC, W>(ts, seq, kOpFactor, n, __float_as_int(shift), 0);
  team_factor<NC, W, 0>(s, ts, P, M, n, shift, 0);
}

template <int NC, int W>
__device__ __forceinline__ void team_symv_lead(Smem<NC>& s, TeamSmem<NC, W>& ts, int& seq,
                                               const f4 (&M)[TeamCfg<NC, W>::SLOTS], int n,
                                               const float* in, float* out) {
  CMPC_T0(t_sv);
  const int off = (int)(reinterpret_cast<const char*>(in) - reinterpret_cast<const char*>(&s));
  CMPC_T0(t_a);
  team_issue<NC, W>(ts, seq, kOpSymv, n, off, 0);
  CMPC_ACC(24, t_a);
  CMPC_T0(t_b);
  team_symv_part<NC, W, 0>(ts, M, n, in, 0);
  CMPC_ACC(25, t_b);
  CMPC_T0(t_c);
  team_barrier();
  CMPC_ACC(26, t_c);
  CMPC_T0(t_d);
  team_symv_reduce<NC, W>(ts, n, out);
  CMPC_ACC(27, t_d);
  CMPC_ACC(3, t_sv);
  CMPC_CNT(13, 1);
}

// helpers 1..W-1, each with its wave index as a compile-time constant; they follow the leader
// through the five bins (heaviest first, as solve_team_kernel drains them)
template <int W, int WV>
__device__ __forceinline__ void team_helpers(Smem<192>& s3, TeamSmem<192, W>& t3, Smem<160>& s2,
                                             TeamSmem<160, W>& t2, Smem<128>& s1,
                                             TeamSmem<128, W>& t1, Smem<96>& s0,
                                             TeamSmem<96, W>& t0, const KParams& P,
                                             float* __restrict__ park, int w, int& seq) {
  if constexpr (WV < W) {
    if (w == WV) {
      team_helper<192, W, WV>(s3, t3, P, park, seq);
#pragma unroll 1
      for (int q = 0; q < 2; ++q) team_helper<160, W, WV>(s2, t2, P, park, seq);  // bins 160, 144
      team_helper<128, W, WV>(s1, t1, P, park, seq);
      team_helper<96, W, WV>(s0, t0, P, park, seq);
    } else {
      team_helpers<W, WV + 1>(s3, t3, s2, t2, s1, t1, s0, t0, P, park, w, seq);
    }
  }
}
