// cmpc_leg.hip -- the reference's 1 kHz leg controller for a batch of robots, on the device: the
// consumer of the QP's first contact forces (stance torque mapping).
//
// Per robot and leg, LegController.compute_leg_torque (leg_controller.py:43-112):
//   stance: tau = J_foot' (-f)                                              (:100-101)
//   swing:  tau = J_foot' (KP e_p + KD e_v + Lambda (a_des - Jdot dq)) + (C dq + g)[leg]
//           Lambda = (J_full M^-1 J_full')^-1                               (:75-98)
// with the swing trajectory planned at take-off (Gait.compute_swing_traj_and_touchdown +
// make_swing_trajectory, gait.py:77-174: touchdown prediction, minimum-jerk + z-bump) and the
// motor clip of the loop (test_MPC.py:227-228).  The Pinocchio quantities are inputs; the
// controller's memory (last mask, take-off time, swing start / touchdown) is a per-robot state
// buffer that persists across ticks.
//
// One 64-lane wave per robot, fp64 (the reference's arithmetic): the robot's matrices are staged
// in LDS with all loads in flight; only when a leg swings (a wave-uniform branch) M is factored
// (Cholesky, all 171 lower entries updated in parallel per column step), Y = L^-1 J_full' is one
// parallel forward substitution over the 12 Jacobian rows, and J M^-1 J' = Y'Y; lanes 0..3 then
// finish one leg each.
// HBM-bound: ~7.7 KB read per robot (M, C, J_full dominate), 0.35 KB written.
//
// This file is compiled as part of cmpc_host.hip (single translation unit).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cmpc {

constexpr double kKpSwing = 500.0;     // leg_controller.py:10
constexpr double kKdSwing = 200.0;     // leg_controller.py:11
constexpr double kHeightSwing = 0.1;   // gait.py:9
constexpr int kNv = 18;                // floating base (6) + 12 leg joints

// lower-triangle entry e of an 18 x 18 matrix -> (row, column), row-major over rows
struct TriTable {
  uint8_t i[kNv * (kNv + 1) / 2], k[kNv * (kNv + 1) / 2];
  constexpr TriTable() : i(), k() {
    int e = 0;
    for (int r = 0; r < kNv; ++r)
      for (int c = 0; c <= r; ++c) { i[e] = (uint8_t)r; k[e] = (uint8_t)c; ++e; }
  }
};
__constant__ constexpr TriTable kTri{};
#define kTriI kTri.i
#define kTriK kTri.k

struct LegArgs {
  const double* t;        // [B]
  const double* gait;     // [B][6]
  const float* force;     // [B] rows of 12 (U[:, 0]), row stride force_stride floats
  int64_t force_stride;
  const double* J_foot;   // [B][4][3][3]
  const double* J_full;   // [B][4][3][18]
  const double* M;        // [B][18][18]
  const double* C;        // [B][18][18]
  const double* g;        // [B][18]
  const double* dq;       // [B][18]
  const double* Jdot_dq;  // [B][4][3]
  const double* foot_pos; // [B][4][3]
  const double* foot_vel; // [B][4][3]
  const double* body;     // [B][16]
  const double* hip;      // [4][3]
  double* state;          // [B][4][8]
  double tau_max;
  double* tau;            // [B][12]
};

__global__ void __launch_bounds__(64, 4) leg_kernel(int64_t B, LegArgs a) {
  __shared__ double Ms[kNv * kNv];     // M, then its Cholesky factor (lower)
  __shared__ double Cs[12 * kNv];      // rows 6..17 of C (the leg joints)
  __shared__ double Jr[12 * kNv];      // J_full rows (3 per leg), then Y = L^-1 J_full' by rows
  __shared__ double Li[4][9];          // J_full M^-1 J_full' per leg
  __shared__ double hs[12];            // (C dq + g) of the 12 leg joints
  __shared__ double dqs[kNv];
  __shared__ double Ld[kNv];           // 1 / diag(L)
  const int lane = threadIdx.x;
  for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
    const double t = a.t[b];
    const double period = a.gait[b * 6], duty = a.gait[b * 6 + 1];
    // gait.py:21-37 current mask at t (lanes 0..3 = legs)
    bool st = false;
    if (lane < 4) st = stance_at(t + 0.0 / 2, period, duty, a.gait[b * 6 + 2 + lane]);
    const uint64_t smask = __ballot(st);
    const bool any_swing = (smask & 0xfull) != 0xfull;
    // stage this robot's matrices in LDS: every load of the robot in flight at once
    {
      const double* Cg = a.C + (b * kNv + 6) * kNv;
      double cv[4], dv = 0.0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = lane + 64 * i;
        cv[i] = (e < 12 * kNv) ? Cg[e] : 0.0;
      }
      if (lane < kNv) dv = a.dq[b * kNv + lane];
      if (any_swing) {  // uniform: M and J_full only matter to swing legs
        const double* Mg = a.M + b * kNv * kNv;
        const double* Jg = a.J_full + b * 12 * kNv;
        double mv[6], jv[4];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          const int e = lane + 64 * i;
          mv[i] = (e < kNv * kNv) ? Mg[e] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = lane + 64 * i;
          jv[i] = (e < 12 * kNv) ? Jg[e] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          const int e = lane + 64 * i;
          if (e < kNv * kNv) Ms[e] = mv[i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = lane + 64 * i;
          if (e < 12 * kNv) Jr[e] = jv[i];
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = lane + 64 * i;
        if (e < 12 * kNv) Cs[e] = cv[i];
      }
      if (lane < kNv) dqs[lane] = dv;
    }
    __syncthreads();
    // (C dq + g) for the leg joints 6..17 (leg_controller.py:98)
    if (lane < 12) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < kNv; ++k) acc = fma(Cs[lane * kNv + k], dqs[k], acc);
      hs[lane] = acc + a.g[b * kNv + 6 + lane];
    }
    if (any_swing) {  // uniform: Lambda is only needed by swing legs
      // Cholesky M = L L', right-looking, all lanes at once: lane-slot e = lane + 64 s owns the
      // lower entry (i, k) = kTri[e].  Step j reads column j (unscaled) and writes it scaled,
      // A[i][k] -= A[i][j] A[k][j] / A[j][j] for k > j; one wave, so LDS reads issued before the
      // writes see the old values and the next step sees the new ones (wave-ordered LDS).
      int ti[3], tk[3];  // this lane's lower entries (loop-invariant; -1: none)
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int e = lane + 64 * q;
        const bool ok = e < kNv * (kNv + 1) / 2;
        ti[q] = ok ? kTriI[ok ? e : 0] : -1;
        tk[q] = ok ? kTriK[ok ? e : 0] : -1;
      }
      for (int j = 0; j < kNv; ++j) {
        const double ajj = Ms[j * kNv + j];
        const double rs = 1.0 / sqrt(ajj), ri = rs * rs;
        if (lane == 0) Ld[j] = rs;  // 1 / L[j][j] for the substitution
        double nv[3];
        int at[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          at[q] = -1;
          if (ti[q] >= 0) {
            const int i = ti[q], k = tk[q];
            if (k == j && i >= j) {
              nv[q] = (i == j) ? ajj * rs : Ms[i * kNv + j] * rs;
              at[q] = i * kNv + j;
            } else if (k > j) {
              nv[q] = Ms[i * kNv + k] - Ms[i * kNv + j] * Ms[k * kNv + j] * ri;
              at[q] = i * kNv + k;
            }
          }
        }
        WSYNC();
#pragma unroll
        for (int q = 0; q < 3; ++q)
          if (at[q] >= 0) Ms[at[q]] = nv[q];
        WSYNC();
      }
      // Y = L^-1 J_full' (18 x 12): forward substitution, lane-slot e = lane + 64 s owns
      // (row r of J_full, entry m) = (e / 18, e % 18); then J M^-1 J' = Y' Y
      for (int i = 0; i < kNv; ++i) {
        const double ri = Ld[i];
        double nv[4];
        int at[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int e = lane + 64 * q;
          at[q] = -1;
          if (e < 12 * kNv) {
            const int r = e / kNv, m = e - r * kNv;
            if (m == i) {
              nv[q] = Jr[r * kNv + i] * ri;
              at[q] = e;
            } else if (m > i) {
              nv[q] = Jr[e] - Ms[m * kNv + i] * Jr[r * kNv + i] * ri;
              at[q] = e;
            }
          }
        }
        WSYNC();
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (at[q] >= 0) Jr[at[q]] = nv[q];
        WSYNC();
      }
      if (lane < 36) {  // (J_full M^-1 J_full')[leg][r][c] = sum_m Y[m][3 leg + r] Y[m][3 leg + c]
        const int leg = lane / 9, r = (lane % 9) / 3, c = lane % 3;
        const double* yr = &Jr[(3 * leg + r) * kNv];
        const double* yc = &Jr[(3 * leg + c) * kNv];
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < kNv; ++k) acc = fma(yr[k], yc[k], acc);
        Li[leg][r * 3 + c] = acc;
      }
    }
    __syncthreads();
    if (lane < 4) {
      const int leg = lane;
      double* S = a.state + (b * 4 + leg) * 8;
      const double* Jf = a.J_foot + (b * 4 + leg) * 9;  // [3][3], row = Cartesian axis
      double f[3], tq[3];
      const double last = S[0];
      const double cur = st ? 1.0 : 0.0;
      if (!st) {
        const double t_swing = (1.0 - duty) * period, t_stance = duty * period;
        const double* fp = a.foot_pos + (b * 4 + leg) * 3;
        const double* fv = a.foot_vel + (b * 4 + leg) * 3;
        if (last != cur) {
          // take-off: gait.py:77-133 touchdown prediction, swing from the current foot position
          const double* bd = a.body + b * 16;
          const double* h = a.hip + leg * 3;
          const double cz = cos(bd[9]), sz = sin(bd[9]);
          const double hwx = bd[0] + (cz * h[0] - sz * h[1] + 0.0 * h[2]);
          const double hwy = bd[1] + (sz * h[0] + cz * h[1] + 0.0 * h[2]);
          const double T = t_swing + 0.5 * t_stance;
          const double pred = T / 2.0;
          const double kvx = 0.4 * T, kpx = 0.1, kvy = 0.2 * T, kpy = 0.05;
          const double dth = bd[10] * pred;
          const double rx = hwx - bd[0], ry = hwy - bd[1];
          S[1] = t;
          S[2] = fp[0]; S[3] = fp[1]; S[4] = fp[2];
          S[5] = hwx + bd[13] * pred + kpx * (bd[3] - bd[11]) + kvx * (bd[6] - bd[13]) + (-dth * ry);
          S[6] = hwy + bd[14] * pred + kpy * (bd[4] - bd[12]) + kvy * (bd[7] - bd[14]) + dth * rx;
          S[7] = kTdHeight + 0.0 + 0.0 + 0.0 + 0.0;
        }
        // gait.py:141-172 minimum-jerk + z-bump at t - take-off time
        const double T = t_swing;
        double s = (t - S[1]) / T;
        s = s < 0.0 ? 0.0 : (s > 1.0 ? 1.0 : s);
        const double s2 = s * s, s3 = s2 * s, s4 = s3 * s, s5 = s4 * s;
        const double mj = 10 * s3 - 15 * s4 + 6 * s5;
        const double dmj = 30 * s2 - 60 * s3 + 30 * s4;
        const double d2mj = 60 * s - 180 * s2 + 120 * s3;
        const double u = 1.0 - s;
        const double bz = 64 * s3 * (u * u * u);
        const double dbz = 192 * s2 * (u * u) * (1 - 2 * s);
        const double d2bz = 192 * (2 * s * (u * u) * (1 - 2 * s) - 2 * s2 * u * (1 - 2 * s) -
                                   2 * s2 * (u * u));
        double p[3], v[3], ac[3];
        for (int i = 0; i < 3; ++i) {
          const double dp = S[5 + i] - S[2 + i];
          p[i] = S[2 + i] + dp * mj;
          v[i] = (dp * dmj) / T;
          ac[i] = (dp * d2mj) / (T * T);
        }
        p[2] += kHeightSwing * bz;
        v[2] += kHeightSwing * dbz / T;
        ac[2] += kHeightSwing * d2bz / (T * T);
        // Lambda = inv(J M^-1 J') (3x3, adjugate)
        const double* K = Li[leg];
        const double c00 = K[4] * K[8] - K[5] * K[7], c01 = K[5] * K[6] - K[3] * K[8],
                     c02 = K[3] * K[7] - K[4] * K[6];
        const double id = 1.0 / (K[0] * c00 + K[1] * c01 + K[2] * c02);
        const double Lam[9] = {c00 * id, (K[2] * K[7] - K[1] * K[8]) * id,
                               (K[1] * K[5] - K[2] * K[4]) * id, c01 * id,
                               (K[0] * K[8] - K[2] * K[6]) * id, (K[2] * K[3] - K[0] * K[5]) * id,
                               c02 * id, (K[1] * K[6] - K[0] * K[7]) * id,
                               (K[0] * K[4] - K[1] * K[3]) * id};
        const double* jd = a.Jdot_dq + (b * 4 + leg) * 3;
        double w[3];
        for (int i = 0; i < 3; ++i) w[i] = ac[i] - jd[i];
        for (int i = 0; i < 3; ++i) {
          const double fff = Lam[3 * i] * w[0] + Lam[3 * i + 1] * w[1] + Lam[3 * i + 2] * w[2];
          f[i] = kKpSwing * (p[i] - fp[i]) + kKdSwing * (v[i] - fv[i]) + fff;
        }
        for (int j = 0; j < 3; ++j)
          tq[j] = Jf[j] * f[0] + Jf[3 + j] * f[1] + Jf[6 + j] * f[2] + hs[3 * leg + j];
      } else {
        const float* fr = a.force + b * a.force_stride + 3 * leg;
        for (int i = 0; i < 3; ++i) f[i] = -(double)fr[i];
        for (int j = 0; j < 3; ++j) tq[j] = Jf[j] * f[0] + Jf[3 + j] * f[1] + Jf[6 + j] * f[2];
      }
      S[0] = cur;
      for (int j = 0; j < 3; ++j) {
        double v = tq[j];
        if (a.tau_max > 0.0) v = fmin(fmax(v, -a.tau_max), a.tau_max);
        a.tau[b * 12 + 3 * leg + j] = v;
      }
    }
    __syncthreads();
  }
}

}  // namespace cmpc
