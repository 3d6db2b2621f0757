// cmpc_traj.hip -- the reference's per-tick reference trajectory, contact table and foot levers
// for a batch of robots, on the device (com_trajectory.py:27-207,
// gait.py:21-74).
//
// One 64-lane wave per group of kTrajGroup robots.  Per robot, with lane = 4k + leg (k < N <= 16):
//   * the desired-position clamp (:47-60), a uniform scalar computation;
//   * x_ref (N x 12, :66-104): 3 entries per lane, written coalesced;
//   * the contact table (:106 -> gait.py:26-37): lane e computes entry e of the (4, N) table at
//     mid-step time;
//   * the foot levers (:108-201).  The reference walks the horizon serially, holding the last
//     predicted touchdown per leg.  Unrolled, the lever of (k, leg) is 0 in swing (mask at the
//     step's start time), the current lever if the leg has not taken off at any step <= k, and
//     otherwise the touchdown predicted at the LAST take-off step j <= k (gait.py:40-74) minus
//     the base position at j.  The start-of-step masks and take-off flags of all (k, leg) are two
//     wave ballots, so each lane finds its j with one bit scan and evaluates the prediction
//     itself, from the step's yaw rotation precomputed for the group (below).
// Time, phase and the contact mask are float64 with the reference's operation order, so the
// stance pattern is bit-identical to gait.py's; the rest is float64 rounded to fp32 on store.
//
// This file is compiled as part of cmpc_host.hip (single translation unit).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cmpc {

constexpr double kMaxPosError = 0.1;  // com_trajectory.py:47
constexpr double kTdHeight = 0.02;    // gait.py:57

// gait.py:33-36: stance = mod(offset + t / period, 1) < duty (np.mod: result has the divisor's
// sign).  No FMA contraction anywhere in this file: the reference's NumPy rounds every product.
__device__ __forceinline__ bool stance_at(double t, double period, double duty, double off) {
#pragma clang fp contract(off)
  double ph = fmod(off + t / period, 1.0);
  if (ph < 0.0) ph += 1.0;
  return ph < duty;
}

// ---- grouped form: kTrajGroup robots per wave ----
// The per-robot scalars (clamp, velocities, the three fp64 sin/cos pairs) were computed by all
// 64 lanes redundantly, and every lane evaluated its own take-off step's sin/cos.  Here a wave
// takes kTrajGroup robots: phase A computes each robot's
// scalars with lane = robot, phase B the 16 per-step yaw rotations of 4 robots per round with
// lane = (robot, step), and phase C walks the robots with the (step, leg) lane map as above,
// reading both from LDS.  Same arithmetic, same operation order, same results.
struct TrajRobot {
  double pdx, pdy, pdz, vwx, vwy, vbx, vby, yaw, wz, period, duty, tn, pred;
  double off[4];
};

constexpr int kTrajGroup = 16;  // robots per wave (enough waves to fill the SIMDs)

__global__ void __launch_bounds__(64) traj_group_kernel(int N, double dt, int64_t B,
                                                        const float* __restrict__ x0,
                                                        double* __restrict__ pos_des,
                                                        const float* __restrict__ cmd,
                                                        const double* __restrict__ t_now,
                                                        const double* __restrict__ gait,
                                                        const float* __restrict__ foot_lever,
                                                        const float* __restrict__ hip,
                                                        float* __restrict__ xref,
                                                        uint8_t* __restrict__ contact,
                                                        float* __restrict__ r_feet) {
#pragma clang fp contract(off)
  __shared__ TrajRobot R[kTrajGroup];
  __shared__ double CS[kTrajGroup][16][2];  // cos, sin of yaw_traj[j] (robot, step)
  const int lane = threadIdx.x;
  const int leg = lane & 3, k = lane >> 2;
  const double hx = hip[leg * 3], hy = hip[leg * 3 + 1];
  for (int64_t b0 = (int64_t)blockIdx.x * kTrajGroup; b0 < B;
       b0 += (int64_t)gridDim.x * kTrajGroup) {
    const int nr = (B - b0) < kTrajGroup ? (int)(B - b0) : kTrajGroup;
    // ---- phase A: lane = robot ----
    if (lane < nr) {
      const int64_t b = b0 + lane;
      const float* xs = x0 + b * 12;
      const double px = xs[0], py = xs[1], roll = xs[3], pitch = xs[4], yaw = xs[5];
      const double vxb = cmd[b * 4], vyb = cmd[b * 4 + 1], zdes = cmd[b * 4 + 2], wz = cmd[b * 4 + 3];
      const double period = gait[b * 6], duty = gait[b * 6 + 1];
      double pdx = pos_des[b * 3], pdy = pos_des[b * 3 + 1];
      if (pdx - px > kMaxPosError) pdx = px + kMaxPosError;
      if (px - pdx > kMaxPosError) pdx = px - kMaxPosError;
      if (pdy - py > kMaxPosError) pdy = py + kMaxPosError;
      if (py - pdy > kMaxPosError) pdy = py - kMaxPosError;
      const double cy = cos(yaw), sy = sin(yaw);
      const double vwx = cy * vxb - sy * vyb, vwy = sy * vxb + cy * vyb;
      const double cr = cos(roll), sr = sin(roll), cp = cos(pitch), sp = sin(pitch);
      TrajRobot& r = R[lane];
      r.pdx = pdx; r.pdy = pdy; r.pdz = zdes; r.vwx = vwx; r.vwy = vwy;
      r.vbx = (cy * cp) * vwx + (sy * cp) * vwy;
      r.vby = (cy * sp * sr - sy * cr) * vwx + (sy * sp * sr + cy * cr) * vwy;
      r.yaw = yaw; r.wz = wz; r.period = period; r.duty = duty; r.tn = t_now[b];
      const double t_swing = (1.0 - duty) * period, t_stance = duty * period;
      r.pred = (t_swing + 0.5 * t_stance) / 2.0;
#pragma unroll
      for (int l = 0; l < 4; ++l) r.off[l] = gait[b * 6 + 2 + l];
      pos_des[b * 3] = pdx; pos_des[b * 3 + 1] = pdy; pos_des[b * 3 + 2] = zdes;
    }
    __syncthreads();
    // ---- phase B: lane = (robot, step), 4 robots per round ----
    for (int rr = 0; rr < nr; rr += 4) {
      const int r = rr + (lane >> 4), j = lane & 15;
      if (r < nr && j < N) {
        const double t = (double)(j + 1) * dt;
        const double yj = R[r].yaw + R[r].wz * t;
        CS[r][j][0] = cos(yj);
        CS[r][j][1] = sin(yj);
      }
    }
    __syncthreads();
    // ---- phase C: one robot at a time, lane = (step, leg) ----
    for (int r = 0; r < nr; ++r) {
      const int64_t b = b0 + r;
      const TrajRobot& u = R[r];
      const double pdx = u.pdx, pdy = u.pdy, pdz = u.pdz, vwx = u.vwx, vwy = u.vwy;
      const double yaw = u.yaw, wz = u.wz, period = u.period, duty = u.duty, tn = u.tn;
      float* xr = xref + b * (int64_t)N * 12;
      for (int e = lane; e < N * 12; e += 64) {
        const int kk = e / 12, c = e - 12 * kk;
        const double t = (double)(kk + 1) * dt;
        double v = 0.0;
        switch (c) {
          case 0: v = pdx + vwx * t; break;
          case 1: v = pdy + vwy * t; break;
          case 2: v = pdz + 0.0 * t; break;
          case 5: v = yaw + wz * t; break;
          case 6: v = vwx; break;
          case 7: v = vwy; break;
          case 11: v = wz; break;
          default: break;
        }
        xr[e] = (float)v;
      }
      if (lane < 4 * N) {
        const int cl = lane / N, ck = lane - cl * N;
        double t = tn + (double)ck * dt;
        t = t + dt / 2;
        contact[b * 4 * N + lane] = stance_at(t, period, duty, u.off[cl]) ? 1 : 0;
      }
      const bool active = k < N;
      const bool m = active && stance_at(tn + (double)k * dt, period, duty, u.off[leg]);
      const uint64_t mbits = __ballot(m);
      const bool prev_stance = (k == 0) ? true : ((mbits >> (lane - 4)) & 1ull) != 0;
      const bool to = active && !m && (k == 0 || prev_stance);
      const uint64_t tbits = __ballot(to);
      if (active) {
        double r0 = 0.0, r1 = 0.0, r2 = 0.0;
        if (m) {
          const uint64_t legbits = 0x1111111111111111ull << leg;
          const uint64_t upto = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
          const uint64_t cand = tbits & legbits & upto;
          if (cand == 0) {
            const float* fl = foot_lever + (b * 4 + leg) * 3;
            r0 = fl[0]; r1 = fl[1]; r2 = fl[2];
          } else {
            const int j = (63 - __clzll((long long)cand)) >> 2;
            const double t = (double)(j + 1) * dt;
            const double bx = pdx + vwx * t, by = pdy + vwy * t, bz = pdz + 0.0 * t;
            const double cj = CS[r][j][0], sj = CS[r][j][1];
            const double pred = u.pred;
            const double hwx = cj * hx - sj * hy, hwy = sj * hx + cj * hy;
            const double nx = bx + hwx, ny = by + hwy;
            const double dth = wz * pred;
            const double rx = nx - bx, ry = ny - by;
            const double tdx = nx + u.vbx * pred + (-dth * ry);
            const double tdy = ny + u.vby * pred + dth * rx;
            const double tdz = kTdHeight + 0.0 + 0.0;
            r0 = tdx - bx; r1 = tdy - by; r2 = tdz - bz;
          }
        }
        float* rf = r_feet + (b * (int64_t)N * 4 + lane) * 3;
        rf[0] = (float)r0; rf[1] = (float)r1; rf[2] = (float)r2;
      }
    }
    __syncthreads();
  }
}

}  // namespace cmpc
