// cmpc_traj.hip -- the reference's per-tick reference trajectory, contact table and foot levers
// for a batch of robots, on the device (com_trajectory.py:27-207,
// gait.py:21-74).
//
// One 64-lane wave per robot, lane = 4k + leg (step k < N <= 16).  Per robot:
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
//     itself.
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

__global__ void __launch_bounds__(64) traj_kernel(int N, double dt, int64_t B,
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
  const int lane = threadIdx.x;
  const int leg = lane & 3, k = lane >> 2;
  const double hx = hip[leg * 3], hy = hip[leg * 3 + 1];
  for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
    // ---- per-robot scalars (uniform loads) ----
    const float* xs = x0 + b * 12;
    const double px = xs[0], py = xs[1], roll = xs[3], pitch = xs[4], yaw = xs[5];
    const double vxb = cmd[b * 4], vyb = cmd[b * 4 + 1], zdes = cmd[b * 4 + 2], wz = cmd[b * 4 + 3];
    const double period = gait[b * 6], duty = gait[b * 6 + 1];
    const double tn = t_now[b];

    // :47-60 desired position clamp (x, y), z commanded
    double pdx = pos_des[b * 3], pdy = pos_des[b * 3 + 1];
    if (pdx - px > kMaxPosError) pdx = px + kMaxPosError;
    if (px - pdx > kMaxPosError) pdx = px - kMaxPosError;
    if (pdy - py > kMaxPosError) pdy = py + kMaxPosError;
    if (py - pdy > kMaxPosError) pdy = py - kMaxPosError;
    const double pdz = zdes;

    // :72-73 world velocity command R_z(yaw) [vx, vy, 0]
    const double cy = cos(yaw), sy = sin(yaw);
    const double vwx = cy * vxb - sy * vyb, vwy = sy * vxb + cy * vyb;
    // :125-130 body-frame base velocity R_world_to_body v_world, R_world_to_body = (R_z R_y R_x)'
    // of the current state (go2_robot_data.py:211-216): rows 0, 1 of R' = columns 0, 1 of R;
    // v_world has no z component
    const double cr = cos(roll), sr = sin(roll), cp = cos(pitch), sp = sin(pitch);
    const double vbx = (cy * cp) * vwx + (sy * cp) * vwy;
    const double vby = (cy * sp * sr - sy * cr) * vwx + (sy * sp * sr + cy * cr) * vwy;

    // ---- x_ref (N x 12), entries e = lane + 64 j ----
    float* xr = xref + b * (int64_t)N * 12;
    for (int e = lane; e < N * 12; e += 64) {
      const int kk = e / 12, c = e - 12 * kk;
      const double t = (double)(kk + 1) * dt;  // :68
      double v = 0.0;
      switch (c) {
        case 0: v = pdx + vwx * t; break;      // :86-88
        case 1: v = pdy + vwy * t; break;
        case 2: v = pdz + 0.0 * t; break;
        case 5: v = yaw + wz * t; break;       // :98
        case 6: v = vwx; break;                // :92
        case 7: v = vwy; break;
        case 11: v = wz; break;                // :103
        default: break;                        // roll, pitch, vz, wx, wy = 0
      }
      xr[e] = (float)v;
    }

    // ---- contact table (4, N) at mid-step times (:106, gait.py:29-30) ----
    if (lane < 4 * N) {
      const int cl = lane / N, ck = lane - cl * N;
      double t = tn + (double)ck * dt;
      t = t + dt / 2;
      contact[b * 4 * N + lane] = stance_at(t, period, duty, gait[b * 6 + 2 + cl]) ? 1 : 0;
    }

    // ---- foot levers (:108-201) ----
    const double off = gait[b * 6 + 2 + leg];
    const bool active = k < N;
    // mask at the step's start time: compute_current_mask(time_now + i dt) (:120, gait.py:21-24)
    const bool m = active && stance_at(tn + (double)k * dt, period, duty, off);
    const uint64_t mbits = __ballot(m);
    // take-off at step k: swing now, stance (or the initial "2" state at k = 0) before
    const bool prev_stance = (k == 0) ? true : ((mbits >> (lane - 4)) & 1ull) != 0;
    const bool to = active && !m && (k == 0 || prev_stance);
    const uint64_t tbits = __ballot(to);
    if (active) {
      double r0 = 0.0, r1 = 0.0, r2 = 0.0;
      if (m) {
        // take-offs of this leg at steps <= k
        const uint64_t legbits = 0x1111111111111111ull << leg;
        const uint64_t upto = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
        const uint64_t cand = tbits & legbits & upto;
        if (cand == 0) {
          // no take-off yet: the lever at the initial touchdown state (:113, :146)
          const float* fl = foot_lever + (b * 4 + leg) * 3;
          r0 = fl[0]; r1 = fl[1]; r2 = fl[2];
        } else {
          const int j = (63 - __clzll((long long)cand)) >> 2;  // last take-off step
          // dummy model at step j (:122-132): base = pos_traj[:, j], R_z(yaw_traj[j])
          const double t = (double)(j + 1) * dt;
          const double bx = pdx + vwx * t, by = pdy + vwy * t, bz = pdz + 0.0 * t;
          const double yj = yaw + wz * t;
          const double cj = cos(yj), sj = sin(yj);
          // gait.py:40-74 touchdown prediction at take-off
          const double t_swing = (1.0 - duty) * period, t_stance = duty * period;
          const double pred = (t_swing + 0.5 * t_stance) / 2.0;
          const double hwx = cj * hx - sj * hy, hwy = sj * hx + cj * hy;
          const double nx = bx + hwx, ny = by + hwy;
          const double dth = wz * pred;
          const double rx = nx - bx, ry = ny - by;
          const double tdx = nx + vbx * pred + (-dth * ry);
          const double tdy = ny + vby * pred + dth * rx;
          const double tdz = kTdHeight + 0.0 + 0.0;
          r0 = tdx - bx; r1 = tdy - by; r2 = tdz - bz;
        }
      }
      float* rf = r_feet + (b * (int64_t)N * 4 + lane) * 3;  // [N][4][3]: (k, leg) = lane
      rf[0] = (float)r0; rf[1] = (float)r1; rf[2] = (float)r2;
    }
    if (lane < 3) pos_des[b * 3 + lane] = lane == 0 ? pdx : (lane == 1 ? pdy : pdz);
  }
}

}  // namespace cmpc
