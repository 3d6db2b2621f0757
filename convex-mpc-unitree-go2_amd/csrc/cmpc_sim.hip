// cmpc_sim.hip -- a vectorised single-rigid-body plant that closes the loop on the device.
//
// The reference closes its loop through MuJoCo (test_MPC.py:160-236, mujoco_model.py), which is
// absent from this image.  This kernel is the stand-in used by the
// closed-loop test and bench (config 4 shape: a batch of robots, MPC every MPC_DT, ground forces
// held between ticks): per robot, the nonlinear rigid-body dynamics the MPC linearises
// (com_trajectory.py:221-270) -- p'' = sum f / m + g, I_w w' + w x I_w w = sum (foot - p) x f,
// ZYX-Euler kinematics for rpy -- integrated semi-implicitly over `nsub` substeps.  Each leg
// applies U[:, 0] while the gait holds it in stance (gait.py:21-37 at the substep time); a leg
// that lands is placed at its hip plus half a stance of the COM velocity (the Raibert rule the
// reference's planner also uses, gait.py:40-74).  One thread per robot, fp32.
//
// This file is compiled as part of cmpc_host.hip (single translation unit).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cmpc {

__global__ void __launch_bounds__(256) srb_kernel(int64_t B, int nsub, double dt,
                                                  const double* __restrict__ t_now,
                                                  const double* __restrict__ gait,
                                                  const float* __restrict__ mass,
                                                  const float* __restrict__ inertia_body,
                                                  const float* __restrict__ force,
                                                  int64_t force_stride,
                                                  const float* __restrict__ hip,
                                                  float* __restrict__ x, float* __restrict__ feet,
                                                  uint8_t* __restrict__ in_contact) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float s[12], ft[4][3], f[4][3];
  for (int i = 0; i < 12; ++i) s[i] = x[b * 12 + i];
  for (int l = 0; l < 4; ++l)
    for (int a = 0; a < 3; ++a) {
      ft[l][a] = feet[(b * 4 + l) * 3 + a];
      f[l][a] = force[b * force_stride + 3 * l + a];
    }
  const float m = mass[b];
  float Ib[9];
  for (int i = 0; i < 9; ++i) Ib[i] = inertia_body[b * 9 + i];
  const double period = gait[b * 6], duty = gait[b * 6 + 1];
  const float t_stance = (float)(duty * period);
  uint8_t cmask = in_contact[b];
  double t = t_now[b];
  const float h = (float)dt;
  for (int it = 0; it < nsub; ++it) {
    // contact state at the substep time; a landing leg is placed under its hip + v t_stance / 2
    const float cr = cosf(s[3]), sr = sinf(s[3]), cp = cosf(s[4]), sp = sinf(s[4]);
    const float cy = cosf(s[5]), sy = sinf(s[5]);
    uint8_t nm = 0;
    for (int l = 0; l < 4; ++l) {
      const bool st = stance_at(t, period, duty, gait[b * 6 + 2 + l]);
      if (st) nm |= (uint8_t)(1u << l);
      if (st && !(cmask & (1u << l))) {
        const float hx = hip[l * 3], hy = hip[l * 3 + 1];
        ft[l][0] = s[0] + cy * hx - sy * hy + s[6] * 0.5f * t_stance;
        ft[l][1] = s[1] + sy * hx + cy * hy + s[7] * 0.5f * t_stance;
        ft[l][2] = 0.f;
      }
    }
    cmask = nm;
    // R = Rz(y) Ry(p) Rx(r); I_w = R I_b R'
    const float R[9] = {cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr,
                        sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr,
                        -sp,     cp * sr,                cp * cr};
    float RI[9], Iw[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        RI[i * 3 + j] = R[i * 3] * Ib[j] + R[i * 3 + 1] * Ib[3 + j] + R[i * 3 + 2] * Ib[6 + j];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        Iw[i * 3 + j] = RI[i * 3] * R[j * 3] + RI[i * 3 + 1] * R[j * 3 + 1] + RI[i * 3 + 2] * R[j * 3 + 2];
    float F[3] = {0.f, 0.f, -9.81f * m}, T[3] = {0.f, 0.f, 0.f};
    for (int l = 0; l < 4; ++l) {
      if (!(cmask & (1u << l))) continue;
      const float rx = ft[l][0] - s[0], ry = ft[l][1] - s[1], rz = ft[l][2] - s[2];
      F[0] += f[l][0]; F[1] += f[l][1]; F[2] += f[l][2];
      T[0] += ry * f[l][2] - rz * f[l][1];
      T[1] += rz * f[l][0] - rx * f[l][2];
      T[2] += rx * f[l][1] - ry * f[l][0];
    }
    const float* w = &s[9];
    const float Iww[3] = {Iw[0] * w[0] + Iw[1] * w[1] + Iw[2] * w[2],
                          Iw[3] * w[0] + Iw[4] * w[1] + Iw[5] * w[2],
                          Iw[6] * w[0] + Iw[7] * w[1] + Iw[8] * w[2]};
    const float rhs[3] = {T[0] - (w[1] * Iww[2] - w[2] * Iww[1]),
                          T[1] - (w[2] * Iww[0] - w[0] * Iww[2]),
                          T[2] - (w[0] * Iww[1] - w[1] * Iww[0])};
    // w' = I_w^-1 rhs (adjugate)
    const float c00 = Iw[4] * Iw[8] - Iw[5] * Iw[7], c01 = Iw[5] * Iw[6] - Iw[3] * Iw[8],
                c02 = Iw[3] * Iw[7] - Iw[4] * Iw[6];
    const float id = 1.f / (Iw[0] * c00 + Iw[1] * c01 + Iw[2] * c02);
    const float Inv[9] = {c00 * id, (Iw[2] * Iw[7] - Iw[1] * Iw[8]) * id,
                          (Iw[1] * Iw[5] - Iw[2] * Iw[4]) * id, c01 * id,
                          (Iw[0] * Iw[8] - Iw[2] * Iw[6]) * id, (Iw[2] * Iw[3] - Iw[0] * Iw[5]) * id,
                          c02 * id, (Iw[1] * Iw[6] - Iw[0] * Iw[7]) * id,
                          (Iw[0] * Iw[4] - Iw[1] * Iw[3]) * id};
    // semi-implicit Euler: velocities first, positions with the new velocities
    for (int i = 0; i < 3; ++i) s[6 + i] += h * F[i] / m;
    for (int i = 0; i < 3; ++i)
      s[9 + i] += h * (Inv[i * 3] * rhs[0] + Inv[i * 3 + 1] * rhs[1] + Inv[i * 3 + 2] * rhs[2]);
    for (int i = 0; i < 3; ++i) s[i] += h * s[6 + i];
    // ZYX Euler rates from the world angular velocity
    const float rd = (cy * s[9] + sy * s[10]) / cp;
    const float pd = -sy * s[9] + cy * s[10];
    const float yd = s[11] + sp * rd;
    s[3] += h * rd; s[4] += h * pd; s[5] += h * yd;
    t += dt;
  }
  for (int i = 0; i < 12; ++i) x[b * 12 + i] = s[i];
  for (int l = 0; l < 4; ++l)
    for (int a = 0; a < 3; ++a) feet[(b * 4 + l) * 3 + a] = ft[l][a];
  in_contact[b] = cmask;
}

}  // namespace cmpc
