// cmpc_dynamics.hip -- the reference's discrete dynamics for a batch of robots, on the device
// (com_trajectory.py:221-286).
//
// Ac (com_trajectory.py:224-238) has nonzero blocks only at (pos, vel) = I and (rpy, omega) =
// R_z(yaw_avg)', so Ac^2 = 0 and the zero-order hold of :278 (cont2discrete 'zoh') is exactly
//   Ad   = I + Ac dt,
//   Bd_k = (I dt + Ac dt^2/2) Bc_k,    Bc_k = [0; 0; (1/m)[I I I I]; I^-1[r_1]x .. I^-1[r_4]x]
// and the 50-sample trapezoid of :281-284 integrates the linear expm(Ac t) gc exactly:
//   gd = (I dt + Ac dt^2/2) gc = [0,0,-g dt^2/2, 0,0,0, 0,0,-g dt, 0,0,0].
// Per instance this is a 3x3 inverse, one rotation and 4N 3x3 products: one 64-lane wave per
// robot computes them in fp64, stages Bd (N x 144 floats) in LDS and writes it with coalesced
// 16-byte stores.  HBM-bound: ~1.6 KB read + 9.8 KB written per robot at N = 16.
//
// This file is compiled as part of cmpc_host.hip (single translation unit).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cmpc {

constexpr double kGravity = 9.81;  // com_trajectory.py:268

__global__ void __launch_bounds__(64) dynamics_kernel(int N, double dt, int64_t B,
                                                      const float* __restrict__ mass,
                                                      const float* __restrict__ inertia,
                                                      const float* __restrict__ r_feet,
                                                      const float* __restrict__ xref,
                                                      float* __restrict__ Ad,
                                                      float* __restrict__ Bd,
                                                      float* __restrict__ gd) {
  __shared__ __attribute__((aligned(16))) float bd[16 * 144];
  const int lane = threadIdx.x;
  const double h2 = 0.5 * dt * dt;
  for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
    // per-robot scalars, redundantly per lane (uniform loads): 1/m, I^-1, R_z(yaw_avg)'
    const double minv = 1.0 / (double)mass[b];
    double I[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) I[i] = (double)inertia[b * 9 + i];
    const double c00 = I[4] * I[8] - I[5] * I[7], c01 = I[5] * I[6] - I[3] * I[8],
                 c02 = I[3] * I[7] - I[4] * I[6];
    const double det = I[0] * c00 + I[1] * c01 + I[2] * c02;
    const double id = 1.0 / det;
    double Iinv[9];  // inverse = adjugate / det (row-major)
    Iinv[0] = c00 * id;
    Iinv[1] = (I[2] * I[7] - I[1] * I[8]) * id;
    Iinv[2] = (I[1] * I[5] - I[2] * I[4]) * id;
    Iinv[3] = c01 * id;
    Iinv[4] = (I[0] * I[8] - I[2] * I[6]) * id;
    Iinv[5] = (I[2] * I[3] - I[0] * I[5]) * id;
    Iinv[6] = c02 * id;
    Iinv[7] = (I[1] * I[6] - I[0] * I[7]) * id;
    Iinv[8] = (I[0] * I[4] - I[1] * I[3]) * id;
    // yaw_avg = mean of the reference yaw over the horizon: lanes 0..N-1 load one step each
    // (all in flight at once), summed over the first 16 lanes in fp64 via LDS
    __shared__ double ys[16];
    if (lane < 16) ys[lane] = (lane < N) ? (double)xref[(b * N + lane) * 12 + 5] : 0.0;
    __syncthreads();
    double ysum = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) ysum += ys[k];
    const double yaw = ysum / N;
    const double cy = cos(yaw), sy = sin(yaw);
    // R_z' = [[c, s, 0], [-s, c, 0], [0, 0, 1]]
    const double Rt[9] = {cy, sy, 0.0, -sy, cy, 0.0, 0.0, 0.0, 1.0};

    // Bd_k column block of leg l (12 x 3), lane = 4k + l
    if (lane < 4 * N) {
      const int k = lane >> 2, l = lane & 3;
      const float* r = r_feet + ((b * N + k) * 4 + l) * 3;
      const double rx = r[0], ry = r[1], rz = r[2];
      const double S[9] = {0.0, -rz, ry, rz, 0.0, -rx, -ry, rx, 0.0};  // [r]x
      double W[9], V[9];  // W = I^-1 [r]x (rows 9-11 of Bc), V = R_z' W
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          W[i * 3 + j] = Iinv[i * 3] * S[j] + Iinv[i * 3 + 1] * S[3 + j] + Iinv[i * 3 + 2] * S[6 + j];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          V[i * 3 + j] = Rt[i * 3] * W[j] + Rt[i * 3 + 1] * W[3 + j] + Rt[i * 3 + 2] * W[6 + j];
      float* blk = bd + k * 144 + 3 * l;
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          const double e = (i == a) ? minv : 0.0;
          blk[i * 12 + a] = (float)(h2 * e);               // pos rows: dt^2/2 (1/m) I
          blk[(3 + i) * 12 + a] = (float)(h2 * V[i * 3 + a]);  // rpy rows: dt^2/2 R_z' I^-1 [r]x
          blk[(6 + i) * 12 + a] = (float)(dt * e);          // vel rows: dt (1/m) I
          blk[(9 + i) * 12 + a] = (float)(dt * W[i * 3 + a]);  // omega rows: dt I^-1 [r]x
        }
    }
    __syncthreads();
    // coalesced stores: Bd (N*36 float4), Ad (36 float4), gd (3 float4)
    float4* bo = reinterpret_cast<float4*>(Bd + b * (int64_t)N * 144);
    const float4* bs = reinterpret_cast<const float4*>(bd);
    for (int e = lane; e < N * 36; e += 64) bo[e] = bs[e];
    if (lane < 36) {  // Ad = I + Ac dt, four entries per lane
      float4 v;
      float* pv = reinterpret_cast<float*>(&v);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int o = 4 * lane + q, i = o / 12, j = o % 12;
        double a = (i == j) ? 1.0 : 0.0;
        if (i < 3 && j == i + 6) a += dt;                          // p' = v
        if (i >= 3 && i < 6 && j >= 9) a += dt * Rt[(i - 3) * 3 + (j - 9)];  // rpy' = R_z' w
        pv[q] = (float)a;
      }
      reinterpret_cast<float4*>(Ad + b * 144)[lane] = v;
    }
    if (lane < 12) {
      double g = 0.0;
      if (lane == 2) g = -kGravity * h2;
      if (lane == 8) g = -kGravity * dt;
      gd[b * 12 + lane] = (float)g;
    }
    __syncthreads();
  }
}

}  // namespace cmpc
