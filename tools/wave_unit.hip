// Unit harness (diagnostic, not part of the product): exercises the one-wave building blocks
// of cmpc_wave.hip (block-sweep inversion, symv) on host-given matrices.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I include \
//         -I convex-mpc-unitree-go2_amd/csrc tools/wave_unit.hip -o tools/libwave_unit.so
#include "cmpc_wave.hip"

using namespace cmpc;

// S: NC x NC row-major (only [0,n) used); out: NC x NC row-major inverse (lower tiles mirrored);
// y = inv * x for x given (NC)
template <int NC>
__global__ void __launch_bounds__(64, Cfg<NC>::WPE) k_invert(const float* S, int n, float* out,
                                                            const float* x, float* y) {
  using C = Cfg<NC>;
  __shared__ Smem<NC> s;
  const int lane = threadIdx.x, g = lane >> 4, c = lane & 15;
  f4 M[C::NTL];
#pragma unroll
  for (int I = 0; I < C::TT; ++I)
#pragma unroll
    for (int J = 0; J <= I; ++J) {
      f4 v;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * I + 4 * g + q, col = 16 * J + c;
        v[q] = (row < n && col < n) ? S[row * 192 + col] : (row == col ? 1.f : 0.f);
      }
      M[tile_index(I, J)] = v;
    }
  invert_tiles<NC>(s, M, n);
  for (int p = lane; p < NC; p += 64) s.r[p] = (p < n) ? x[p] : 0.f;
  symv<NC>(s, M, n, s.r, s.dl);
  for (int p = lane; p < NC; p += 64) y[p] = s.dl[p];
#pragma unroll
  for (int I = 0; I < C::TT; ++I)
#pragma unroll
    for (int J = 0; J <= I; ++J) {
      const f4 v = M[tile_index(I, J)];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * I + 4 * g + q, col = 16 * J + c;
        out[row * 192 + col] = v[q];
        out[col * 192 + row] = v[q];
      }
    }
}

extern "C" int wave_invert(const float* S, int n, float* out, const float* x, float* y) {
  float *dS, *dO, *dx, *dy;
  const size_t bytes = 192 * 192 * 4;
  (void)hipMalloc(&dS, bytes); (void)hipMalloc(&dO, bytes);
  (void)hipMalloc(&dx, 768); (void)hipMalloc(&dy, 768);
  (void)hipMemcpy(dS, S, bytes, hipMemcpyHostToDevice);
  (void)hipMemcpy(dx, x, 768, hipMemcpyHostToDevice);
  (void)hipMemset(dO, 0, bytes);
  if (n <= 128) hipLaunchKernelGGL(k_invert<128>, dim3(1), dim3(64), 0, 0, dS, n, dO, dx, dy);
  else if (n <= 160) hipLaunchKernelGGL(k_invert<160>, dim3(1), dim3(64), 0, 0, dS, n, dO, dx, dy);
  else hipLaunchKernelGGL(k_invert<192>, dim3(1), dim3(64), 0, 0, dS, n, dO, dx, dy);
  hipError_t e = hipDeviceSynchronize();
  (void)hipMemcpy(out, dO, bytes, hipMemcpyDeviceToHost);
  (void)hipMemcpy(y, dy, 768, hipMemcpyDeviceToHost);
  (void)hipFree(dS); (void)hipFree(dO); (void)hipFree(dx); (void)hipFree(dy);
  return (int)e;
}

// condensation of one instance (ADMM basis, shift 0): out = H + diag(Rt) over NC x NC
__global__ void __launch_bounds__(64) k_condense(KParams P, const float* Ad, const float* Bd,
                                                 const uint8_t* contact, float* img, float* out,
                                                 int* nout, const float* dvec, const float* vin,
                                                 float* gout, float* Eout) {
  constexpr int NC = 128;
  using C = Cfg<NC>;
  __shared__ Smem<NC> s;
  const int lane = threadIdx.x, g = lane >> 4, c = lane & 15;
  const int N = P.N;
  if (lane < 12) { s.Q2[lane] = P.Q2[lane]; s.R2[lane] = P.R2[lane]; }
  for (int e = lane; e < 144; e += 64) s.A[e] = Ad[e];
  const bool stc = (lane < 4 * N) ? (contact[(lane & 3) * N + (lane >> 2)] != 0) : false;
  const int pos = wave_excl_scan4(stc ? 1 : 0);
  const int ntri = wave_total4(stc ? 1 : 0);
  if (stc) s.tri[pos] = lane;
  if (lane < 4 * N) s.tri_of[lane] = stc ? pos : -1;
  for (int o = lane; o < 12 * N; o += 64) s.D[o] = dvec[o];
  build_admm_basis<NC>(s, P, Bd, ntri);
  const int n = 3 * ntri;
  for (int p = lane; p < n; p += 64) s.v[p] = vin[p];
  gradient<NC>(s, P, n, s.v, s.g);
  for (int p = lane; p < n; p += 64) gout[p] = s.g[p];
  for (int o = lane; o < 12 * N; o += 64) Eout[o] = s.E[o];
  f4 M[C::NTL];
  condense_tiles<NC>(s, P, M, n, 0.f);
  (void)img;
#pragma unroll
  for (int I = 0; I < C::TT; ++I)
#pragma unroll
    for (int J = 0; J <= I; ++J) {
      const f4 v = M[tile_index(I, J)];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * I + 4 * g + q, col = 16 * J + c;
        out[row * NC + col] = v[q];
        out[col * NC + row] = v[q];
      }
    }
  if (lane == 0) *nout = n;
}

extern "C" int wave_condense(const float* Q2, const float* R2, int N, const float* Ad,
                             const float* Bd, const uint8_t* contact, float* out, int* n,
                             const float* dvec, const float* vin, float* gout, float* Eout) {
  KParams P{};
  P.N = N;
  for (int i = 0; i < 12; ++i) { P.Q2[i] = Q2[i]; P.R2[i] = R2[i]; }
  float *dA, *dB, *dimg, *dout;
  uint8_t* dc;
  int* dn;
  (void)hipMalloc(&dA, 144 * 4); (void)hipMalloc(&dB, N * 144 * 4);
  (void)hipMalloc(&dc, 4 * N); (void)hipMalloc(&dimg, Cfg<128>::SLAB * 4);
  (void)hipMalloc(&dout, 128 * 128 * 4); (void)hipMalloc(&dn, 4);
  (void)hipMemset(dimg, 0, Cfg<128>::SLAB * 4);
  float *dd, *dv, *dg, *dE;
  (void)hipMalloc(&dd, 192 * 4); (void)hipMalloc(&dv, 192 * 4);
  (void)hipMalloc(&dg, 192 * 4); (void)hipMalloc(&dE, 192 * 4);
  (void)hipMemcpy(dd, dvec, 192 * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dv, vin, 192 * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dA, Ad, 144 * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, Bd, N * 144 * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dc, contact, 4 * N, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_condense, dim3(1), dim3(64), 0, 0, P, dA, dB, dc, dimg, dout, dn, dd, dv,
                     dg, dE);
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(gout, dg, 192 * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(Eout, dE, 192 * 4, hipMemcpyDeviceToHost);
  hipError_t e = hipDeviceSynchronize();
  (void)hipMemcpy(out, dout, 128 * 128 * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(n, dn, 4, hipMemcpyDeviceToHost);
  (void)hipFree(dA); (void)hipFree(dB); (void)hipFree(dc); (void)hipFree(dimg);
  (void)hipFree(dout); (void)hipFree(dn);
  return (int)e;
}
