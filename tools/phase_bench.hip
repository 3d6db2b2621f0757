// Diagnostic microbenchmark: throughput cost of each solver phase of cmpc_wave.hip at the
// product occupancy (persistent waves, NC = 128, one synthetic QP per wave), in ns per call per
// wave and in CU-cycles per call.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -I include \
//         -I convex-mpc-unitree-go2_amd/csrc tools/phase_bench.hip -o tools/phase_bench
#include <cstdio>
#include "cmpc_wave.hip"
using namespace cmpc;

template <int NC, int PHASE>
__global__ void __launch_bounds__(64, Cfg<NC>::WPE) phase_kernel(KParams P, int n, int reps,
                                                                 float* sink) {
  using C = Cfg<NC>;
  __shared__ Smem<NC> s;
  const int lane = threadIdx.x;
  // synthetic but well-posed instance: A = I + small, B columns random-ish, trot-like params
  for (int e = lane; e < 144; e += 64) s.A[e] = ((e / 12) == (e % 12) ? 1.f : 0.f) + 0.01f * ((e * 7) % 5);
  if (lane < 12) { s.Q2[lane] = P.Q2[lane]; s.R2[lane] = P.R2[lane]; }
  for (int p = lane; p < NC; p += 64) {
    s.Rt[p] = 2e-5f;
    s.par[p] = (p < n) ? (p * P.N) / n : 0;
    s.x[p] = (p < n) ? 1.f : 0.f;
    s.v[p] = s.x[p];
  }
  for (int e = lane; e < NC * 12; e += 64) s.Bt[e] = 0.01f * (((e * 13) % 17) - 8);
  for (int k = lane; k <= P.N; k += 64) {
    int c = 0;
    for (int p = 0; p < n; ++p) c += ((p * P.N) / n < k) ? 1 : 0;
    s.off[k] = c;
  }
  for (int o = lane; o < 12 * P.N; o += 64) { s.D[o] = 0.1f; s.Dt[o] = 0.1f; }
  __syncthreads();
  f4 M[C::NTL];
  condense_tiles<NC>(s, P, M, n, 1e-4f);
  invert_tiles<NC>(s, M, n);
  for (int r = 0; r < reps; ++r) {
    if (PHASE == 0) condense_tiles<NC>(s, P, M, n, 1e-4f + 1e-9f * r);
    if (PHASE == 1) invert_tiles<NC>(s, M, n);
    if (PHASE == 2) symv<NC>(s, M, n, s.x, s.dl);
    if (PHASE == 3) gradient<NC>(s, P, n, s.v, s.g);
  }
  float acc = 0.f;
#pragma unroll
  for (int t = 0; t < C::NTL; ++t) acc += M[t][0] + M[t][3];
  acc += s.dl[lane] + s.g[lane];
  if (acc == 1234.5f) sink[blockIdx.x] = acc;
}

template <int PHASE>
void run(const char* name, int n, int reps) {
  KParams P{};
  P.N = 16;
  const float Q[12] = {1, 1, 50, 10, 20, 1, 2, 2, 1, 1, 1, 1};
  for (int i = 0; i < 12; ++i) { P.Q2[i] = 2 * Q[i]; P.R2[i] = 2e-5f; }
  float* sink;
  (void)hipMalloc(&sink, 1 << 20);
  int cus = 0, nb = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, phase_kernel<128, PHASE>, 64, 0);
  const int grid = cus * nb;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float ms0 = 0, ms1 = 0;
  for (int pass = 0; pass < 2; ++pass) {  // reps and 0 reps: the difference is the phase
    const int rr = pass ? reps : 0;
    hipLaunchKernelGGL((phase_kernel<128, PHASE>), dim3(grid), dim3(64), 0, 0, P, n, rr, sink);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((phase_kernel<128, PHASE>), dim3(grid), dim3(64), 0, 0, P, n, rr, sink);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(pass ? &ms1 : &ms0, a, b);
  }
  const double per_call_ms = (ms1 - ms0) / reps;  // per wave (all waves run concurrently)
  const double cu_cycles = per_call_ms * 1e-3 * 2.1e9 / nb;  // CU-cycles per call per instance
  printf("%-10s n=%d waves/CU=%d  %8.2f us per call per wave  ~%8.0f CU-cycles per call (2.1 GHz)\n",
         name, n, nb, per_call_ms * 1e3, cu_cycles);
  (void)hipFree(sink);
}

int main() {
  run<0>("condense", 120, 20);
  run<1>("invert", 120, 20);
  run<2>("symv", 120, 200);
  run<3>("gradient", 120, 200);
  return 0;
}
