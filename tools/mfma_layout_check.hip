// Check of the v_mfma_f32_16x16x4_f32 operand/result maps the solver relies on
// (cdna_hip_programming.md section 3): A operand lane l = A[l&15][l>>4], B operand lane l =
// B[l>>4][l&15], D lane l reg r = D[4*(l>>4)+r][l&15].  Uses the solver's k-permutation
// (step s, lane group g -> k = 4g+s) with asymmetric integer data.
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_layout_check.hip -o /tmp/mfma_check && /tmp/mfma_check
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void k(const float* A, const float* B, float* D) {
  const int l = threadIdx.x, g = l >> 4, c = l & 15;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < 4; ++s) {
    const float a = A[c * 16 + 4 * g + s];  // A[i=c][k=4g+s]
    const float b = B[(4 * g + s) * 16 + c];  // B[k=4g+s][j=c]
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) D[(4 * g + r) * 16 + c] = acc[r];
}

int main() {
  float hA[256], hB[256], hD[256], ref[256];
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      hA[i * 16 + j] = (float)((i * 7 + j * 3) % 11) - 5.f;
      hB[i * 16 + j] = (float)((i * 5 + j * 13) % 9) - 4.f + (i == 2 ? 1.f : 0.f);
    }
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      float s = 0.f;
      for (int q = 0; q < 16; ++q) s += hA[i * 16 + q] * hB[q * 16 + j];
      ref[i * 16 + j] = s;
    }
  float *dA, *dB, *dD;
  hipMalloc(&dA, sizeof hA);
  hipMalloc(&dB, sizeof hB);
  hipMalloc(&dD, sizeof hD);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 256; ++i) bad += hD[i] != ref[i];
  printf("mfma 16x16x4f32 layout check: %s (%d mismatches)\n", bad ? "FAIL" : "OK", bad);
  return bad ? 1 : 0;
}
