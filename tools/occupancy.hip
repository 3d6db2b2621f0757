// Diagnostic: occupancy (blocks per CU) of each bin kernel as the plan computes it.
#include <cstdio>
#include "cmpc_wave.hip"
using namespace cmpc;
template <int NC> void show() {
  int nb = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, solve_bin_kernel<NC>, 64, 0);
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(solve_bin_kernel<NC>));
  printf("NC=%d blocks/CU=%d (err %d) vgpr %d lds %zu private %zu\n", NC, nb, (int)e, a.numRegs,
         a.sharedSizeBytes, a.localSizeBytes);
}
int main() { show<96>(); show<128>(); show<160>(); show<192>(); return 0; }
