// Probe of the gfx950 cross-lane moves used by common.h (permlane16/32 swap, DPP row_ror):
// hipcc --offload-arch=gfx950 -O2 -o /tmp/probe_lanes scripts/probe_lanes.hip && /tmp/probe_lanes
// (lane l prints the values it receives; result recorded in profiles/r3_probe_lanes.txt)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out) {
  const unsigned v = threadIdx.x;
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  const auto q = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  const int d8 = __builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);
  const int d4 = __builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);
  out[threadIdx.x * 6 + 0] = r[0];
  out[threadIdx.x * 6 + 1] = r[1];
  out[threadIdx.x * 6 + 2] = q[0];
  out[threadIdx.x * 6 + 3] = q[1];
  out[threadIdx.x * 6 + 4] = d8;
  out[threadIdx.x * 6 + 5] = d4;
}
int main() {
  int* d;
  if (hipMalloc(&d, 64 * 6 * 4) != hipSuccess) return 1;
  k<<<1, 64>>>(d);
  int h[64 * 6];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int l = 0; l < 64; ++l) printf("%2d: p32 %2d %2d  p16 %2d %2d  ror8 %2d ror4 %2d\n", l, h[l*6], h[l*6+1], h[l*6+2], h[l*6+3], h[l*6+4], h[l*6+5]);
  return 0;
}
