// checks the cross-row broadcast on the GPU (all 4 source rows, random doubles)
#include <hip/hip_runtime.h>
#include <stdio.h>
__device__ __forceinline__ unsigned grp_bcast_u32(unsigned x, int kr) {
  const auto h = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  const unsigned y = (kr < 2) ? h[0] : h[1];
  const auto q = __builtin_amdgcn_permlane16_swap(y, y, false, false);
  return (kr & 1) ? q[1] : q[0];
}
__device__ __forceinline__ double grp_bcast_f64(double v, int kr) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = grp_bcast_u32((unsigned)b, kr), hi = grp_bcast_u32((unsigned)(b >> 32), kr);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__global__ void k(const double* in, double* out) {
  const int l = threadIdx.x;
  const double v = in[l];
#pragma unroll
  for (int kr = 0; kr < 4; ++kr) out[kr * 64 + l] = grp_bcast_f64(v, kr);
}
int main() {
  double h[64], o[256], *di, *dout;
  for (int i = 0; i < 64; ++i) h[i] = 1.0 / (i + 1) + i * 1e10;
  hipMalloc(&di, 512); hipMalloc(&dout, 2048);
  hipMemcpy(di, h, 512, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, di, dout);
  hipMemcpy(o, dout, 2048, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int kr = 0; kr < 4; ++kr)
    for (int l = 0; l < 64; ++l) bad += o[kr * 64 + l] != h[(l & 15) + 16 * kr];
  printf("grp_bcast mismatches: %d\n", bad);
  return bad != 0;
}
