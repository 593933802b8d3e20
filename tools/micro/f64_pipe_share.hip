// Do f64 MFMA and f64 VALU work of two waves on one SIMD overlap on gfx950?
// One 512-thread workgroup per CU (two waves per SIMD): waves 0-3 issue NM independent-chain
// v_mfma_f64_16x16x4_f64, waves 4-7 issue NV f64 (or f32) FMAs in 8 independent chains.  Each
// wave stamps s_memtime around its loop.  Modes: 0 MFMA waves only, 1 VALU waves only, 2 both,
// 3 both with the VALU waves at s_setprio 3.
//   build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o f64_pipe_share f64_pipe_share.hip
//   run:   ./f64_pipe_share
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef double d4 __attribute__((ext_vector_type(4)));

template <bool F32>
__global__ void __launch_bounds__(512) k_share(int mode, int nm, int nv, double* out,
                                               unsigned long long* ticks) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool mw = w < 4;
  unsigned long long t0 = 0, t1 = 0;
  double res = 0.0;
  if (mw && mode != 1) {
    d4 acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = d4{0.0, 0.0, 0.0, 0.0};
    double a = 1.0 + lane * 1e-3, b = 0.5 - lane * 1e-4;
    __syncthreads();
    t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < nm; it += 8) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    t1 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 8; ++i) res += acc[i][0] + acc[i][3];
  } else if (!mw && mode != 0) {
    if (mode == 3) __builtin_amdgcn_s_setprio(3);
    __syncthreads();
    t0 = __builtin_amdgcn_s_memtime();
    if constexpr (F32) {
      float x[8];
      for (int i = 0; i < 8; ++i) x[i] = 1.0f + i * 1e-3f + lane * 1e-5f;
      for (int it = 0; it < nv; it += 8) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = fmaf(x[i], 0.999f, 1e-3f);
      }
      for (int i = 0; i < 8; ++i) res += x[i];
    } else {
      double x[8];
      for (int i = 0; i < 8; ++i) x[i] = 1.0 + i * 1e-3 + lane * 1e-5;
      for (int it = 0; it < nv; it += 8) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = fma(x[i], 0.999, 1e-3);
      }
      for (int i = 0; i < 8; ++i) res += x[i];
    }
    t1 = __builtin_amdgcn_s_memtime();
  } else {
    __syncthreads();
  }
  if (lane == 0) ticks[blockIdx.x * 8 + w] = t1 - t0;
  if (res == 123.456) out[threadIdx.x] = res;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  double* out;
  unsigned long long* tk;
  hipMalloc(&out, 4096 * 8);
  hipMalloc(&tk, (size_t)cus * 8 * 8);
  std::vector<unsigned long long> h((size_t)cus * 8);
  const int nm = 4096, nv = 16384;
  const char* names[4] = {"MFMA waves only", "VALU waves only", "both",
                          "both, VALU prio 3"};
  for (int f32 = 0; f32 < 2; ++f32)
    for (int mode = 0; mode < 4; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {
        if (f32) hipLaunchKernelGGL(k_share<true>, dim3(cus), dim3(512), 0, 0, mode, nm, nv, out, tk);
        else hipLaunchKernelGGL(k_share<false>, dim3(cus), dim3(512), 0, 0, mode, nm, nv, out, tk);
        hipDeviceSynchronize();
      }
      hipMemcpy(h.data(), tk, h.size() * 8, hipMemcpyDeviceToHost);
      std::vector<double> m, v;
      for (int c = 0; c < cus; ++c)
        for (int w = 0; w < 8; ++w) (w < 4 ? m : v).push_back((double)h[c * 8 + w]);
      std::sort(m.begin(), m.end());
      std::sort(v.begin(), v.end());
      printf("%s VALU, %-16s: MFMA waves %8.0f ticks (%.1f per MFMA)   VALU waves %8.0f ticks "
             "(%.2f per FMA)\n", f32 ? "f32" : "f64", names[mode], m[m.size() / 2],
             m[m.size() / 2] / nm, v[v.size() / 2], v[v.size() / 2] / nv);
    }
  return 0;
}
