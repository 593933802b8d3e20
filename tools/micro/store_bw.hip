// HBM write-bandwidth ceiling for the K12 builder's store stream (MI355X, gfx950).
//
// The builder writes n_pad x mp doubles (8.39 GB at C3) and reads almost nothing, so its
// roofline is the chip's WRITE bandwidth, not the 8 TB/s spec (a read+write figure).  This
// measures pure store streams of the same size and shape:
//   lin   : each wave instruction stores 1 KiB contiguous (16 B per lane), grid-stride
//   linnt : the same with nontemporal stores (what the builder issues)
//   tile  : the matrix-core builder's pattern -- per instruction 4 rows x 256 B, rows mp * 8 B
//           apart, 16 B per lane (lanes 0-15 one row)
//   read  : a pure read stream (16 B per lane) of the same buffer, for comparison
//   copy  : read + write of two halves
// usage: store_bw [GB]   (default 8.39)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                               \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                               \
    }                                                                        \
  } while (0)

typedef double nt2 __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(256) k_lin(nt2* __restrict__ p, long n2, double v) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long)gridDim.x * 256)
    p[i] = nt2{v, v + 1.0};
}

__global__ void __launch_bounds__(256) k_linnt(nt2* __restrict__ p, long n2, double v) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long)gridDim.x * 256)
    __builtin_nontemporal_store(nt2{v, v + 1.0}, &p[i]);
}

// rows of mp doubles; a workgroup owns 128 columns (blockIdx.x) and walks 64-row blocks
__global__ void __launch_bounds__(256) k_tile(double* __restrict__ K, long nrb, long mp, double v) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, ln = lane & 15, lq = lane >> 4;
  const long j0 = (long)blockIdx.x * 128;
  for (long rb = blockIdx.y; rb < nrb; rb += gridDim.y) {
    const long ib = rb * 64 + 16 * w;
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long i = ib + lq + 4 * r;
        __builtin_nontemporal_store(nt2{v, v}, reinterpret_cast<nt2*>(&K[i * mp + j0 + 32 * p + 2 * ln]));
      }
  }
}

__global__ void __launch_bounds__(256) k_read(const nt2* __restrict__ p, long n2, double* out) {
  double s = 0.0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long)gridDim.x * 256) {
    const nt2 x = p[i];
    s += x.x + x.y;
  }
  if (s == 12345.678) out[0] = s;   // keeps the loads
}

__global__ void __launch_bounds__(256) k_copy(const nt2* __restrict__ a, nt2* __restrict__ b, long n2) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long)gridDim.x * 256) b[i] = a[i];
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? atof(argv[1]) : 8.39;
  const long mp = 1024;
  long nrb = (long)(gb * 1e9 / (64.0 * mp * 8.0));
  const long bytes = nrb * 64 * mp * 8;
  const long n2 = bytes / 16;
  double* buf = nullptr;
  double* out = nullptr;
  CHK(hipMalloc(&buf, bytes));
  CHK(hipMalloc(&out, 64));
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const int reps = 5;
  printf("buffer %.3f GB, %d CUs\n", bytes / 1e9, cus);
  for (int wpc : {4, 8, 16}) {
    const int grid = cus * wpc;
    for (int kind = 0; kind < 5; ++kind) {
      const char* names[5] = {"lin", "linnt", "tile", "read", "copy"};
      auto launch = [&]() {
        if (kind == 0) hipLaunchKernelGGL(k_lin, dim3(grid), dim3(256), 0, 0, (nt2*)buf, n2, 1.0);
        if (kind == 1) hipLaunchKernelGGL(k_linnt, dim3(grid), dim3(256), 0, 0, (nt2*)buf, n2, 1.0);
        if (kind == 2) hipLaunchKernelGGL(k_tile, dim3(mp / 128, grid / (mp / 128)), dim3(256), 0, 0, buf, nrb, mp, 1.0);
        if (kind == 3) hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, (const nt2*)buf, n2, out);
        if (kind == 4) hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, (const nt2*)buf, (nt2*)(buf + bytes / 16), n2 / 2);
      };
      launch();
      CHK(hipDeviceSynchronize());
      CHK(hipEventRecord(a, 0));
      for (int r = 0; r < reps; ++r) launch();
      CHK(hipEventRecord(b, 0));
      CHK(hipEventSynchronize(b));
      float ms = 0.f;
      CHK(hipEventElapsedTime(&ms, a, b));
      const double t = ms / reps * 1e-3;
      printf("wpc %2d  %-6s %8.3f ms  %6.3f TB/s\n", wpc, names[kind], t * 1e3, bytes / t / 1e12);
      fflush(stdout);
    }
  }
  CHK(hipFree(buf));
  return 0;
}
