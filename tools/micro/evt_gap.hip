// What an event record or a cross-stream wait costs the GPU between two dependent kernels on
// one stream (C2's critical path has several).  Each iteration: kernel A (one workgroup, ~2 us
// of spinning) then kernel B on the same stream, with nothing / an event record / a wait on an
// event already complete on another stream / a wait on an event recorded on another stream
// right before, in between.  Reports the mean GPU time per iteration (events around 200
// iterations).  usage: ./evt_gap
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_spin(double* out, int iters) {
  double v = threadIdx.x;
  for (int i = 0; i < iters; ++i) v = v * 0.999999 + 1e-9;
  if (v == 12345.0) out[threadIdx.x] = v;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  double* out;
  CK(hipMalloc(&out, 4096));
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t t0, t1, ev, ev2, evt;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  CK(hipEventCreate(&evt));
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&ev2, hipEventDisableTiming));
  const int N = 200, spin = 2000;
  const char* names[] = {"plain", "record(notiming)", "record(timing)", "wait(complete,other stream)",
                         "wait(pending,other stream)", "record+wait(same stream event)"};
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 0; mode < 6; ++mode) {
      hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s2, out, 10);
      CK(hipEventRecord(ev2, s2));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(t0, s));
      for (int i = 0; i < N; ++i) {
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, out, spin);
        if (mode == 1) CK(hipEventRecord(ev, s));
        if (mode == 2) CK(hipEventRecord(evt, s));
        if (mode == 3) CK(hipStreamWaitEvent(s, ev2, 0));
        if (mode == 4) {
          hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s2, out, 10);
          CK(hipEventRecord(ev2, s2));
          CK(hipStreamWaitEvent(s, ev2, 0));
        }
        if (mode == 5) {
          CK(hipEventRecord(ev, s));
          CK(hipStreamWaitEvent(s, ev, 0));
        }
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, out, spin);
      }
      CK(hipEventRecord(t1, s));
      CK(hipEventSynchronize(t1));
      float ms;
      CK(hipEventElapsedTime(&ms, t0, t1));
      printf("rep %d %-32s %8.2f us per iteration (2 kernels)\n", rep, names[mode], ms * 1e3 / N);
    }
  return 0;
}
