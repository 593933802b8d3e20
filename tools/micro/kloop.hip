// k-loop anatomy of the f64 MFMA kernels (k_syrk / k_contract shape): 128x128 tile per
// 256-thread workgroup (4 waves as 2x2 of 64x64, 4x4 v_mfma_f64_16x16x4 fragments per wave),
// BK = 16 per step, register-staged double-buffered LDS, one barrier per step, 2 WGs per CU.
// Variants switch off parts of the loop to locate the matrix-pipe bubbles:
//   MODE 0  full loop (global loads -> regs -> LDS, barrier, LDS fragment reads, MFMA)
//   MODE 1  no global loads (LDS stores of register constants)
//   MODE 2  no global loads, no LDS stores (fragment reads + barrier + MFMA)
//   MODE 3  no barrier (fragment reads + MFMA only)
//   MODE 4  MFMA only (fragments in registers)
//   MODE 5  LDS-DMA staging (k_loop_dma)
// k_loop8: the same tile with 8 waves per workgroup (64 x 32 per wave).  MI355X r1: MODE 2
// 74.4 vs 73.1 TF/s, but the full loop 68.1 vs 69.2 (the 4-wave loop stays)
//   build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o kloop kloop.hip ; run: ./kloop
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int BK = 16, SB = 144;

// EPI > 0: a stand-in for the contraction's per-tile epilogue every 64 steps (one m = 1024 tile):
// the waves wait for their accumulators, then sleep EPI x s_sleep(127) (~8k cycles each) without
// issuing anything -- how much of a latency-bound epilogue do the co-resident waves hide?
// EPI >= 100: instead of sleeping, (EPI - 100) x 256 fp64 FMAs in 8 independent chains per wave
// (EPI >= 200: the same count of fp32 FMAs) -- does VALU arithmetic beside a partner's MFMA
// stream cost more than its issue slots?
__device__ __forceinline__ void fake_epilogue(int epi, double a, double* out) {
  if (a == 1234.5) out[threadIdx.x] = a;   // waits for the accumulator chain
  if (epi >= 200) {
    float v[8];
    for (int c = 0; c < 8; ++c) v[c] = (float)a + c;
    for (int e = 0; e < (epi - 200) * 32; ++e)
#pragma unroll
      for (int c = 0; c < 8; ++c) v[c] = fmaf(v[c], 0.999f, 1e-3f);
    float t = 0.f;
    for (int c = 0; c < 8; ++c) t += v[c];
    if (t == 1234.5f) out[threadIdx.x] = t;
  } else if (epi >= 100) {
    double v[8];
    for (int c = 0; c < 8; ++c) v[c] = a + c;
    for (int e = 0; e < (epi - 100) * 32; ++e)
#pragma unroll
      for (int c = 0; c < 8; ++c) v[c] = fma(v[c], 0.999, 1e-3);
    double t = 0.0;
    for (int c = 0; c < 8; ++c) t += v[c];
    if (t == 1234.5) out[threadIdx.x] = t;
  } else {
    for (int e = 0; e < epi; ++e) __builtin_amdgcn_s_sleep(127);
  }
}

template <int MODE, int EPI = 0>
__global__ void __launch_bounds__(256, 2) k_loop(const double* __restrict__ K, int64_t mp,
                                                 int nsteps, double* out) {
  __shared__ __attribute__((aligned(16))) double Ka[2][BK * SB];
  __shared__ __attribute__((aligned(16))) double Kb[2][BK * SB];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int ta = blockIdx.x % 8, tb = (blockIdx.x / 8) % 8;
  const int64_t rbeg = (int64_t)(blockIdx.x / 64) * nsteps * BK;
  d4 acc[4][4];
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 4; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
  const int lrow = tid >> 4, lc = tid & 15;
  const double2* gA = reinterpret_cast<const double2*>(K + (rbeg + lrow) * mp + ta * 128) + lc;
  const double2* gB = reinterpret_cast<const double2*>(K + (rbeg + lrow) * mp + tb * 128) + lc;
  const int64_t gstep = BK * mp / 2;
  double2 va0, va1, va2, va3, vb0, vb1, vb2, vb3;
  va0 = va1 = va2 = va3 = vb0 = vb1 = vb2 = vb3 = make_double2(1.0 + tid * 1e-9, 1.0);
  auto gload = [&](int step) {
    const int64_t o = (int64_t)step * gstep;
    va0 = gA[o]; va1 = gA[o + 16]; va2 = gA[o + 32]; va3 = gA[o + 48];
    vb0 = gB[o]; vb1 = gB[o + 16]; vb2 = gB[o + 32]; vb3 = gB[o + 48];
  };
  auto sstore = [&](int buf) {
    double2* pa = reinterpret_cast<double2*>(&Ka[buf][lrow * SB]) + lc;
    double2* pb = reinterpret_cast<double2*>(&Kb[buf][lrow * SB]) + lc;
    pa[0] = va0; pa[16] = va1; pa[32] = va2; pa[48] = va3;
    pb[0] = vb0; pb[16] = vb1; pb[32] = vb2; pb[48] = vb3;
  };
  if (MODE == 0 || MODE >= 6) gload(0);
  sstore(0);
  sstore(1);
  __syncthreads();
  double rf[4] = {1.0 + lane * 1e-7, 1.0, 1.0, 1.0};
  for (int step = 0; step < nsteps; ++step) {
    const int cur = step & 1;
    if ((MODE == 0 || MODE >= 6) && step + 1 < nsteps) gload(step + 1);
    const double* As = Ka[cur];
    const double* Bs = Kb[cur];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int krow = kk * 4 + (lane >> 4);
      double af[4], bf[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        if (MODE <= 3 || MODE >= 6) {
          af[f] = As[krow * SB + wr * 64 + f * 16 + (lane & 15)];
          bf[f] = Bs[krow * SB + wc * 64 + f * 16 + (lane & 15)];
        } else {
          af[f] = rf[f];
          bf[f] = rf[(f + kk) & 3];
        }
      }
#pragma unroll
      for (int fm = 0; fm < 4; ++fm)
#pragma unroll
        for (int fn = 0; fn < 4; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[fm], bf[fn], acc[fm][fn], 0, 0, 0);
      // MODE 6 / 7: the next step's LDS stores between the MFMAs of sub-step 1 / 2 instead of
      // after the last one (the buffer is free since the previous barrier)
      if ((MODE == 6 && kk == 1) || (MODE == 7 && kk == 2))
        if (step + 1 < nsteps) sstore(cur ^ 1);
    }
    if (MODE <= 1 && step + 1 < nsteps) sstore(cur ^ 1);
    if (MODE <= 2 || MODE >= 6) __syncthreads();
    if (EPI > 0 && (step & 63) == 63) fake_epilogue(EPI, acc[0][0][0] + acc[3][3][3], out);
  }
  double s = 0.0;
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 4; ++b) s += acc[a][b][0] + acc[a][b][1] + acc[a][b][2] + acc[a][b][3];
  if (s == 1234.5) out[tid] = s;
}

// Prefetch distance 2: global loads for step + 2 are issued at the top of step (two staging
// register sets), so one wave per SIMD (its partner in an epilogue) still covers an HBM round
// trip with two steps of MFMAs instead of one.
template <int EPI>
__global__ void __launch_bounds__(256, 2) k_loop_pf2(const double* __restrict__ K, int64_t mp,
                                                     int nsteps, double* out) {
  __shared__ __attribute__((aligned(16))) double Ka[2][BK * SB];
  __shared__ __attribute__((aligned(16))) double Kb[2][BK * SB];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int ta = blockIdx.x % 8, tb = (blockIdx.x / 8) % 8;
  const int64_t rbeg = (int64_t)(blockIdx.x / 64) * nsteps * BK;
  d4 acc[4][4];
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 4; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
  const int lrow = tid >> 4, lc = tid & 15;
  const double2* gA = reinterpret_cast<const double2*>(K + (rbeg + lrow) * mp + ta * 128) + lc;
  const double2* gB = reinterpret_cast<const double2*>(K + (rbeg + lrow) * mp + tb * 128) + lc;
  const int64_t gstep = BK * mp / 2;
  double2 a0, a1, a2, a3, b0, b1, b2, b3;   // staging set of the even steps
  double2 c0, c1, c2, c3, d0, d1, d2, d3;   // and of the odd steps
#define PF_LOAD(step_, A0, A1, A2, A3, B0, B1, B2, B3)                                   \
  {                                                                                     \
    const int64_t o_ = (int64_t)(step_) * gstep;                                        \
    A0 = gA[o_]; A1 = gA[o_ + 16]; A2 = gA[o_ + 32]; A3 = gA[o_ + 48];                  \
    B0 = gB[o_]; B1 = gB[o_ + 16]; B2 = gB[o_ + 32]; B3 = gB[o_ + 48];                  \
  }
#define PF_STORE(buf_, A0, A1, A2, A3, B0, B1, B2, B3)                                  \
  {                                                                                     \
    double2* pa_ = reinterpret_cast<double2*>(&Ka[buf_][lrow * SB]) + lc;               \
    double2* pb_ = reinterpret_cast<double2*>(&Kb[buf_][lrow * SB]) + lc;               \
    pa_[0] = A0; pa_[16] = A1; pa_[32] = A2; pa_[48] = A3;                              \
    pb_[0] = B0; pb_[16] = B1; pb_[32] = B2; pb_[48] = B3;                              \
  }
  auto compute = [&](int cur) {
    const double* As = Ka[cur];
    const double* Bs = Kb[cur];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int krow = kk * 4 + (lane >> 4);
      double af[4], bf[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        af[f] = As[krow * SB + wr * 64 + f * 16 + (lane & 15)];
        bf[f] = Bs[krow * SB + wc * 64 + f * 16 + (lane & 15)];
      }
#pragma unroll
      for (int fm = 0; fm < 4; ++fm)
#pragma unroll
        for (int fn = 0; fn < 4; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[fm], bf[fn], acc[fm][fn], 0, 0, 0);
    }
  };
  PF_LOAD(0, a0, a1, a2, a3, b0, b1, b2, b3);
  PF_LOAD(1, c0, c1, c2, c3, d0, d1, d2, d3);
  PF_STORE(0, a0, a1, a2, a3, b0, b1, b2, b3);
  __syncthreads();
  for (int step = 0; step < nsteps; step += 2) {   // nsteps even
    // even step: its operands are in LDS buffer 0; refill the even set with step + 2
    if (step + 2 < nsteps) PF_LOAD(step + 2, a0, a1, a2, a3, b0, b1, b2, b3);
    compute(0);
    PF_STORE(1, c0, c1, c2, c3, d0, d1, d2, d3);
    __syncthreads();
    // odd step: buffer 1; refill the odd set with step + 3
    if (step + 3 < nsteps) PF_LOAD(step + 3, c0, c1, c2, c3, d0, d1, d2, d3);
    compute(1);
    if (step + 2 < nsteps) PF_STORE(0, a0, a1, a2, a3, b0, b1, b2, b3);
    __syncthreads();
    if (EPI > 0 && ((step + 1) & 63) == 63) fake_epilogue(EPI, acc[0][0][0] + acc[3][3][3], out);
  }
  double s = 0.0;
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 4; ++b) s += acc[a][b][0] + acc[a][b][1] + acc[a][b][2] + acc[a][b][3];
  if (s == 1234.5) out[tid] = s;
}

template <int EPI>
void run_pf2(const double* K, int64_t mp, int nsteps, double* out, int nwg = 512) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k_loop_pf2<EPI>, dim3(nwg), dim3(256), 0, 0, K, mp, nsteps / 4, out);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_loop_pf2<EPI>, dim3(nwg), dim3(256), 0, 0, K, mp, nsteps, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 128 * 128 * 16 * (double)nsteps * nwg;
  printf("PF2 EPI %2d wgs %d: %.3f ms  %.2f TF/s\n", EPI, nwg, ms, flops / (ms * 1e-3) / 1e12);
}

// Intra-wave interleaving (MODE 0's work): loads and stores unconditional (clamped on the last
// step) so a step is one basic block, and sched_group_barrier asks the scheduler for one
// MFMA, then one LDS read, ... with the eight global loads and eight LDS stores spread over
// the step -- the other instructions issue in the shadow of the MFMAs already in the pipe,
// which matters when a wave has its SIMD to itself.  IL: 0 = no pattern (control).
template <int IL>
__global__ void __launch_bounds__(256, 2) k_loop_il(const double* __restrict__ K, int64_t mp,
                                                    int nsteps, double* out) {
  __shared__ __attribute__((aligned(16))) double Ka[2][BK * SB];
  __shared__ __attribute__((aligned(16))) double Kb[2][BK * SB];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int ta = blockIdx.x % 8, tb = (blockIdx.x / 8) % 8;
  const int64_t rbeg = (int64_t)(blockIdx.x / 64) * nsteps * BK;
  d4 acc[4][4];
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 4; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
  const int lrow = tid >> 4, lc = tid & 15;
  const double2* gA = reinterpret_cast<const double2*>(K + (rbeg + lrow) * mp + ta * 128) + lc;
  const double2* gB = reinterpret_cast<const double2*>(K + (rbeg + lrow) * mp + tb * 128) + lc;
  const int64_t gstep = BK * mp / 2;
  double2 va0, va1, va2, va3, vb0, vb1, vb2, vb3;
  {
    va0 = gA[0]; va1 = gA[16]; va2 = gA[32]; va3 = gA[48];
    vb0 = gB[0]; vb1 = gB[16]; vb2 = gB[32]; vb3 = gB[48];
    double2* pa = reinterpret_cast<double2*>(&Ka[0][lrow * SB]) + lc;
    double2* pb = reinterpret_cast<double2*>(&Kb[0][lrow * SB]) + lc;
    pa[0] = va0; pa[16] = va1; pa[32] = va2; pa[48] = va3;
    pb[0] = vb0; pb[16] = vb1; pb[32] = vb2; pb[48] = vb3;
  }
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    const int cur = step & 1;
    const int nx = step + 1 < nsteps ? step + 1 : step;   // clamped: one basic block per step
    const int64_t o = (int64_t)nx * gstep;
    va0 = gA[o]; va1 = gA[o + 16]; va2 = gA[o + 32]; va3 = gA[o + 48];
    vb0 = gB[o]; vb1 = gB[o + 16]; vb2 = gB[o + 32]; vb3 = gB[o + 48];
    const double* As = Ka[cur];
    const double* Bs = Kb[cur];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int krow = kk * 4 + (lane >> 4);
      double af[4], bf[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        af[f] = As[krow * SB + wr * 64 + f * 16 + (lane & 15)];
        bf[f] = Bs[krow * SB + wc * 64 + f * 16 + (lane & 15)];
      }
#pragma unroll
      for (int fm = 0; fm < 4; ++fm)
#pragma unroll
        for (int fn = 0; fn < 4; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[fm], bf[fn], acc[fm][fn], 0, 0, 0);
    }
    {
      double2* pa = reinterpret_cast<double2*>(&Ka[cur ^ 1][lrow * SB]) + lc;
      double2* pb = reinterpret_cast<double2*>(&Kb[cur ^ 1][lrow * SB]) + lc;
      pa[0] = va0; pa[16] = va1; pa[32] = va2; pa[48] = va3;
      pb[0] = vb0; pb[16] = vb1; pb[32] = vb2; pb[48] = vb3;
    }
    if (IL == 1) {
      // 8 VMEM reads first (one per MFMA), LDS reads one per MFMA, LDS writes in the last
      // quarter, one per MFMA
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);          // MFMA
        if (i < 8) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
        if (i < 32) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0); // DS read
        if (i >= 48 && i < 56) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
      }
    } else if (IL == 2) {
      // DS reads two per MFMA slot in the first half, writes spread over the second half
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (i < 8) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        if ((i & 1) == 0) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        if (i >= 32 && (i & 3) == 0) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      }
    }
    __syncthreads();
  }
  double s = 0.0;
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 4; ++b) s += acc[a][b][0] + acc[a][b][1] + acc[a][b][2] + acc[a][b][3];
  if (s == 1234.5) out[tid] = s;
}

template <int IL>
void run_il(const double* K, int64_t mp, int nsteps, double* out, int nwg) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k_loop_il<IL>, dim3(nwg), dim3(256), 0, 0, K, mp, nsteps / 4, out);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_loop_il<IL>, dim3(nwg), dim3(256), 0, 0, K, mp, nsteps, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 128 * 128 * 16 * (double)nsteps * nwg;
  printf("IL %d wgs %d: %.3f ms  %.2f TF/s\n", IL, nwg, ms, flops / (ms * 1e-3) / 1e12);
}

// BK = 32 per step, double-buffered, one workgroup per CU (launch_bounds(256, 1): up to 512
// VGPRs per wave): half the barriers per MFMA of the BK = 16 loop
template <int SBW>
__global__ void __launch_bounds__(256, 1) k_loop32(const double* __restrict__ K, int64_t mp,
                                                   int nsteps, double* out) {
  constexpr int B2 = 32;
  __shared__ __attribute__((aligned(16))) double Ka[2][B2 * SBW];
  __shared__ __attribute__((aligned(16))) double Kb[2][B2 * SBW];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int ta = blockIdx.x % 8, tb = (blockIdx.x / 8) % 8;
  const int64_t rbeg = (int64_t)(blockIdx.x / 64) * nsteps * B2;
  d4 acc[4][4];
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 4; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
  const int lrow = tid >> 4, lc = tid & 15;   // 16 rows per pass, two passes per step
  const double2* gA = reinterpret_cast<const double2*>(K + (rbeg + lrow) * mp + ta * 128) + lc;
  const double2* gB = reinterpret_cast<const double2*>(K + (rbeg + lrow) * mp + tb * 128) + lc;
  const int64_t gstep = B2 * mp / 2, ghalf = 16 * mp / 2;
  double2 va[8], vb[8];
  auto gload = [&](int step) {
    const int64_t o = (int64_t)step * gstep;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        va[h * 4 + q] = gA[o + h * ghalf + 16 * q];
        vb[h * 4 + q] = gB[o + h * ghalf + 16 * q];
      }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      double2* pa = reinterpret_cast<double2*>(&Ka[buf][(lrow + 16 * h) * SBW]) + lc;
      double2* pb = reinterpret_cast<double2*>(&Kb[buf][(lrow + 16 * h) * SBW]) + lc;
#pragma unroll
      for (int q = 0; q < 4; ++q) { pa[16 * q] = va[h * 4 + q]; pb[16 * q] = vb[h * 4 + q]; }
    }
  };
  gload(0);
  sstore(0);
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    const int cur = step & 1;
    if (step + 1 < nsteps) gload(step + 1);
    const double* As = Ka[cur];
    const double* Bs = Kb[cur];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int krow = kk * 4 + (lane >> 4);
      double af[4], bf[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        af[f] = As[krow * SBW + wr * 64 + f * 16 + (lane & 15)];
        bf[f] = Bs[krow * SBW + wc * 64 + f * 16 + (lane & 15)];
      }
#pragma unroll
      for (int fm = 0; fm < 4; ++fm)
#pragma unroll
        for (int fn = 0; fn < 4; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[fm], bf[fn], acc[fm][fn], 0, 0, 0);
    }
    if (step + 1 < nsteps) sstore(cur ^ 1);
    __syncthreads();
  }
  double s = 0.0;
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 4; ++b) s += acc[a][b][0] + acc[a][b][1] + acc[a][b][2] + acc[a][b][3];
  if (s == 1234.5) out[tid] = s;
}

// MODE 5: operands staged by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave instruction =
// one 128-column k-row of an image) straight into the other LDS buffer: no staging VGPRs, no
// ds_write; each wave issues 8 DMAs per step for step + 1, waits for its own (vmcnt(0)) after
// the MFMAs, then the barrier.
__global__ void __launch_bounds__(256, 2) k_loop_dma(const double* __restrict__ K, int64_t mp,
                                                     int nsteps, double* out) {
  __shared__ __attribute__((aligned(16))) double Ka[2][BK * SB];
  __shared__ __attribute__((aligned(16))) double Kb[2][BK * SB];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int ta = blockIdx.x % 8, tb = (blockIdx.x / 8) % 8;
  const int64_t rbeg = (int64_t)(blockIdx.x / 64) * nsteps * BK;
  d4 acc[4][4];
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 4; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
  // wave wv stages k-rows 4 wv .. 4 wv + 3 of both images
  auto dma = [&](int step, int buf) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int kr = 4 * wv + q;
      const int64_t row = rbeg + (int64_t)step * BK + kr;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(K + row * mp + ta * 128 + 2 * lane),
          (__attribute__((address_space(3))) void*)(&Ka[buf][kr * SB]), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(K + row * mp + tb * 128 + 2 * lane),
          (__attribute__((address_space(3))) void*)(&Kb[buf][kr * SB]), 16, 0, 0);
    }
  };
  dma(0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    const int cur = step & 1;
    if (step + 1 < nsteps) dma(step + 1, cur ^ 1);
    const double* As = Ka[cur];
    const double* Bs = Kb[cur];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int krow = kk * 4 + (lane >> 4);
      double af[4], bf[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        af[f] = As[krow * SB + wr * 64 + f * 16 + (lane & 15)];
        bf[f] = Bs[krow * SB + wc * 64 + f * 16 + (lane & 15)];
      }
#pragma unroll
      for (int fm = 0; fm < 4; ++fm)
#pragma unroll
        for (int fn = 0; fn < 4; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[fm], bf[fn], acc[fm][fn], 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);   // this wave's DMAs for step + 1 have landed
    __syncthreads();
  }
  double s = 0.0;
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 4; ++b) s += acc[a][b][0] + acc[a][b][1] + acc[a][b][2] + acc[a][b][3];
  if (s == 1234.5) out[tid] = s;
}

void run_dma(const double* K, int64_t mp, int nsteps, double* out, int nwg = 512) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k_loop_dma, dim3(nwg), dim3(256), 0, 0, K, mp, nsteps / 4, out);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_loop_dma, dim3(nwg), dim3(256), 0, 0, K, mp, nsteps, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 128 * 128 * 16 * (double)nsteps * nwg;
  printf("MODE 5 (LDS-DMA) wgs %d: %.3f ms  %.2f TF/s\n", nwg, ms, flops / (ms * 1e-3) / 1e12);
}

template <int SBW>
void run32(const double* K, int64_t mp, int nsteps16, double* out, int wgs) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int nsteps = nsteps16 / 2;
  hipLaunchKernelGGL(k_loop32<SBW>, dim3(wgs), dim3(256), 0, 0, K, mp, nsteps / 4, out);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_loop32<SBW>, dim3(wgs), dim3(256), 0, 0, K, mp, nsteps, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 128 * 128 * 32 * (double)nsteps * wgs;
  printf("BK32 SB=%d wgs=%d: %.3f ms  %.2f TF/s\n", SBW, wgs, ms, flops / (ms * 1e-3) / 1e12);
}

template <int MODE, int EPI = 0>
void run(const double* K, int64_t mp, int nsteps, double* out, int nwg = 512) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((k_loop<MODE, EPI>), dim3(nwg), dim3(256), 0, 0, K, mp, nsteps / 4, out);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k_loop<MODE, EPI>), dim3(nwg), dim3(256), 0, 0, K, mp, nsteps, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 128 * 128 * 16 * (double)nsteps * nwg;
  printf("MODE %d EPI %2d wgs %d: %.3f ms  %.2f TF/s\n", MODE, EPI, nwg, ms, flops / (ms * 1e-3) / 1e12);
}


// 8 waves per 128x128 workgroup (2 x 4, 64 x 32 per wave: 4 x 2 fragments, 64 accumulator
// VGPRs), 2 WGs per CU = 4 waves per SIMD: more waves to hide LDS / barrier latency at 1.5x
// the fragment reads per MFMA.  MODE as k_loop (0 full, 2 no global loads / LDS stores).
template <int MODE, int EPI = 0>
__global__ void __launch_bounds__(512, 2) k_loop8(const double* __restrict__ K, int64_t mp,
                                                  int nsteps, double* out) {
  __shared__ __attribute__((aligned(16))) double Ka[2][BK * SB];
  __shared__ __attribute__((aligned(16))) double Kb[2][BK * SB];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 2, wc = wv & 3;
  const int ta = blockIdx.x % 8, tb = (blockIdx.x / 8) % 8;
  const int64_t rbeg = (int64_t)(blockIdx.x / 64) * nsteps * BK;
  d4 acc[4][2];
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
  const int lrow = tid >> 5, lc = tid & 31;   // 16 rows x 32 double2 per operand
  const double2* gA = reinterpret_cast<const double2*>(K + (rbeg + lrow) * mp + ta * 128) + lc;
  const double2* gB = reinterpret_cast<const double2*>(K + (rbeg + lrow) * mp + tb * 128) + lc;
  const int64_t gstep = BK * mp / 2;
  double2 va0, va1, vb0, vb1;
  va0 = va1 = vb0 = vb1 = make_double2(1.0 + tid * 1e-9, 1.0);
  auto gload = [&](int step) {
    const int64_t o = (int64_t)step * gstep;
    va0 = gA[o]; va1 = gA[o + 32];
    vb0 = gB[o]; vb1 = gB[o + 32];
  };
  auto sstore = [&](int buf) {
    double2* pa = reinterpret_cast<double2*>(&Ka[buf][lrow * SB]) + lc;
    double2* pb = reinterpret_cast<double2*>(&Kb[buf][lrow * SB]) + lc;
    pa[0] = va0; pa[32] = va1;
    pb[0] = vb0; pb[32] = vb1;
  };
  if (MODE == 0) gload(0);
  sstore(0);
  sstore(1);
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    const int cur = step & 1;
    if (MODE == 0 && step + 1 < nsteps) gload(step + 1);
    const double* As = Ka[cur];
    const double* Bs = Kb[cur];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int krow = kk * 4 + (lane >> 4);
      double af[4], bf[2];
#pragma unroll
      for (int f = 0; f < 4; ++f) af[f] = As[krow * SB + wr * 64 + f * 16 + (lane & 15)];
#pragma unroll
      for (int f = 0; f < 2; ++f) bf[f] = Bs[krow * SB + wc * 32 + f * 16 + (lane & 15)];
#pragma unroll
      for (int fm = 0; fm < 4; ++fm)
#pragma unroll
        for (int fn = 0; fn < 2; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[fm], bf[fn], acc[fm][fn], 0, 0, 0);
    }
    if (MODE <= 1 && step + 1 < nsteps) sstore(cur ^ 1);
    __syncthreads();
    if (EPI > 0 && (step & 63) == 63) fake_epilogue(EPI, acc[0][0][0] + acc[3][1][3], out);
  }
  double s = 0.0;
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 2; ++b) s += acc[a][b][0] + acc[a][b][1] + acc[a][b][2] + acc[a][b][3];
  if (s == 1234.5) out[tid] = s;
}

template <int MODE, int EPI = 0>
void run8(const double* K, int64_t mp, int nsteps, double* out) {
  const int nwg = 512;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((k_loop8<MODE, EPI>), dim3(nwg), dim3(512), 0, 0, K, mp, nsteps / 4, out);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k_loop8<MODE, EPI>), dim3(nwg), dim3(512), 0, 0, K, mp, nsteps, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 128 * 128 * 16 * (double)nsteps * nwg;
  printf("8-wave MODE %d EPI %2d: %.3f ms  %.2f TF/s\n", MODE, EPI, ms, flops / (ms * 1e-3) / 1e12);
}

int main() {
  const int64_t mp = 1024, rows = 8 * 16 * 4000;   // 8 row chunks x 4000 steps
  double *K, *out;
  hipMalloc(&K, rows * mp * 8);
  hipMalloc(&out, 4096);
  {
    // random operands in (0, 1): switching activity like K12 (DVFS lowers the clock on it)
    double* h = (double*)malloc(rows * mp * 8);
    unsigned long long st = 88172645463325252ull;
    for (int64_t i = 0; i < rows * mp; ++i) {
      st ^= st << 13; st ^= st >> 7; st ^= st << 17;
      h[i] = (double)(st >> 11) * (1.0 / 9007199254740992.0);
    }
    (void)hipMemcpy(K, h, rows * mp * 8, hipMemcpyHostToDevice);
    free(h);
  }
  const int nsteps = 4000;
  if (getenv("KLOOP_ALONE")) {   // one workgroup per CU (one wave per SIMD) vs two
    for (int rep = 0; rep < 2; ++rep) {
      run_il<0>(K, mp, nsteps, out, 512);
      run_il<0>(K, mp, nsteps, out, 256);
      run_il<1>(K, mp, nsteps, out, 512);
      run_il<1>(K, mp, nsteps, out, 256);
      run_il<2>(K, mp, nsteps, out, 512);
      run_il<2>(K, mp, nsteps, out, 256);
      run<4>(K, mp, nsteps, out, 512);
      run<4>(K, mp, nsteps, out, 256);
      run<3>(K, mp, nsteps, out, 512);
      run<3>(K, mp, nsteps, out, 256);
      run<2>(K, mp, nsteps, out, 512);
      run<2>(K, mp, nsteps, out, 256);
      run<0>(K, mp, nsteps, out, 512);
      run<0>(K, mp, nsteps, out, 256);
    }
    return 0;
  }
  if (getenv("KLOOP_EPI")) {   // epilogue-hiding comparison only
    for (int rep = 0; rep < 2; ++rep) {
      run<0>(K, mp, nsteps, out);
      run<0, 6>(K, mp, nsteps, out);
      run<0, 12>(K, mp, nsteps, out);
      run_pf2<0>(K, mp, nsteps, out);
      run_pf2<6>(K, mp, nsteps, out);
      run_pf2<12>(K, mp, nsteps, out);
      run<0, 200>(K, mp, nsteps, out);
      run<0, 201>(K, mp, nsteps, out);
      run<0, 204>(K, mp, nsteps, out);
      run<0, 208>(K, mp, nsteps, out);
      run<0, 216>(K, mp, nsteps, out);
      run_pf2<204>(K, mp, nsteps, out);
    }
    return 0;
  }
  run<0>(K, mp, nsteps, out);
  run_dma(K, mp, nsteps, out);
  run<0>(K, mp, nsteps, out);
  run_dma(K, mp, nsteps, out);
  run32<144>(K, mp, nsteps, out, 256);
  run32<144>(K, mp, nsteps, out, 512);
  run<0>(K, mp, nsteps, out);
  run<1>(K, mp, nsteps, out);
  run<2>(K, mp, nsteps, out);
  run<3>(K, mp, nsteps, out);
  run<4>(K, mp, nsteps, out);
  run<0>(K, mp, nsteps, out);
  run8<0>(K, mp, nsteps, out);
  run8<2>(K, mp, nsteps, out);
  run8<0>(K, mp, nsteps, out);
  run<0>(K, mp, nsteps, out);
  return 0;
}
