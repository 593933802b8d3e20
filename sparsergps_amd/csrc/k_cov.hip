// Covariance-matrix builders and their theta-derivatives on gfx950.
//
// Reference semantics (luisdamiano/sparseRGPs):
//   make_cov_matC / make_cov_mat_ardC   src/covariance_functionsC.cpp:72-169, 191-252
//   dsig_dthetaC / dsig_dtheta_ardC     src/covariance_function_derivativesC.cpp:307-552, 555-722
// The reference fills each matrix with a scalar double loop that copies two rows and looks
// parameters up by name per pair; here one thread owns one (i, j) pair per iteration, rows
// are staged in LDS, knots live in registers and stores are coalesced along the output's
// contiguous dimension.  These kernels are HBM-write-bound (8 B stored per pair).
#include <stdlib.h>

#include "sgp_internal.h"
#include "sgp_probe.h"

namespace {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// kernel value from raw coordinate differences (xi - uj computed per coordinate).  DT is a
// compile-time bound on d (8 or SGP_MAXD): the coordinate loops unroll with a c < d guard, so
// the callers' coordinate arrays stay in registers (runtime-indexed ones went to scratch).
template <int DT>
__device__ __forceinline__ double kvalue(const KernParams& kp, const double* xi,
                                         const double* uj) {
  const int d = kp.d;
  double s = 0.0;
  if (kp.kernel == 0) {
#pragma unroll
    for (int c = 0; c < DT; ++c)
      if (c < d) { double t = xi[c] - uj[c]; s = fma(t, t, s); }
    return kp.sig2 * exp(kp.coef * s);
  } else if (kp.kernel == 1) {
#pragma unroll
    for (int c = 0; c < DT; ++c)
      if (c < d) { double t = (xi[c] - uj[c]) * kp.rl[c]; s = fma(t, t, s); }
    return kp.sig2 * exp(-s / 2.0);
  } else {
#pragma unroll
    for (int c = 0; c < DT; ++c)
      if (c < d) s += fabs(xi[c] - uj[c]);
    return kp.sig2 * exp(kp.coef * s);
  }
}

// d K / d log theta_param for one pair (covariance_function_derivativesC.cpp:35-171, 232-301)
template <int DT>
__device__ __forceinline__ double dkvalue(const KernParams& kp, const double* xi,
                                          const double* uj, int param, bool sym) {
  const int d = kp.d;
  if (param == kp.P - 1) {  // tau: 2 tau^2 iff all(x1 == x2)   (l.157-163)
    if (kp.kernel == 2 && !sym) return 0.0;   // exp cross-mode returns zeros (l.520)
    bool eq = true;
#pragma unroll
    for (int c = 0; c < DT; ++c)
      if (c < d) eq = eq && (xi[c] == uj[c]);
    return eq ? 2.0 * kp.tau * kp.tau : 0.0;
  }
  if (kp.kernel == 0) {
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < DT; ++c)
      if (c < d) { double t = xi[c] - uj[c]; s = fma(t, t, s); }
    double e = exp(kp.coef * s);
    if (param == 0) return 2.0 * kp.sigma * e * kp.sigma;                       // l.47
    return (kp.sig2 * e) * ((1.0 / (kp.l[0] * kp.l[0] * kp.l[0])) * s) * kp.l[0];  // l.98-99
  } else if (kp.kernel == 1) {
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < DT; ++c)
      if (c < d) { double t = (xi[c] - uj[c]) * kp.rl[c]; s = fma(t, t, s); }
    double e = exp(-(s / 2.0));
    if (param == 0) return 2.0 * kp.sigma * e * kp.sigma;                       // l.78
    const int c = param - 1;
    const double lc = kp.l[c];
    double dc = 0.0;   // xi[c] - uj[c] without a runtime register index
#pragma unroll
    for (int q = 0; q < DT; ++q)
      if (q == c) dc = xi[q] - uj[q];
    return (kp.sig2 * e) * ((1.0 / (lc * lc * lc)) * (dc * dc)) * lc;          // l.133-134
  } else {  // exp: derivatives use the L2 distance (quirk Q12, l.244, 264)
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < DT; ++c)
      if (c < d) { double t = xi[c] - uj[c]; s = fma(t, t, s); }
    double dist = sqrt(s);
    double e = exp(-(1.0 / kp.l[0]) * dist);
    if (param == 0) return 2.0 * kp.sigma * e * kp.sigma;
    return (kp.sig2 * e) * ((1.0 / (kp.l[0] * kp.l[0])) * dist) * kp.l[0];
  }
}

// Layer-1 filler: out (n x np, column-major).  Block = 64 rows x 4 column lanes.
template <bool DERIV, int DT>
__global__ void __launch_bounds__(256) k_fill(KernParams kp, const double* __restrict__ x,
                                              int64_t n, int64_t ldx,
                                              const double* __restrict__ xp, int64_t np,
                                              int64_t ldxp, int sym, int param,
                                              double* __restrict__ out, int64_t ldo,
                                              int cols_per_block) {
  const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
  const int64_t j0 = (int64_t)blockIdx.y * cols_per_block;
  double xi[DT], uj[DT];
#pragma unroll
  for (int c = 0; c < DT; ++c) xi[c] = (i < n && c < kp.d) ? x[i + c * ldx] : 0.0;
  for (int64_t jj = threadIdx.y; jj < cols_per_block; jj += 4) {
    const int64_t j = j0 + jj;
    if (j >= np) break;
#pragma unroll
    for (int c = 0; c < DT; ++c) uj[c] = (c < kp.d) ? xp[j + c * ldxp] : 0.0;
    if (i >= n) continue;
    double v;
    if (DERIV) {
      v = dkvalue<DT>(kp, xi, uj, param, sym != 0);
    } else {
      v = kvalue<DT>(kp, xi, uj);
      if (sym && i == j) v = v + kp.tau2 + kp.delta;   // covariance_functionsC.cpp:91
    }
    out[i + j * ldo] = v;
  }
}

// K12 row-major (n_pad x mp).  Block: 64 knot columns (lanes) x 4 row groups; each block
// walks 64-row blocks blockIdx.y, blockIdx.y + gridDim.y, ...  Row coordinates (pre-scaled by
// 1/l_c for ARD) are staged in LDS and read as wave-wide broadcasts; the lane's knot stays in
// registers; one coalesced 512-B store per row.  Row blocks [rb0, rb1).
template <bool ARD, int DT>
__global__ void __launch_bounds__(256) k_build_knm(KernParams kp, const double* __restrict__ X,
                                                   int64_t ldx, int64_t n,
                                                   const double* __restrict__ U, int64_t ldu,
                                                   int64_t m, int64_t mp,
                                                   double* __restrict__ K,
                                                   const double* __restrict__ rvec,
                                                   double* __restrict__ tslab, int64_t rb0,
                                                   int64_t rb1) {
  // block: 128 knot columns (two adjacent per lane, one 16-byte store per lane and row: 1 KiB
  // per wave-instruction) x 4 row groups
  __shared__ __attribute__((aligned(16))) double xs[64 * DT];
  __shared__ double rsh[64];
  __shared__ double tsh[4][128];
  const int d = kp.d;
  const int64_t j = (int64_t)blockIdx.x * 128 + 2 * threadIdx.x;
  const int tid = threadIdx.y * 64 + threadIdx.x;
  double u0[DT], u1[DT];
  const bool jv0 = j < m, jv1 = j + 1 < m;
#pragma unroll
  for (int c = 0; c < DT; ++c) {
    const double sc = ARD ? kp.rl[c] : 1.0;
    u0[c] = (jv0 && c < d) ? (ARD ? U[j + c * ldu] * sc : U[j + c * ldu]) : 0.0;
    u1[c] = (jv1 && c < d) ? (ARD ? U[j + 1 + c * ldu] * sc : U[j + 1 + c * ldu]) : 0.0;
  }
  const double sig2 = kp.sig2;
  const double scale = ARD ? -0.5 : kp.coef;
  for (int64_t rb = rb0 + blockIdx.y; rb < rb1; rb += gridDim.y) {
    const int64_t i0 = rb * 64;
    __syncthreads();   // the previous row block's xs / rsh / tsh reads are done
    for (int e = tid; e < 64 * DT; e += 256) {
      const int r = e / DT, c = e % DT;
      const int64_t i = i0 + r;
      double v = 0.0;
      if (c < d && i < n) v = ARD ? X[i + c * ldx] * kp.rl[c] : X[i + c * ldx];
      xs[e] = v;
    }
    if (rvec && tid < 64) rsh[tid] = (i0 + tid < n) ? rvec[i0 + tid] : 0.0;
    double tp0 = 0.0, tp1 = 0.0;
    __syncthreads();
    for (int r = threadIdx.y; r < 64; r += 4) {
      const int64_t i = i0 + r;
      const double2* xr = reinterpret_cast<const double2*>(&xs[r * DT]);
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int c2 = 0; c2 < DT / 2; ++c2) {
        const double2 xv = xr[c2];
        const double a0 = xv.x - u0[2 * c2], a1 = xv.y - u0[2 * c2 + 1];
        const double b0 = xv.x - u1[2 * c2], b1 = xv.y - u1[2 * c2 + 1];
        s0 = fma(a0, a0, s0);
        s0 = fma(a1, a1, s0);
        s1 = fma(b0, b0, s1);
        s1 = fma(b1, b1, s1);
      }
      const bool iv = i < n;
      const double v0 = (jv0 && iv) ? sig2 * sgp_exp_nonpos(scale * s0) : 0.0;
      const double v1 = (jv1 && iv) ? sig2 * sgp_exp_nonpos(scale * s1) : 0.0;
      // streaming store (nontemporal): K12 is re-read only by the next kernel, long after it
      // has left the caches
      typedef double nt2 __attribute__((ext_vector_type(2)));
      __builtin_nontemporal_store(nt2{v0, v1}, reinterpret_cast<nt2*>(&K[i * mp + j]));
      if (rvec) {
        tp0 = fma(v0, rsh[r], tp0);
        tp1 = fma(v1, rsh[r], tp1);
      }
    }
    if (rvec) {   // t_j partial of this block's 64 rows, fixed combination order
      tsh[threadIdx.y][2 * threadIdx.x] = tp0;
      tsh[threadIdx.y][2 * threadIdx.x + 1] = tp1;
      __syncthreads();
      if (threadIdx.y < 2) {
        const int cc = threadIdx.y * 64 + threadIdx.x;
        tslab[rb * mp + (int64_t)blockIdx.x * 128 + cc] =
            ((tsh[0][cc] + tsh[1][cc]) + tsh[2][cc]) + tsh[3][cc];
      }
    }
  }
}

// K12 row-major (n_pad x mp) on the matrix cores, d <= 4 NC (NC = 2, 4, 8), sqexp / ARD.
// The exponent log(sig2) - 1/2 |x~ - u~|^2 (x~ = (x - ctr) / l per coordinate, ctr = the
// knots' mean) is one GEMM with inner dimension 4 NC + 4 over augmented coordinates
//   A_i = [x~_i (4 NC), -|x~_i|^2 / 2, 1, 1, 0]    B_j = [u~_j (4 NC), 1, -|u~_j|^2 / 2, log sig2, 0]
// i.e. NC + 1 v_mfma_f64_16x16x4_f64 per 16 x 16 tile (lane l >> 4 feeds coordinates
// 4 k + (l >> 4) of chunk k), so the VALU only evaluates exp (the per-pair coordinate
// differences of k_build_knm cost ~40 % of its VALU work, which then matched the store time);
// padding rows / knots carry -1e300 in the |.|^2 slot, so the clamped exponent gives exactly 0
// there without a select.  The expansion's rounding is ~1e-16 (|x~|^2 + |u~|^2) absolute in the
// exponent -- ~1e-14 relative in K at the configs' scales, centring keeps it there for data far
// from the origin.  Block: 4 waves x 16 rows of a 64-row block, 128 knots; tile 2p (2p+1) holds
// knots j0 + 32p + 2 l' (+1) in MFMA column l' = lane & 15, so each lane stores its two adjacent
// knots as one 16-byte store (lanes 0-15: 256 contiguous bytes of one row).  Persistent over
// row blocks rb0 + blockIdx.y + k gridDim.y; with t, the workgroup's t = K^T r partial over all
// its row blocks goes to slot slot0 + blockIdx.y of tslab (fixed order: deterministic).
// t's running sums live in LDS, not registers: lane (w, lq, l') owns the two doubles of its
// columns in tacc_s[w][lq], a private read-modify-write per tile pair and row block (no other
// lane touches them, so no atomics), and r reaches the lanes as one value per lane (row ia)
// broadcast by shuffles.  In registers (8 sums, 4 + 4 r values) the with-t builder needed 162
// VGPRs, i.e. 3 workgroups per CU against the t-free builder's 4 (VI's build 1.67 ms against
// FITC's 1.50 ms for the same K12); the sums and their reduction order are unchanged, so t is
// bit-identical to the register form.
template <bool WITH_T, int NC>
__global__ void __launch_bounds__(256, NC > 4 ? (WITH_T ? 2 : 3) : ((WITH_T && NC == 2) ? SGP_BUILD_OCC_T2 : 4))
k_build_knm_mfma(KernParams kp, const double* __restrict__ X, int64_t ldx, int64_t n,
                 const double* __restrict__ U, int64_t ldu, int64_t m, int64_t mp,
                 double* __restrict__ K, const double* __restrict__ rvec,
                 double* __restrict__ tslab, int64_t slot0, int64_t rb0, int64_t rb1) {
  typedef double nt2 __attribute__((ext_vector_type(2)));
  __shared__ nt2 tacc_s[WITH_T ? 16 : 1][64];   // [wave][lq][tile pair p][lane & 15]
  __shared__ double etab[32];
  if (threadIdx.x < 32) etab[threadIdx.x] = kp.et[threadIdx.x];
  if (WITH_T)
    for (int e = threadIdx.x; e < 16 * 64; e += 256) tacc_s[e >> 6][e & 63] = nt2{0.0, 0.0};
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ln = lane & 15, lq = lane >> 4;
  const int d = kp.d;
  bool fc[NC];                  // this lane's coordinate of chunk k: 4 k + lq
  double ct[NC], rl[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    fc[k] = 4 * k + lq < d;
    ct[k] = fc[k] ? kp.ctr[4 * k + lq] : 0.0;
    rl[k] = fc[k] ? kp.rl[4 * k + lq] : 0.0;
  }
  const int64_t j0 = (int64_t)blockIdx.x * 128;
  // knot fragments: in registers for d <= 8 without t; for wider d (4 NC + 4 per lane and
  // tile), or beside t's row values, they would not fit within 128 VGPRs (4 workgroups per
  // CU), so they sit in LDS as [chunk][tile][lane] (each read one conflict-free ds_read_b64),
  // written by wave w for tiles 2w, 2w + 1
  constexpr bool BL = NC > 2 || WITH_T;
  __shared__ double sbf[BL ? (NC + 1) * 8 * 64 : 1];
  double bc[BL ? 1 : NC][8], b2[BL ? 1 : 8];
#pragma unroll
  for (int tt = 0; tt < 8; ++tt) {
    if (BL && (tt >> 1) != w) continue;
    const int64_t j = j0 + 32 * (tt >> 1) + 2 * ln + (tt & 1);
    const bool jv = j < m;
    double u2 = 0.0;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const double u = (jv && fc[k]) ? (U[j + (4 * k + lq) * ldu] - ct[k]) * rl[k] : 0.0;
      if constexpr (BL) sbf[(k * 8 + tt) * 64 + lane] = u;
      else bc[k][tt] = u;
      u2 = fma(u, u, u2);
    }
    u2 += __shfl_xor(u2, 16, 64);
    u2 += __shfl_xor(u2, 32, 64);
    // padding knots: an exponent of -1e300 (clamped to -746 below) gives K = 0 with no
    // per-pair select
    const double bv = lq == 0 ? 1.0 : (lq == 1 ? (jv ? -0.5 * u2 : -1e300) : (lq == 2 ? kp.lsig2 : 0.0));
    if constexpr (BL) sbf[(NC * 8 + tt) * 64 + lane] = bv;
    else b2[tt] = bv;
  }
  if constexpr (BL) __syncthreads();
  auto bfr = [&](int k, int tt) -> double {
    if constexpr (BL) return sbf[(k * 8 + tt) * 64 + lane];
    else return k < NC ? bc[k][tt] : b2[tt];
  };
  const double ehi = kp.lsig2;
  nt2* const tl = &tacc_s[4 * w + lq][0];       // this lane's t sums: tl[16 p + ln]
  // The next row block's coordinates and r are loaded before this block's stores: vmcnt
  // counts loads and stores in issue order, so loads issued after the stores would make every
  // block wait for the previous block's 16 stores to drain.
  double xn[NC], rn = 0.0;
  auto load_rows = [&](int64_t rb) {
    const int64_t ia = rb * 64 + 16 * w + ln;   // X (and r) are zero-padded to n_pad rows
#pragma unroll
    for (int k = 0; k < NC; ++k) xn[k] = fc[k] ? X[ia + (4 * k + lq) * ldx] : 0.0;
    if (WITH_T) rn = rvec[ia];
  };
#pragma unroll
  for (int k = 0; k < NC; ++k) xn[k] = 0.0;
  if (rb0 + (int64_t)blockIdx.y < rb1) load_rows(rb0 + blockIdx.y);
  for (int64_t rb = rb0 + blockIdx.y; rb < rb1; rb += gridDim.y) {
    const int64_t ib = rb * 64 + 16 * w;
    const int64_t ia = ib + ln;                 // this lane's A row
    double ac[NC], x2 = 0.0;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      ac[k] = fc[k] ? (xn[k] - ct[k]) * rl[k] : 0.0;
      x2 = fma(ac[k], ac[k], x2);
    }
    const double rcur = rn;
    if (rb + gridDim.y < rb1) load_rows(rb + gridDim.y);
    double rr[4];   // r of this lane's output rows lq + 4 r (held by lanes lq + 4 r)
#pragma unroll
    for (int r = 0; r < 4; ++r) rr[r] = WITH_T ? __shfl(rcur, lq + 4 * r, 64) : 0.0;
    x2 += __shfl_xor(x2, 16, 64);
    x2 += __shfl_xor(x2, 32, 64);
    // exponent = x~.u~ - |x~|^2 / 2 - |u~|^2 / 2 + log(sig2); padding rows as padding knots
    const double a2 = lq == 0 ? (ia < n ? -0.5 * x2 : -1e300) : (lq <= 2 ? 1.0 : 0.0);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const d4 z = {0.0, 0.0, 0.0, 0.0};
      d4 e0 = __builtin_amdgcn_mfma_f64_16x16x4f64(ac[0], bfr(0, 2 * p), z, 0, 0, 0);
      d4 e1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ac[0], bfr(0, 2 * p + 1), z, 0, 0, 0);
#pragma unroll
      for (int k = 1; k < NC; ++k) {
        e0 = __builtin_amdgcn_mfma_f64_16x16x4f64(ac[k], bfr(k, 2 * p), e0, 0, 0, 0);
        e1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ac[k], bfr(k, 2 * p + 1), e1, 0, 0, 0);
      }
      e0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a2, bfr(NC, 2 * p), e0, 0, 0, 0);
      e1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a2, bfr(NC, 2 * p + 1), e1, 0, 0, 0);
      nt2 ta = WITH_T ? tl[16 * p + ln] : nt2{0.0, 0.0};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // K = exp(exponent) <= sig2: clamp the rounding above log(sig2), and below at -746
        // (where exp underflows to 0)
        const double v0 = sgp_exp_tab(fmin(fmax(e0[r], -746.0), ehi), kp, etab);
        const double v1 = sgp_exp_tab(fmin(fmax(e1[r], -746.0), ehi), kp, etab);
        const int64_t i = ib + lq + 4 * r;
        __builtin_nontemporal_store(nt2{v0, v1},
                                    reinterpret_cast<nt2*>(&K[i * mp + j0 + 32 * p + 2 * ln]));
        if (WITH_T) {
          ta.x = fma(v0, rr[r], ta.x);
          ta.y = fma(v1, rr[r], ta.y);
        }
      }
      if (WITH_T) tl[16 * p + ln] = ta;
      // keep each tile pair's four stores where they are: left to itself the scheduler sinks
      // all 16 to the end of the block, so a wave alternates a store burst with a long
      // store-free VALU stretch
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (WITH_T) {
    // column cc = 32 p + 2 l' + h: per wave (lq 0 + lq 1) + (lq 2 + lq 3), then the waves in order
    __syncthreads();
    if (threadIdx.x < 128) {
      const int cc = threadIdx.x, sl = 16 * (cc >> 5) + ((cc >> 1) & 15), h = cc & 1;
      double v[4];
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) {
        const double* q0 = reinterpret_cast<const double*>(&tacc_s[4 * ww][sl]) + h;
        v[ww] = (q0[0] + q0[128]) + (q0[256] + q0[384]);
      }
      tslab[(slot0 + blockIdx.y) * mp + j0 + cc] = ((v[0] + v[1]) + v[2]) + v[3];
    }
  }
}

// K22 (mp x mp, row-major) with diagonal ((sig2 + tau2 + delta) - diag_sub), identity padding.
// K22 (symmetric mode, nugget on the diagonal).  DT = compile-time coordinate bound so the
// knot coordinates stay in registers (a runtime-sized local array went to scratch: 108 us at
// m = 1024 against ~5 us).  Same per-pair arithmetic and summation order as kvalue().
template <int DT>
__global__ void __launch_bounds__(256) k_build_kmm(KernParams kp, const double* __restrict__ U,
                                                   int64_t ldu, int64_t m, int64_t mp,
                                                   double diag_sub, double* __restrict__ K22,
                                                   double* __restrict__ K22b) {
  const int64_t k = (int64_t)blockIdx.x * 64 + threadIdx.x;
  const int64_t j = (int64_t)blockIdx.y * 4 + threadIdx.y;
  if (j >= mp || k >= mp) return;
  double v;
  if (j < m && k < m) {
    const int d = kp.d;
    double s = 0.0;
    if (kp.kernel == 0) {
#pragma unroll
      for (int c = 0; c < DT; ++c)
        if (c < d) { const double t = U[j + c * ldu] - U[k + c * ldu]; s = fma(t, t, s); }
      v = kp.sig2 * exp(kp.coef * s);
    } else if (kp.kernel == 1) {
#pragma unroll
      for (int c = 0; c < DT; ++c)
        if (c < d) {
          const double t = (U[j + c * ldu] - U[k + c * ldu]) * kp.rl[c];
          s = fma(t, t, s);
        }
      v = kp.sig2 * exp(-s / 2.0);
    } else {
#pragma unroll
      for (int c = 0; c < DT; ++c)
        if (c < d) s += fabs(U[j + c * ldu] - U[k + c * ldu]);
      v = kp.sig2 * exp(kp.coef * s);
    }
    if (j == k) v = ((v + kp.tau2) + kp.delta) - diag_sub;
  } else {
    v = (j == k) ? 1.0 : 0.0;
  }
  K22[j * mp + k] = v;
  if (K22b) K22b[j * mp + k] = v;   // the copy the in-place inverse starts from
}

// sum_{j,k<m} G22_jk dK22^p_jk with
//   G22 = a u_j u_k + b (Ainv - Binv)_jk + c M3_jk + e (v_j w_k + w_j v_k)   (v, w optional).
// Per block partial sums of P records: sigma, the length scales, and the tau-coincidence sum
// sum_{u_j == u_k} G22_jk (dK22/dlog tau = 2 tau^2 there; used by the Laplace path, whose
// K22 keeps tau^2 -- the Gaussian paths zero dK22/dtau, vi_functions.R:313-316).
template <int DT>
__global__ void __launch_bounds__(256) k_contract_kmm(KernParams kp, const double* __restrict__ U,
                                                      int64_t ldu, int64_t m, int64_t mp,
                                                      const double* __restrict__ uvec,
                                                      const double* __restrict__ Ainv,
                                                      const double* __restrict__ Binv,
                                                      const double* __restrict__ M3, double a,
                                                      double b, double c,
                                                      const double* __restrict__ vvec,
                                                      const double* __restrict__ wvec, double e2,
                                                      double* __restrict__ slab) {
  // one block per knot row j; compile-time coordinate loops keep everything in registers
  __shared__ double red[4][DT + 2];
  const int np = kp.P, d = kp.d;
  const int64_t j = blockIdx.x;
  double uj[DT], acc[DT + 2];
#pragma unroll
  for (int q = 0; q < DT; ++q) uj[q] = (q < d) ? U[j + q * ldu] : 0.0;
#pragma unroll
  for (int p = 0; p < DT + 2; ++p) acc[p] = 0.0;
  const double auj = a * uvec[j];
  const double vj = vvec ? vvec[j] : 0.0, wj = vvec ? wvec[j] : 0.0;
  for (int64_t k = threadIdx.x; k < m; k += 256) {
    double uk[DT];
    bool same = true;
#pragma unroll
    for (int q = 0; q < DT; ++q) {
      uk[q] = (q < d) ? U[k + q * ldu] : 0.0;
      same = same && (uj[q] == uk[q]);
    }
    const int64_t o = j * mp + k;
    double g = auj * uvec[k] + b * (Ainv[o] - Binv[o]) + c * M3[o];
    if (vvec) g += e2 * (vj * wvec[k] + wj * vvec[k]);
    const double kv = kvalue<DT>(kp, uj, uk);
    const double gk = g * kv;
    acc[0] += 2.0 * gk;                                   // sigma: dK/dlog sigma = 2K
    if (kp.kernel == 0) {
      double s = 0.0;
#pragma unroll
      for (int q = 0; q < DT; ++q) {
        if (q < d) { const double t = uj[q] - uk[q]; s = fma(t, t, s); }
      }
      acc[1] += gk * s * kp.rl2[0];
    } else {
#pragma unroll
      for (int q = 0; q < DT; ++q) {
        if (q < d) {
          const double t = (uj[q] - uk[q]) * kp.rl[q];
          acc[1 + q] += gk * t * t;
        }
      }
    }
    if (same) acc[DT + 1] += g;                           // tau coincidence sum
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int p = 0; p < DT + 2; ++p) {
    const double v = wave_sum(acc[p]);
    if (lane == 0) red[w][p] = v;
  }
  __syncthreads();
  // record layout: [sigma, length scales (L), tau-coincidence] -> P fields
  if (threadIdx.x < np) {
    const int src = (threadIdx.x == np - 1) ? DT + 1 : threadIdx.x;
    slab[j * np + threadIdx.x] = red[0][src] + red[1][src] + red[2][src] + red[3][src];
  }
}

// Knot part of the m x m contraction for d K22 / d u_kc = e_k v^T + v e_k^T,
// v_l = K22_lk (u_lc - u_kc) / l_c^2: one block per knot k, out[k*d + c] =
// 2 sum_l G22_kl K22_kl (u_lc - u_kc) (raw coordinates; the 1/l_c^2 is applied by the caller).
template <int DT>
__global__ void __launch_bounds__(256) k_knot_kmm(KernParams kp, const double* __restrict__ U,
                                                  int64_t ldu, int64_t m, int64_t mp,
                                                  const double* __restrict__ uvec,
                                                  const double* __restrict__ Ainv,
                                                  const double* __restrict__ Binv,
                                                  const double* __restrict__ M3, double a,
                                                  double b, double c,
                                                  const double* __restrict__ vvec,
                                                  const double* __restrict__ wvec, double e2,
                                                  double* __restrict__ out) {
  __shared__ double red[4][DT];
  const int64_t k = blockIdx.x;
  double uk[DT], acc[DT];
#pragma unroll
  for (int q = 0; q < DT; ++q) {
    uk[q] = (q < kp.d) ? U[k + q * ldu] : 0.0;
    acc[q] = 0.0;
  }
  for (int64_t l = threadIdx.x; l < m; l += 256) {
    double ul[DT];
#pragma unroll
    for (int q = 0; q < DT; ++q) ul[q] = (q < kp.d) ? U[l + q * ldu] : 0.0;
    const int64_t o = k * mp + l;
    double g = a * uvec[k] * uvec[l] + b * (Ainv[o] - Binv[o]) + c * M3[o];
    if (vvec) g += e2 * (vvec[k] * wvec[l] + wvec[k] * vvec[l]);
    const double gk = 2.0 * g * kvalue<DT>(kp, ul, uk);
#pragma unroll
    for (int q = 0; q < DT; ++q) acc[q] = fma(gk, ul[q] - uk[q], acc[q]);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < DT; ++q) {
    double v = wave_sum(acc[q]);
    if (lane == 0) red[w][q] = v;
  }
  __syncthreads();
  if (threadIdx.x < kp.d)
    out[k * kp.d + threadIdx.x] =
        red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

}  // namespace

hipError_t launch_knot_kmm(const KernParams& kp, const double* U, int64_t ldu, int64_t m,
                           int64_t mp, const double* uvec, const double* Ainv,
                           const double* Binv, const double* M3, double a, double b, double c,
                           const double* vvec, const double* wvec, double e2, double* out,
                           hipStream_t s) {
  if (kp.d <= 8)
    hipLaunchKernelGGL(k_knot_kmm<8>, dim3((unsigned)m), dim3(256), 0, s, kp, U, ldu, m, mp, uvec,
                       Ainv, Binv, M3, a, b, c, vvec, wvec, e2, out);
  else
    hipLaunchKernelGGL(k_knot_kmm<SGP_MAXD>, dim3((unsigned)m), dim3(256), 0, s, kp, U, ldu, m,
                       mp, uvec, Ainv, Binv, M3, a, b, c, vvec, wvec, e2, out);
  return hipGetLastError();
}

hipError_t launch_fill_cov(const KernParams& kp, const double* x, int64_t n, int64_t ldx,
                           const double* xp, int64_t np, int64_t ldxp, bool sym, double* out,
                           int64_t ldo, hipStream_t s) {
  const int cpb = 64;
  dim3 grid((unsigned)((n + 63) / 64), (unsigned)((np + cpb - 1) / cpb));
  if (n == 0 || np == 0) return hipSuccess;
  if (kp.d > 8)
    hipLaunchKernelGGL((k_fill<false, SGP_MAXD>), grid, dim3(64, 4), 0, s, kp, x, n, ldx, xp, np,
                       ldxp, sym ? 1 : 0, 0, out, ldo, cpb);
  else
    hipLaunchKernelGGL((k_fill<false, 8>), grid, dim3(64, 4), 0, s, kp, x, n, ldx, xp, np, ldxp,
                       sym ? 1 : 0, 0, out, ldo, cpb);
  return hipGetLastError();
}

hipError_t launch_fill_dcov(const KernParams& kp, const double* x, int64_t n, int64_t ldx,
                            const double* xp, int64_t np, int64_t ldxp, bool sym, int param,
                            double* out, int64_t ldo, hipStream_t s) {
  const int cpb = 64;
  dim3 grid((unsigned)((n + 63) / 64), (unsigned)((np + cpb - 1) / cpb));
  if (n == 0 || np == 0) return hipSuccess;
  if (kp.d > 8)
    hipLaunchKernelGGL((k_fill<true, SGP_MAXD>), grid, dim3(64, 4), 0, s, kp, x, n, ldx, xp, np,
                       ldxp, sym ? 1 : 0, param, out, ldo, cpb);
  else
    hipLaunchKernelGGL((k_fill<true, 8>), grid, dim3(64, 4), 0, s, kp, x, n, ldx, xp, np, ldxp,
                       sym ? 1 : 0, param, out, ldo, cpb);
  return hipGetLastError();
}

// One builder launch over row blocks [rb0, rb1) with at most wpc workgroups per CU.  t
// partials (rvec != nullptr) go to tslab rows [slot0, slot0 + *slots): one per workgroup row
// for the matrix-core builder, one per row block for the VALU builder (exp kernel, wide spans).
static hipError_t build_knm_range(const KernParams& kp, const double* X, int64_t ldx, int64_t n,
                                  const double* U, int64_t ldu, int64_t m, int64_t mp, double* K,
                                  const double* r, double* tslab, int64_t slot0, int64_t* slots,
                                  int64_t rb0, int64_t rb1, int wpc, hipStream_t s) {
  static int cus = 0, occ[2][3];   // [with t][NC = 2, 4, 8]
  if (cus == 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    cus = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
              ? prop.multiProcessorCount : 256;
    const void* fns[2][3] = {
        {(const void*)k_build_knm_mfma<false, 2>, (const void*)k_build_knm_mfma<false, 4>,
         (const void*)k_build_knm_mfma<false, 8>},
        {(const void*)k_build_knm_mfma<true, 2>, (const void*)k_build_knm_mfma<true, 4>,
         (const void*)k_build_knm_mfma<true, 8>}};
    for (int t = 0; t < 2; ++t)
      for (int q = 0; q < 3; ++q)
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[t][q], fns[t][q], 256, 0) !=
                hipSuccess || occ[t][q] < 1)
          occ[t][q] = 2;
  }
  if (slots) *slots = 0;
  if (rb1 <= rb0) return hipSuccess;
  if (kp.kernel == 2) return hipErrorInvalidValue;
  const int64_t ncb = mp / 128;   // 128 knot columns per block
  const bool ard = kp.kernel == 1;
  if (knm_mfma_ok(kp)) {
    // persistent: one residency round of workgroups, each walking its share of row blocks
    const int q = kp.d <= 8 ? 0 : (kp.d <= 16 ? 1 : 2);
    const int oc = occ[r ? 1 : 0][q];
    const int per_cu = wpc < oc ? wpc : oc;
    int64_t gy = ((int64_t)cus * per_cu) / (ncb > 0 ? ncb : 1);
    gy = gy < 1 ? 1 : (gy > rb1 - rb0 ? rb1 - rb0 : gy);
    dim3 grid((unsigned)ncb, (unsigned)gy);
#define SGP_BUILD_MFMA(T, NCV)                                                                 \
  hipLaunchKernelGGL((k_build_knm_mfma<T, NCV>), grid, dim3(256), 0, s, kp, X, ldx, n, U, ldu, m, \
                     mp, K, r, tslab, slot0, rb0, rb1)
    if (r) {
      if (q == 0) SGP_BUILD_MFMA(true, 2);
      else if (q == 1) SGP_BUILD_MFMA(true, 4);
      else SGP_BUILD_MFMA(true, 8);
    } else {
      if (q == 0) SGP_BUILD_MFMA(false, 2);
      else if (q == 1) SGP_BUILD_MFMA(false, 4);
      else SGP_BUILD_MFMA(false, 8);
    }
#undef SGP_BUILD_MFMA
    if (slots) *slots = gy;
    return hipGetLastError();
  }
  int64_t gy = ((int64_t)cus * wpc) / (ncb > 0 ? ncb : 1);
  gy = gy < 1 ? 1 : (gy > rb1 - rb0 ? rb1 - rb0 : gy);
  dim3 grid((unsigned)ncb, (unsigned)gy);
  // the VALU builder writes one t partial per row block, at tslab row rb
  if (r && slot0 != rb0) return hipErrorInvalidValue;
  if (ard) hipLaunchKernelGGL((k_build_knm<true, SGP_MAXD>), grid, dim3(64, 4), 0, s, kp, X, ldx, n, U, ldu, m, mp, K, r, tslab, rb0, rb1);
  else hipLaunchKernelGGL((k_build_knm<false, SGP_MAXD>), grid, dim3(64, 4), 0, s, kp, X, ldx, n, U, ldu, m, mp, K, r, tslab, rb0, rb1);
  if (slots) *slots = rb1 - rb0;
  return hipGetLastError();
}

// Full-occupancy builder (more than fit: the occupancy limit applies).
constexpr int BUILD_WPC_FULL = 64;
// While the K22 Gauss-Jordan chain runs on the high-priority aux stream (FITC / Laplace phase
// 1), a builder at full occupancy leaves no CU room for the chain's workgroups (they queue
// behind the builder's and the next pass then waits for the chain).  The first row blocks are
// therefore built at BUILD_WPC_SHARED workgroups per CU, sized to last about as long as the
// chain, and the rest at full occupancy.
constexpr int BUILD_WPC_SHARED = 2;

static hipError_t build_knm_impl(const KernParams& kp, const double* X, int64_t ldx, int64_t n,
                                 int64_t n_pad, const double* U, int64_t ldu, int64_t m,
                                 int64_t mp, double* K, const double* r, double* tslab,
                                 int64_t shared_rb, int64_t* t_rows, hipStream_t s) {
  const int64_t nrb = n_pad / 64;
  if (shared_rb > nrb) shared_rb = nrb;
  if (shared_rb < 0) shared_rb = 0;
  int64_t s1 = 0, s2 = 0;
  hipError_t e = build_knm_range(kp, X, ldx, n, U, ldu, m, mp, K, r, tslab, 0, &s1, 0, shared_rb,
                                 BUILD_WPC_SHARED, s);
  if (e != hipSuccess) return e;
  // the VALU builder's partial rows are indexed by row block
  const int64_t slot0 = knm_mfma_ok(kp) ? s1 : shared_rb;
  e = build_knm_range(kp, X, ldx, n, U, ldu, m, mp, K, r, tslab, slot0, &s2, shared_rb, nrb,
                      BUILD_WPC_FULL, s);
  if (t_rows) *t_rows = slot0 + s2;
  return e;
}

// Row blocks built at shared occupancy beside the K22 chain: ~60 us per 64-wide Gauss-Jordan
// step beside the builder (+ build and first pivot) at ~2.8 GB/ms for the shared-occupancy
// builder (measured, m = 1024).
static int64_t chain_shared_rb(int64_t mp) {
  const double chain_us = SGP_CHAIN_US_STEP * (double)(mp / 64) + SGP_CHAIN_US_FIX;
  return (int64_t)(chain_us * 2.8e6 / (64.0 * (double)mp * 8.0)) + 1;   // 2.8 GB/ms = 2.8e6 B/us
}

hipError_t launch_build_knm(const KernParams& kp, const double* X, int64_t ldx, int64_t n,
                            int64_t n_pad, const double* U, int64_t ldu, int64_t m, int64_t mp,
                            double* K, hipStream_t s, bool beside_chain) {
  return build_knm_impl(kp, X, ldx, n, n_pad, U, ldu, m, mp, K, nullptr, nullptr,
                        beside_chain ? chain_shared_rb(mp) : 0, nullptr, s);
}

hipError_t launch_build_knm_t(const KernParams& kp, const double* X, int64_t ldx, int64_t n,
                              int64_t n_pad, const double* U, int64_t ldu, int64_t m, int64_t mp,
                              double* K, const double* r, double* tslab, int64_t* t_rows,
                              hipStream_t s, bool beside_chain) {
  return build_knm_impl(kp, X, ldx, n, n_pad, U, ldu, m, mp, K, r, tslab,
                        beside_chain ? chain_shared_rb(mp) : 0, t_rows, s);
}

hipError_t launch_build_kmm(const KernParams& kp, const double* U, int64_t ldu, int64_t m,
                            int64_t mp, double diag_sub, double* K22, hipStream_t s,
                            double* K22_copy) {
  dim3 grid((unsigned)(mp / 64), (unsigned)((mp + 3) / 4));
  if (kp.d <= 8)
    hipLaunchKernelGGL(k_build_kmm<8>, grid, dim3(64, 4), 0, s, kp, U, ldu, m, mp, diag_sub, K22,
                       K22_copy);
  else
    hipLaunchKernelGGL(k_build_kmm<SGP_MAXD>, grid, dim3(64, 4), 0, s, kp, U, ldu, m, mp,
                       diag_sub, K22, K22_copy);
  return hipGetLastError();
}

hipError_t launch_contract_kmm(const KernParams& kp, const double* U, int64_t ldu, int64_t m,
                               int64_t mp, const double* uvec, const double* Ainv,
                               const double* Binv, const double* M3, double a, double b,
                               double c, const double* vvec, const double* wvec, double e2,
                               double* slab, int64_t slab_cap, int* nblocks, hipStream_t s) {
  const int nb = (int)(m > 0 ? m : 1);   // one block (and one record) per knot row
  *nblocks = nb;
  if ((int64_t)nb * kp.P > slab_cap) return hipErrorInvalidValue;
  if (m <= 0) return hipSuccess;
  if (kp.d <= 8)
    hipLaunchKernelGGL(k_contract_kmm<8>, dim3(nb), dim3(256), 0, s, kp, U, ldu, m, mp, uvec,
                       Ainv, Binv, M3, a, b, c, vvec, wvec, e2, slab);
  else
    hipLaunchKernelGGL(k_contract_kmm<SGP_MAXD>, dim3(nb), dim3(256), 0, s, kp, U, ldu, m, mp,
                       uvec, Ainv, Binv, M3, a, b, c, vvec, wvec, e2, slab);
  return hipGetLastError();
}
