// m x m dense algebra and row reductions for the sparse-GP evaluation on gfx950.
//
// The reference calls base-R chol()/solve() (LAPACK dpotrf/dgesv) on the m x m matrices
// Sigma22 and Sigma22 + t(Sigma12) %*% (B * Sigma12) (R/vi_functions.R:96, 231, 239).  Here
// both are inverted by dense_spd_inverse: a blocked Gauss-Jordan (sweep) SPD inverse, one
// launch per 64-wide pivot, whose trailing updates are f64 MFMA products; the pivots are the
// Cholesky factor's squared diagonal, so log-determinants and R's chol() failure order come
// out of the same pass.
// Reductions are two-stage with fixed order (deterministic, run-to-run bit-identical).
#include <stdlib.h>

#include <atomic>

#include "sgp_internal.h"
#include "sgp_probe.h"

namespace {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double block_sum(double v, double* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_sum(v);
  if (lane == 0) sh[w] = v;
  __syncthreads();
  double t = 0.0;
  const int nw = blockDim.x >> 6;
  for (int q = 0; q < nw; ++q) t += sh[q];
  __syncthreads();
  return t;
}

// ---------------------------------------------------------------- blocked Gauss-Jordan
// 1/sqrt(p) for p > 0: hardware rsq seed + two Newton steps (full double accuracy).
__device__ __forceinline__ double rsqrt_nr(double p) {
  double y = __builtin_amdgcn_rsq(p);
  y = y * fma(-0.5 * p * y, y, 1.5);
  y = y * fma(-0.5 * p * y, y, 1.5);
  return y;
}

// Pivot of the SPD Gauss-Jordan inverse: P = inv(B) for a 64x64 SPD block B (a Schur
// complement) read from B[i * ldb + j] (global or LDS), by the symmetric sweep operator
// applied in four 16-wide blocks K (sweeps compose, so sweeping K at once equals its 16
// scalar sweeps in turn):
//   W_KK <- Q = -inv(W_KK)          16 scalar sweeps by the one wave that owns rows K, in
//                                   registers, lanes exchanging by ds_bpermute: no barriers
//   W_RK <- -F_R,  F = W_:K Q       one 16x16x16 MFMA product per wave
//   W_KR <- -Q W_RK^T
//   W_RR <- W_RR + F_R W_RK^T       rank-16 update, MFMA
// so a pivot costs 64 barrier-free scalar sweeps plus 12 block barriers instead of 64
// block-wide barriers.  Layout: wave w owns rows 16w..16w+15 as four 16x16 MFMA
// accumulator tiles (lane l: column l & 15, rows (l >> 4) + 4q).  The scalar sweeps keep
// the reference arithmetic of the sweep operator; the final W is -inv(B).  The sweep pivots
// d_k are the Schur complements L_kk^2 of the Cholesky factor, so *logd_slot = sum log L_kk
// = 1/2 sum log d_k; a non-positive pivot sets status = gofs + k + 1 (R's chol() order).
// lds: GJ_PIVOT_LDS doubles.  Called by all 256 threads of the block.
constexpr int GJP_LD = 17;                                  // padded row stride (doubles)
constexpr int GJ_PIVOT_LDS = 2 * 64 * GJP_LD + 64 * GJP_LD + 16 * GJP_LD + 64;

__device__ __forceinline__ double rcp_nr(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = r * fma(-d, r, 2.0);
  r = r * fma(-d, r, 2.0);
  return r;
}

// lane `src`'s value to every lane (scalar register path)
__device__ __forceinline__ double readlane_f64(double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, src);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// lane K of every 16-lane row to the whole row (DPP row_newbcast, gfx90a+)
template <int K>
__device__ __forceinline__ double row_bcast_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, 0x150 + K, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0x150 + K, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// runtime-k form for unrolled loops (folds to one case once k is a constant)
__device__ __forceinline__ double row_bcast_f64(double v, int k) {
  switch (k) {
    case 0: return row_bcast_f64<0>(v);    case 1: return row_bcast_f64<1>(v);
    case 2: return row_bcast_f64<2>(v);    case 3: return row_bcast_f64<3>(v);
    case 4: return row_bcast_f64<4>(v);    case 5: return row_bcast_f64<5>(v);
    case 6: return row_bcast_f64<6>(v);    case 7: return row_bcast_f64<7>(v);
    case 8: return row_bcast_f64<8>(v);    case 9: return row_bcast_f64<9>(v);
    case 10: return row_bcast_f64<10>(v);  case 11: return row_bcast_f64<11>(v);
    case 12: return row_bcast_f64<12>(v);  case 13: return row_bcast_f64<13>(v);
    case 14: return row_bcast_f64<14>(v);  default: return row_bcast_f64<15>(v);
  }
}

// Sweep K of the 16x16 pivot block t (accumulator layout: lane (lr, lc) holds rows lr + 4q of
// column lc): W_ij <- W_ij + W_iK (-r W_Kj), one DPP64 v_fmac_f64_dpp per register (W_iK read
// from lane K of the 16-lane row; on column K itself nvj = r - 1 gives W_iK r), then row K set
// apart: W_Kj <- r W_Kj, W_KK <- -r (r = 1 / W_KK).  Against the DPP moves, products and selects
// of the element-wise form: 68 vs 89 ns per sweep (tools/micro/gj_sweep.hip), same accuracy.
// s_nop 1: the two wait states a DPP read of a VGPR needs after a VALU write of it (inline asm
// is invisible to the compiler's hazard recognizer).
template <int K>
__device__ __forceinline__ void gj_sweep_dpp(d4& t, double (&dk)[16], int lr, int lc) {
  constexpr int kq = K >> 2, kr = K & 3;
  const double vc = __shfl(t[kq], lc + 16 * kr, 64);                      // W_K,lc
  const double d = readlane_f64(t[kq], K + 16 * kr);                      // W_KK (uniform)
  const double r = rcp_nr(d);
  dk[K] = d;
  const double rowk = t[kq];
  const double nvj = (lc == K) ? r - 1.0 : -(r * vc);
  double a0 = t[0], a1 = t[1], a2 = t[2], a3 = t[3];
  asm volatile("s_nop 1\n"
               "v_fmac_f64_dpp %0, %0, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n"
               "v_fmac_f64_dpp %1, %1, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n"
               "v_fmac_f64_dpp %2, %2, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n"
               "v_fmac_f64_dpp %3, %3, %4 row_newbcast:%5 row_mask:0xf bank_mask:0xf\n"
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
               : "v"(nvj), "i"(K));
  t[0] = a0;
  t[1] = a1;
  t[2] = a2;
  t[3] = a3;
  const double rk = (lc == K) ? -r : r * rowk;
  t[kq] = (lr == kr) ? rk : t[kq];
}
__device__ __forceinline__ void gj_sweeps16(d4& t, double (&dk)[16], int lr, int lc) {
  gj_sweep_dpp<0>(t, dk, lr, lc);   gj_sweep_dpp<1>(t, dk, lr, lc);
  gj_sweep_dpp<2>(t, dk, lr, lc);   gj_sweep_dpp<3>(t, dk, lr, lc);
  gj_sweep_dpp<4>(t, dk, lr, lc);   gj_sweep_dpp<5>(t, dk, lr, lc);
  gj_sweep_dpp<6>(t, dk, lr, lc);   gj_sweep_dpp<7>(t, dk, lr, lc);
  gj_sweep_dpp<8>(t, dk, lr, lc);   gj_sweep_dpp<9>(t, dk, lr, lc);
  gj_sweep_dpp<10>(t, dk, lr, lc);  gj_sweep_dpp<11>(t, dk, lr, lc);
  gj_sweep_dpp<12>(t, dk, lr, lc);  gj_sweep_dpp<13>(t, dk, lr, lc);
  gj_sweep_dpp<14>(t, dk, lr, lc);  gj_sweep_dpp<15>(t, dk, lr, lc);
}

template <bool SC1 = false>   // SC1: P stored write-through (k_gj_persist's hand-off)
__device__ __forceinline__ void gj_pivot_body(const double* B, int64_t ldb, int64_t gofs,
                                              double* __restrict__ P,
                                              double* __restrict__ logd_slot,
                                              int* __restrict__ status, double* lds,
                                              const double* B2 = nullptr, double beta = 0.0) {
  double* Es0 = lds;                          // [2][64][GJP_LD]  column panel W_:K (old)
  double* Fs = lds + 2 * 64 * GJP_LD;         // [64][GJP_LD]     F = W_:K Q (own rows per wave)
  double* Qs = Fs + 64 * GJP_LD;              // [16][GJP_LD]     Q = -inv(W_KK)
  double* piv = Qs + 16 * GJP_LD;             // [64]             sweep pivots
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int lr = lane >> 4, lc = lane & 15;
  d4 acc[4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[ct][q] = B[(16 * wv + lr + 4 * q) * ldb + 16 * ct + lc];
  if (B2) {   // the block of B + beta B2 (the first pivot of dense_spd_inverse_sum)
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        acc[ct][q] = fma(beta, B2[(16 * wv + lr + 4 * q) * ldb + 16 * ct + lc], acc[ct][q]);
  }
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    double* Es = Es0 + (kb & 1) * 64 * GJP_LD;
    // publish the column panel E = W_:K (every wave's tile kb)
#pragma unroll
    for (int q = 0; q < 4; ++q) Es[(16 * wv + lr + 4 * q) * GJP_LD + lc] = acc[kb][q];
    __syncthreads();
    if (wv == kb) {
      // 16 scalar sweeps of W_KK in registers: lane (lr, lc) holds rows lr + 4q of column lc
      double dk[16];                                                       // the pivots
      gj_sweeps16(acc[kb], dk, lr, lc);
#pragma unroll
      for (int q = 0; q < 4; ++q) Qs[(lr + 4 * q) * GJP_LD + lc] = acc[kb][q];
      // record the pivots; the first non-positive one (R's chol() leading-minor order) sets
      // status unless an earlier block already did
      double dl = dk[0];
#pragma unroll
      for (int k = 1; k < 16; ++k) dl = (lane == k) ? dk[k] : dl;
      const bool bad = lane < 16 && (!(dl > 0.0) || !isfinite(dl));
      const unsigned long long badm = __ballot(bad);
      if (lane < 16) piv[16 * kb + lane] = dl;
      if (lane == 0 && badm)
        atomicCAS(status, 0, (int)(gofs + 16 * kb + __builtin_ctzll(badm) + 1));
    }
    __syncthreads();
    if (wv == kb) {
      // W_KR <- -Q E_R^T  (tiles ct != kb of the pivot rows)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        if (ct == kb) continue;
        d4 t = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int sk = 0; sk < 4; ++sk) {
          const double af = -Qs[lc * GJP_LD + 4 * sk + lr];
          const double bf = Es[(16 * ct + lc) * GJP_LD + 4 * sk + lr];
          t = __builtin_amdgcn_mfma_f64_16x16x4f64(af, bf, t, 0, 0, 0);
        }
        acc[ct] = t;
      }
    } else {
      // F_w = E_w Q; W_wK <- -F_w; W_wR <- W_wR + F_w E_R^T
      d4 f = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int sk = 0; sk < 4; ++sk) {
        const double af = Es[(16 * wv + lc) * GJP_LD + 4 * sk + lr];
        const double bf = Qs[(4 * sk + lr) * GJP_LD + lc];
        f = __builtin_amdgcn_mfma_f64_16x16x4f64(af, bf, f, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) Fs[(16 * wv + lr + 4 * q) * GJP_LD + lc] = f[q];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        if (ct == kb) continue;
#pragma unroll
        for (int sk = 0; sk < 4; ++sk) {
          const double af = Fs[(16 * wv + lc) * GJP_LD + 4 * sk + lr];
          const double bf = Es[(16 * ct + lc) * GJP_LD + 4 * sk + lr];
          acc[ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(af, bf, acc[ct], 0, 0, 0);
        }
      }
      acc[kb] = -f;
    }
  }
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      double* d = &P[(16 * wv + lr + 4 * q) * 64 + 16 * ct + lc];
      if constexpr (SC1) __hip_atomic_store(d, -acc[ct][q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else *d = -acc[ct][q];
    }
  __syncthreads();
  double lg = (tid < 64) ? log(piv[tid]) : 0.0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) lg += __shfl_xor(lg, off, 64);
  if (tid == 0) *logd_slot = 0.5 * lg;
}

// Pivot step k as its own launch (the first pivot of dense_spd_inverse).
__global__ void __launch_bounds__(256) k_gj_pivot(const double* __restrict__ A, int64_t lda,
                                                  int k, double* __restrict__ P,
                                                  double* __restrict__ logd,
                                                  int* __restrict__ status,
                                                  const double* __restrict__ A2, double beta) {
  __shared__ double lds[GJ_PIVOT_LDS];
  const int64_t o = (int64_t)k * 64;
  gj_pivot_body(A + o * lda + o, lda, o, P, logd + k, status, lds, A2 ? A2 + o * lda + o : nullptr,
                beta);
}

// One Gauss-Jordan step k, out of place (Ao -> An), every 64x64 tile (i, j) in one launch:
//   i == k: An_kj = P_k Ao_kj (An_kk = P_k);   j == k: An_ik = -Ao_ik P_k;
//   else    An_ij = Ao_ij - (Ao_ik P_k) Ao_kj                       (two 64^3 f64-MFMA products)
// Look-ahead: the workgroup owning tile (k+1, k+1) factors its fresh tile right away and writes
// the next pivot inverse P_{k+1}, so a step costs one launch instead of pivot + panel + update.
// LDS row stride (doubles).  The A-operand fragment reads of gj_mm64 are paired into
// ds_read2_b64 (banks (a/4) mod 32, 16-lane groups): 16 rows per group need distinct double
// slots mod 16, i.e. an odd stride (70 gave 2-way conflicts on every A read: 0.25 of the LDS
// cycles in the r2 PMC pass).  The B reads are 16 contiguous columns at any stride.
constexpr int GJ_LS = 65;

__device__ __forceinline__ void gj_mm64(const double* As, const double* Bs, d4 (&acc)[2][2]) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wr = wv >> 1, wc = wv & 1;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll SGP_GJ_MM_UNROLL
  for (int kk = 0; kk < 16; ++kk) {
    const int kx = kk * 4 + (lane >> 4);
    double af[2], bf[2];
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      af[f] = As[(wr * 32 + f * 16 + (lane & 15)) * GJ_LS + kx];
      bf[f] = Bs[kx * GJ_LS + wc * 32 + f * 16 + (lane & 15)];
    }
#pragma unroll
    for (int fm = 0; fm < 2; ++fm)
#pragma unroll
      for (int fn = 0; fn < 2; ++fn)
        acc[fm][fn] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[fm], bf[fn], acc[fm][fn], 0, 0, 0);
  }
}

// Global loads of a 64x64 tile into registers (16 per thread, coalesced rows) and their LDS
// stores, split so that every load of a step is in flight before the first one is waited on.
__device__ __forceinline__ void gj_ld(double (&v)[16], const double* G, int64_t ldg) {
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = threadIdx.x + 256 * q;
    v[q] = G[(int64_t)(e >> 6) * ldg + (e & 63)];
  }
}
// the same tile of G + beta G2 (step 0 of dense_spd_inverse_sum: the matrix is formed as it is
// read, no separate axpby launch); SUM = false is gj_ld
template <bool SUM>
__device__ __forceinline__ void gj_ld2(double (&v)[16], const double* G, const double* G2,
                                       double beta, int64_t ldg) {
  if constexpr (!SUM) {
    gj_ld(v, G, ldg);
  } else {
    double w[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = threadIdx.x + 256 * q;
      v[q] = G[(int64_t)(e >> 6) * ldg + (e & 63)];
      w[q] = G2[(int64_t)(e >> 6) * ldg + (e & 63)];
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = fma(beta, w[q], v[q]);
  }
}
__device__ __forceinline__ void gj_st(double* S, const double (&v)[16]) {
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = threadIdx.x + 256 * q;
    S[(e >> 6) * GJ_LS + (e & 63)] = v[q];
  }
}

// SUM (step 0 of dense_spd_inverse_sum): Ao is read as Ao + beta A2.
template <bool SUM>
__global__ void __launch_bounds__(256) k_gj_step(const double* __restrict__ Ao,
                                                 double* __restrict__ An, int64_t lda, int k,
                                                 int nb, const double* __restrict__ Pk,
                                                 double* __restrict__ Pn,
                                                 double* __restrict__ logd,
                                                 int* __restrict__ status,
                                                 const double* __restrict__ A2, double beta) {
  __shared__ double lds[2 * 64 * GJ_LS];
  double* S0 = lds;
  double* S1 = lds + 64 * GJ_LS;
  const int i = blockIdx.y, j = blockIdx.x;
  const int64_t oi = (int64_t)i * 64, oj = (int64_t)j * 64, ok = (int64_t)k * 64;
  SGP_PROBE_GJ_DECL();   // timing probe hooks (sgp_probe.h): empty in the product
#define GJ_STAMP(p_) SGP_PROBE_GJ_STAMP(p_)
  GJ_STAMP(0);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  d4 acc[2][2];
  double v0[16], v1[16];
  if (i == k) {
    if (j == k) {
      for (int e = threadIdx.x; e < 4096; e += 256)
        An[(oi + (e >> 6)) * lda + oj + (e & 63)] = Pk[e];
      return;
    }
    gj_ld(v0, Pk, 64);
    gj_ld2<SUM>(v1, Ao + ok * lda + oj, A2 + ok * lda + oj, beta, lda);
    gj_st(S0, v0);
    gj_st(S1, v1);
    __syncthreads();
    gj_mm64(S0, S1, acc);
#pragma unroll
    for (int fm = 0; fm < 2; ++fm)
#pragma unroll
      for (int fn = 0; fn < 2; ++fn)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = wr * 32 + fm * 16 + (lane >> 4) + 4 * q;
          const int c = wc * 32 + fn * 16 + (lane & 15);
          An[(oi + r) * lda + oj + c] = acc[fm][fn][q];
        }
    return;
  }
  gj_ld2<SUM>(v0, Ao + oi * lda + ok, A2 + oi * lda + ok, beta, lda);   // C_i = Ao_ik
  gj_ld(v1, Pk, 64);
  if (j == k) {
    gj_st(S0, v0);
    gj_st(S1, v1);
    __syncthreads();
    gj_mm64(S0, S1, acc);                        // C_i P_k
#pragma unroll
    for (int fm = 0; fm < 2; ++fm)
#pragma unroll
      for (int fn = 0; fn < 2; ++fn)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = wr * 32 + fm * 16 + (lane >> 4) + 4 * q;
          const int c = wc * 32 + fn * 16 + (lane & 15);
          An[(oi + r) * lda + oj + c] = -acc[fm][fn][q];
        }
    return;
  }
  // the remaining operands (Ao_kj, and Ao_ij in the accumulator layout) are loaded now as well
  double v2[16], aij[2][2][4];
  gj_ld2<SUM>(v2, Ao + ok * lda + oj, A2 + ok * lda + oj, beta, lda);
#pragma unroll
  for (int fm = 0; fm < 2; ++fm)
#pragma unroll
    for (int fn = 0; fn < 2; ++fn)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = wr * 32 + fm * 16 + (lane >> 4) + 4 * q;
        const int c = wc * 32 + fn * 16 + (lane & 15);
        aij[fm][fn][q] = Ao[(oi + r) * lda + oj + c];
        if constexpr (SUM) aij[fm][fn][q] = fma(beta, A2[(oi + r) * lda + oj + c], aij[fm][fn][q]);
      }
  gj_st(S0, v0);
  gj_st(S1, v1);
  __syncthreads();
  GJ_STAMP(1);
  gj_mm64(S0, S1, acc);                          // C_i P_k
  __syncthreads();                               // everyone is done reading S0 / S1
  GJ_STAMP(2);
#pragma unroll
  for (int fm = 0; fm < 2; ++fm)
#pragma unroll
    for (int fn = 0; fn < 2; ++fn)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = wr * 32 + fm * 16 + (lane >> 4) + 4 * q;
        const int c = wc * 32 + fn * 16 + (lane & 15);
        S0[r * GJ_LS + c] = acc[fm][fn][q];
      }
  gj_st(S1, v2);                                 // Ao_kj
  __syncthreads();
  gj_mm64(S0, S1, acc);                          // (C_i P_k) Ao_kj
  const bool look_ahead = (i == k + 1) && (j == k + 1);
  if (look_ahead) __syncthreads();               // S0 is reused for the fresh tile below
#pragma unroll
  for (int fm = 0; fm < 2; ++fm)
#pragma unroll
    for (int fn = 0; fn < 2; ++fn)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = wr * 32 + fm * 16 + (lane >> 4) + 4 * q;
        const int c = wc * 32 + fn * 16 + (lane & 15);
        const double v = aij[fm][fn][q] - acc[fm][fn][q];
        An[(oi + r) * lda + oj + c] = v;
        if (look_ahead) S0[r * GJ_LS + c] = v;
      }
  if (look_ahead) {
    __syncthreads();
    GJ_STAMP(3);
    gj_pivot_body(S0, GJ_LS, (int64_t)(k + 1) * 64, Pn, logd + k + 1, status, S1);
    GJ_STAMP(4);
  }
#undef GJ_STAMP
}

// ---------------------------------------------------------------- persistent Gauss-Jordan
// The whole chain of an SPD inverse in one launch (nb <= GJ_NB_MAX): G workgroups claim tasks
// from a ticket counter in dependency order and run them in place on the matrix, so a step's
// tiles start as soon as their own inputs exist instead of at a launch boundary, and the next
// pivot's workgroup (task 1 of each step) is never queued behind the step's other tiles.
// Tasks, in ticket order:  0: pivot P_0 of tile (0, 0);  then per step k (nb^2 tasks):
//   interior (i, j), i, j != k:  A_ij <- A_ij - (A_ik P_k) A_kj; the first one is (k+1, k+1),
//                                which then factors its fresh tile into P_{k+1} (look-ahead);
//                                in shell order max(a, b), a = i - k - 1, b = j - k - 1 (mod nb),
//                                so the tiles step k+1's look-ahead needs come first
//   column (i, k):  A_ik <- -A_ik P_k       row (k, j):  A_kj <- P_k A_kj       (k, k): P_k
// A task waits only for tasks with smaller tickets, and a ticket is only claimed by a running
// workgroup, so the smallest unfinished ticket can always proceed: no co-residency is assumed
// (the K22 chain on `aux` may hold CUs at the same time).  Flags (device-scope release /
// acquire): ver[i][j] = steps applied to tile (i, j); loaded[i][j] = k + 1 once interior task
// (k, i, j) holds A_ik and A_kj (the in-place column / row tasks overwrite them only then);
// piv[k] = P_k is in memory.  The last workgroup to leave zeroes the sync words for the next
// launch (allocated zeroed).  Arithmetic per tile is k_gj_step's: results are bit-identical.
constexpr int GJ_NB_MAX = 64;
constexpr int GJ_SYNC_PIV = 64, GJ_SYNC_VER = GJ_SYNC_PIV + GJ_NB_MAX;

// Hand-offs between workgroups (MI355X_MICROARCH.md, inter-workgroup visibility, first row of
// the sc1 table): every byte handed over is stored write-through (sc1) and loaded sc1 (L1
// bypassed), each storing wave drains its stores (s_waitcnt vmcnt(0)) before the workgroup
// barrier behind which one lane stores the flag (sc1); a consumer polls with sc1 loads in one
// wave and the others load after the barrier it then joins.  No cache-wide fences: an acquire
// fence per task, or polling with acquire loads, made a step at m = 1024 five times slower.
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned ldu_sc1(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stu_sc1(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Threads tid < cnt (wave 0) wait for their flag (ptr(tid)) to reach v, then the workgroup
// proceeds.  Watchdog: a wait that outlasts ~2^24 polls (seconds; a real wait is microseconds)
// marks the chain aborted (sync[2], status -1, reported by the host as an internal error) and
// every later wait returns at once, so the grid always drains.
constexpr unsigned GJ_SPIN_MAX = 1u << 24;
template <typename F>
__device__ __forceinline__ void gj_wait(int cnt, F ptr, unsigned v, unsigned* sync, int* status) {
  if ((int)threadIdx.x < cnt) {
    const unsigned* f = ptr((int)threadIdx.x);
    unsigned it = 0;
    while (ldu_sc1(f) < v) {
      if ((++it & 255u) == 0) {
        if (it >= GJ_SPIN_MAX) {
          stu_sc1(sync + 2, 1u);
          atomicCAS(status, 0, -1);
          break;
        }
        if (ldu_sc1(sync + 2)) break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}
// the workgroup's (sc1) stores drained, then flag = v
__device__ __forceinline__ void gj_publish(unsigned* f, unsigned v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) stu_sc1(f, v);
}
// A 64x64 tile (row stride ldg) by 16-byte sc1 buffer loads (the 8-byte form runs at ~0.6 of
// the rate, MI355X_MICROARCH.md): thread t holds columns c = 2 (t & 31), c + 1 of rows
// (t >> 5) + 8 q in v[2 q], v[2 q + 1]; gj_st16 stores that layout to an LDS tile
typedef unsigned int gj_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gj_rsrc(const double* G) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(G), (short)0, 0x7fffffff,
                                           0x00020000);
}
__device__ __forceinline__ int gj_off16(int q, int64_t ldg) {   // byte offset of thread's pair q
  return (int)((((int64_t)(threadIdx.x >> 5) + 8 * q) * ldg + 2 * (threadIdx.x & 31)) * 8);
}
__device__ __forceinline__ void gj_ld16_sc1(double (&v)[16], const double* G, int64_t ldg) {
  const __amdgpu_buffer_rsrc_t rs = gj_rsrc(G);
  gj_u4 w[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) w[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, gj_off16(q, ldg), 0, 16);
#pragma unroll
  for (int q = 0; q < 8; ++q) __builtin_memcpy(&v[2 * q], &w[q], 16);
}
__device__ __forceinline__ void gj_st16(double* S, const double (&v)[16]) {
  const int c = 2 * (threadIdx.x & 31), r0 = threadIdx.x >> 5;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    S[(r0 + 8 * q) * GJ_LS + c] = v[2 * q];
    S[(r0 + 8 * q) * GJ_LS + c + 1] = v[2 * q + 1];
  }
}

template <bool SC1>
__device__ __forceinline__ void gj_store_acc(double* T, int64_t ld, const d4 (&acc)[2][2],
                                             double sgn) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, wr = wv >> 1, wc = wv & 1;
#pragma unroll
  for (int fm = 0; fm < 2; ++fm)
#pragma unroll
    for (int fn = 0; fn < 2; ++fn)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = wr * 32 + fm * 16 + (lane >> 4) + 4 * q;
        const int c = wc * 32 + fn * 16 + (lane & 15);
        if constexpr (SC1) st_sc1(&T[r * ld + c], sgn * acc[fm][fn][q]);
        else T[r * ld + c] = sgn * acc[fm][fn][q];
      }
}

// withhold: a ticket whose flag publish is skipped (fault injection of the watchdog test, armed
// only in probe builds, SGP_PROBE_GJ_WITHHOLD; -1 in the product)
__global__ void __launch_bounds__(256) k_gj_persist(const double* src0, const double* src0b,
                                                    double beta, double* buf, int64_t lda,
                                                    int nb, double* __restrict__ P,
                                                    double* __restrict__ logd,
                                                    int* __restrict__ status,
                                                    unsigned* __restrict__ sync, int withhold) {
  __shared__ double lds[4 * 64 * GJ_LS];
  __shared__ int tk;
  double* S0 = lds;
  double* S1 = lds + 64 * GJ_LS;
  double* S2 = lds + 2 * 64 * GJ_LS;
  double* S3 = lds + 3 * 64 * GJ_LS;
  unsigned* piv = sync + GJ_SYNC_PIV;
  unsigned* ver = sync + GJ_SYNC_VER;
  unsigned* loaded = ver + nb * nb;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int nn = nb * nb, n1 = nb - 1;
  auto tile = [&](const double* A, int i, int j) { return A + (int64_t)i * 64 * lda + (int64_t)j * 64; };
  auto wtile = [&](int i, int j) { return buf + (int64_t)i * 64 * lda + (int64_t)j * 64; };
  // step k's operand (i, j): step 0 reads src0 (+ beta src0b), later steps the matrix itself
  // every load of the matrix and P is sc1 (src0 too: in place it is the matrix)
  // (gj_ld16_sc1 layout; stored with gj_st16)
  auto ld_tile = [&](double (&v)[16], int k, int i, int j) {
    gj_ld16_sc1(v, tile(k == 0 ? src0 : buf, i, j), lda);
    if (k == 0 && src0b) {
      const double* B = tile(src0b, i, j);
      const int c = 2 * (threadIdx.x & 31), r0 = threadIdx.x >> 5;
#pragma unroll
      for (int q = 0; q < 16; ++q)
        v[q] = fma(beta, B[(int64_t)(r0 + 8 * (q >> 1)) * lda + c + (q & 1)], v[q]);
    }
  };
  int pk_have = -1;   // the step whose P is in S1 (a workgroup often runs several of a step)
  auto ld_pk = [&](int k) {   // P_k -> S1
    if (pk_have == k) return;
    gj_wait(1, [&](int) { return piv + k; }, 1u, sync, status);
    double v[16];
    gj_ld16_sc1(v, P + (int64_t)k * 4096, 64);
    gj_st16(S1, v);
    pk_have = k;
  };
  // A_ij (step k's operand) in the accumulator layout of gj_mm64
  auto ld_acc = [&](double (&aij)[2][2][4], int k, int i, int j) {
    const double* Aij = tile(k == 0 ? src0 : buf, i, j);
    const double* Bij = (k == 0 && src0b) ? tile(src0b, i, j) : nullptr;
#pragma unroll
    for (int fm = 0; fm < 2; ++fm)
#pragma unroll
      for (int fn = 0; fn < 2; ++fn)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rr = wr * 32 + fm * 16 + (lane >> 4) + 4 * q;
          const int c = wc * 32 + fn * 16 + (lane & 15);
          aij[fm][fn][q] = ld_sc1(&Aij[rr * lda + c]);
          if (Bij) aij[fm][fn][q] = fma(beta, Bij[rr * lda + c], aij[fm][fn][q]);
        }
  };
  // out tile (i, j) = aij - acc into memory, or (X) only into LDS: the look-ahead's fresh tile
  // is read by nothing but its own pivot (step k+1's (k+1, k+1) task overwrites the tile with
  // P_{k+1}, and no task of step k+1 reads it), so it is neither stored nor published
  auto st_out = [&](int i, int j, const double (&aij)[2][2][4], const d4 (&acc)[2][2], double* X) {
    double* Tij = wtile(i, j);
#pragma unroll
    for (int fm = 0; fm < 2; ++fm)
#pragma unroll
      for (int fn = 0; fn < 2; ++fn)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rr = wr * 32 + fm * 16 + (lane >> 4) + 4 * q;
          const int c = wc * 32 + fn * 16 + (lane & 15);
          const double v = aij[fm][fn][q] - acc[fm][fn][q];
          if (X) X[rr * GJ_LS + c] = v;
          else st_sc1(&Tij[rr * lda + c], v);
        }
  };
  // units of a step: the look-ahead tile (k+1, k+1) alone (not in the last step), the other
  // interior tiles of each row i = k+1+a paired along the row (one A_ik P_k product serves two
  // tiles: three 64^3 products and six tile loads for two tiles instead of four and eight),
  // then the column / row tasks and (k, k)
  const int half = (n1 + 1) / 2;                                   // units of a full row
  const int u_reg = 1 + n1 / 2 + (n1 - 1) * half + 2 * n1 + 1;    // per step before the last
  const int u_last = n1 * half + 2 * n1 + 1;
  const int ntask = 1 + n1 * u_reg + u_last;
  for (;;) {
    if (threadIdx.x == 0) tk = (int)__hip_atomic_fetch_add(sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int t = tk;
    __syncthreads();
    if (t >= ntask) break;
    if (t == 0) {   // P_0
      double v[16];
      ld_tile(v, 0, 0, 0);
      gj_st16(S0, v);
      __syncthreads();
      gj_pivot_body<true>(S0, GJ_LS, 0, P, logd, status, S1);
      if (t != withhold) gj_publish(piv, 1u);
      pk_have = -1;
      continue;
    }
    int k, r;
    {
      const int s = t - 1;
      k = s / u_reg;
      if (k >= n1) k = n1;
      r = s - k * u_reg;
    }
    const bool last = k == n1;
    d4 acc[2][2];
    int ia = -1, b0 = 0, b1 = -1;    // interior unit: row offset a, column offsets b0 (, b1)
    if (!last && r == 0) {
      ia = 0;                        // the look-ahead tile
    } else {
      int q = last ? r : r - 1;
      for (int a = 0; a < n1; ++a) {
        const int skip = (a == 0 && !last) ? 1 : 0;
        const int cnt = n1 - skip, u = (cnt + 1) / 2;
        if (q < u) {
          ia = a;
          b0 = skip + 2 * q;
          b1 = b0 + 1 < n1 ? b0 + 1 : -1;
          break;
        }
        q -= u;
      }
      if (ia < 0) r = q + 0;         // past the interior units: q counts the column / row tasks
    }
    if (ia >= 0) {
      const int i = (k + 1 + ia) % nb, j0 = (k + 1 + b0) % nb;
      const bool two = b1 >= 0;
      const int j1 = two ? (k + 1 + b1) % nb : j0;
      const bool look_ahead = !last && ia == 0 && b0 == 0;
      if (k > 0) {
        const int f0 = i * nb + j0, f1 = i * nb + k, f2 = k * nb + j0, f3 = i * nb + j1,
                  f4 = k * nb + j1;
        gj_wait(two ? 5 : 3,
                [&](int q) {
                  return ver + (q == 0 ? f0 : q == 1 ? f1 : q == 2 ? f2 : q == 3 ? f3 : f4);
                },
                (unsigned)k, sync, status);
      }
      double v0[16], v2[16], aij0[2][2][4], aij1[2][2][4];
      ld_tile(v0, k, i, k);
      ld_tile(v2, k, k, j0);
      ld_acc(aij0, k, i, j0);
      gj_st16(S0, v0);
      gj_st16(S2, v2);
      if (two) {
        ld_tile(v2, k, k, j1);
        ld_acc(aij1, k, i, j1);
        gj_st16(S3, v2);
      }
      __syncthreads();   // A_ik and A_kj are in LDS: the column / row tasks may overwrite them
      if (threadIdx.x == 0) {
        stu_sc1(loaded + i * nb + j0, (unsigned)(k + 1));
        if (two) stu_sc1(loaded + i * nb + j1, (unsigned)(k + 1));
      }
      ld_pk(k);
      __syncthreads();
      gj_mm64(S0, S1, acc);                      // A_ik P_k
      __syncthreads();
      gj_store_acc<false>(S0, GJ_LS, acc, 1.0);
      __syncthreads();
      gj_mm64(S0, S2, acc);                      // (A_ik P_k) A_kj0
      if (look_ahead) __syncthreads();           // S0 takes the fresh tile
      st_out(i, j0, aij0, acc, look_ahead ? S0 : nullptr);
      if (two) {
        gj_mm64(S0, S3, acc);                    // (A_ik P_k) A_kj1
        st_out(i, j1, aij1, acc, nullptr);
      }
      if (!look_ahead) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
          stu_sc1(ver + i * nb + j0, (unsigned)(k + 1));
          if (two) stu_sc1(ver + i * nb + j1, (unsigned)(k + 1));
        }
      } else {
        __syncthreads();
        gj_pivot_body<true>(S0, GJ_LS, (int64_t)(k + 1) * 64, P + (int64_t)(k + 1) * 4096,
                      logd + k + 1, status, S1);
        if (t != withhold) gj_publish(piv + k + 1, 1u);
        pk_have = -1;   // S1 was the pivot's scratch
      }
      continue;
    }
    if (r < 2 * n1) {
      // column task (i, k): -A_ik P_k, or row task (k, j): P_k A_kj
      const bool col = r < n1;
      const int x = (k + 1 + (col ? r : r - n1)) % nb;
      const int i = col ? x : k, j = col ? k : x;
      if (k > 0) gj_wait(1, [&](int) { return ver + i * nb + j; }, (unsigned)k, sync, status);
      double v[16];
      ld_tile(v, k, i, j);
      gj_st16(col ? S0 : S2, v);
      ld_pk(k);
      __syncthreads();
      if (col) gj_mm64(S0, S1, acc);
      else gj_mm64(S1, S2, acc);
      // every interior task of row i (column j) of this step holds its copy of this tile
      if (col)
        gj_wait(nb, [&](int q) { return loaded + i * nb + (q == k ? (k + 1) % nb : q); },
                (unsigned)(k + 1), sync, status);
      else
        gj_wait(nb, [&](int q) { return loaded + (q == k ? (k + 1) % nb : q) * nb + j; },
                (unsigned)(k + 1), sync, status);
      gj_store_acc<true>(wtile(i, j), lda, acc, col ? -1.0 : 1.0);
      gj_publish(ver + i * nb + j, (unsigned)(k + 1));
      continue;
    }
    // (k, k) <- P_k
    gj_wait(1, [&](int) { return piv + k; }, 1u, sync, status);
    {
      const __amdgpu_buffer_rsrc_t rp = gj_rsrc(P + (int64_t)k * 4096), rt = gj_rsrc(wtile(k, k));
      gj_u4 w[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) w[q] = __builtin_amdgcn_raw_buffer_load_b128(rp, gj_off16(q, 64), 0, 16);
#pragma unroll
      for (int q = 0; q < 8; ++q) __builtin_amdgcn_raw_buffer_store_b128(w[q], rt, gj_off16(q, lda), 0, 16);
    }
    gj_publish(ver + k * nb + k, (unsigned)(k + 1));
  }
  // the last workgroup out resets the sync words (no other workgroup touches them any more)
  if (threadIdx.x == 0) tk = (int)__hip_atomic_fetch_add(sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (tk == (int)gridDim.x - 1) {
    for (int e = threadIdx.x; e < 2 * nn; e += 256) ver[e] = 0u;
    for (int e = threadIdx.x; e < nb; e += 256) piv[e] = 0u;
    if (threadIdx.x < 3) sync[threadIdx.x] = 0u;
  }
}

__global__ void __launch_bounds__(256) k_axpby(double a, const double* __restrict__ A, double b,
                                               const double* __restrict__ B,
                                               double* __restrict__ C, int64_t count) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < count;
       e += (int64_t)gridDim.x * 256)
    C[e] = a * A[e] + b * B[e];
}

// y = scale * A x, one wave per row
__global__ void __launch_bounds__(256) k_gemv(const double* __restrict__ A, int64_t mp,
                                              const double* __restrict__ x, double scale,
                                              double* __restrict__ y) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= mp) return;
  double s = 0.0;
  for (int64_t j = lane; j < mp; j += 64) s = fma(A[row * mp + j], x[j], s);
  s = wave_sum(s);
  if (lane == 0) y[row] = scale * s;
}

__global__ void __launch_bounds__(256) k_dot_partial(const double* __restrict__ a,
                                                     const double* __restrict__ b, int64_t count,
                                                     double* __restrict__ partial) {
  __shared__ double sh[4];
  double s = 0.0;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < count;
       e += (int64_t)gridDim.x * 256)
    s = b ? fma(a[e], b[e], s) : s + a[e];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_sum_vec(const double* __restrict__ v, int64_t count,
                                                 double* __restrict__ out) {
  __shared__ double sh[4];
  double s = 0.0;
  for (int64_t e = threadIdx.x; e < count; e += 256) s += v[e];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) out[0] = s;
}

// out[k] = sum_r slab[r*ncol + k]; one block per column
__global__ void __launch_bounds__(256) k_colsum(const double* __restrict__ slab, int64_t nrows,
                                                int64_t ncol, double* __restrict__ out) {
  __shared__ double sh[4];
  const int64_t k = blockIdx.x;
  double s = 0.0;
  for (int64_t r = threadIdx.x; r < nrows; r += 256) s += slab[r * ncol + k];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) out[k] = s;
}

// k_sum_vec (block 0) and k_diag (every block) in one launch: the tail of the K22 chain
__global__ void __launch_bounds__(256) k_sum_and_diag(const double* __restrict__ v, int64_t count,
                                                      double* __restrict__ sum,
                                                      const double* __restrict__ A, int64_t mp,
                                                      int64_t lda, double* __restrict__ out) {
  __shared__ double sh[4];
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j < mp) out[j] = A[j * lda + j];
  if (blockIdx.x == 0) {
    double s = 0.0;
    for (int64_t e = threadIdx.x; e < count; e += 256) s += v[e];
    s = block_sum(s, sh);
    if (threadIdx.x == 0) sum[0] = s;
  }
}

__global__ void __launch_bounds__(256) k_diag(const double* __restrict__ A, int64_t mp,
                                              int64_t lda, double* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j < mp) out[j] = A[j * lda + j];
}

__global__ void __launch_bounds__(256) k_fitc_z(const double* __restrict__ q, int64_t n,
                                                int64_t n_pad, double c0, double* __restrict__ w,
                                                double* __restrict__ slab) {
  __shared__ double sh[4];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_pad; i += (int64_t)gridDim.x * 256) {
    if (i < n) {
      const double z = c0 - q[i];
      w[i] = 1.0 / z;
      s += log(z);
    } else {
      w[i] = 0.0;
    }
  }
  s = block_sum(s, sh);
  if (threadIdx.x == 0) slab[blockIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_fitc_omega(const double* __restrict__ alpha,
                                                    const double* __restrict__ w,
                                                    const double* __restrict__ p, int64_t n,
                                                    int64_t n_pad, double* __restrict__ omega,
                                                    double* __restrict__ slab) {
  __shared__ double sh[4];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_pad; i += (int64_t)gridDim.x * 256) {
    double o = 0.0;
    if (i < n) o = alpha[i] * alpha[i] - (w[i] - w[i] * w[i] * p[i]);
    omega[i] = o;
    s += o;
  }
  s = block_sum(s, sh);
  if (threadIdx.x == 0) slab[blockIdx.x] = s;
}

// VI phase-2 row pass over the m x m operands, one wave per row j (replaces a GEMV, an axpby
// and a dot-product pair):  u_j = invz (Binv t)_j,  P_j: = a K22inv_j: + b Binv_j:,
// part_j = sum_k Binv_jk S_jk.  The GEMV keeps k_gemv's lane-strided summation order.
__global__ void __launch_bounds__(256) k_vi_mm_rows(const double* __restrict__ Binv,
                                                    const double* __restrict__ K22inv,
                                                    const double* __restrict__ S,
                                                    const double* __restrict__ t, int64_t mp,
                                                    double invz, double a, double b,
                                                    double* __restrict__ u,
                                                    double* __restrict__ P,
                                                    double* __restrict__ part) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= mp) return;
  const int64_t o = row * mp;
  double su = 0.0, sp = 0.0;
  for (int64_t j = lane; j < mp; j += 64) {
    const double bv = Binv[o + j];
    su = fma(bv, t[j], su);
    sp = fma(bv, S[o + j], sp);
    P[o + j] = a * K22inv[o + j] + b * bv;
  }
  su = wave_sum(su);
  sp = wave_sum(sp);
  if (lane == 0) {
    u[row] = invz * su;
    part[row] = sp;
  }
}

// sc[0] = t . u, sc[1] = sum part (= tr(Binv S)), sc[2] = *rr; one block, fixed order
__global__ void __launch_bounds__(256) k_vi_mm_scalars(const double* __restrict__ t,
                                                       const double* __restrict__ u,
                                                       const double* __restrict__ part,
                                                       int64_t mp, const double* __restrict__ rr,
                                                       double* __restrict__ tu_out,
                                                       double* __restrict__ trbs_out,
                                                       double* __restrict__ rr_out) {
  __shared__ double sh[4];
  double a = 0.0, c = 0.0;
  for (int64_t j = threadIdx.x; j < mp; j += 256) {
    a = fma(t[j], u[j], a);
    c += part[j];
  }
  a = block_sum(a, sh);
  c = block_sum(c, sh);
  if (threadIdx.x == 0) {
    *tu_out = a;
    *trbs_out = c;
    *rr_out = *rr;
  }
}

}  // namespace

hipError_t launch_vi_mm_rows(const double* Binv, const double* K22inv, const double* S,
                             const double* t, int64_t mp, double invz, double a, double b,
                             double* u, double* P, double* part, hipStream_t s) {
  hipLaunchKernelGGL(k_vi_mm_rows, dim3((unsigned)((mp + 3) / 4)), dim3(256), 0, s, Binv, K22inv,
                     S, t, mp, invz, a, b, u, P, part);
  return hipGetLastError();
}

hipError_t launch_vi_mm_scalars(const double* t, const double* u, const double* part, int64_t mp,
                                const double* rr, double* tu_out, double* trbs_out,
                                double* rr_out, hipStream_t s) {
  hipLaunchKernelGGL(k_vi_mm_scalars, dim3(1), dim3(256), 0, s, t, u, part, mp, rr, tu_out,
                     trbs_out, rr_out);
  return hipGetLastError();
}

hipError_t launch_fitc_z(const double* q, int64_t n, int64_t n_pad, double c0, double* w,
                         double* slab, int* nblocks, hipStream_t s) {
  int nb = (int)((n_pad + 255) / 256);
  if (nb > 1024) nb = 1024;
  *nblocks = nb;
  hipLaunchKernelGGL(k_fitc_z, dim3(nb), dim3(256), 0, s, q, n, n_pad, c0, w, slab);
  return hipGetLastError();
}

hipError_t launch_fitc_omega(const double* alpha, const double* w, const double* p, int64_t n,
                             int64_t n_pad, double* omega, double* slab, int* nblocks,
                             hipStream_t s) {
  int nb = (int)((n_pad + 255) / 256);
  if (nb > 1024) nb = 1024;
  *nblocks = nb;
  hipLaunchKernelGGL(k_fitc_omega, dim3(nb), dim3(256), 0, s, alpha, w, p, n, n_pad, omega, slab);
  return hipGetLastError();
}

// Dynamic LDS added to each step's workgroup so that only one fits per CU (66.6 KB static +
// this > 80 KB).  Two chains run side by side (VI phase 2: K22's and Bm's inverses); with two
// workgroups per CU a step's look-ahead workgroup (the chain's critical path: next pivot)
// shared its CU with the other chain's tile updates.  One per CU, the other chain's step
// fills the CUs the short tile updates free.  SGP_GJ_PAD_KB overrides (0 = off).
static size_t gj_step_pad() {
  static long pad = -1;
  if (pad < 0) {
    const char* e = getenv("SGP_GJ_PAD_KB");
    pad = e ? atol(e) * 1024 : 24 * 1024;
  }
  return (size_t)pad;
}

// Workgroups of one persistent chain: at m = 1024 a step's 255 other tiles (~4 us each) must
// finish within the look-ahead task's ~14 us; two chains (K22's, Bm's) may run together.
static int gj_workgroups(int nb) {
  const int cap = SGP_GJ_GMAX;
  return nb * nb < cap ? nb * nb : cap;
}

// the ticket whose publish the next launch withholds: -1, except once per process in a probe
// build run with SGP_PROBE_GJ_WITHHOLD=<ticket> (the watchdog test, tests/test_gpu_gj.py)
static int gj_withhold_ticket() {
#ifdef SGP_PROBE_BUILD
  static std::atomic<int> armed{-2};
  int a = armed.load();
  if (a == -2) {
    const char* e = getenv("SGP_PROBE_GJ_WITHHOLD");
    int want = e ? atoi(e) : -1;
    if (armed.compare_exchange_strong(a, want)) a = want;
  }
  if (a >= 0 && armed.compare_exchange_strong(a, -1)) return a;
#endif
  return -1;
}

static hipError_t gj_persist(const double* src0, const double* src0b, double beta, double* buf,
                             int64_t mp, double* P, double* logd, int* status, unsigned* sync,
                             hipStream_t s) {
  const int nb = (int)(mp / SGP_DB);
  hipLaunchKernelGGL(k_gj_persist, dim3(gj_workgroups(nb)), dim3(256), 0, s, src0, src0b, beta,
                     buf, mp, nb, P, logd, status, sync, gj_withhold_ticket());
  return hipGetLastError();
}

hipError_t dense_spd_inverse(double* A, int64_t mp, double* R, double* P, double* logd,
                             int* status, unsigned* sync, hipStream_t s) {
  const int nb = (int)(mp / SGP_DB);
  return dense_spd_inverse_chain(A, mp, R, P, logd, status, sync, s,
                                 nb > GJ_NB_MAX || SGP_GJ_STEPS);
}

hipError_t dense_spd_inverse_sum(const double* A0, double beta, const double* B0, double* out,
                                 int64_t mp, double* R, double* P, double* logd, int* status,
                                 unsigned* sync, hipStream_t s) {
  const int nb = (int)(mp / SGP_DB);
  return dense_spd_inverse_sum_chain(A0, beta, B0, out, mp, R, P, logd, status, sync, s,
                                     nb > GJ_NB_MAX || SGP_GJ_STEPS);
}

hipError_t dense_spd_inverse_chain(double* A, int64_t mp, double* R, double* P, double* logd,
                                   int* status, unsigned* sync, hipStream_t s, bool per_step) {
  // in place; R: mp x mp ping-pong buffer of the launch-per-step chain (nb > GJ_NB_MAX);
  // P: nb 64x64 pivot inverses (mp * 64 doubles)
  const int nb = (int)(mp / SGP_DB);
  if (!per_step) {
    if (nb > GJ_NB_MAX) return hipErrorInvalidValue;
    return gj_persist(A, nullptr, 0.0, A, mp, P, logd, status, sync, s);
  }
  hipLaunchKernelGGL(k_gj_pivot, dim3(1), dim3(256), 0, s, A, mp, 0, P, logd, status,
                     (const double*)nullptr, 0.0);
  double* src = A;
  double* dst = R;
  for (int k = 0; k < nb; ++k) {
    double* Pn = (k + 1 < nb) ? P + (int64_t)(k + 1) * 4096 : P;
    hipLaunchKernelGGL(k_gj_step<false>, dim3(nb, nb), dim3(256), gj_step_pad(), s, src, dst, mp,
                       k, nb, P + (int64_t)k * 4096, Pn, logd, status, (const double*)nullptr,
                       0.0);
    double* t = src;
    src = dst;
    dst = t;
  }
  if (src != A)
    return hipMemcpyAsync(A, src, sizeof(double) * mp * mp, hipMemcpyDeviceToDevice, s);
  return hipGetLastError();
}

hipError_t dense_spd_inverse_sum_chain(const double* A0, double beta, const double* B0,
                                       double* out, int64_t mp, double* R, double* P, double* logd,
                                       int* status, unsigned* sync, hipStream_t s, bool per_step) {
  // out = inv(A0 + beta B0), the sum formed as step 0 reads it (no axpby launch).  Launch per
  // step (nb > GJ_NB_MAX): step k writes buf[(nb - 1 - k) % 2] (buf = {out, R}), so the last
  // step always lands in out and no copy follows
  const int nb = (int)(mp / SGP_DB);
  if (!per_step) {
    if (nb > GJ_NB_MAX) return hipErrorInvalidValue;
    return gj_persist(A0, B0, beta, out, mp, P, logd, status, sync, s);
  }
  double* buf[2] = {out, R};
  hipLaunchKernelGGL(k_gj_pivot, dim3(1), dim3(256), 0, s, A0, mp, 0, P, logd, status, B0, beta);
  for (int k = 0; k < nb; ++k) {
    double* Pn = (k + 1 < nb) ? P + (int64_t)(k + 1) * 4096 : P;
    double* dst = buf[(nb - 1 - k) % 2];
    if (k == 0)
      hipLaunchKernelGGL(k_gj_step<true>, dim3(nb, nb), dim3(256), gj_step_pad(), s, A0, dst,
                         mp, k, nb, P, Pn, logd, status, B0, beta);
    else
      hipLaunchKernelGGL(k_gj_step<false>, dim3(nb, nb), dim3(256), gj_step_pad(), s,
                         (const double*)buf[(nb - k) % 2], dst, mp, k, nb,
                         P + (int64_t)k * 4096, Pn, logd, status, (const double*)nullptr, 0.0);
  }
  return hipGetLastError();
}

hipError_t dense_axpby(double a, const double* A, double b, const double* B, double* C,
                       int64_t count, hipStream_t s) {
  int nb = (int)((count + 255) / 256);
  if (nb > 4096) nb = 4096;
  hipLaunchKernelGGL(k_axpby, dim3(nb), dim3(256), 0, s, a, A, b, B, C, count);
  return hipGetLastError();
}

hipError_t dense_gemv(const double* A, int64_t mp, const double* x, double scale, double* y,
                      hipStream_t s) {
  hipLaunchKernelGGL(k_gemv, dim3((unsigned)((mp + 3) / 4)), dim3(256), 0, s, A, mp, x, scale,
                     y);
  return hipGetLastError();
}

hipError_t launch_dot(const double* a, const double* b, int64_t count, double* partial,
                      double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_dot_partial, dim3(256), dim3(256), 0, s, a, b, count, partial);
  hipLaunchKernelGGL(k_sum_vec, dim3(1), dim3(256), 0, s, partial, (int64_t)256, out);
  return hipGetLastError();
}

hipError_t launch_colsum(const double* slab, int64_t nrows, int64_t ncol, double* out,
                         hipStream_t s) {
  if (ncol <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_colsum, dim3((unsigned)ncol), dim3(256), 0, s, slab, nrows, ncol, out);
  return hipGetLastError();
}

hipError_t launch_diag(const double* A, int64_t mp, int64_t lda, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_diag, dim3((unsigned)((mp + 255) / 256)), dim3(256), 0, s, A, mp, lda,
                     out);
  return hipGetLastError();
}

hipError_t launch_sum_and_diag(const double* v, int64_t count, double* sum, const double* A,
                               int64_t mp, int64_t lda, double* diag, hipStream_t s) {
  hipLaunchKernelGGL(k_sum_and_diag, dim3((unsigned)((mp + 255) / 256)), dim3(256), 0, s, v,
                     count, sum, A, mp, lda, diag);
  return hipGetLastError();
}

hipError_t launch_sum_small(const double* v, int64_t count, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_sum_vec, dim3(1), dim3(256), 0, s, v, count, out);
  return hipGetLastError();
}
