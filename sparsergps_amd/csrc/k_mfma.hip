// fp64 matrix-core (v_mfma_f64_16x16x4_f64) kernels for gfx950.
//
//  k_syrk_blk  S = K^T diag(w) K over n rows (split-K over row chunks, deterministic slabs, the
//              lower 64-blocks packed 4 per workgroup), plus t = K^T diag(w) r and
//              rr = r^T diag(w) r.  Replaces the reference's `t(Sigma12) %*% ((1/Z) * Sigma12)`
//              (R/vi_functions.R:96, 231, 239).
//  k_contract  G = alpha u^T + K P fused with the d K12/d log(theta) contraction: the GEMM
//              result never leaves registers; the epilogue recomputes K_ij and the pairwise
//              distances and reduces sum_ij G_ij dK_ij/dtheta_p for every p at once.  Replaces
//              the reference's per-parameter loop of ~13 n x m^2 products
//              (R/vi_functions.R:259-419).
//  k_gemm64    small generic GEMM for the m x m dense algebra.
//
// MFMA f64 16x16x4 lane maps (cdna_hip_programming.md Sec.3):
//   A: lane l holds A[l&15][l>>4];  B: lane l holds B[l>>4][l&15];
//   C/D: register r of lane l is C[(l>>4) + 4r][l&15].
#include <algorithm>
#include <vector>

#include "sgp_internal.h"
#include "sgp_probe.h"

namespace {

constexpr int T128 = 128;
constexpr int BK = 16;
constexpr int SB = 144;   // LDS row stride (doubles) of [k][128] operand images: 2*144 % 64 == 32
// LDS row stride of the [128][16] A image.  Odd, because hipcc fuses the A-fragment reads of
// two k-substeps into ds_read2_b64, which banks 16-lane groups mod 32 dwords: an even stride of
// 18 put rows r and r+8 on one bank (2-way conflicts on every A read); 17 is conflict-free for
// ds_read2_b64 and ds_write_b64 alike (rows are then 8-byte aligned only: no b128 stores)
constexpr int SA = 17;
constexpr int SYRK_RGRP = 16;   // slabs summed per group by k_syrk_reduce_grp

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// bijective XCD-aware remap: work items that share operands get consecutive ids on one XCD
__device__ __forceinline__ int64_t xcd_remap(int64_t orig, int64_t nwg) {
  const int64_t x = orig % 8, q = nwg / 8, r = nwg % 8;
  const int64_t base = (x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + orig / 8;
}

__device__ __forceinline__ void load8(const double* __restrict__ g, double2 (&v)[4]) {
  const double2* p = reinterpret_cast<const double2*>(g);
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = p[q];
}
__device__ __forceinline__ void store8(double* s, const double2 (&v)[4]) {
  double2* p = reinterpret_cast<double2*>(s);
#pragma unroll
  for (int q = 0; q < 4; ++q) p[q] = v[q];
}

// ============================================================================ SYRK, 64-blocks
// S = K^T diag(w) K without the diagonal tiles' redundant upper halves.  The lower triangle of
// 64 x 64 blocks (nb64 = mp/64 block rows) is covered by workgroups of 4 blocks (one per wave):
//   * every strictly-lower 128-tile (a > b): its 4 blocks (2a+r, 2b+c), operands = the 128-col
//     K blocks a (image A) and b (image B);
//   * the diagonal 128-tiles' 3 lower blocks D0 = (2t,2t), L = (2t+1,2t), D1 = (2t+1,2t+1) are
//     packed: group g (g < G = ceil(3 nb / 4)) takes tile g's three blocks from image A = K block
//     g, plus one block of tile G + k/3 (k = g; block kind k % 3) from image B = that K block,
//     so G groups cover all 3 nb diagonal blocks.
// At m = 1024 that is 28 + 6 = 34 workgroups per row chunk instead of 36 (5.6% fewer flops).
// Weights scale the A-side fragment in registers (a wave may take both operands from one
// image).  The per-(split, block) slabs are reduced in fixed order by k_syrk_reduce_blk.
__device__ __forceinline__ void syrk_group(int64_t gi, int nb, int wv, int& ta, int& tb, int& rs,
                                           int& cs, int& rp, int& cp) {
  const int64_t noff = (int64_t)nb * (nb - 1) / 2;
  if (gi < noff) {
    int a = (int)((sqrtf(8.0f * (float)gi + 1.0f) + 1.0f) * 0.5f);
    while ((int64_t)a * (a - 1) / 2 > gi) --a;
    while ((int64_t)(a + 1) * a / 2 <= gi) ++a;
    const int b = (int)(gi - (int64_t)a * (a - 1) / 2);
    ta = a; tb = b;
    const int wr = wv >> 1, wc = wv & 1;
    rs = wr; cs = 2 + wc;
    rp = 2 * a + wr; cp = 2 * b + wc;
    return;
  }
  const int g = (int)(gi - noff), G = (3 * nb + 3) / 4;
  const int te = G + g / 3, kind = g % 3;
  ta = g;
  tb = (te < nb) ? te : g;
  if (wv == 0) { rs = 0; cs = 0; rp = 2 * g; cp = 2 * g; }
  else if (wv == 1) { rs = 1; cs = 0; rp = 2 * g + 1; cp = 2 * g; }
  else if (wv == 2) { rs = 1; cs = 1; rp = 2 * g + 1; cp = 2 * g + 1; }
  else if (te < nb) {
    if (kind == 0) { rs = 2; cs = 2; rp = 2 * te; cp = 2 * te; }
    else if (kind == 1) { rs = 3; cs = 2; rp = 2 * te + 1; cp = 2 * te; }
    else { rs = 3; cs = 3; rp = 2 * te + 1; cp = 2 * te + 1; }
  } else {
    rs = cs = rp = cp = -1;   // idle wave (nb too small to pack)
  }
}

// t = K^T (w r) slices (a kernel argument): group gi computes columns [slice * W, slice * W +
// W) of K column panel `panel` (entry panel * S + slice, W = 128 / S; -1: none), spread so that
// no workgroup of the single residency round carries more than one slice (syrk_t_table).
struct SyrkTMap {
  signed char e[128];   // per group: panel * S + slice, or -1
  int S;                // slices per panel
};

// Issue order of one k-step (64 MFMAs, 32 LDS fragment reads, 8 global loads, 8 LDS stores)
// as a scheduling request: each MFMA is followed by at most one LDS read (the first 32), one
// global load (the first 8) and, late in the step, one LDS store.  The compiler's own order
// front-loads every read and store and then waits on the global loads before the stores, so a
// wave that has its SIMD to itself (the co-resident workgroup in an epilogue) leaves the
// matrix pipe idle for the load latency; interleaved, the other instructions issue while the
// MFMAs already queued execute.  tools/micro/kloop.hip (IL 1): 68.4 -> 73.9 TF/s with two
// workgroups per CU, 60.3 -> 70.0 with one.  Needs the step to be a single basic block.
// SPREAD: one LDS read per two MFMAs over the whole step (fragments read one sub-step ahead:
// fewer live registers, for kernels whose epilogue shares the register budget).
// PAT (experiments, tools/micro/con_trace.hip): where the LDS stores go (0: MFMA slots 48-55,
// 2: 56-63, 3: 32-39, 4: not grouped)
// NVMEM: global loads of the step placed one per MFMA slot (the 8 operand loads).
// NMFMA: MFMAs in the step (64; 32 for the contraction's 128 x 64 tail tiles), the store slots
// keeping their distance from the end of the step.
template <bool SPREAD = false, int PAT = 0, int NVMEM = 8, int NMFMA = 64>
__device__ __forceinline__ void mfma_interleave() {
#pragma unroll
  for (int i = 0; i < NMFMA; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                      // MFMA
    if (i >= SGP_IL_VMEM0 && i < SGP_IL_VMEM0 + NVMEM)
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                    // VMEM read
    if (SPREAD ? (i & 1) == 0 : i < 32)
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                    // DS read
    constexpr int w0 = PAT == 2 ? NMFMA - 8 : PAT == 3 ? NMFMA / 2 : NMFMA - 16;
    if (PAT != 4 && i >= w0 && i < w0 + 8)
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);                    // DS write
  }
}
// With-t SYRK: the next k-step's operand loads pinned to the top of the step (a scheduling
// barrier after them, no VMEM groups in the interleave).  The group-barrier request alone
// leaves the loads at MFMA slots 16-54 of 64 with their vmcnt wait 4-30 slots later
// (tools/isa_step.py); pinned, the t-carrying SYRK runs 1.7 % faster (FITC C3 17.95 -> 17.64
// ms), but the same pin made the VI SYRK 10 % and the contraction 1.5 % slower and the omega
// SYRK 5 % slower (profiles/r3/gload_pin_ab.txt), so only the t variants use it.

// Balanced plan (syrk_plan_bal): a diagonal 128-tile t of S -- 36 lower 16x16 fragments -- split
// over the 4 waves of one workgroup as fragment rows v and 7 - v (9 fragments each: 36 MFMAs per
// step, not the 64 of a packed 64-block wave); these workgroups take longer row chunks so that
// they finish with the strictly-lower tiles' (k_syrk_blk's off-diagonal groups).  Operands from
// one staged image (K's column panel t).  WMODE 2 stages sqrt(w)-scaled rows (both operands
// scaled), WMODE 1 scales the two A fragments of a k-substep.  TMODE != 0 (with WMODE 1): the
// workgroup also forms panel t's slice of t = K^T (w o r) (TMODE 1) or K^T tv (TMODE 2) over its
// rows from the same image -- column tid % 128, the step's rows tid / 128, +2, ... -- and, for
// t == 0, rr = sum (w r) r or sum tv r (the off-diagonal groups of k_syrk_blk<.., 3, ..> carry
// no t work).
template <int V, int WMODE, int TMODE>
__device__ __forceinline__ void syrk_dt_body(const double* __restrict__ K, int64_t mp,
                                             const double* __restrict__ w,
                                             const double* __restrict__ r,
                                             const double* __restrict__ tv, int t, int64_t rbeg,
                                             int nsteps, double (*Ka)[BK * SB], double (*ws)[BK],
                                             double (*rw)[BK], double& tacc, double& rrp,
                                             double* __restrict__ out) {
  constexpr int R0 = V, R1 = 7 - V, N0 = R0 + 1, N1 = R1 + 1;
  constexpr bool WITH_T = TMODE != 0;
  const int tid = threadIdx.x, lane = tid & 63;
  d4 acc0[N0], acc1[N1];
#pragma unroll
  for (int c = 0; c < N0; ++c) acc0[c] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int c = 0; c < N1; ++c) acc1[c] = d4{0.0, 0.0, 0.0, 0.0};
  const int lrow = tid >> 4, lc = tid & 15;
  const double2* gA = reinterpret_cast<const double2*>(K + (rbeg + lrow) * mp + t * (int64_t)T128) + lc;
  const int64_t gstep = BK * mp / 2;
  double2 v[4];
  double vw = 1.0, vsa = 1.0, vrr = 0.0, vr = 0.0;
  double t4[4] = {0.0, 0.0, 0.0, 0.0};
  const int tcol = tid & (T128 - 1), trow = tid >> 7;
#define SDT_GLOAD(step)                                                         \
  {                                                                             \
    const int64_t o_ = (int64_t)(step) * gstep;                                 \
    const int64_t rr_ = rbeg + (int64_t)(step) * BK + (tid & (BK - 1));        \
    _Pragma("unroll") for (int q = 0; q < 4; ++q) v[q] = gA[o_ + 16 * q];       \
    if constexpr (WMODE == 1) vw = w[rr_];                                      \
    if constexpr (WMODE == 2) vsa = w[rbeg + (int64_t)(step) * BK + lrow];      \
    if constexpr (WITH_T) {                                                     \
      vrr = r[rr_];                                                             \
      if constexpr (TMODE == 2) vr = tv[rr_];                                   \
    }                                                                           \
  }
#define SDT_SSTORE(buf, fold)                                                   \
  {                                                                             \
    double2* p_ = reinterpret_cast<double2*>(&Ka[buf][lrow * SB]) + lc;         \
    _Pragma("unroll") for (int q = 0; q < 4; ++q) {                             \
      double2 x_ = v[q];                                                        \
      if constexpr (WMODE == 2) { x_.x *= vsa; x_.y *= vsa; }                   \
      p_[16 * q] = x_;                                                          \
    }                                                                           \
    if constexpr (WMODE == 1) ws[buf][tid & (BK - 1)] = vw;                     \
    if constexpr (WITH_T) {                                                     \
      const double rw_ = TMODE == 2 ? vr : vw * vrr;                            \
      rw[buf][tid & (BK - 1)] = rw_;                                            \
      rrp = fma(rw_ * (fold), vrr, rrp);                                        \
    }                                                                           \
  }
  if (nsteps > 0) {
    SDT_GLOAD(0);
    SDT_SSTORE(0, 1.0);
  }
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    const int cur = step & 1;
    const bool more = step + 1 < nsteps;
    SDT_GLOAD(more ? step + 1 : step);   // one basic block per step
    const double* Kc = Ka[cur];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int krow = kk * 4 + (lane >> 4);
      const double* row = Kc + krow * SB + (lane & 15);
      double a0 = row[R0 * 16], a1 = row[R1 * 16];
      if constexpr (WMODE == 1) {
        const double wk = ws[cur][krow];
        a0 *= wk;
        a1 *= wk;
      }
#pragma unroll
      for (int c = 0; c < N1; ++c) {
        const double b = row[c * 16];
        if (c < N0) acc0[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b, acc0[c], 0, 0, 0);
        acc1[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b, acc1[c], 0, 0, 0);
      }
    }
    if constexpr (WITH_T) {
      // the t slice from the current image: rows trow, trow + 2, ... of the step
#pragma unroll
      for (int k = 0; k < BK / 2; ++k) {
        const int q = trow + 2 * k;
        t4[k & 3] = fma(rw[cur][q], Kc[q * SB + tcol], t4[k & 3]);
      }
    }
    SDT_SSTORE(cur ^ 1, more ? 1.0 : 0.0);   // on the last step into the idle buffer
    if constexpr (SGP_SDT_IL && WMODE != 1) mfma_interleave<false, 2, 4, 36>();
    __syncthreads();
  }
#undef SDT_GLOAD
#undef SDT_SSTORE
  tacc = (t4[0] + t4[1]) + (t4[2] + t4[3]);
  // fragment (R, c) of tile t -> 64-block (2t + R/4, 2t + c/4) of the slab
#pragma unroll
  for (int c = 0; c < N1; ++c)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      if (hh == 0 && c >= N0) continue;
      const int R = hh == 0 ? R0 : R1;
      const d4& a = hh == 0 ? acc0[c] : acc1[c];
      const int rp = 2 * t + R / 4, cp = 2 * t + c / 4;
      double* blk = out + (int64_t)(rp * (rp + 1) / 2 + cp) * 4096;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        blk[((R % 4) * 16 + (lane >> 4) + 4 * q) * 64 + (c % 4) * 16 + (lane & 15)] = a[q];
    }
}

// slab_t / slab_rr: split sd's [nb][128] t partials and its rr partial (TMODE != 0)
template <int WMODE, int TMODE>
__device__ __forceinline__ void syrk_dtile(const double* __restrict__ K, int64_t n_pad,
                                           int64_t mp, const double* __restrict__ w,
                                           const double* __restrict__ r,
                                           const double* __restrict__ tv, int t, int nb,
                                           int64_t sd, int64_t chunk, double (*Ka)[BK * SB],
                                           double (*ws)[BK], double (*rw)[BK],
                                           double* __restrict__ out,
                                           double* __restrict__ slab_t,
                                           double* __restrict__ slab_rr) {
  const int64_t rbeg = sd * chunk;
  int64_t rend = rbeg + chunk;
  if (rend > n_pad) rend = n_pad;
  const int nsteps = rend > rbeg ? (int)((rend - rbeg) / BK) : 0;
  double tacc = 0.0, rrp = 0.0;
  switch (threadIdx.x >> 6) {   // wave-uniform
    case 0: syrk_dt_body<0, WMODE, TMODE>(K, mp, w, r, tv, t, rbeg, nsteps, Ka, ws, rw, tacc, rrp, out); break;
    case 1: syrk_dt_body<1, WMODE, TMODE>(K, mp, w, r, tv, t, rbeg, nsteps, Ka, ws, rw, tacc, rrp, out); break;
    case 2: syrk_dt_body<2, WMODE, TMODE>(K, mp, w, r, tv, t, rbeg, nsteps, Ka, ws, rw, tacc, rrp, out); break;
    default: syrk_dt_body<3, WMODE, TMODE>(K, mp, w, r, tv, t, rbeg, nsteps, Ka, ws, rw, tacc, rrp, out); break;
  }
  if constexpr (TMODE != 0) {
    // the two row halves of each column, then rr from the BK staging lanes of tile 0
    const int tid = threadIdx.x;
    double* tsh = &Ka[0][0];   // every wave is past its last read of the images
    tsh[tid] = tacc;
    __syncthreads();
    if (tid < T128) slab_t[(sd * nb + t) * T128 + tid] = tsh[tid] + tsh[tid + T128];
    if (t == 0 && tid < 64) {
      double v = tid < BK ? rrp : 0.0;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (tid == 0) slab_rr[sd] = v;
    }
  }
}

// WMODE: how rows are weighted.  0: not (VI; compiled out, the k-loop would otherwise multiply
// every A fragment by 1.0); 1: by w on the A fragments, between their LDS reads and the MFMAs
// (16 fp64 VALU per step on the MFMA operand path; any sign: FITC, Laplace's a and the
// t-carrying forms); 2 (S only): w >= 0 given as sqrt(w) (k_sqrt_rows), scaling both staged
// images as they are stored -- the same VALU count, but on the staging path of the next step
// instead of in front of this step's MFMAs (Laplace's NR objectives S_B and S_Z: 2.7-4 %).
// TMODE: 0 no t; 1 t = K^T (w o r) with rr = sum w r^2; 2 t = K^T tv with rr = sum tv r.
// TR: rows of the t slice per thread and step, 8 / S for S slices per panel (syrk_t_table)
template <int TMODE, int WMODE, int TR = 2>
__global__ void __launch_bounds__(256, 2)
k_syrk_blk(const double* __restrict__ K, int64_t n_pad, int64_t mp, const double* __restrict__ w,
           const double* __restrict__ r, const double* __restrict__ tv,
           int64_t chunk, int ngroups, int nb, double* __restrict__ slab,
           double* __restrict__ slab_t, double* __restrict__ slab_rr, SyrkTMap tm,
           int64_t nwg_blk, int64_t chunk_d, double* __restrict__ slab_d) {
  __shared__ __attribute__((aligned(16))) double Ka[2][BK * SB];
  __shared__ __attribute__((aligned(16))) double Kb[2][BK * SB];
  __shared__ double ws[2][BK];
  __shared__ double rw[2][BK];   // with_t: (w r)_i or tv_i of the step's rows

  // the balanced plan's diagonal-tile workgroups follow the packed groups' grid (with t: they
  // form it, the off-diagonal groups of WMODE 3 carry none)
  if constexpr (TMODE == 0 || WMODE == 3) {
    if ((int64_t)blockIdx.x >= nwg_blk) {
      const int64_t loc = (int64_t)blockIdx.x - nwg_blk;
      const int t = (int)(loc % nb);
      const int64_t sd = loc / nb;
      syrk_dtile<WMODE == 3 ? 1 : WMODE, TMODE>(
          K, n_pad, mp, w, r, tv, t, nb, sd, chunk_d, Ka, ws, rw,
          slab_d + sd * ((int64_t)(2 * nb) * (2 * nb + 1) / 2) * 4096, slab_t, slab_rr);
      return;
    }
  }
  const int64_t nwg = nwg_blk;
  const int64_t wgid = xcd_remap(blockIdx.x, nwg);
  const int split = (int)(wgid / ngroups);
  const int64_t gi = wgid % ngroups;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int ta, tb, rs, cs, rp, cp;
  syrk_group(gi, nb, wv, ta, tb, rs, cs, rp, cp);
  const bool active = rs >= 0;
  // t = K^T (w r) (or K^T tv): this group's slice of one of its two K column panels
  // (c_tmap); rr from diagonal group 0.
  const int64_t noff = (int64_t)nb * (nb - 1) / 2;
  const int dg = (gi >= noff) ? (int)(gi - noff) : -1;
  constexpr bool WITH_T = TMODE != 0 && WMODE != 3;   // WMODE 3: t on the diagonal tiles
  constexpr bool with_t = WITH_T;
  static_assert(!(WMODE == 2 && TMODE != 0), "sqrt(w)-scaled images: S only");
  // WMODE 3 (balanced plan only, every group off-diagonal: rows from image A, columns from
  // image B): image A staged as w o K, image B as K -- no per-fragment weight, any sign
  constexpr bool SCALE_A = WMODE == 2 || WMODE == 3, SCALE_B = WMODE == 2;
  // tm.S == 0 (more groups than the table holds, m > 1920): one whole-panel slice per panel,
  // panel a >= 1 on the strictly-lower group (a, 0) and panel 0 on diagonal group 0 -- distinct
  // groups, each holding its panel as image A
  int tmap = -1;
  if (with_t) {
    if (tm.S > 0) tmap = (int)tm.e[gi];
    else if (gi < noff) tmap = (tb == 0) ? ta : -1;
    else if (dg == 0) tmap = 0;
  }
  const int tS = (with_t && tm.S > 0) ? tm.S : 1, tW = T128 / tS;
  const int tpan = tmap >= 0 ? tmap / tS : -1;
  // all 256 threads share the slice: column tid % tW, rows trg, trg + tng, ... of each step
  const int tng = 256 / tW, trg = tid / tW;
  const int tcol = tmap >= 0 ? (tmap % tS) * tW + tid % tW : 0;   // column within the panel
  const bool t_on = with_t && tmap >= 0;
  const bool t_inb = tpan != ta;                               // panel held as image B
  // rr = sum (w r)_i r_i: each of the BK staging threads of diagonal group 0 folds in its own
  // row as it stages it (no per-step loop over the BK rows on one thread)
  const bool t_rr = with_t && dg == 0 && tid < BK;
  double rrp = 0.0;
  double tacc4[4] = {0.0, 0.0, 0.0, 0.0}, vrr = 0.0, vr = 0.0;
  const int64_t rbeg = (int64_t)split * chunk;
  int64_t rend = rbeg + chunk;
  if (rend > n_pad) rend = n_pad;
  const int nsteps = (int)((rend - rbeg) / BK);

  d4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};

  const int lrow = tid >> 4, lc = tid & 15;
  // with t: (w r)_i, or tv_i when the caller passes tv (Laplace); every lane stages the row
  // tid % BK so the step has no lane-dependent branch
  constexpr bool has_tv = TMODE == 2;
  const double2* gA = reinterpret_cast<const double2*>(K + (rbeg + lrow) * mp + ta * (int64_t)T128) + lc;
  const double2* gB = reinterpret_cast<const double2*>(K + (rbeg + lrow) * mp + tb * (int64_t)T128) + lc;
  const int64_t gstep = BK * mp / 2;
  double2 va0, va1, va2, va3, vb0, vb1, vb2, vb3;
  double vw = 1.0, vsa = 1.0;   // vw: row tid % BK's weight (WMODE 1); vsa: row lrow's sqrt(w)
  // operand images and column offsets of this wave's row / column panels
  const int ra = (rs >> 1) & 1, ro = (rs & 1) * 64;
  const int ca_ = (cs >> 1) & 1, co = (cs & 1) * 64;

#define SYRKB_GLOAD(step)                                                       \
  {                                                                             \
    const int64_t o_ = (int64_t)(step) * gstep;                                 \
    va0 = gA[o_]; va1 = gA[o_ + 16]; va2 = gA[o_ + 32]; va3 = gA[o_ + 48];      \
    vb0 = gB[o_]; vb1 = gB[o_ + 16]; vb2 = gB[o_ + 32]; vb3 = gB[o_ + 48];      \
    /* one block: every lane stages row tid % BK (16 lanes per row) */          \
    const int64_t rr_ = rbeg + (int64_t)(step) * BK + (tid & (BK - 1));        \
    if constexpr (WMODE == 1) vw = w[rr_];                                      \
    if constexpr (SCALE_A) vsa = w[rbeg + (int64_t)(step) * BK + lrow];        \
    if constexpr (WITH_T) {                                                     \
      vrr = r[rr_];                                                             \
      if constexpr (has_tv) vr = tv[rr_];                                       \
    }                                                                           \
  }
// fold: 1 when the staged rows are a new step's (rr counts each row once), 0 for the last
// step's reload of its own rows
#define SYRKB_SSTORE(buf, fold)                                                 \
  {                                                                             \
    double2* pa_ = reinterpret_cast<double2*>(&Ka[buf][lrow * SB]) + lc;        \
    double2* pb_ = reinterpret_cast<double2*>(&Kb[buf][lrow * SB]) + lc;        \
    if constexpr (SCALE_A) {             /* sqrt(w) K (WMODE 2) or w o K (3) */ \
      va0.x *= vsa; va0.y *= vsa; va1.x *= vsa; va1.y *= vsa;                   \
      va2.x *= vsa; va2.y *= vsa; va3.x *= vsa; va3.y *= vsa;                   \
    }                                                                           \
    if constexpr (SCALE_B) {                                                    \
      vb0.x *= vsa; vb0.y *= vsa; vb1.x *= vsa; vb1.y *= vsa;                   \
      vb2.x *= vsa; vb2.y *= vsa; vb3.x *= vsa; vb3.y *= vsa;                   \
    }                                                                           \
    pa_[0] = va0; pa_[16] = va1; pa_[32] = va2; pa_[48] = va3;                  \
    pb_[0] = vb0; pb_[16] = vb1; pb_[32] = vb2; pb_[48] = vb3;                  \
    if constexpr (WMODE == 1) ws[buf][tid & (BK - 1)] = vw;                     \
    if constexpr (WITH_T) {                                                     \
      double rw_;                                  /* tv_i or (w r)_i */        \
      if constexpr (has_tv) rw_ = vr;                                           \
      else rw_ = vw * vrr;                                                      \
      rw[buf][tid & (BK - 1)] = rw_;                                            \
      rrp = fma(rw_ * (fold), vrr, rrp);   /* used by the t_rr lanes only */    \
    }                                                                           \
  }

  if (nsteps > 0) {
    SYRKB_GLOAD(0);
    SYRKB_SSTORE(0, 1.0);
  }
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    const int cur = step & 1;
    // One basic block per step, which the interleaved schedule below needs: the last step
    // reloads its own rows (and weights) and stores them into the idle buffer (t variants: with
    // fold = 0, so rr counts them once); inactive waves run their MFMAs on valid LDS operands
    // (results never written).  The t slice is accumulated inside the block (below).
    const bool more = step + 1 < nsteps;
    SYRKB_GLOAD(more ? step + 1 : step);
    if constexpr (WITH_T) __builtin_amdgcn_sched_barrier(0);
    const double* As = (ra ? Kb[cur] : Ka[cur]) + ro;
    const double* Bs = (ca_ ? Kb[cur] : Ka[cur]) + co;
    {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int krow = kk * 4 + (lane >> 4);
        double af[4], bf[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          af[f] = As[krow * SB + f * 16 + (lane & 15)];
          bf[f] = Bs[krow * SB + f * 16 + (lane & 15)];
        }
        if constexpr (WMODE == 1) {
          const double wk = ws[cur][krow];
#pragma unroll
          for (int f = 0; f < 4; ++f) af[f] *= wk;
        }
#pragma unroll
        for (int fm = 0; fm < 4; ++fm)
#pragma unroll
          for (int fn = 0; fn < 4; ++fn)
            acc[fm][fn] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[fm], bf[fn], acc[fm][fn], 0, 0, 0);
      }
    }
    SYRKB_SSTORE(cur ^ 1, more ? 1.0 : 0.0);
    // VMEM groups for the operand loads in the first 8 MFMA slots (the compiler still places
    // them at slots 16-54: tools/isa_step.py; giving the row scalars slots of their own as
    // well, ahead of the operands, was 3 % slower at C3 FITC); the t variants pin them instead
    mfma_interleave<false, SGP_SYRK_IL_PAT, WITH_T ? 0 : 8>();
    // t: at most one W-column slice per workgroup, shared by all four waves (TR = BK / (256 / W)
    // rows per thread and step), from the current buffer (the stores above went to the other).
    // Branch-free, so it stays inside the step's basic block and its LDS reads interleave with
    // the MFMAs: workgroups without a slice read column 0 and never use the sums.  (Round 2-3:
    // a branch after the block, its loop over rows waiting on each read in turn, cost the
    // with-t SYRK 16 % against the same SYRK without t.)
    if constexpr (WITH_T) {
      const double* img = (t_inb ? Kb[cur] : Ka[cur]) + tcol;
      double a_[TR], b_[TR];
#pragma unroll
      for (int k = 0; k < TR; ++k) {
        const int q = trg + k * (BK / TR);
        a_[k] = rw[cur][q];
        b_[k] = img[q * SB];
      }
#pragma unroll
      for (int k = 0; k < TR; ++k) tacc4[k & 3] = fma(a_[k], b_[k], tacc4[k & 3]);
    }
    __syncthreads();
  }
#undef SYRKB_GLOAD
#undef SYRKB_SSTORE

  if constexpr (WITH_T) {
    // the row groups' partials of each column, combined in a fixed order (every thread of the
    // block reaches these barriers: t_on is uniform per workgroup)
    __syncthreads();                          // the operand images are no longer read
    double* tsh = &Ka[0][0];
    if (t_on) tsh[tid] = (tacc4[0] + tacc4[1]) + (tacc4[2] + tacc4[3]);
    __syncthreads();
    if (t_on && tid < tW) {
      double v = 0.0;
      for (int g = 0; g < tng; ++g) v += tsh[tid + g * tW];
      slab_t[((int64_t)split * nb + tpan) * T128 + tcol] = v;
    }
  }
  if (dg == 0 && with_t && wv == 0) {          // lanes 0..BK-1 of wave 0 hold the partials
    double v = t_rr ? rrp : 0.0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (tid == 0) slab_rr[split] = v;
  }
  if (!active) return;
  const int64_t bid = (int64_t)rp * (rp + 1) / 2 + cp;
  const int64_t nblk = (int64_t)(2 * nb) * (2 * nb + 1) / 2;
  double* out = slab + ((int64_t)split * nblk + bid) * 4096;
#pragma unroll
  for (int fm = 0; fm < 4; ++fm)
#pragma unroll
    for (int fn = 0; fn < 4; ++fn)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = fm * 16 + (lane >> 4) + 4 * q;
        const int col = fn * 16 + (lane & 15);
        out[row * 64 + col] = acc[fm][fn][q];
      }
}

// sqrt of non-negative row weights for k_syrk_blk<.., WMODE 2, ..> (NaN for a negative one, which
// then surfaces as a failed factorisation instead of a silently wrong S)
__global__ void __launch_bounds__(256)
k_sqrt_rows(const double* __restrict__ w, int64_t n, double* __restrict__ sw) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) sw[i] = sqrt(w[i]);
}

// S (mp x mp full symmetric) from the per-split lower 64-blocks, fixed split order
__global__ void __launch_bounds__(256)
k_syrk_reduce_grp(double* __restrict__ slab, int splits, int64_t nblk) {
  // first stage for many splits (small m): split group g = blockIdx.z sums its SYRK_RGRP
  // slabs in order into the group's first slab (each element touched by one thread only)
  const int64_t bid = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int s0 = blockIdx.z * SYRK_RGRP;
  const int s1 = s0 + SYRK_RGRP < splits ? s0 + SYRK_RGRP : splits;
  // all the group's loads in flight before the (ordered) sum: the loop form waited on each
  double a[SYRK_RGRP];
#pragma unroll
  for (int q = 0; q < SYRK_RGRP; ++q)
    a[q] = s0 + q < s1 ? slab[((int64_t)(s0 + q) * nblk + bid) * 4096 + e] : 0.0;
  double v = 0.0;
#pragma unroll
  for (int q = 0; q < SYRK_RGRP; ++q)
    if (s0 + q < s1) v += a[q];
  slab[((int64_t)s0 * nblk + bid) * 4096 + e] = v;
}

__global__ void __launch_bounds__(256)
k_syrk_reduce_blk(const double* __restrict__ slab, int splits, int64_t nblk, int64_t mp,
                  double* __restrict__ red, int stride, const double* __restrict__ rr_src,
                  double* __restrict__ rr_dst, int packed, const double* __restrict__ slab_d,
                  int splits_d, int stride_d) {
  const int64_t bid = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;   // element of the 64 x 64 block
  // a precomputed r^T r, and the 7 padding words after it zeroed (VI's red1 tail: a multi-GPU
  // all-reduce sums them, so they must not be whatever the buffer held)
  if (rr_src && bid == 0 && e < 8) rr_dst[e] = e == 0 ? *rr_src : 0.0;
  int rp = (int)((sqrtf(8.0f * (float)bid + 1.0f) - 1.0f) * 0.5f);
  while ((int64_t)(rp + 1) * (rp + 2) / 2 <= bid) ++rp;
  while ((int64_t)rp * (rp + 1) / 2 > bid) --rp;
  const int cp = (int)(bid - (int64_t)rp * (rp + 1) / 2);
  // a diagonal 64-block's upper fragments are not written by k_syrk_s256: the lower element of
  // each symmetric pair writes both (a, b) and (b, a), for both SYRK kernels (packed: the
  // block as it is, its upper fragments zero; k_unpack_lower64 mirrors).  Inside a diagonal
  // 16 x 16 fragment both elements of a pair are computed; with weights they differ in the last
  // bit ((w_k K_ka) K_kb against (w_k K_kb) K_ka), so only the lower one (row >= column) may
  // write the pair -- two writers of one address made FITC and Laplace non-deterministic
  const bool upper = rp == cp && (e / 64) / 16 < (e % 64) / 16;
  if (upper && !packed) return;
  if (!packed && rp == cp && (e / 64) < (e % 64)) return;
  // the balanced plan keeps the diagonal 128-tiles' blocks in their own slab region
  if (slab_d && rp / 2 == cp / 2) {
    slab = slab_d;
    splits = splits_d;
    stride = stride_d;
  }
  double v = 0.0;
  if (!upper)
    for (int sp0 = 0; sp0 < splits; sp0 += 16 * stride) {   // 16 loads in flight, summed in order
      double a[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int sp = sp0 + q * stride;
        a[q] = sp < splits ? slab[((int64_t)sp * nblk + bid) * 4096 + e] : 0.0;
      }
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (sp0 + q * stride < splits) v += a[q];
    }
  if (packed) {
    red[bid * 4096 + e] = v;
    return;
  }
  const int64_t a = (int64_t)rp * 64 + e / 64, b = (int64_t)cp * 64 + e % 64;
  red[a * mp + b] = v;
  red[b * mp + a] = v;
}

// k_syrk_reduce_grp and k_syrk_reduce_blk in one launch (one slab region, splits > SYRK_RGRP):
// group g of a 256-element slice sums its SYRK_RGRP slabs as k_syrk_reduce_grp does and stores
// the total write-through (sc1); the slice's last group to finish (a ticket per slice,
// rsync[bid * 16 + x]) sums the group totals in group order -- the same order and values as
// k_syrk_reduce_blk -- and resets the ticket.  Nothing waits on another workgroup.
__global__ void __launch_bounds__(256)
k_syrk_reduce_last(double* __restrict__ slab, int splits, int64_t nblk, int64_t mp,
                   double* __restrict__ red, const double* __restrict__ rr_src,
                   double* __restrict__ rr_dst, int packed, unsigned* __restrict__ rsync) {
  const int64_t bid = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int ng = (int)gridDim.z;
  const int s0 = blockIdx.z * SYRK_RGRP;
  const int s1 = s0 + SYRK_RGRP < splits ? s0 + SYRK_RGRP : splits;
  double a[SYRK_RGRP];
#pragma unroll
  for (int q = 0; q < SYRK_RGRP; ++q)
    a[q] = s0 + q < s1 ? slab[((int64_t)(s0 + q) * nblk + bid) * 4096 + e] : 0.0;
  double v = 0.0;
#pragma unroll
  for (int q = 0; q < SYRK_RGRP; ++q)
    if (s0 + q < s1) v += a[q];
  __hip_atomic_store(slab + ((int64_t)s0 * nblk + bid) * 4096 + e, v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's totals have landed
  __syncthreads();
  __shared__ int s_last;
  unsigned* tk = rsync + bid * 16 + blockIdx.x;
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (int)(t == (unsigned)(ng - 1));
    if (s_last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;
  if (rr_src && bid == 0 && e < 8) rr_dst[e] = e == 0 ? *rr_src : 0.0;
  int rp = (int)((sqrtf(8.0f * (float)bid + 1.0f) - 1.0f) * 0.5f);
  while ((int64_t)(rp + 1) * (rp + 2) / 2 <= bid) ++rp;
  while ((int64_t)rp * (rp + 1) / 2 > bid) --rp;
  const int cp = (int)(bid - (int64_t)rp * (rp + 1) / 2);
  // which elements write, as in k_syrk_reduce_blk
  const bool upper = rp == cp && (e / 64) / 16 < (e % 64) / 16;
  if (upper && !packed) return;
  if (!packed && rp == cp && (e / 64) < (e % 64)) return;
  double t = 0.0;
  if (!upper)
    for (int g0 = 0; g0 < ng; g0 += 16) {   // 16 loads in flight, summed in group order
      double b[16];
#pragma unroll
      for (int q = 0; q < 16; ++q)
        b[q] = g0 + q < ng ? __hip_atomic_load(slab + ((int64_t)(g0 + q) * SYRK_RGRP * nblk +
                                                       bid) * 4096 + e,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                           : 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (g0 + q < ng) t += b[q];
    }
  if (packed) {
    red[bid * 4096 + e] = t;
    return;
  }
  const int64_t ra = (int64_t)rp * 64 + e / 64, rb = (int64_t)cp * 64 + e % 64;
  red[ra * mp + rb] = t;
  red[rb * mp + ra] = t;
}

// Full symmetric S (mp x mp) from its packed lower 64-blocks (k_syrk_reduce_blk, packed): an
// element on or below the diagonal is read as stored, the rest from its mirror.
__global__ void __launch_bounds__(256)
k_unpack_lower64(const double* __restrict__ packed, int64_t mp, double* __restrict__ S) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= mp * mp) return;
  const int64_t a = idx / mp, b = idx % mp;
  const int64_t ra = a / 64, rb = b / 64;
  const int ia = (int)(a % 64), ib = (int)(b % 64);
  // the lower element of every pair (row >= column), also inside a diagonal 16 x 16 fragment,
  // where both are stored: S comes out exactly symmetric, as the unpacked reduction writes it
  const bool lower = ra > rb || (ra == rb && ia >= ib);
  const int64_t r = lower ? ra : rb, c = lower ? rb : ra;
  const int i = lower ? ia : ib, j = lower ? ib : ia;
  S[idx] = packed[(r * (r + 1) / 2 + c) * 4096 + i * 64 + j];
}

// ============================================================================ SYRK, mp = 256
// S = K^T diag(w) K for mp = 256 (C2's knot count), without t.  The packed 64-block kernel
// above runs 12 wave-blocks per row chunk there for 8 of algorithmic work (its diagonal
// 64-blocks whole and two idle packing slots: 1.5 n m^2 executed), and every packed workgroup
// keeps one full-cost wave, so skipping work inside it does not shorten the barrier-bound step
// (profiles/r4/syrk_kind_skip_ab.txt).  Here the 136 lower 16x16 fragments of S are split evenly
// over the 8 waves of a row chunk's two workgroups: wave v owns fragment rows v and 15 - v
// (v + 1 and 16 - v fragments: 17 each), so the chunk executes 136 / 128 = 1.06 n m^2 and every
// wave has the same MFMA count.  Each workgroup stages the chunk's whole 16 x 256 row slab (two
// workgroups per CU: one waits at its step barrier while the other computes -- one 512-thread
// workgroup sharing a single staged slab ran 20 % slower); the weights scale the two A
// fragments of a k-substep (2 multiplies, not 4).  The lower fragments land in the 64-block
// slabs of k_syrk_blk (k_syrk_reduce_blk mirrors a diagonal block's lower fragments and skips
// its upper ones, which are never written).
constexpr int SB2 = 272;   // [k][256] image row stride: 2 * 272 % 64 == 32, as SB

template <int V, bool WEIGHTED>
__device__ __forceinline__ void syrk256_body(const double* __restrict__ K,
                                             const double* __restrict__ w, int64_t rbeg,
                                             int nsteps, double (*Ks)[BK * SB2],
                                             double (*ws)[BK], double* __restrict__ out) {
  constexpr int R0 = V, R1 = 15 - V, N0 = R0 + 1, N1 = R1 + 1;
  const int tid = threadIdx.x, lane = tid & 63;
  d4 acc0[N0], acc1[N1];
#pragma unroll
  for (int c = 0; c < N0; ++c) acc0[c] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int c = 0; c < N1; ++c) acc1[c] = d4{0.0, 0.0, 0.0, 0.0};
  // loader: row tid >> 4 of the step, double2 columns (tid & 15) + 16 q, q < 8
  const int lrow = tid >> 4, lc = tid & 15;
  const double2* gK = reinterpret_cast<const double2*>(K + (rbeg + lrow) * 256) + lc;
  constexpr int64_t gstep = BK * 256 / 2;
  double2 v[8];
  double vw = 1.0;
#define S256_GLOAD(step)                                                        \
  {                                                                             \
    const int64_t o_ = (int64_t)(step) * gstep;                                 \
    _Pragma("unroll") for (int q = 0; q < 8; ++q) v[q] = gK[o_ + 16 * q];       \
    if constexpr (WEIGHTED) vw = w[rbeg + (int64_t)(step) * BK + (tid & (BK - 1))]; \
  }
#define S256_SSTORE(buf)                                                        \
  {                                                                             \
    double2* p_ = reinterpret_cast<double2*>(&Ks[buf][lrow * SB2]) + lc;        \
    _Pragma("unroll") for (int q = 0; q < 8; ++q) p_[16 * q] = v[q];            \
    if constexpr (WEIGHTED) ws[buf][tid & (BK - 1)] = vw;                       \
  }
  if (nsteps > 0) {
    S256_GLOAD(0);
    S256_SSTORE(0);
  }
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    const int cur = step & 1;
    S256_GLOAD(step + 1 < nsteps ? step + 1 : step);   // one basic block per step
    const double* Kc = Ks[cur];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int krow = kk * 4 + (lane >> 4);
      const double* row = Kc + krow * SB2 + (lane & 15);
      double a0 = row[R0 * 16], a1 = row[R1 * 16];
      if constexpr (WEIGHTED) {
        const double wk = ws[cur][krow];
        a0 *= wk;
        a1 *= wk;
      }
#pragma unroll
      for (int c = 0; c < N1; ++c) {
        const double b = row[c * 16];
        if (c < N0) acc0[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b, acc0[c], 0, 0, 0);
        acc1[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b, acc1[c], 0, 0, 0);
      }
    }
    S256_SSTORE(cur ^ 1);   // on the last step into the idle buffer
    if constexpr (SGP_S256_IL) mfma_interleave<false, 2, 8, 68>();
    __syncthreads();
  }
#undef S256_GLOAD
#undef S256_SSTORE
  // fragment (R, c) -> 64-block (R / 4, c / 4) of the slab, element ((R % 4) * 16 + row) * 64 +
  // (c % 4) * 16 + col
#pragma unroll
  for (int c = 0; c < N1; ++c)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      if (hh == 0 && c >= N0) continue;
      const int R = hh == 0 ? R0 : R1;
      const d4& a = hh == 0 ? acc0[c] : acc1[c];
      const int rp = R / 4, cp = c / 4;
      double* blk = out + (int64_t)(rp * (rp + 1) / 2 + cp) * 4096;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        blk[((R % 4) * 16 + (lane >> 4) + 4 * q) * 64 + (c % 4) * 16 + (lane & 15)] = a[q];
    }
}

template <bool WEIGHTED>
__global__ void __launch_bounds__(256, 2)
k_syrk_s256(const double* __restrict__ K, int64_t n_pad, const double* __restrict__ w,
            int64_t chunk, double* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) double Ks[2][BK * SB2];
  __shared__ double ws[2][BK];
  const int64_t nwg = (int64_t)gridDim.x;
  const int64_t wgid = xcd_remap(blockIdx.x, nwg);   // a chunk's two workgroups on one XCD
  const int64_t split = wgid >> 1;
  const int v = (int)(wgid & 1) * 4 + (threadIdx.x >> 6);
  const int64_t rbeg = split * chunk;
  int64_t rend = rbeg + chunk;
  if (rend > n_pad) rend = n_pad;
  const int nsteps = rend > rbeg ? (int)((rend - rbeg) / BK) : 0;
  double* out = slab + split * 10 * 4096;   // nblk = 10 lower 64-blocks at mp = 256
#define S256_CASE(v_)                                                          \
  case v_:                                                                     \
    syrk256_body<v_, WEIGHTED>(K, w, rbeg, nsteps, Ks, ws, out);               \
    break;
  switch (v) {   // wave-uniform: each wave runs its own fragment rows' k-loop
    S256_CASE(0) S256_CASE(1) S256_CASE(2) S256_CASE(3)
    S256_CASE(4) S256_CASE(5) S256_CASE(6) S256_CASE(7)
  }
#undef S256_CASE
}

// ============================================================================ TN GEMM
// C = A^T B over n rows (A: n_pad x ma, B: n_pad x mb, both row-major; ma, mb multiples of
// 128): split-K over row chunks like k_syrk_blk, one 128x128 tile per workgroup, deterministic
// slabs [split][tile][128 x 128].  grid = splits * (ma/128) * (mb/128).
__global__ void __launch_bounds__(256, 2)
k_gemm_tn(const double* __restrict__ A, int64_t lda, const double* __restrict__ B, int64_t ldb,
          int64_t n_pad, int nta, int ntb, int64_t chunk, double* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) double Ka[2][BK * SB];
  __shared__ __attribute__((aligned(16))) double Kb[2][BK * SB];
  const int64_t nwg = (int64_t)gridDim.x;
  const int64_t wgid = xcd_remap(blockIdx.x, nwg);
  const int ntile = nta * ntb;
  const int split = (int)(wgid / ntile);
  const int tile = (int)(wgid % ntile);
  const int ta = tile / ntb, tb = tile % ntb;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int64_t rbeg = (int64_t)split * chunk;
  int64_t rend = rbeg + chunk;
  if (rend > n_pad) rend = n_pad;
  const int nsteps = (int)((rend - rbeg) / BK);
  d4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
  const int lrow = tid >> 4, lc = tid & 15;   // double2 columns lc + 16 q (as k_syrk_blk)
  const double2* gA = reinterpret_cast<const double2*>(A + (rbeg + lrow) * lda + ta * (int64_t)T128) + lc;
  const double2* gB = reinterpret_cast<const double2*>(B + (rbeg + lrow) * ldb + tb * (int64_t)T128) + lc;
  const int64_t sa = BK * lda / 2, sb = BK * ldb / 2;
  double2 va0, va1, va2, va3, vb0, vb1, vb2, vb3;
#define TN_GLOAD(step)                                                          \
  {                                                                             \
    const int64_t oa_ = (int64_t)(step) * sa, ob_ = (int64_t)(step) * sb;       \
    va0 = gA[oa_]; va1 = gA[oa_ + 16]; va2 = gA[oa_ + 32]; va3 = gA[oa_ + 48];  \
    vb0 = gB[ob_]; vb1 = gB[ob_ + 16]; vb2 = gB[ob_ + 32]; vb3 = gB[ob_ + 48];  \
  }
#define TN_SSTORE(buf)                                                          \
  {                                                                             \
    double2* pa_ = reinterpret_cast<double2*>(&Ka[buf][lrow * SB]) + lc;        \
    double2* pb_ = reinterpret_cast<double2*>(&Kb[buf][lrow * SB]) + lc;        \
    pa_[0] = va0; pa_[16] = va1; pa_[32] = va2; pa_[48] = va3;                  \
    pb_[0] = vb0; pb_[16] = vb1; pb_[32] = vb2; pb_[48] = vb3;                  \
  }
  if (nsteps > 0) {
    TN_GLOAD(0);
    TN_SSTORE(0);
  }
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    const int cur = step & 1;
    if (step + 1 < nsteps) TN_GLOAD(step + 1);
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
    if (step + 1 < nsteps) TN_SSTORE(cur ^ 1);
    __syncthreads();
  }
#undef TN_GLOAD
#undef TN_SSTORE
  double* out = slab + ((int64_t)split * ntile + tile) * (T128 * T128);
#pragma unroll
  for (int fm = 0; fm < 4; ++fm)
#pragma unroll
    for (int fn = 0; fn < 4; ++fn)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = wr * 64 + fm * 16 + (lane >> 4) + 4 * q;
        const int col = wc * 64 + fn * 16 + (lane & 15);
        out[row * T128 + col] = acc[fm][fn][q];
      }
}

// C[a][b] (row-major, ld = ntb*128) = sum over splits of the tile slabs
__global__ void __launch_bounds__(256)
k_gemm_tn_reduce(const double* __restrict__ slab, int splits, int nta, int ntb,
                 double* __restrict__ C) {
  const int tile = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int ntile = nta * ntb;
  double s = 0.0;
  for (int sp = 0; sp < splits; ++sp) s += slab[((int64_t)sp * ntile + tile) * (T128 * T128) + e];
  const int ta = tile / ntb, tb = tile % ntb;
  const int64_t a = (int64_t)ta * T128 + e / T128, b = (int64_t)tb * T128 + e % T128;
  C[a * (int64_t)ntb * T128 + b] = s;
}

__global__ void __launch_bounds__(256)
k_syrk_reduce_t(const double* __restrict__ slab_t, const double* __restrict__ slab_rr,
                int splits, int nb, int64_t mp, double* __restrict__ red) {
  const int64_t a = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (a < mp) {
    const int ta = (int)(a / T128), col = (int)(a % T128);
    double s = 0.0;
    for (int sp = 0; sp < splits; ++sp) s += slab_t[((int64_t)sp * nb + ta) * T128 + col];
    red[mp * mp + a] = s;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    double s = 0.0;
    for (int sp = 0; sp < splits; ++sp) s += slab_rr[sp];
    red[mp * mp + mp] = s;
  }
}

// ============================================================================ contraction
// One kernel, two epilogues, both on the tile T = K[i-block, :] * M[:, j-block] held in
// f64-MFMA accumulators:
//   EPI_GRAD     G_ij = alpha_i u_j + rs_i T_ij, contracted with dK_ij/dlog(theta) for all
//                parameters at once (record per tile: sum G*K, sum G*K*w_c, tau-coincidence
//                sums, alpha^T alpha);
//   EPI_ROWQUAD  per-row partial sum_j K_ij T_ij (= diag(K M K^T) after summing the column
//                tiles) into rowq[tj][row].
// When uvec != nullptr, alpha_i = (r_i - K_i u) * iz_i is computed in the same k-loop from the
// staged K values (iz_i = invz_vec ? invz_vec[i] : invz), optionally written to alpha_out.
enum { EPI_GRAD = 0, EPI_ROWQUAD = 1 };

// KU (row quadratic forms without u: the Z pass): false compiles the K u fold out of the k-loop
// T2 (FROM_T only): a second stored product folded in (ConArgs::tin2)
constexpr int CON_A_SZ = T128 * SA;   // 2176 (keeps the B image 16-byte aligned)
constexpr int CON_B_SZ = BK * SB;     // 2304
constexpr int CON_LDS = 2 * (CON_A_SZ + CON_B_SZ);

// The part of a tile's k range one workgroup computes (k_contract_sk, the balanced launch): the
// whole range (CON_FULL, also every tile of k_contract), its tail (CON_TAIL: the partial product
// and partial K u are handed to the workgroup that holds the head, no epilogue) or its head
// (CON_HEAD: adds the handed-over tail, then the epilogue)
enum { CON_FULL = 0, CON_TAIL = 1, CON_HEAD = 2 };
constexpr int64_t CON_SK_SLOT = 65 * 256;   // doubles per hand-over slot: 64 accumulators + K u
struct ConSK {
  double* ws = nullptr;          // [slots][CON_SK_SLOT]
  int dp = -1;                   // whole rounds run as the grid first (-1: all but the last)
  unsigned* flags = nullptr;     // per slot: the launch epoch once the slot is written
  unsigned epoch = 0;
  int64_t slot = 0;              // CON_TAIL: the slot written; CON_HEAD: the slot read
  int* status = nullptr;         // -1: a hand-over wait expired (reported by the host)
};

__device__ __forceinline__ unsigned con_ldu_sc1(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// SKM: which hand-over code is compiled in -- 0 none (CON_FULL), CON_TAIL (the body ends after
// the k-loop), CON_HEAD (`part` chooses at run time between CON_HEAD and CON_FULL).  The tail and
// the head never share one copy of the body: compiled together the accumulators spilled
// ~250 VGPRs
template <int DT, int EPI, bool V2, bool KNOT, bool FROM_T, bool KU, bool T2, int SKM>
__device__ __forceinline__ void con_tile(
    const KernParams& kp, const double* __restrict__ K, const double* __restrict__ M,
    const double* __restrict__ X, int64_t ldx, int64_t n, int64_t n_pad,
    const double* __restrict__ U, int64_t ldu, int64_t m, int64_t mp, const ConArgs& ca,
    double* __restrict__ slab, int nrec, double* __restrict__ rowq, int64_t ti, int64_t tj,
    int64_t wgid, int kb, int ke, double* lds, double (*red)[SGP_MAXD + 5], double (*s_uk)[BK],
    const ConSK& sk, int part, int tid_in) {
  const double* __restrict__ r = ca.r;
  const double* __restrict__ uvec = ca.uvec;
  const double* __restrict__ cdiag = ca.cdiag;
  constexpr int A_SZ = CON_A_SZ, B_SZ = CON_B_SZ;
  const int64_t ntj = mp / T128;
  const int64_t nwg = (n_pad / T128) * ntj;   // tiles (the record slab's row length)
  const int64_t i0 = ti * T128, j0 = tj * T128;

  const int tid = tid_in, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const bool with_u = KU && (uvec != nullptr) && (ca.alpha_in == nullptr);   // fuse K u into the loop
  constexpr bool with_v = V2;   // second rank-1 term (Laplace), compiled in only where used

  d4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};

  // A loader: 128 rows x 16 k, thread -> (row = tid>>1, 8 doubles at (tid&1)*8)
  const int arow = tid >> 1, acol = (tid & 1) * 8;
  const double2* gA = reinterpret_cast<const double2*>(K + (i0 + arow) * mp + acol);
  // B loader: 16 k x 128 cols, thread -> (k = tid>>4, double2 columns (tid&15) + 16 q):
  // 8 consecutive lanes store 128 contiguous bytes (conflict-free ds_write_b128)
  const int bk = tid >> 4, bc = tid & 15;
  const double2* gB = reinterpret_cast<const double2*>(M + (int64_t)bk * mp + j0) + bc;
  const int64_t bstep = BK * mp / 2;
  double2 va0, va1, va2, va3, vb0, vb1, vb2, vb3;
  // alpha folded into the k-loop: each thread dots the 8 K values it stages with u.
  double ku = 0.0, vuk = 0.0;
  // the step is one basic block (mfma_interleave): the u slice is fetched, staged and folded
  // unconditionally -- from M when there is no u (valid memory; ku is then never used)
  const double* __restrict__ uk_src = with_u ? uvec : M;

  // The alpha dot products K_i . u ride on the A stream: 16 threads fetch the step's u slice
  // with the operands, it is staged in LDS with them, and each thread folds its 8 staged K
  // values in at the top of the next step (no global load waited on inside the loop).
#define CON_GLOAD(step)                                                          \
  {                                                                              \
    const int64_t oa_ = (int64_t)(step) * (BK / 2), ob_ = (int64_t)(step) * bstep; \
    va0 = gA[oa_]; va1 = gA[oa_ + 1]; va2 = gA[oa_ + 2]; va3 = gA[oa_ + 3];      \
    vb0 = gB[ob_]; vb1 = gB[ob_ + 16]; vb2 = gB[ob_ + 32]; vb3 = gB[ob_ + 48];   \
    if constexpr (KU) vuk = uk_src[(int64_t)(step) * BK + (tid & (BK - 1))];     \
  }
#define CON_SSTORE(buf)                                                          \
  {                                                                              \
    double* As_ = lds + (buf) * (A_SZ + B_SZ);                                   \
    double* pa_ = &As_[arow * SA + acol];                                        \
    double2* pb_ = reinterpret_cast<double2*>(&As_[A_SZ + bk * SB]) + bc;        \
    pa_[0] = va0.x; pa_[1] = va0.y; pa_[2] = va1.x; pa_[3] = va1.y;              \
    pa_[4] = va2.x; pa_[5] = va2.y; pa_[6] = va3.x; pa_[7] = va3.y;              \
    pb_[0] = vb0; pb_[16] = vb1; pb_[32] = vb2; pb_[48] = vb3;                   \
    if constexpr (KU) s_uk[buf][tid & (BK - 1)] = vuk;   /* 16 lanes per address */ \
  }
#define CON_KU(buf)                                                              \
  {                                                                              \
    const double* u_ = &s_uk[buf][acol];                                         \
    ku = fma(va0.x, u_[0], ku); ku = fma(va0.y, u_[1], ku);                      \
    ku = fma(va1.x, u_[2], ku); ku = fma(va1.y, u_[3], ku);                      \
    ku = fma(va2.x, u_[4], ku); ku = fma(va2.y, u_[5], ku);                      \
    ku = fma(va3.x, u_[6], ku); ku = fma(va3.y, u_[7], ku);                      \
  }

  SGP_PROBE_CON_STAMP(0);
  if constexpr (FROM_T) {
    // the product tile T = K M was stored by an earlier row-quadratic pass over the same K and
    // M (launch_rowquad_knm with tstore): read it instead of recomputing 2 n m^2 flops
#pragma unroll
    for (int fm = 0; fm < 4; ++fm)
#pragma unroll
      for (int fn = 0; fn < 4; ++fn)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          acc[fm][fn][q] = ca.tin[(i0 + wr * 64 + fm * 16 + (lane >> 4) + 4 * q) * mp + j0 +
                                  wc * 64 + fn * 16 + (lane & 15)];
  } else {
  CON_GLOAD(kb);
  CON_SSTORE(0);
  __syncthreads();
  for (int step = kb; step < ke; ++step) {
    const int cur = (step - kb) & 1;
    if constexpr (KU) CON_KU(cur);   // va still holds this step's staged K values
    CON_GLOAD(step + 1 < ke ? step + 1 : step);   // the last step reloads its own slice
    const double* As = lds + cur * (A_SZ + B_SZ);
    const double* Bs = As + A_SZ;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int kx = kk * 4 + (lane >> 4);
      double af[4], bf[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        af[f] = As[(wr * 64 + f * 16 + (lane & 15)) * SA + kx];
        bf[f] = Bs[kx * SB + wc * 64 + f * 16 + (lane & 15)];
      }
#pragma unroll
      for (int fm = 0; fm < 4; ++fm)
#pragma unroll
        for (int fn = 0; fn < 4; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[fm], bf[fn], acc[fm][fn], 0, 0, 0);
    }
    CON_SSTORE(cur ^ 1);   // on the last step into the idle buffer
    mfma_interleave<SGP_CON_IL_SPREAD, SGP_CON_IL_PAT>();
    __syncthreads();
  }
  }   // !FROM_T
#undef CON_GLOAD
#undef CON_SSTORE
#undef CON_KU

  if constexpr (SKM == CON_TAIL) {
    // hand the partial product over: every value stored write-through (sc1), the stores
    // drained, then the slot's flag (the head's workgroup may run on another XCD)
    double* w = sk.ws + sk.slot * CON_SK_SLOT;
#pragma unroll
    for (int fm = 0; fm < 4; ++fm)
#pragma unroll
      for (int fn = 0; fn < 4; ++fn)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          __hip_atomic_store(&w[((fm * 4 + fn) * 4 + q) * 256 + tid], acc[fm][fn][q],
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&w[64 * 256 + tid], ku, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      __hip_atomic_store(&sk.flags[sk.slot], sk.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if (SKM == CON_HEAD && part == CON_HEAD) {
    // the tail was computed at the start of the next workgroup's range: long done by now.
    // Watchdog: a wait past ~2^22 polls marks the launch failed and goes on (the grid drains)
    if (tid == 0) {
      unsigned it = 0;
      while (con_ldu_sc1(&sk.flags[sk.slot]) != sk.epoch) {
        if (++it >= (1u << 22)) {
          atomicExch(sk.status, -1);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    const double* w = sk.ws + sk.slot * CON_SK_SLOT;
    // in groups of 16 values: the scheduler would otherwise issue all 64 loads up front and
    // need 128 more VGPRs beside the accumulators
#pragma unroll
    for (int fm = 0; fm < 4; ++fm) {
      double t[4][4];
#pragma unroll
      for (int fn = 0; fn < 4; ++fn)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          t[fn][q] = __hip_atomic_load(&w[((fm * 4 + fn) * 4 + q) * 256 + tid], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int fn = 0; fn < 4; ++fn)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[fm][fn][q] += t[fn][q];
      __builtin_amdgcn_sched_barrier(0);
    }
    ku += __hip_atomic_load(&w[64 * 256 + tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  SGP_PROBE_CON_STAMP(1);
  if constexpr (SGP_CON_EPI_PRIO > 0) __builtin_amdgcn_s_setprio(SGP_CON_EPI_PRIO);
  SGP_PROBE_CON_SKIP_EPILOGUE()   // timing probe hook (sgp_probe.h): empty in the product
  // ---------------- alpha (per row), shared by both epilogues ----------------
  double* s_alpha = lds;                    // 128
  double* s_rs = s_alpha + T128;            // 128
  double* s_u = s_rs + T128;                // 128
  double* s_cd = s_u + T128;                // 128
  double* s_beta = s_cd + T128;             // 128
  double* s_v = s_beta + T128;              // 128
  double* s_xs = s_v + T128;                // MFMA B image [x~ | x~^2] of one coordinate chunk
  double* s_us = s_xs + T128 * 16;          // 128 x 9 ([col][c], scaled; odd stride: 16
                                            // columns on distinct banks)
  // T2: the second product's row scales, past the gradient epilogue's K stage (s_us, 2 x 16
  // x 136 doubles of stage: 3968 + 4352 doubles in)
  double* s_rs2 = lds + 8320;
  static_assert(8320 + T128 <= 2 * (A_SZ + B_SZ), "s_rs2 fits the LDS image");
  ku += __shfl_xor(ku, 1, 64);                       // the two halves of row `arow`
  double a2 = 0.0;                                    // alpha^2, counted once (tj == 0)
  if ((tid & 1) == 0) {
    const int64_t i = i0 + arow;
    const double iz = ca.invz_vec ? ca.invz_vec[i] : ca.invz;
    const double al = ca.alpha_in ? ca.alpha_in[i]
                                  : (with_u ? (r[i] - ku) * iz : 0.0);   // padded rows -> 0
    // rows past n: every row factor 0, so G = 0 there and the epilogue needs no validity mask
    // (K12 is exactly 0 in the padded columns j >= m, and T = K M is finite: W = G o K = 0)
    const bool iv = i < n;
    s_alpha[arow] = iv ? al : 0.0;
    s_rs[arow] = iv ? (ca.rs_vec ? ca.rs * ca.rs_vec[i] : ca.rs) : 0.0;
    if constexpr (T2) s_rs2[arow] = iv ? (ca.rs_vec2 ? ca.rs2 * ca.rs_vec2[i] : ca.rs2) : 0.0;
    s_beta[arow] = (with_v && iv) ? ca.beta_in[i] : 0.0;
    if (tj == 0) {
      if (ca.count_a2 && i < n) a2 = al * al;
      if (ca.alpha_out) ca.alpha_out[i] = al;
    }
  }
  const double* Kt = K + i0 * mp + j0;

  if constexpr (EPI == EPI_ROWQUAD) {
    if (ca.tstore != nullptr) {   // keep T = K M for a later FROM_T gradient pass
#pragma unroll
      for (int fm = 0; fm < 4; ++fm)
#pragma unroll
        for (int fn = 0; fn < 4; ++fn)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            ca.tstore[(i0 + wr * 64 + fm * 16 + (lane >> 4) + 4 * q) * mp + j0 + wc * 64 +
                      fn * 16 + (lane & 15)] = acc[fm][fn][q];
    }
    __syncthreads();
    double* s_q = s_cd;                       // [2][128] (reuses s_cd / s_xs space)
    // per lane: 16 rows (fm, q) x 4 cols (fn) -> row sums over this wave's 64 columns
#pragma unroll
    for (int fm = 0; fm < 4; ++fm) {
      double kv[4][4];   // the 16 K values of this row fragment, issued together
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int fn = 0; fn < 4; ++fn)
          kv[q][fn] = Kt[(int64_t)(wr * 64 + fm * 16 + (lane >> 4) + 4 * q) * mp +
                         wc * 64 + fn * 16 + (lane & 15)];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = wr * 64 + fm * 16 + (lane >> 4) + 4 * q;
        double v = 0.0;
#pragma unroll
        for (int fn = 0; fn < 4; ++fn)
          v = fma(kv[q][fn], acc[fm][fn][q], v);   // K = 0 outside (n, m)
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 8, 64);
        if ((lane & 15) == 0) s_q[wc * T128 + row] = v;
      }
    }
    __syncthreads();
    if (tid < T128) rowq[tj * n_pad + i0 + tid] = s_q[tid] + s_q[T128 + tid];
    return;
  } else {
    // ---------------- gradient epilogue ----------------
    const int d = kp.d;
    constexpr int sus = 9;                 // s_us row stride: one chunk of 8, odd
    const bool ard = (kp.kernel == 1);
    const double rl2s = kp.rl2[0];
    const int L = kp.L;
    for (int e = tid; e < T128; e += 256) {
      const int64_t j = j0 + e;
      s_u[e] = (uvec && j < m) ? uvec[j] : 0.0;
      s_v[e] = (with_v && j < m) ? ca.vvec[j] : 0.0;
      s_cd[e] = (cdiag && j < m) ? cdiag[j] : 0.0;
    }
    double e_sig = 0.0;
    double e_sq = 0.0;                           // one length scale: sum over all coordinates
    double* s_kn;
    static_assert(DT % 8 == 0, "coordinates are processed in chunks of 8");
    constexpr int NCH = DT / 8;
    {
      // MFMA epilogue.  With W = G o K (zero outside (n, m)) and x~, u~ the (ARD-scaled)
      // coordinates, every per-pair sum the gradient needs is a small product over rows:
      //   D[j][c']   = sum_i W_ij XB_ic',  XB = [x~ | x~^2]  (c' < 8 | c' >= 8)
      //   C_j        = sum_i W_ij
      //   e_l[c]     = sum_ij W_ij (x~_ic - u~_jc)^2 = sum_j D[j][8+c] - 2 u~_jc D[j][c] + u~_jc^2 C_j
      //   knot (j,c) = sum_i W_ij (x~_ic - u~_jc)   = D[j][c] - u~_jc C_j
      // The C fragment of K P is read directly as the A operand of v_mfma_f64_16x16x4 (its lane
      // map is that of W^T), so D costs 4 MFMAs per 16x16 fragment instead of ~3 d VALU ops
      // per pair.
      // K_ij is read back through LDS: per half of a 16-row fragment fm, the 16 tile rows the
      // four waves need are copied global -> LDS by LDS-DMA (one 1 KiB row per
      // wave-instruction, no VGPRs held), double-buffered, the first two before the coordinate
      // staging so their latency hides behind it.  (Fragment-shaped loads straight to VGPRs
      // serialised on one HBM round trip per fragment at this register pressure.)
      // Coordinates go through the D products in chunks of 8 (DT / 8 chunks): the first chunk
      // rides on the pass that forms W; each further chunk restages [x~ | x~^2] and u~ and adds
      // one 16-column MFMA product over the W kept in the accumulators.
      constexpr int KST = 136;                  // stage row stride (doubles)
      // this lane's source in the first stage row of its wave (row (wv >> 1) 64 + 4 (wv & 1)
      // + q of a stage; stage s adds 16 (s >> 1) + 8 (s & 1) rows): every stage address is this
      // pointer plus a wave-uniform row offset times mp -- one 64-bit add per DMA instead of a
      // 64-bit multiply-add chain (the co-resident k-loop pays for every VALU cycle here)
      const double* const kq0 = K + (i0 + (wv >> 1) * 64 + 4 * (wv & 1)) * mp + j0 + 2 * lane;
      double* kst = s_us + ((T128 * sus + 1) & ~1);   // 2 x 16 x KST, 16-byte aligned
      // chunk ch of the coordinates: s_xs = [x~ | x~^2] (128 x 16), s_us = u~ (128 x sus)
#define CON_XSTAGE(ch_)                                                                  \
      _Pragma("unroll") for (int e = tid; e < T128 * 8; e += 256) {                      \
        const int rr = e % T128, c = e / T128, cg = 8 * (ch_) + c;                       \
        const int64_t i = i0 + rr, j = j0 + rr;                                          \
        double xv = 0.0;                                                                 \
        if (cg < d) {                                                                    \
          const double sc = ard ? kp.rl[cg] : 1.0;                                       \
          xv = (i < n) ? X[i + cg * ldx] * sc : 0.0;                                     \
          s_us[rr * sus + c] = (j < m) ? U[j + cg * ldu] * sc : 0.0;                     \
        }                                                                                \
        s_xs[rr * 16 + c] = xv;                                                          \
        s_xs[rr * 16 + 8 + c] = xv * xv;                                                 \
      }
      // Eight half-height stages (16 rows: the 8 rows a lane's q pair needs, of each 64-row
      // half), double-buffered in the LDS one 32-row stage took, each issued one half-stage
      // ahead of its use (round 3; four single-buffered 32-row stages before: the same time at
      // C3, 31.3-31.4 ms, and 1-3 % more at C2, profiles/r3/kdb_ab.txt).  The compiler waits
      // vmcnt(0) after each issue (it tracks the DMA as an LDS write it cannot tell apart from
      // the stage being read); a real two-ahead prefetch (inline-asm DMA, three buffers) was no
      // faster -- the stage phase is bound by the issue slots the co-resident workgroup's k-loop
      // leaves, not by the load latency (profiles/r3/con_epi_dma_ab.txt)
#ifdef SGP_CON_PROBE_NO_KDMA   // timing probe (wrong results): the K stages are not loaded
#define CON_KHALF(s_)
#else
#define CON_KHALF(s_)                                                                    \
      _Pragma("unroll") for (int q_ = 0; q_ < 4; ++q_) {                                 \
        const int rho_ = wv * 4 + q_;                                                    \
        __builtin_amdgcn_global_load_lds(                                                \
            (const __attribute__((address_space(1))) void*)(                             \
                kq0 + (int64_t)(((s_) >> 1) * 16 + ((s_) & 1) * 8 + q_) * mp),          \
            (__attribute__((address_space(3))) void*)(kst + ((s_) & 1) * 16 * KST + rho_ * KST), \
            16, 0, 0);                                                                   \
      }
#endif
      // T2: the second stored product's values of a half-stage (rows 2h, 2h + 1 of fragment fm,
      // four column fragments), loaded into registers one half-stage ahead beside the K stage's
      // DMA (the same vmcnt(0) waits cover both)
      double t2n[2][4];
#define CON_T2LOAD(s_)                                                                   \
      if constexpr (T2) {                                                                \
        _Pragma("unroll") for (int r2_ = 0; r2_ < 2; ++r2_)                              \
        _Pragma("unroll") for (int fn_ = 0; fn_ < 4; ++fn_)                              \
          t2n[r2_][fn_] = ca.tin2[(i0 + wr * 64 + ((s_) >> 1) * 16 + (lane >> 4) +        \
                                   4 * (2 * ((s_) & 1) + r2_)) * mp + j0 + wc * 64 +      \
                                  fn_ * 16 + (lane & 15)];                                \
      }
      CON_KHALF(0);
      CON_KHALF(1);
      CON_T2LOAD(0);
      CON_XSTAGE(0);
      __builtin_amdgcn_s_waitcnt(0);            // K stage 0 (LDS-DMA) landed
      __syncthreads();
      s_kn = kst;                               // KNOT: [2 (wr)][128 cols][8] per chunk
                                                // (aliases the K stage, after its last use)
      SGP_PROBE_CON_STAMP(4);

      d4 P[4];
      double Cc[4], ucol[4], vcol[4];
#pragma unroll
      for (int fn = 0; fn < 4; ++fn) {
        const int col = wc * 64 + fn * 16 + (lane & 15);
        P[fn] = d4{0.0, 0.0, 0.0, 0.0};
        Cc[fn] = 0.0;
        ucol[fn] = s_u[col];
        vcol[fn] = with_v ? s_v[col] : 0.0;
      }
      {
#pragma unroll
        for (int hs = 0; hs < 8; ++hs) {
          const int fm = hs >> 1, h = hs & 1;
          if (hs > 0) {                         // half-stage hs landed (and is visible to all);
            __builtin_amdgcn_s_waitcnt(0);      // everyone is done with hs - 1's buffer
            __syncthreads();
            if (hs < 7) { CON_KHALF(hs + 1); }
          }
          double t2c[2][4];
          if constexpr (T2) {
#pragma unroll
            for (int r2 = 0; r2 < 2; ++r2)
#pragma unroll
              for (int fn = 0; fn < 4; ++fn) t2c[r2][fn] = t2n[r2][fn];
            if (hs < 7) { CON_T2LOAD(hs + 1); }
          }
          const double* kb = kst + h * 16 * KST;
          double xb[2];
#pragma unroll
          for (int r2 = 0; r2 < 2; ++r2)
            xb[r2] = s_xs[(wr * 64 + fm * 16 + 4 * (2 * h + r2) + (lane >> 4)) * 16 + (lane & 15)];
#pragma unroll
          for (int fn = 0; fn < 4; ++fn) {
            const int col = wc * 64 + fn * 16 + (lane & 15);
            double kv[2];
#pragma unroll
            for (int r2 = 0; r2 < 2; ++r2) kv[r2] = kb[(wr * 8 + (lane >> 4) + 4 * r2) * KST + col];
#pragma unroll
            for (int r2 = 0; r2 < 2; ++r2) {
              const int q = 2 * h + r2;
              const int row = wr * 64 + fm * 16 + (lane >> 4) + 4 * q;
              double G = s_rs[row] * acc[fm][fn][q];
              if constexpr (T2) G = fma(s_rs2[row], t2c[r2][fn], G);
              if constexpr (V2) G = fma(s_beta[row], vcol[fn], G);
              G = fma(s_alpha[row], ucol[fn], G);
              // no validity mask: padded rows have G = 0 and padded columns K = 0.  (The former
              // `valid ? G * kv : 0` became a branch per element around its LDS reads -- an
              // exposed LDS round trip and an exec-mask block each -- and every VALU cycle here
              // is taken from the co-resident workgroup's MFMA stream)
              double w = G * kv[r2];
              // the passes over stored products (FROM_T: FITC's / Laplace's one-pass gradient)
              // keep the select (measured 5 % slower without it) and so does Laplace with knot
              // gradients (without it its 256 VGPRs spill)
              if constexpr ((V2 && KNOT) || FROM_T) w = (j0 + col < m && i0 + row < n) ? w : 0.0;
              Cc[fn] += w;
              acc[fm][fn][q] = w;
            }
          }
#pragma unroll
          for (int r2 = 0; r2 < 2; ++r2)
#pragma unroll
            for (int fn = 0; fn < 4; ++fn)
#ifndef SGP_CON_PROBE_NO_EPI_MFMA
              P[fn] = __builtin_amdgcn_mfma_f64_16x16x4f64(acc[fm][fn][2 * h + r2], xb[r2], P[fn],
                                                           0, 0, 0);
#else   // timing probe (wrong results): a VALU stand-in for the D products
              P[fn][r2] = fma(acc[fm][fn][2 * h + r2], xb[r2], P[fn][r2]);
#endif
          if (hs == 1) SGP_PROBE_CON_STAMP(3);
        }
        __syncthreads();                        // everyone is done reading the last stage
      }
#undef CON_KHALF
#undef CON_T2LOAD
      SGP_PROBE_CON_STAMP(5);
      // D fragment fn: lane l, register q -> column wc*64 + fn*16 + (l>>4) + 4q, c' = l & 15
      const int cp = lane & 15, cc = cp & 7;
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        if (8 * ch >= d) break;                 // d is uniform: every thread breaks alike
        if (ch > 0) {
          __syncthreads();                      // the previous chunk's s_xs / s_us are read
          CON_XSTAGE(ch);
          __syncthreads();
#pragma unroll
          for (int fn = 0; fn < 4; ++fn) P[fn] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int fm = 0; fm < 4; ++fm) {
            double xb[4];
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4)
              xb[r4] = s_xs[(wr * 64 + fm * 16 + 4 * r4 + (lane >> 4)) * 16 + (lane & 15)];
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4)
#pragma unroll
              for (int fn = 0; fn < 4; ++fn)
                P[fn] = __builtin_amdgcn_mfma_f64_16x16x4f64(acc[fm][fn][r4], xb[r4], P[fn], 0,
                                                             0, 0);
          }
        }
        const bool cok = 8 * ch + cc < d;
        double E = 0.0;
#pragma unroll
        for (int fn = 0; fn < 4; ++fn) {
          double C = Cc[fn];
          C += __shfl_xor(C, 16, 64);
          C += __shfl_xor(C, 32, 64);            // every lane: C of column (lane & 15)
          if (ch == 0 && (lane >> 4) == 0) e_sig += C;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int jl = wc * 64 + fn * 16 + (lane >> 4) + 4 * q;
            const double Cq = __shfl(C, (lane >> 4) + 4 * q, 64);
            const double u = cok ? s_us[jl * sus + cc] : 0.0;
            const double pv = P[fn][q];
            E += (cp >= 8) ? pv : u * fma(u, Cq, -2.0 * pv);
            if constexpr (KNOT) {
              if (cp < 8) s_kn[(wr * T128 + jl) * 8 + cc] = pv - u * Cq;
            }
          }
        }
        E += __shfl_xor(E, 8, 64);
        E += __shfl_xor(E, 16, 64);
        E += __shfl_xor(E, 32, 64);              // lanes c (0..7): sum_ij W_ij (x~_ic - u~_jc)^2
        if (ard) {
          if (lane < 8 && 8 * ch + lane < d) red[wv][1 + 8 * ch + lane] = E;
        } else {
          double t = E;
          t += __shfl_xor(t, 1, 64);
          t += __shfl_xor(t, 2, 64);
          t += __shfl_xor(t, 4, 64);
          e_sq += t;
        }
        if constexpr (KNOT) {
          // this chunk's knot partials: the two 64-row halves (wr) combined, [tile][col][d]
          __syncthreads();
          for (int e = tid; e < T128 * 8; e += 256) {
            const int col = e >> 3, c = e & 7, cg = 8 * ch + c;
            if (cg < d)
              ca.knot_slab[(ti * mp + j0 + col) * d + cg] =
                  s_kn[col * 8 + c] + s_kn[(T128 + col) * 8 + c];
          }
        }
      }
#undef CON_XSTAGE
    }

    SGP_PROBE_CON_STAMP(6);
    // record = [e_sig, e_l[0..L-1], c_sum, c_cnt, c_dg, alpha^T alpha]
    // (the coincidence fields stay zero here; k_coinc adds them)
    double v;
    v = wave_sum(e_sig);
    if (lane == 0) red[wv][0] = v;
    if (!ard && lane == 0) red[wv][1] = e_sq * rl2s;   // ARD: red[wv][1 + c] written above
    v = wave_sum(a2);
    if (lane == 0) {
      red[wv][1 + L] = 0.0;
      red[wv][2 + L] = 0.0;
      red[wv][3 + L] = 0.0;
      red[wv][4 + L] = v;
    }
    __syncthreads();
    if (tid < nrec)   // field-major [nrec][nwg]: coalesced for the reduction (launch_rowsum)
      slab[tid * nwg + wgid] = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
    SGP_PROBE_CON_STAMP(2);
  }
  if constexpr (SGP_CON_EPI_PRIO > 0) __builtin_amdgcn_s_setprio(0);
}

// one 128 x 128 output tile per workgroup (grid = tiles), XCD-aware tile order
template <int DT, int EPI, bool V2 = false, bool KNOT = false, bool FROM_T = false, bool KU = true,
          bool T2 = false>
__global__ void __launch_bounds__(256, 2)
k_contract(KernParams kp, const double* __restrict__ K, const double* __restrict__ M,
           const double* __restrict__ X, int64_t ldx, int64_t n, int64_t n_pad,
           const double* __restrict__ U, int64_t ldu, int64_t m, int64_t mp, ConArgs ca,
           double* __restrict__ slab, int nrec, double* __restrict__ rowq) {
  __shared__ __attribute__((aligned(16))) double lds[CON_LDS];
  __shared__ double red[4][SGP_MAXD + 5];
  __shared__ double s_uk[2][BK];   // u slice of the staged k-step (fused alpha)
  const int64_t ntj = mp / T128;
  const int64_t nwg = (n_pad / T128) * ntj;
  const int64_t wgid = xcd_remap(blockIdx.x, nwg);
  con_tile<DT, EPI, V2, KNOT, FROM_T, KU, T2, 0>(
      kp, K, M, X, ldx, n, n_pad, U, ldu, m, mp, ca, slab, nrec, rowq, wgid / ntj, wgid % ntj,
      wgid, 0, (int)(mp / BK), lds, red, s_uk, ConSK{}, CON_FULL, (int)threadIdx.x);
}

// The balanced form of VI's gradient contraction for grids whose last residency round would
// be mostly empty (C2: 1564 tiles over 512 slots = 3.05 rounds run as 4; the 8-GPU shard: 15.3
// as 16).  A persistent grid of G = resident workgroups: the first R - 1 whole rounds
// (R = tiles / G) as the one-tile grid runs them -- in round r workgroup v takes tile r G + v,
// v the XCD-aware index, so the tiles resident on one XCD together share their K row panels and
// P column panels in its L2 as before -- and the last round plus the remainder (G + tiles mod G
// tiles) Stream-K style: their k-steps, in tile order, split evenly over the G workgroups
// (each range covers at least one tile's steps, so a tile meets at most two workgroups).  A
// range that starts inside a tile computes that tile's tail FIRST, before its whole rounds, and
// hands it to workgroup v - 1, which holds the tile's head at the very end of its own work and
// adds the tail before the tile's one epilogue.
template <int DT, bool KNOT>
__global__ void __launch_bounds__(256, 2)
k_contract_sk(KernParams kp, const double* __restrict__ K, const double* __restrict__ M,
              const double* __restrict__ X, int64_t ldx, int64_t n, int64_t n_pad,
              const double* __restrict__ U, int64_t ldu, int64_t m, int64_t mp, ConArgs ca,
              double* __restrict__ slab, int nrec, ConSK sk) {
  __shared__ __attribute__((aligned(16))) double lds[CON_LDS];
  __shared__ double red[4][SGP_MAXD + 5];
  __shared__ double s_uk[2][BK];
  const int64_t ntj = mp / T128;
  const int64_t ntiles = (n_pad / T128) * ntj;
  const int S = (int)(mp / BK);
  const int64_t G = gridDim.x, v = xcd_remap(blockIdx.x, G);
  // the host launches this with ntiles >= G
  const int64_t dp_rounds = (sk.dp >= 0 && sk.dp < ntiles / G) ? sk.dp : ntiles / G - 1;
  const int64_t t0 = dp_rounds * G;           // the balanced region: tiles [t0, ntiles)
  const int64_t Usk = (ntiles - t0) * S;
  const int64_t u1 = Usk * (v + 1) / G;
  int64_t u = Usk * v / G;
  if (u % S != 0) {   // the range starts inside a tile: its tail, handed to workgroup v - 1
    const int64_t tile = t0 + u / S;
    const int kb = (int)(u % S);
    ConSK p = sk;
    p.slot = v;
    con_tile<DT, EPI_GRAD, false, KNOT, false, true, false, CON_TAIL>(
        kp, K, M, X, ldx, n, n_pad, U, ldu, m, mp, ca, slab, nrec, nullptr, tile / ntj,
        tile % ntj, tile, kb, S, lds, red, s_uk, p, CON_TAIL, (int)threadIdx.x);
    u += S - kb;
    __syncthreads();
  }
  int64_t r = 0;
  for (;;) {   // the whole rounds, then the range's whole tiles, then maybe a head
    int64_t tile;
    int ke;
    if (r < dp_rounds) {
      tile = r * G + v;
      ke = S;
      ++r;
    } else if (u < u1) {
      tile = t0 + u / S;
      ke = (int)((u1 - u) < (int64_t)S ? (u1 - u) : S);
      u += ke;
    } else {
      break;
    }
    ConSK p = sk;
    p.slot = v + 1;
    // the thread index passed through an opaque move each iteration: every per-thread offset
    // of the tile body is then recomputed inside the loop instead of hoisted out of it and
    // kept live across the k-loop
    int tid;
    asm volatile("v_mov_b32 %0, %1" : "=v"(tid) : "v"((int)threadIdx.x));
    con_tile<DT, EPI_GRAD, false, KNOT, false, true, false, CON_HEAD>(
        kp, K, M, X, ldx, n, n_pad, U, ldu, m, mp, ca, slab, nrec, nullptr, tile / ntj,
        tile % ntj, tile, 0, ke, lds, red, s_uk, p, ke < S ? CON_HEAD : CON_FULL, tid);
    __syncthreads();   // the next tile's operand staging reuses the epilogue's LDS
  }
}

// knot partials: part[r][col] = sum_{ti = r, r+G, ...} slab[ti][col]   (grid: ncol/256 x G).
// Four independent accumulators keep four loads in flight per thread (the column sum is
// latency-bound: ~60 rows per thread at n = 1e6).
__global__ void __launch_bounds__(256)
k_knot_reduce1(const double* __restrict__ slab, int64_t ntiles, int64_t ncol,
               double* __restrict__ part) {
  const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r = blockIdx.y, G = gridDim.y;
  if (col >= ncol) return;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  int64_t t = r;
  for (; t + 3 * G < ntiles; t += 4 * G) {
    s0 += slab[t * ncol + col];
    s1 += slab[(t + G) * ncol + col];
    s2 += slab[(t + 2 * G) * ncol + col];
    s3 += slab[(t + 3 * G) * ncol + col];
  }
  for (; t < ntiles; t += G) s0 += slab[t * ncol + col];
  part[r * ncol + col] = (s0 + s1) + (s2 + s3);
}

// out[col] (+)= sum_r part[r][col]: 64 columns x 4 row groups per block, LDS combine
__global__ void __launch_bounds__(256)
k_knot_reduce2(const double* __restrict__ part, int rows, int64_t ncol, double* __restrict__ out,
               int accumulate) {
  __shared__ double sh[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 64 + tx;
  double s0 = 0.0, s1 = 0.0;
  if (col < ncol) {
    int r = ty;
    for (; r + 4 < rows; r += 8) {
      s0 += part[(int64_t)r * ncol + col];
      s1 += part[(int64_t)(r + 4) * ncol + col];
    }
    for (; r < rows; r += 4) s0 += part[(int64_t)r * ncol + col];
  }
  sh[ty][tx] = s0 + s1;
  __syncthreads();
  if (ty == 0 && col < ncol) {
    const double s = (sh[0][tx] + sh[1][tx]) + (sh[2][tx] + sh[3][tx]);
    out[col] = accumulate ? out[col] + s : s;
  }
}

// ============================================================================ coincidences
// tau's dK12/dlog(tau) = 2 tau^2 exactly where a data row equals a knot (quirk Q5).  Knots are
// hashed on the host (khash sorted, kidx the knot of each hash); thread i hashes row i,
// binary-searches, verifies the coordinates and, per match j, recomputes
//   G_ij = alpha_i u_j + beta_i v_j + rs_i (K M)_ij
// with one length-m dot product.  Per-row sums, block partials [nb][3] = {sum G, count,
// sum cdiag_j}: deterministic, and O(n d) work when nothing coincides.
__device__ __forceinline__ uint64_t coord_hash(const double* x, int64_t stride, int d) {
  uint64_t h = 1469598103934665603ull;
  for (int c = 0; c < d; ++c) {
    double v = x[c * stride];
    if (v == 0.0) v = 0.0;   // +0 and -0 compare equal in R
    uint64_t b = (uint64_t)__double_as_longlong(v);
    for (int k = 0; k < 8; ++k) {
      h ^= (b >> (8 * k)) & 0xffu;
      h *= 1099511628211ull;
    }
  }
  return h;
}

// Coincidence scan of block `bid` of `nblk` (tau's dK12/dtau = 2 tau^2 pairs)
struct CoincArgs {
  const double* X; int64_t ldx, n; int d;
  const double* U; int64_t ldu, m;
  const uint64_t* khash; const int* kidx;
  const double* K; int64_t mp; const double* M;
  const double* alpha; const double* uvec; const double* beta; const double* vvec;
  const double* rs_vec; double rs; const double* cdiag;
  uint8_t* cflag; int flag_mode;
  const double* M2; const double* rs_vec2; double rs2;   // ConArgs::M2 (fused two-product pass)
};

__device__ __forceinline__ void coinc_body(const CoincArgs& ca, int64_t bid, int64_t nblk,
                                           double* __restrict__ part) {
  const double* __restrict__ X = ca.X;
  const double* __restrict__ U = ca.U;
  const double* __restrict__ K = ca.K;
  const double* __restrict__ M = ca.M;
  const int64_t ldx = ca.ldx, n = ca.n, ldu = ca.ldu, m = ca.m, mp = ca.mp;
  const int d = ca.d, flag_mode = ca.flag_mode;
  const uint64_t* __restrict__ khash = ca.khash;
  const int* __restrict__ kidx = ca.kidx;
  const double *alpha = ca.alpha, *uvec = ca.uvec, *beta = ca.beta, *vvec = ca.vvec;
  const double *rs_vec = ca.rs_vec, *cdiag = ca.cdiag;
  const double rs = ca.rs;
  uint8_t* cflag = ca.cflag;
  // flag_mode 1: hash every row and record in cflag whether it equals some knot;
  //           2: cflag is current for this knot set -- only flagged rows are revisited
  double a[3] = {0.0, 0.0, 0.0};
  for (int64_t i = bid * 256 + threadIdx.x; i < n; i += nblk * 256) {
    if (flag_mode == 2 && !cflag[i]) continue;
    bool any = false;
    const uint64_t h = coord_hash(X + i, ldx, d);
    int64_t lo = 0, hi = m;   // first position with khash >= h
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (khash[mid] < h) lo = mid + 1; else hi = mid;
    }
    for (int64_t p = lo; p < m && khash[p] == h; ++p) {
      const int64_t j = kidx[p];
      bool eq = true;
      for (int c = 0; c < d; ++c) eq = eq && (X[i + c * ldx] == U[j + c * ldu]);
      if (!eq) continue;
      any = true;
      double t = 0.0;
      for (int64_t k = 0; k < m; ++k) t = fma(K[i * mp + k], M[k * mp + j], t);
      double g = (rs_vec ? rs * rs_vec[i] : rs) * t;
      if (ca.M2) {
        double t2 = 0.0;
        for (int64_t k = 0; k < m; ++k) t2 = fma(K[i * mp + k], ca.M2[k * mp + j], t2);
        g = fma(ca.rs_vec2 ? ca.rs2 * ca.rs_vec2[i] : ca.rs2, t2, g);
      }
      if (beta) g = fma(beta[i], vvec[j], g);
      if (alpha && uvec) g = fma(alpha[i], uvec[j], g);
      a[0] += g;
      a[1] += 1.0;
      a[2] += cdiag ? cdiag[j] : 0.0;
    }
    if (flag_mode == 1) cflag[i] = any ? 1 : 0;
  }
  __shared__ double sh[4][3];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int k = 0; k < 3; ++k) {
    const double v = wave_sum(a[k]);
    if (lane == 0) sh[w][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < 3)
    part[bid * 3 + threadIdx.x] =
        sh[0][threadIdx.x] + sh[1][threadIdx.x] + sh[2][threadIdx.x] + sh[3][threadIdx.x];
}

// The contraction's record reduction, first pass, in one launch: blocks [0, nbc) run the
// coincidence scan (partials part_c[b][3]); blocks [nbc, nbc + nrow * G) sum field c's
// per-tile records over the tile range of group g (partials part_r[c][g]).
__global__ void __launch_bounds__(256)
k_rec_pass1(CoincArgs ca, int nbc, const double* __restrict__ slab, int64_t len, int G,
            double* __restrict__ part_r, double* __restrict__ part_c) {
  if ((int)blockIdx.x < nbc) {
    coinc_body(ca, blockIdx.x, nbc, part_c);
    return;
  }
  __shared__ double sh[4];
  const int64_t bid = (int64_t)blockIdx.x - nbc, c = bid / G, g = bid % G;
  const int64_t b = len * g / G, e = len * (g + 1) / G;
  double v = 0.0;
  for (int64_t k = b + threadIdx.x; k < e; k += 256) v += slab[c * len + k];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) part_r[c * G + g] = sh[0] + sh[1] + sh[2] + sh[3];
}

// Second pass (one block, fixed summation orders): rec[c] = sum_g part_r[c][g] for c < nrow,
// and the coincidence sums added to rec[coff + 0..2].
__device__ __forceinline__ void rec_pass2_body(const RecPass2& p) {
  __shared__ double sh[3][4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  for (int b = tid; b < p.nbc; b += 256) {
    s0 += p.part_c[b * 3];
    s1 += p.part_c[b * 3 + 1];
    s2 += p.part_c[b * 3 + 2];
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (lane == 0) {
    sh[0][wv] = s0;
    sh[1][wv] = s1;
    sh[2][wv] = s2;
  }
  __syncthreads();
  if (tid < p.nrow) {
    double v = 0.0;
    for (int g = 0; g < p.G; ++g) v += p.part_r[tid * p.G + g];
    const int q = tid - p.coff;
    if (q >= 0 && q < 3) v += sh[q][0] + sh[q][1] + sh[q][2] + sh[q][3];
    p.rec[tid] = v;
  }
}

__global__ void __launch_bounds__(256) k_rec_pass2(RecPass2 p) { rec_pass2_body(p); }

// The readback kernel (capi.hip Readback::wait): the deferred pass 2, then the segments into
// pinned host memory (the records it just wrote among them: same workgroup, ordered by the barrier)
__global__ void __launch_bounds__(256) k_rec_gather(RecPass2 p, GatherSegs g,
                                                    double* __restrict__ dst) {
  if (p.rec != nullptr) {
    rec_pass2_body(p);
    __syncthreads();
  }
  for (int q = 0; q < g.count; ++q)
    for (int i = threadIdx.x; i < g.n[q]; i += 256) dst[g.off[q] + i] = g.src[q][i];
  __threadfence_system();
}

// rowq[tj][i] summed over the column tiles -> out[i] (deterministic order)
__global__ void __launch_bounds__(256)
k_rowq_reduce(const double* __restrict__ rowq, int64_t ntj, int64_t n_pad,
              double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n_pad) return;
  double s = 0.0;
  for (int64_t t = 0; t < ntj; ++t) s += rowq[t * n_pad + i];
  out[i] = s;
}

// ============================================================================ generic 64x64 GEMM
// [64][16] A image stride.  The compiler pairs the fragment reads into ds_read2_b64, which banks
// (a/4) mod 32 in 16-lane groups: the 16 rows a group reads must fall on distinct double slots
// mod 16, i.e. an odd stride (18 gave 2-way conflicts: 0.25 of the LDS cycles, r2 PMC pass)
constexpr int GA = 17;
constexpr int GB = 80;   // [16][64] B image stride: 2*80 % 64 == 32
template <bool TA, bool TB>
__global__ void __launch_bounds__(256)
k_gemm64(int64_t M, int64_t N, int64_t Kd, double alpha, const double* __restrict__ A,
         int64_t lda, const double* __restrict__ B, int64_t ldb, double beta,
         double* C, int64_t ldc, int lower_only) {
  // double-buffered LDS with the next k-step's operands prefetched into registers while the
  // current step's MFMAs run (Kd is a multiple of 16 at every call site: padded m x m blocks)
  __shared__ double As[2][64 * GA];
  __shared__ double Bs[2][16 * GB];
  const int64_t tn = blockIdx.x, tm = blockIdx.y;
  if (lower_only && tm < tn) return;
  const int64_t i0 = tm * 64, j0 = tn * 64;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  d4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
  double ra[4], rb[4];
  auto gload = [&](int64_t k0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + q * 256;
      int row, kk;
      if (!TA) { row = e >> 4; kk = e & 15; } else { kk = e >> 6; row = e & 63; }
      ra[q] = TA ? A[(k0 + kk) * lda + i0 + row] : A[(i0 + row) * lda + k0 + kk];
      int col, kb;
      if (!TB) { kb = e >> 6; col = e & 63; } else { col = e >> 4; kb = e & 15; }
      rb[q] = TB ? B[(j0 + col) * ldb + k0 + kb] : B[(k0 + kb) * ldb + j0 + col];
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + q * 256;
      int row, kk;
      if (!TA) { row = e >> 4; kk = e & 15; } else { kk = e >> 6; row = e & 63; }
      As[buf][row * GA + kk] = ra[q];
      int col, kb;
      if (!TB) { kb = e >> 6; col = e & 63; } else { col = e >> 4; kb = e & 15; }
      Bs[buf][kb * GB + col] = rb[q];
    }
  };
  if (Kd > 0) {
    gload(0);
    sstore(0);
  }
  __syncthreads();
  int cur = 0;
  for (int64_t k0 = 0; k0 < Kd; k0 += 16) {
    const bool more = k0 + 16 < Kd;
    if (more) gload(k0 + 16);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int kx = kk * 4 + (lane >> 4);
      double af[2], bf[2];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        af[f] = As[cur][(wr * 32 + f * 16 + (lane & 15)) * GA + kx];
        bf[f] = Bs[cur][kx * GB + wc * 32 + f * 16 + (lane & 15)];
      }
#pragma unroll
      for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int fn = 0; fn < 2; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[fm], bf[fn], acc[fm][fn], 0, 0, 0);
    }
    if (more) sstore(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
#pragma unroll
  for (int fm = 0; fm < 2; ++fm)
#pragma unroll
    for (int fn = 0; fn < 2; ++fn)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t row = i0 + wr * 32 + fm * 16 + (lane >> 4) + 4 * q;
        const int64_t col = j0 + wc * 32 + fn * 16 + (lane & 15);
        double v = alpha * acc[fm][fn][q];
        if (beta != 0.0) v = fma(beta, C[row * ldc + col], v);
        C[row * ldc + col] = v;
      }
}

struct SyrkPlan {
  int nb, T, splits;
  int64_t chunk;
};

SyrkPlan syrk_plan(int64_t n_pad, int64_t mp) {
  // One resident "round" = 256 CUs x 2 workgroups (216 VGPRs, 74 KB LDS each).  Pick the
  // split count so splits * T fills an integer number of rounds as fully as possible.
  constexpr int64_t kSlots = 512;
  SyrkPlan p;
  p.nb = (int)(mp / T128);
  p.T = p.nb * (p.nb + 1) / 2;
  const int64_t max_splits = n_pad / BK > 0 ? n_pad / BK : 1;
  int64_t best = 1;
  double best_fill = 0.0;
  for (int64_t rounds = 1; rounds <= 4; ++rounds) {
    int64_t sp = rounds * kSlots / p.T;
    if (sp < 1) sp = 1;
    if (sp > max_splits) sp = max_splits;
    const double fill = (double)(sp * p.T) / (double)(((sp * p.T + kSlots - 1) / kSlots) * kSlots);
    if (fill > best_fill + 1e-9) { best_fill = fill; best = sp; }
    if (best_fill >= 0.95) break;
  }
  int64_t chunk = (n_pad + best - 1) / best;
  chunk = (chunk + BK - 1) / BK * BK;
  p.chunk = chunk;
  p.splits = (int)((n_pad + chunk - 1) / chunk);
  return p;
}

// k_syrk_blk: the same split rule over its packed groups (T = workgroups per row chunk)
// Host mirror of syrk_group's image panels (ta, tb) of group gi.
static void syrk_group_panels(int64_t gi, int nb, int& ta, int& tb) {
  const int64_t noff = (int64_t)nb * (nb - 1) / 2;
  if (gi < noff) {
    int a = 1;
    while ((int64_t)(a + 1) * a / 2 <= gi) ++a;
    ta = a;
    tb = (int)(gi - (int64_t)a * (a - 1) / 2);
    return;
  }
  const int g = (int)(gi - noff), G = (3 * nb + 3) / 4, te = G + g / 3;
  ta = g;
  tb = te < nb ? te : g;
}

// t slices: S slices per panel (4, 2 or 1: the largest a greedy matching places with at most
// one slice per group; panels with the fewest holding groups first).  Returns S.
static int syrk_t_table(int nb, int ngroups, int* tmap) {
  for (int S = 4; S >= 1; S >>= 1) {
    std::vector<int> used(ngroups, -1);
    std::vector<std::vector<int>> holders(nb);
    for (int gi = 0; gi < ngroups; ++gi) {
      int ta, tb;
      syrk_group_panels(gi, nb, ta, tb);
      holders[ta].push_back(gi);
      if (tb != ta) holders[tb].push_back(gi);
    }
    std::vector<int> order(nb);
    for (int p = 0; p < nb; ++p) order[p] = p;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
      return holders[x].size() < holders[y].size();
    });
    bool ok = true;
    for (int p : order) {
      for (int sl = 0; sl < S && ok; ++sl) {
        bool placed = false;
        for (int gi : holders[p])
          if (used[gi] < 0) { used[gi] = p * S + sl; placed = true; break; }
        ok = placed;
      }
    }
    if (ok) {
      for (int gi = 0; gi < ngroups; ++gi) tmap[gi] = used[gi];
      return S;
    }
  }
  return 0;   // no placement (does not happen for nb >= 1: S = 1 needs nb distinct holders)
}

SyrkPlan syrk_plan_blk(int64_t n_pad, int64_t mp) {
  SyrkPlan p = syrk_plan(n_pad, mp);   // nb, and a starting point
  const int nb = p.nb;
  const int groups = nb * (nb - 1) / 2 + (3 * nb + 3) / 4;
  constexpr int64_t kSlots = 512;
  const int64_t max_splits = n_pad / BK > 0 ? n_pad / BK : 1;
  int64_t best = 1;
  double best_fill = 0.0;
  for (int64_t rounds = 1; rounds <= 4; ++rounds) {
    int64_t sp = rounds * kSlots / groups;
    if (sp < 1) sp = 1;
    if (sp > max_splits) sp = max_splits;
    const double fill = (double)(sp * groups) /
                        (double)(((sp * groups + kSlots - 1) / kSlots) * kSlots);
    if (fill > best_fill + 1e-9) { best_fill = fill; best = sp; }
    if (best_fill >= 0.95) break;
  }
  int64_t chunk = (n_pad + best - 1) / best;
  chunk = (chunk + BK - 1) / BK * BK;
  p.T = groups;
  p.chunk = chunk;
  p.splits = (int)((n_pad + chunk - 1) / chunk);
  return p;
}

// Balanced plan (nb >= 3): the strictly-lower 128-tiles as k_syrk_blk's packed groups with S_o
// row chunks (64 MFMAs per wave-step), the nb diagonal 128-tiles as syrk_dtile workgroups with
// S_d longer chunks (36 MFMAs per wave-step, no redundant upper fragments), one residency round
// between them.  wd: a diagonal-tile wave-step's cost in MFMA slots (36 issued, plus the
// per-fragment weights and the t slice where they apply).  Unweighted or sqrt(w)-staged S:
// used when its makespan, max(64 chunk_o, wd chunk_d), beats the packed plan's 64 chunk by
// more than 2 % (C5's m = 512: 1.143 -> 1.049 n MFMA-steps per row; at m = 1024 the round's
// integer split counts leave no gain).  force (signed weights or t, WMODE 3): always -- there
// it moves the per-fragment weights and the t slice off the off-diagonal groups.
struct SyrkBal {
  bool on = false;
  int S_o = 0, S_d = 0;
  int64_t chunk_o = 0, chunk_d = 0;
};

static double syrk_dtile_cost(bool weighted, bool with_t) {
  return (double)SGP_SDT_W + (weighted ? (double)SGP_SDT_WW : 0.0) +
         (with_t ? (double)SGP_SDT_WT : 0.0);
}

static SyrkBal syrk_plan_bal(int64_t n_pad, int64_t mp, double wd, bool force) {
  SyrkBal b;
  const int nb = (int)(mp / T128);
  if (nb < 3 || !SGP_SYRK_BAL) return b;
  const int noff = nb * (nb - 1) / 2;
  constexpr int64_t kSlots = 512;
  const int64_t max_splits = n_pad / BK > 0 ? n_pad / BK : 1;
  auto chunk_of = [&](int64_t S) {
    int64_t c = (n_pad + S - 1) / S;
    return (c + BK - 1) / BK * BK;
  };
  double best = 0.0;
  for (int64_t So = 1; So * noff < kSlots && So <= max_splits; ++So) {
    int64_t Sd = (kSlots - So * noff) / nb;
    if (Sd < 1) break;
    if (Sd > max_splits) Sd = max_splits;
    const int64_t co = chunk_of(So), cd = chunk_of(Sd);
    const double T = std::max(64.0 * (double)co, wd * (double)cd);
    if (!b.on || T < best) {
      b.on = true;
      best = T;
      b.chunk_o = co;
      b.chunk_d = cd;
      b.S_o = (int)((n_pad + co - 1) / co);
      b.S_d = (int)((n_pad + cd - 1) / cd);
    }
  }
  if (!b.on || force) return b;
  // the packed plan: one or more rounds of equal workgroups
  const SyrkPlan q = syrk_plan_blk(n_pad, mp);
  const int64_t rounds = ((int64_t)q.splits * q.T + kSlots - 1) / kSlots;
  const double T_pack = 64.0 * (double)q.chunk * (double)rounds;
  b.on = best < 0.98 * T_pack;
  return b;
}

// k_syrk_s256 (mp = 256): two workgroups per row chunk, as many chunks as fill one residency
// round
static SyrkPlan syrk_plan_s256(int64_t n_pad) {
  SyrkPlan p;
  p.nb = 2;
  p.T = 2;
  constexpr int64_t kSlots = 512;
  const int64_t max_splits = n_pad / BK > 0 ? n_pad / BK : 1;
  int64_t sp = kSlots / p.T;
  if (sp > max_splits) sp = max_splits;
  int64_t chunk = (n_pad + sp - 1) / sp;
  chunk = (chunk + BK - 1) / BK * BK;
  p.chunk = chunk;
  p.splits = (int)((n_pad + chunk - 1) / chunk);
  return p;
}

}  // namespace

// the fragment-balanced k_syrk_s256 serves the SYRKs without t at mp = 256
bool syrk_use_s256(int64_t mp, bool with_t) { return mp == 256 && !with_t; }

namespace {

int64_t syrk_slab_doubles_mp(int64_t n_pad, int64_t mp) {
  SyrkPlan q = syrk_plan_blk(n_pad, mp);
  const int64_t nblk = (int64_t)(2 * q.nb) * (2 * q.nb + 1) / 2;
  int64_t need = (int64_t)q.splits * nblk * 4096 + (int64_t)q.splits * q.nb * T128 + q.splits +
                 n_pad;   // + the sqrt(w) rows of WMODE 2
  // every balanced plan launch_syrk_aug may pick (its split counts depend on the weights / t).
  // Its diagonal-tile splits are laid out like the others, over all nblk lower 64-blocks,
  // although syrk_dtile writes only the 3 nb inside the diagonal 128-tiles: ~3.5 MB per diagonal
  // split at m = 1024, of the order of 100 MB per context at C3 -- kept for the uniform block
  // index of the reductions (288 GB of HBM per GPU; a compact layout would save it)
  for (int v = 0; v < 3; ++v) {   // unweighted / sqrt(w); signed weights; weights and t
    const SyrkBal bal = syrk_plan_bal(n_pad, mp, syrk_dtile_cost(v > 0, v > 1), v > 0);
    if (bal.on)
      need = std::max(need, (int64_t)(bal.S_o + bal.S_d) * nblk * 4096 +
                                (int64_t)std::max(bal.S_o, bal.S_d) * (q.nb * T128 + 1) + n_pad);
  }
  if (mp == 256) {
    SyrkPlan r = syrk_plan_s256(n_pad);
    need = std::max(need, (int64_t)r.splits * (10 * 4096 + 2 * T128 + 1) + n_pad);   // as laid out
  }
  return need;
}
}  // namespace

// slab capacity for every knot count up to mp (an evaluation may use fewer knots than the
// context was created for, and the small-m plans have more splits)
int64_t syrk_slab_doubles(int64_t n_pad, int64_t mp) {
  int64_t need = 0;
  for (int64_t q = T128; q <= mp; q += T128) need = std::max(need, syrk_slab_doubles_mp(n_pad, q));
  return need;
}

hipError_t launch_syrk_aug(const double* K, int64_t n_pad, int64_t mp, const double* r,
                           const double* w, double* slab, int64_t slab_cap, double* red,
                           hipStream_t s, int part, const double* tv, int with_t,
                           const double* rr_src, bool packed, bool w_nonneg, unsigned* rsync) {
  if (packed && with_t) return hipErrorInvalidValue;   // the packed layout is VI's (no t)
  {   // the packed 64-block kernel (no redundant diagonal-tile halves), or at mp = 256 the
      // fragment-balanced k_syrk_s256 (same slab layout and reduction)
    const bool s256 = syrk_use_s256(mp, with_t != 0);
    SyrkPlan q = s256 ? syrk_plan_s256(n_pad) : syrk_plan_blk(n_pad, mp);
    // nb >= 3: signed weights or t -> WMODE 3 on the balanced plan (the off-diagonal groups
    // stage w o K as their A image and carry no t; the diagonal tiles keep the per-fragment
    // weights and form t); unweighted or sqrt(w)-staged S -> the balanced plan when it beats
    // the packed one (syrk_plan_bal)
    const bool wsq = w && w_nonneg && !with_t;
    bool use3 = !s256 && w && !wsq && SGP_SYRK_W3 && q.nb >= 3;
    SyrkBal bal;
    if (use3) bal = syrk_plan_bal(n_pad, mp, syrk_dtile_cost(true, with_t != 0), true);
    else if (!s256 && !with_t) bal = syrk_plan_bal(n_pad, mp, syrk_dtile_cost(false, false), false);
    // no balanced plan fits one residency round once the strictly-lower groups alone fill it
    // (nb >= 32, m > 3968): the per-fragment weights on the packed plan (WMODE 1) instead
    if (use3 && !bal.on) use3 = false;
    if (bal.on) {
      q.T = q.nb * (q.nb - 1) / 2;   // the packed kernel's strictly-lower groups only
      q.splits = bal.S_o;
      q.chunk = bal.chunk_o;
    }
    const int64_t nblk = (int64_t)(2 * q.nb) * (2 * q.nb + 1) / 2;
    double* sl_s = slab;
    double* sl_d = sl_s + (int64_t)q.splits * nblk * 4096;   // the diagonal tiles' region
    double* sl_t = sl_d + (bal.on ? (int64_t)bal.S_d * nblk * 4096 : 0);
    // t partials: per row chunk of whichever workgroups form t (WMODE 3: the diagonal tiles)
    const int t_splits = use3 ? bal.S_d : q.splits;
    double* sl_rr = sl_t + (int64_t)t_splits * q.nb * T128;
    if (sl_rr + t_splits + n_pad > slab + slab_cap) return hipErrorInvalidValue;   // + sqrt(w)
    const int64_t nwg_blk = (int64_t)q.splits * q.T;
    const dim3 grid((unsigned)(nwg_blk + (bal.on ? (int64_t)bal.S_d * q.nb : 0)));
    SyrkTMap tm{};
    tm.S = 1;
    if ((part & 1) && with_t) {
      // the balanced slice table when the groups fit it; otherwise tm.S = 0 selects the
      // one-slice-per-panel rule inside the kernel (k_syrk_blk)
      tm.S = 0;
      if (q.T <= 128) {
        int tmap[128];
        tm.S = syrk_t_table(q.nb, q.T, tmap);
        for (int gi = 0; gi < q.T; ++gi) tm.e[gi] = (signed char)(tm.S > 0 ? tmap[gi] : -1);
      }
    }
    if ((part & 1) && s256) {
      if (w)
        hipLaunchKernelGGL((k_syrk_s256<true>), grid, dim3(256), 0, s, K, n_pad, w, q.chunk, sl_s);
      else
        hipLaunchKernelGGL((k_syrk_s256<false>), grid, dim3(256), 0, s, K, n_pad, w, q.chunk, sl_s);
    } else if (part & 1) {
      // with t: the weighted forms only (FITC phase 1: w = 1/Z; Laplace: w = B with tv)
      if (with_t && !w) return hipErrorInvalidValue;
      // rows of the t slice per thread: 8 / S (tm.S == 0: one slice per panel)
      const int tr = tm.S >= 4 ? 2 : tm.S == 2 ? 4 : 8;
      // non-negative weights without t: their square roots scale the staged images (with t
      // the extra staging work made FITC's phase-1 SYRK 4.6 % slower, 17.66 -> 18.47 ms at
      // C3, against 2.7 % faster NR objectives at C5: profiles/r4/syrk_sqrt_rows_ab.txt)
      const double* wk = w;
      if (wsq) {
        double* sw = sl_rr + t_splits;   // n_pad doubles past the partial sums
        hipLaunchKernelGGL(k_sqrt_rows, dim3((unsigned)((n_pad + 255) / 256)), dim3(256), 0, s,
                           w, n_pad, sw);
        wk = sw;
      }
#define SYRK_T_LAUNCH(tmode_, wmode_, tr_)                                                     \
  hipLaunchKernelGGL((k_syrk_blk<tmode_, wmode_, tr_>), grid, dim3(256), 0, s, K, n_pad, mp, wk, \
                     r, tv, q.chunk, q.T, q.nb, sl_s, sl_t, sl_rr, tm, nwg_blk, bal.chunk_d, sl_d)
      if (use3) {
        if (with_t && tv) SYRK_T_LAUNCH(2, 3, 2);
        else if (with_t) SYRK_T_LAUNCH(1, 3, 2);
        else SYRK_T_LAUNCH(0, 3, 2);
      } else if (with_t && tv) {
        if (tr == 2) SYRK_T_LAUNCH(2, 1, 2);
        else if (tr == 4) SYRK_T_LAUNCH(2, 1, 4);
        else SYRK_T_LAUNCH(2, 1, 8);
      } else if (with_t) {
        if (tr == 2) SYRK_T_LAUNCH(1, 1, 2);
        else if (tr == 4) SYRK_T_LAUNCH(1, 1, 4);
        else SYRK_T_LAUNCH(1, 1, 8);
      } else if (wsq) {
        SYRK_T_LAUNCH(0, 2, 2);
      } else if (w) {
        SYRK_T_LAUNCH(0, 1, 2);
      } else {
        SYRK_T_LAUNCH(0, 0, 2);
      }
#undef SYRK_T_LAUNCH
    }
    if (part & 2) {
      // many splits (small m): a first pass sums groups of SYRK_RGRP slabs in parallel, the
      // final pass then sums the group totals (fixed order either way: deterministic)
      int stride = 1, stride_d = 1;
      if (rsync && !bal.on && q.splits > SYRK_RGRP && nblk * 16 <= SGP_SYRK_RSYNC_WORDS) {
        const unsigned ng = (unsigned)((q.splits + SYRK_RGRP - 1) / SYRK_RGRP);
        hipLaunchKernelGGL(k_syrk_reduce_last, dim3(4096 / 256, (unsigned)nblk, ng), dim3(256),
                           0, s, sl_s, q.splits, nblk, mp, red, rr_src,
                           red + (packed ? nblk * 4096 : mp * mp) + mp, packed ? 1 : 0, rsync);
        if (with_t)
          hipLaunchKernelGGL(k_syrk_reduce_t, dim3((unsigned)((mp + 255) / 256)), dim3(256), 0, s,
                             sl_t, sl_rr, t_splits, q.nb, mp, red);
        return hipGetLastError();
      }
      if (q.splits > SYRK_RGRP) {
        const unsigned ng = (unsigned)((q.splits + SYRK_RGRP - 1) / SYRK_RGRP);
        hipLaunchKernelGGL(k_syrk_reduce_grp, dim3(4096 / 256, (unsigned)nblk, ng), dim3(256), 0,
                           s, sl_s, q.splits, nblk);
        stride = SYRK_RGRP;
      }
      if (bal.on && bal.S_d > SYRK_RGRP) {
        const unsigned ng = (unsigned)((bal.S_d + SYRK_RGRP - 1) / SYRK_RGRP);
        hipLaunchKernelGGL(k_syrk_reduce_grp, dim3(4096 / 256, (unsigned)nblk, ng), dim3(256), 0,
                           s, sl_d, bal.S_d, nblk);
        stride_d = SYRK_RGRP;
      }
      hipLaunchKernelGGL(k_syrk_reduce_blk, dim3(4096 / 256, (unsigned)nblk), dim3(256), 0, s,
                         sl_s, q.splits, nblk, mp, red, stride, rr_src,
                         red + (packed ? nblk * 4096 : mp * mp) + mp, packed ? 1 : 0,
                         bal.on ? sl_d : nullptr, bal.S_d, stride_d);
      if (with_t)
        hipLaunchKernelGGL(k_syrk_reduce_t, dim3((unsigned)((mp + 255) / 256)), dim3(256), 0, s,
                           sl_t, sl_rr, t_splits, q.nb, mp, red);
    }
    return hipGetLastError();
  }
}

int64_t syrk_packed_doubles(int64_t mp) {
  const int64_t nb64 = mp / 64;
  return nb64 * (nb64 + 1) / 2 * 4096;
}

hipError_t launch_unpack_lower64(const double* packed, int64_t mp, double* S, hipStream_t s) {
  hipLaunchKernelGGL(k_unpack_lower64, dim3((unsigned)((mp * mp + 255) / 256)), dim3(256), 0, s,
                     packed, mp, S);
  return hipGetLastError();
}

int64_t gemm_tn_splits(int64_t n_pad, int ntile) {
  constexpr int64_t kSlots = 512;
  int64_t sp = kSlots / ntile;
  if (sp < 1) sp = 1;
  const int64_t max_splits = n_pad / BK > 0 ? n_pad / BK : 1;
  return sp > max_splits ? max_splits : sp;
}

int64_t gemm_tn_slab_doubles(int64_t n_pad, int64_t ma, int64_t mb) {
  const int ntile = (int)((ma / T128) * (mb / T128));
  return gemm_tn_splits(n_pad, ntile) * ntile * T128 * T128;
}

hipError_t launch_gemm_tn(const double* A, int64_t lda, int64_t ma, const double* B, int64_t ldb,
                          int64_t mb, int64_t n_pad, double* slab, int64_t slab_cap, double* C,
                          hipStream_t s) {
  const int nta = (int)(ma / T128), ntb = (int)(mb / T128), ntile = nta * ntb;
  int64_t splits = gemm_tn_splits(n_pad, ntile);
  int64_t chunk = (n_pad + splits - 1) / splits;
  chunk = (chunk + BK - 1) / BK * BK;
  splits = (n_pad + chunk - 1) / chunk;
  if (splits * ntile * T128 * T128 > slab_cap) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_gemm_tn, dim3((unsigned)(splits * ntile)), dim3(256), 0, s, A, lda, B, ldb,
                     n_pad, nta, ntb, chunk, slab);
  hipLaunchKernelGGL(k_gemm_tn_reduce, dim3(T128 * T128 / 256, ntile), dim3(256), 0, s, slab,
                     (int)splits, nta, ntb, C);
  return hipGetLastError();
}

hipError_t launch_rec_gather(const RecPass2& p2, const GatherSegs& g, double* dst, hipStream_t s) {
  hipLaunchKernelGGL(k_rec_gather, dim3(1), dim3(256), 0, s, p2, g, dst);
  return hipGetLastError();
}

hipError_t launch_records(const double* slab, int64_t nrow, int64_t len, const double* X,
                          int64_t ldx, int64_t n, int d, const double* U, int64_t ldu, int64_t m,
                          const uint64_t* khash, const int* kidx, const double* K, int64_t mp,
                          const double* M, const ConArgs& cg, const double* alpha, double* part,
                          int64_t part_cap, int coff, double* rec, uint8_t* cflag, int flag_mode,
                          hipStream_t s, RecPass2* defer) {
  if (nrow <= 0 || nrow > 256 || coff < 0 || coff + 3 > nrow) return hipErrorInvalidValue;
  const int G = 32;
  int64_t nbc = (n + 255) / 256;
  if (nbc > 1024) nbc = 1024;
  if (nbc < 1) nbc = 1;
  if (nrow * G + 3 * nbc > part_cap) return hipErrorInvalidValue;
  double* part_r = part;
  double* part_c = part + nrow * G;
  CoincArgs ca{X, ldx, n, d, U, ldu, m, khash, kidx, K, mp, M, alpha, cg.uvec, cg.beta_in,
               cg.vvec, cg.rs_vec, cg.rs, cg.cdiag, cflag, flag_mode, cg.M2, cg.rs_vec2,
               cg.rs2};
  hipLaunchKernelGGL(k_rec_pass1, dim3((unsigned)(nbc + nrow * G)), dim3(256), 0, s, ca,
                     (int)nbc, slab, len, G, part_r, part_c);
  RecPass2 p2;
  p2.part_r = part_r;
  p2.part_c = part_c;
  p2.rec = rec;
  p2.G = G;
  p2.nrow = (int)nrow;
  p2.nbc = (int)nbc;
  p2.coff = coff;
  if (defer != nullptr) *defer = p2;
  else hipLaunchKernelGGL(k_rec_pass2, dim3(1), dim3(256), 0, s, p2);
  return hipGetLastError();
}

hipError_t launch_knot_reduce(const double* knot_slab, int64_t ntiles, int64_t mp, int d,
                              double* part, int64_t part_cap, double* out, bool accumulate,
                              hipStream_t s) {
  const int64_t ncol = mp * d;
  const unsigned gx = (unsigned)((ncol + 255) / 256);
  // enough row groups that each thread of the first pass sums ~32 rows (latency, not
  // bandwidth, bounds this tall column sum), within the partials' capacity
  int64_t gy = ntiles / 32;
  if (gy > 256) gy = 256;
  if (gy > part_cap / ncol) gy = part_cap / ncol;
  if (gy < 1) gy = 1;
  if (gy * ncol > part_cap) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_knot_reduce1, dim3(gx, (unsigned)gy), dim3(256), 0, s, knot_slab, ntiles,
                     ncol, part);
  hipLaunchKernelGGL(k_knot_reduce2, dim3((unsigned)((ncol + 63) / 64)), dim3(256), 0, s, part,
                     (int)gy, ncol, out, accumulate ? 1 : 0);
  return hipGetLastError();
}

// dynamic LDS of the gradient-contraction launches: SGP_CON_SHMEM (sgp_probe.h) is 0 in the
// product; tools/micro/con_trace.hip builds with a pad that leaves one workgroup per CU
// The balanced launch when the tile grid's last residency round would be mostly empty: more
// than 2 % of the rounds' capacity idle, and a workgroup's range at least one tile's k-steps
static bool con_use_sk(const ConArgs& ca, int64_t nwg, int64_t mp) {
  if (ca.sk_ws == nullptr || ca.sk_slots < 1 || nwg < ca.sk_slots) return false;
  const int64_t G = ca.sk_slots, S = mp / BK;
  const int64_t rounds = (nwg + G - 1) / G;
  const double idle = 1.0 - (double)nwg / (double)(rounds * G);
  return idle > 0.02 && nwg * S / G >= S;
}

template <int DT, bool KNOT = false>
static void launch_con_grad(bool v2, const KernParams& kp, const double* K, const double* M,
                            const double* X, int64_t ldx, int64_t n, int64_t n_pad,
                            const double* U, int64_t ldu, int64_t m, int64_t mp,
                            const ConArgs& ca, double* slab, int nrec, int64_t nwg,
                            hipStream_t s) {
  if (!v2 && con_use_sk(ca, nwg, mp)) {
    ConSK sk;
    sk.ws = ca.sk_ws;
    sk.flags = ca.sk_flags;
    sk.epoch = ca.sk_epoch;
    sk.status = ca.sk_status;
    sk.dp = ca.sk_dp;
    hipLaunchKernelGGL((k_contract_sk<DT, KNOT>), dim3((unsigned)ca.sk_slots), dim3(256), 0, s,
                       kp, K, M, X, ldx, n, n_pad, U, ldu, m, mp, ca, slab, nrec, sk);
    return;
  }
  if (v2)
    hipLaunchKernelGGL((k_contract<DT, EPI_GRAD, true, KNOT>), dim3((unsigned)nwg), dim3(256), SGP_CON_SHMEM,
                       s, kp, K, M, X, ldx, n, n_pad, U, ldu, m, mp, ca, slab, nrec,
                       (double*)nullptr);
  else
    hipLaunchKernelGGL((k_contract<DT, EPI_GRAD, false, KNOT>), dim3((unsigned)nwg), dim3(256), SGP_CON_SHMEM,
                       s, kp, K, M, X, ldx, n, n_pad, U, ldu, m, mp, ca, slab, nrec,
                       (double*)nullptr);
}

// the gradient pass over a stored product T = K M (FROM_T: no k-loop)
template <int DT, bool T2>
static void launch_con_from_t2(bool v2, bool kn, const KernParams& kp, const double* K,
                               const double* M, const double* X, int64_t ldx, int64_t n,
                               int64_t n_pad, const double* U, int64_t ldu, int64_t m, int64_t mp,
                               const ConArgs& ca, double* slab, int nrec, int64_t nwg,
                               hipStream_t s) {
  const dim3 g((unsigned)nwg), b(256);
  if (v2 && kn)
    hipLaunchKernelGGL((k_contract<DT, EPI_GRAD, true, true, true, true, T2>), g, b, 0, s, kp, K,
                       M, X, ldx, n, n_pad, U, ldu, m, mp, ca, slab, nrec, (double*)nullptr);
  else if (v2)
    hipLaunchKernelGGL((k_contract<DT, EPI_GRAD, true, false, true, true, T2>), g, b, 0, s, kp, K,
                       M, X, ldx, n, n_pad, U, ldu, m, mp, ca, slab, nrec, (double*)nullptr);
  else if (kn)
    hipLaunchKernelGGL((k_contract<DT, EPI_GRAD, false, true, true, true, T2>), g, b, 0, s, kp, K,
                       M, X, ldx, n, n_pad, U, ldu, m, mp, ca, slab, nrec, (double*)nullptr);
  else
    hipLaunchKernelGGL((k_contract<DT, EPI_GRAD, false, false, true, true, T2>), g, b, 0, s, kp,
                       K, M, X, ldx, n, n_pad, U, ldu, m, mp, ca, slab, nrec, (double*)nullptr);
}

template <int DT>
static void launch_con_from_t(bool v2, bool kn, const KernParams& kp, const double* K,
                              const double* M, const double* X, int64_t ldx, int64_t n,
                              int64_t n_pad, const double* U, int64_t ldu, int64_t m, int64_t mp,
                              const ConArgs& ca, double* slab, int nrec, int64_t nwg,
                              hipStream_t s) {
  if constexpr (DT == 8) {   // the two-product pass: d <= 8 only (spill-free at 246-256 VGPRs)
    if (ca.tin2 != nullptr) {
      launch_con_from_t2<DT, true>(v2, kn, kp, K, M, X, ldx, n, n_pad, U, ldu, m, mp, ca, slab,
                                   nrec, nwg, s);
      return;
    }
  }
    launch_con_from_t2<DT, false>(v2, kn, kp, K, M, X, ldx, n, n_pad, U, ldu, m, mp, ca, slab,
                                  nrec, nwg, s);
}

int64_t sgp_con_sk_doubles(int slots) { return (int64_t)(slots + 1) * CON_SK_SLOT; }

hipError_t launch_contract_args(const KernParams& kp, const double* K, const double* M,
                                const double* X, int64_t ldx, int64_t n, int64_t n_pad,
                                const double* U, int64_t ldu, int64_t m, int64_t mp,
                                const ConArgs& ca, double* slab, int64_t* nrec_out,
                                int64_t* nwg_out, hipStream_t s) {
  const int64_t nwg = (n_pad / T128) * (mp / T128);
  const int nrec = kp.L + 5;
  *nrec_out = nrec;
  *nwg_out = nwg;
  if ((ca.tin2 != nullptr) != (ca.M2 != nullptr) || (ca.tin2 && (!ca.tin || kp.d > 8)))
    return hipErrorInvalidValue;   // the second product: beside a first, with its M, d <= 8
  if (ca.tin != nullptr) {   // stored product: no k-loop (alpha from alpha_in)
    if (ca.uvec != nullptr && ca.alpha_in == nullptr) return hipErrorInvalidValue;
    const bool v2 = ca.beta_in != nullptr, kn = ca.knot_slab != nullptr;
    if (kp.d <= 8) launch_con_from_t<8>(v2, kn, kp, K, M, X, ldx, n, n_pad, U, ldu, m, mp, ca, slab,
                                        nrec, nwg, s);
    else launch_con_from_t<SGP_MAXD>(v2, kn, kp, K, M, X, ldx, n, n_pad, U, ldu, m, mp, ca, slab,
                                     nrec, nwg, s);
    return hipGetLastError();
  }
  if (ca.knot_slab != nullptr) {
    const bool v2 = ca.beta_in != nullptr;
    if (kp.d <= 8) launch_con_grad<8, true>(v2, kp, K, M, X, ldx, n, n_pad, U, ldu, m, mp, ca,
                                            slab, nrec, nwg, s);
    else launch_con_grad<SGP_MAXD, true>(v2, kp, K, M, X, ldx, n, n_pad, U, ldu, m, mp, ca, slab,
                                         nrec, nwg, s);
  } else {
    // coordinate bound DT: one chunk of 8 (C3 and below) or up to SGP_MAXD in chunks of 8
    const bool v2 = ca.beta_in != nullptr;   // FITC / Laplace two-term epilogue
    if (kp.d <= 8) launch_con_grad<8>(v2, kp, K, M, X, ldx, n, n_pad, U, ldu, m, mp, ca, slab,
                                      nrec, nwg, s);
    else launch_con_grad<SGP_MAXD>(v2, kp, K, M, X, ldx, n, n_pad, U, ldu, m, mp, ca, slab, nrec,
                                   nwg, s);
  }
  return hipGetLastError();
}

hipError_t launch_contract_knm(const KernParams& kp, const double* K, const double* M,
                               const double* X, int64_t ldx, int64_t n, int64_t n_pad,
                               const double* U, int64_t ldu, int64_t m, int64_t mp,
                               const double* r, double invz, const double* invz_vec,
                               const double* uvec, const double* rs_vec, double rs,
                               const double* coinc_diag, int count_a2, double* slab,
                               int64_t* nrec_out, int64_t* nwg_out, hipStream_t s) {
  ConArgs ca;
  ca.r = r;
  ca.invz = invz;
  ca.invz_vec = invz_vec;
  ca.uvec = uvec;
  ca.rs_vec = rs_vec;
  ca.rs = rs;
  ca.cdiag = coinc_diag;
  ca.count_a2 = count_a2;
  return launch_contract_args(kp, K, M, X, ldx, n, n_pad, U, ldu, m, mp, ca, slab, nrec_out,
                              nwg_out, s);
}

hipError_t launch_rowquad_knm(const KernParams& kp, const double* K, const double* M, int64_t n,
                              int64_t n_pad, int64_t m, int64_t mp, const double* r,
                              double invz, const double* invz_vec, const double* uvec,
                              double* alpha_out, double* rowq_slab, double* out,
                              hipStream_t s, double* tstore) {
  const int64_t nwg = (n_pad / T128) * (mp / T128);
  ConArgs ca;
  ca.r = r;
  ca.invz = invz;
  ca.invz_vec = invz_vec;
  ca.uvec = uvec;
  ca.alpha_out = alpha_out;
  ca.tstore = tstore;
  if (uvec != nullptr || SGP_CON_ROWQ_KU)
    hipLaunchKernelGGL((k_contract<8, EPI_ROWQUAD>), dim3((unsigned)nwg), dim3(256), 0, s, kp, K, M,
                       (const double*)nullptr, (int64_t)0, n, n_pad, (const double*)nullptr,
                       (int64_t)0, m, mp, ca, (double*)nullptr, 0, rowq_slab);
  else   // the Z pass: no K u fold in the k-loop
    hipLaunchKernelGGL((k_contract<8, EPI_ROWQUAD, false, false, false, false>),
                       dim3((unsigned)nwg), dim3(256), 0, s, kp, K, M, (const double*)nullptr,
                       (int64_t)0, n, n_pad, (const double*)nullptr, (int64_t)0, m, mp, ca,
                       (double*)nullptr, 0, rowq_slab);
  hipLaunchKernelGGL(k_rowq_reduce, dim3((unsigned)((n_pad + 255) / 256)), dim3(256), 0, s,
                     rowq_slab, mp / T128, n_pad, out);
  return hipGetLastError();
}

hipError_t launch_gemm64(bool transA, bool transB, bool lower_only, int64_t M, int64_t N,
                         int64_t K, double alpha, const double* A, int64_t lda,
                         const double* B, int64_t ldb, double beta, double* C, int64_t ldc,
                         hipStream_t s) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (M % 64 || N % 64 || K % 16 || K < 0) return hipErrorInvalidValue;   // tile-padded shapes only
  dim3 grid((unsigned)(N / 64), (unsigned)(M / 64));
  const int lo = lower_only ? 1 : 0;
  if (!transA && !transB)
    hipLaunchKernelGGL((k_gemm64<false, false>), grid, dim3(256), 0, s, M, N, K, alpha, A, lda,
                       B, ldb, beta, C, ldc, lo);
  else if (!transA && transB)
    hipLaunchKernelGGL((k_gemm64<false, true>), grid, dim3(256), 0, s, M, N, K, alpha, A, lda, B,
                       ldb, beta, C, ldc, lo);
  else if (transA && !transB)
    hipLaunchKernelGGL((k_gemm64<true, false>), grid, dim3(256), 0, s, M, N, K, alpha, A, lda, B,
                       ldb, beta, C, ldc, lo);
  else
    hipLaunchKernelGGL((k_gemm64<true, true>), grid, dim3(256), 0, s, M, N, K, alpha, A, lda, B,
                       ldb, beta, C, ldc, lo);
  return hipGetLastError();
}
