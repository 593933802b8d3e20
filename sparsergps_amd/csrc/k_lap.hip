// Per-row kernels of the Poisson sparse-Laplace path (newtrap_sparseGP + dlogq_dcov_par in
// adjoint form) and the two HBM-bound K12 matrix-vector passes it needs.
//
// Every kernel here is a single streaming pass: the n-vectors are ~8 B/row each, the GEMVs
// read K12 (n_pad x mp, row-major) once.  Per-block partial sums go to a slab reduced by
// launch_colsum (deterministic, no atomics), so all ranks / reruns see identical bits.
//
// Row semantics follow the reference (R/derivative_functions_of_data_likelihoods.R:7-61,
// R/newtrap_sparseGP.R:234-325, R/laplace_approx_obj_funs.R:108-174,
// R/laplace_approx_gradient.R:133-336) with a = exposure (`m` in the reference's Poisson
// helpers, "a vector of the areas of each grid cell", derivative_functions_of_data_likelihoods.R:
// 38): W = d2 = d3 = -a e^f, d1 = y - a e^f.  a is per row: av[i] when the context holds a
// per-row exposure (sgp_lap_set_expo), the scalar expo otherwise (av == nullptr).
#include "sgp_internal.h"
#include "sgp_probe.h"

namespace {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide sums of NV values into slab[blockIdx.x * NV + k]
template <int NV>
__device__ __forceinline__ void block_store_sums(const double (&v)[NV], double* slab) {
  __shared__ double sh[4][NV];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const double s = wave_sum(v[k]);
    if (lane == 0) sh[w][k] = s;
  }
  __syncthreads();
  if (threadIdx.x < NV)
    slab[(int64_t)blockIdx.x * NV + threadIdx.x] =
        sh[0][threadIdx.x] + sh[1][threadIdx.x] + sh[2][threadIdx.x] + sh[3][threadIdx.x];
}

#define ROW_LOOP(i) \
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_pad; i += (int64_t)gridDim.x * 256)

// Z_i = c0 - q_i (newtrap_sparseGP.R:63-66), zinv = 1/Z; padded rows Z = 1, zinv = 0.
__global__ void __launch_bounds__(256) k_lap_z(const double* __restrict__ q, int64_t n,
                                               int64_t n_pad, double c0, double* __restrict__ Z,
                                               double* __restrict__ zinv) {
  ROW_LOOP(i) {
    const bool v = i < n;
    const double z = v ? c0 - q[i] : 1.0;
    Z[i] = z;
    zinv[i] = v ? 1.0 / z : 0.0;
  }
}

// Objective row terms at f (laplace_approx_obj_funs.R:108-174): SYRK weights
// B = 1/(Z - 1/W) (the R2/R3 weight: -W/Z2 = B), rf = f - mu, tv = rf/Z,
// slab = [sum log p(y_i|f_i), sum log Z2_i],  Z2 = 1 + sqrt(-W) Z sqrt(-W).
__global__ void __launch_bounds__(256) k_lap_obj(int64_t n, int64_t n_pad,
                                                 const double* __restrict__ f,
                                                 const double* __restrict__ y,
                                                 const double* __restrict__ mu,
                                                 const double* __restrict__ Z,
                                                 const double* __restrict__ zinv, double expo,
                                                 double logexpo, const double* __restrict__ av,
                                                 double* __restrict__ B,
                                                 double* __restrict__ rf, double* __restrict__ tv,
                                                 double* __restrict__ slab) {
  double acc[2] = {0.0, 0.0};
  ROW_LOOP(i) {
    if (i < n) {
      const double fi = f[i], yi = y[i], zi = Z[i];
      const double ai = av ? av[i] : expo, lai = av ? log(ai) : logexpo;
      const double e = exp(fi);
      const double W = -ai * e;
      B[i] = 1.0 / (zi - 1.0 / W);
      const double r = fi - mu[i];
      rf[i] = r;
      tv[i] = zinv[i] * r;
      acc[0] += yi * lai - lgamma(yi + 1.0) - ai * e + yi * fi;
      const double sw = sqrt(-W);
      acc[1] += log(1.0 + sw * zi * sw);
    } else {
      B[i] = 0.0;
      rf[i] = 0.0;
      tv[i] = 0.0;
    }
  }
  block_store_sums<2>(acc, slab);
}

// NR step, part a (grad_loglik_fn_pois + the first half of newtrap_sparseGP_update):
//   g = y - a e^f, omzw = 1 - Z W, gpsi = g - (rf - y1)/Z   (y1 = K Bm_Z^-1 t_Z),
//   v = gpsi / omzw (input of the K^T pass), slab = [#{|gpsi_i| > tol}]; gpsi itself is kept
//   (newtrap_sparseGP's returned `gradient`, R/newtrap_sparseGP.R:178-185).
__global__ void __launch_bounds__(256) k_lap_nr_a(int64_t n, int64_t n_pad,
                                                  const double* __restrict__ f,
                                                  const double* __restrict__ y,
                                                  const double* __restrict__ mu,
                                                  const double* __restrict__ Z,
                                                  const double* __restrict__ zinv, double expo,
                                                  const double* __restrict__ av,
                                                  const double* __restrict__ y1, double tol,
                                                  double* __restrict__ g, double* __restrict__ omzw,
                                                  double* __restrict__ v,
                                                  double* __restrict__ gpsi,
                                                  double* __restrict__ slab) {
  double acc[1] = {0.0};
  ROW_LOOP(i) {
    if (i < n) {
      const double ai = av ? av[i] : expo;
      const double e = exp(f[i]);
      const double W = -ai * e;
      const double gi = -ai * e + y[i];
      const double zi = Z[i], iz = zinv[i];
      const double om = 1.0 - zi * W;
      const double gp = gi + (-iz * (f[i] - mu[i]) + iz * y1[i]);
      g[i] = gi;
      omzw[i] = om;
      v[i] = (1.0 / om) * gp;
      gpsi[i] = gp;
      if (fabs(gp) > tol) acc[0] += 1.0;
    } else {
      g[i] = 0.0;
      omzw[i] = 1.0;
      v[i] = 0.0;
      gpsi[i] = 0.0;
    }
  }
  block_store_sums<1>(acc, slab);
}

// NR step, part b: f += (Z/omzw) g - rf/omzw + y1/omzw + y2/omzw  (y2 = K C K^T v)
// (newtrap_sparseGP.R:252-289: A11 - A12 + A13 + A2).
__global__ void __launch_bounds__(256) k_lap_nr_b(int64_t n, int64_t n_pad,
                                                  double* __restrict__ f,
                                                  const double* __restrict__ mu,
                                                  const double* __restrict__ Z,
                                                  const double* __restrict__ g,
                                                  const double* __restrict__ omzw,
                                                  const double* __restrict__ y1,
                                                  const double* __restrict__ y2) {
  ROW_LOOP(i) {
    if (i < n) {
      const double om = omzw[i], fi = f[i];
      const double a11 = (Z[i] / om) * g[i];
      const double a12 = (1.0 / om) * (fi - mu[i]);
      const double a13 = y1[i] / om;
      const double a2 = y2[i] / om;
      f[i] = fi + (a11 - a12 + a13 + a2);
    }
  }
}

// Gradient rows, part a (laplace_approx_gradient.R:133-178): with p_i = k_i^T C k_i,
//   c2 = rf/Z - y1/Z (left as passed in when y1 == nullptr), B = 1/(Z - 1/W), dMt = B - B^2 p  (diag of Sigma~^-1),
//   comp4 = -1/D + (1/(Z D))^2 p  (D = W - 1/Z),  sv = comp4 (-W3)(-1/W),  bsv = B sv.
__global__ void __launch_bounds__(256) k_lap_grad_a(int64_t n, int64_t n_pad,
                                                    const double* __restrict__ f,
                                                    const double* __restrict__ y,
                                                    const double* __restrict__ mu,
                                                    const double* __restrict__ Z,
                                                    const double* __restrict__ zinv, double expo,
                                                    const double* __restrict__ av,
                                                    const double* __restrict__ y1,
                                                    const double* __restrict__ p,
                                                    double* __restrict__ c2,
                                                    double* __restrict__ g,
                                                    double* __restrict__ B,
                                                    double* __restrict__ dMt,
                                                    double* __restrict__ sv,
                                                    double* __restrict__ bsv) {
  ROW_LOOP(i) {
    if (i < n) {
      const double ai = av ? av[i] : expo;
      const double e = exp(f[i]);
      const double W = -ai * e, W3 = W;
      const double zi = Z[i], iz = zinv[i];
      const double bi = 1.0 / (zi - 1.0 / W);
      const double pi = p[i];
      if (y1) c2[i] = iz * (f[i] - mu[i]) - iz * y1[i];   // else c2 came with p (fused alpha)
      g[i] = -ai * e + y[i];
      B[i] = bi;
      dMt[i] = bi - bi * bi * pi;
      const double D = W - 1.0 / zi;
      const double coef = iz * (1.0 / D);
      const double comp4 = -(1.0 / D) + coef * coef * pi;
      const double s = comp4 * (-W3) * (-1.0 / W);
      sv[i] = s;
      bsv[i] = bi * s;
    } else {
      c2[i] = 0.0;
      g[i] = 0.0;
      B[i] = 0.0;
      dMt[i] = 0.0;
      sv[i] = 0.0;
      bsv[i] = 0.0;
    }
  }
}

// Gradient rows, part b: h = B sv - B (K C w)  (= Sigma~^-1 sv),
//   a = -dMt/2 + c2^2/2 - h g/2 (the coefficient of A = d diag Sigma~), slab = [sum a].
__global__ void __launch_bounds__(256) k_lap_grad_b(int64_t n, int64_t n_pad,
                                                    const double* __restrict__ B,
                                                    const double* __restrict__ sv,
                                                    const double* __restrict__ y3,
                                                    const double* __restrict__ dMt,
                                                    const double* __restrict__ c2,
                                                    const double* __restrict__ g,
                                                    double* __restrict__ h,
                                                    double* __restrict__ a,
                                                    double* __restrict__ slab) {
  double acc[1] = {0.0};
  ROW_LOOP(i) {
    if (i < n) {
      const double bi = B[i];
      const double hi = bi * sv[i] - bi * y3[i];
      const double ci = c2[i];
      const double ai = -0.5 * dMt[i] + 0.5 * ci * ci - 0.5 * hi * g[i];
      h[i] = hi;
      a[i] = ai;
      acc[0] += ai;
    } else {
      h[i] = 0.0;
      a[i] = 0.0;
    }
  }
  block_store_sums<1>(acc, slab);
}

#undef ROW_LOOP

// y1 = K x1 (and y2 = K x2 when x2 != nullptr): one wave per row, double2 loads.
__global__ void __launch_bounds__(256) k_gemv_rows(const double* __restrict__ K, int64_t n_pad,
                                                   int64_t mp, const double* __restrict__ x1,
                                                   const double* __restrict__ x2,
                                                   double* __restrict__ y1,
                                                   double* __restrict__ y2) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t h = mp / 2;
  const double2* X1 = reinterpret_cast<const double2*>(x1);
  const double2* X2 = reinterpret_cast<const double2*>(x2);
  for (int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n_pad; i += nw) {
    const double2* row = reinterpret_cast<const double2*>(K + i * mp);
    double s1 = 0.0, s2 = 0.0;
    for (int64_t c = lane; c < h; c += 64) {
      const double2 k = row[c];
      const double2 a = X1[c];
      s1 = fma(k.x, a.x, s1);
      s1 = fma(k.y, a.y, s1);
      if (x2) {
        const double2 b = X2[c];
        s2 = fma(k.x, b.x, s2);
        s2 = fma(k.y, b.y, s2);
      }
    }
    s1 = wave_sum(s1);
    if (x2) s2 = wave_sum(s2);
    if (lane == 0) {
      y1[i] = s1;
      if (x2) y2[i] = s2;
    }
  }
}

// part[ch][v][j] = sum_{i in chunk ch} K_ij V_v[i]  for v < NV (V_v = V + v * ldv)
template <int NV>
__global__ void __launch_bounds__(128) k_gemv_cols(const double* __restrict__ K, int64_t n_pad,
                                                   int64_t mp, const double* __restrict__ V,
                                                   int64_t ldv, int64_t chunk,
                                                   double* __restrict__ part) {
  const int64_t j = (int64_t)blockIdx.x * 128 + threadIdx.x;
  const int64_t ch = blockIdx.y;
  const int64_t i0 = ch * chunk;
  const int64_t i1 = (i0 + chunk < n_pad) ? i0 + chunk : n_pad;
  double acc[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) acc[v] = 0.0;
  int64_t i = i0;
  for (; i + 4 <= i1; i += 4) {
    double k[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) k[u] = K[(i + u) * mp + j];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < NV; ++v) acc[v] = fma(k[u], V[v * ldv + i + u], acc[v]);
  }
  for (; i < i1; ++i) {
    const double k = K[i * mp + j];
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] = fma(k, V[v * ldv + i], acc[v]);
  }
  double* o = part + (ch * NV) * mp + j;
#pragma unroll
  for (int v = 0; v < NV; ++v) o[v * mp] = acc[v];
}

// Newton-step passes over K12 that each replace a row GEMV, a per-row kernel and a column GEMV
// (two K reads) by one read (k_lap_rowstream below):
// LAP_PASS_A (NR part a): x = x1, the k_lap_nr_a update (y1 = d, g, omzw, gpsi), v = gpsi/omzw,
//   scalars = [stop-rule count].
// LAP_PASS_B (NR part b + the next objective's t): x = x2, the k_lap_nr_b update of f
//   (y2 = d), v = tv = (f - mu)/Z at the new f (t = K^T tv), scalars = [sum tv (f - mu)];
//   k_lap_obj then forms B, rf, tv and the likelihood sums in its own (cheap, fully parallel)
//   pass and S_B comes from the weighted SYRK without t.
// One workgroup per row chunk; part[ch][0..mp) and the scalars sc[ch][..] are reduced by
// launch_colsum (fixed order).  mp <= 2048.
enum { LAP_PASS_A = 0, LAP_PASS_B = 1 };

struct LapPassArgs {
  const double* x;                            // x1 (A) / x2 (B), mp
  const double* f;                            // mode f at the step's start
  double* f_out;                              // B: the updated f (may alias f)
  const double *y, *mu, *Z, *zinv;
  const double *g_in, *omzw_in, *y1_in;       // B
  double expo, tol;                           // A
  const double* av;                           // A: per-row exposure (nullptr: expo)
  double *y1, *g, *omzw, *v, *gpsi;           // A outputs
  double* part;                               // [nch][mp]
  double* sc;                                 // [nch][NS]
};

// The two Newton-step passes, streamed: each wave loads its rows straight into registers (lane l holds columns 2l + 128q, 2l + 128q + 1 of RF rows at a time),
// forms d_i = K_i x with its lanes' x slice and one wave reduction per row, applies the row
// update (every lane; lane 0 stores), and folds v_i K_i into its lanes' column sums from the same
// registers -- no barrier inside the row loop (round 3's form staged 64 KB row blocks in LDS
// behind two barriers per block and stalled on each block's loads: 4.9 against 5.1-5.6 TB/s
// at C5, profiles/r4/lap_rowstream_ab.txt).  The four
// waves' column sums are combined in fixed order at the end.  NQM: double2 columns per lane per
// row (mp / 128 rounded up to 2, 4, 8 or 16), RF rows in flight per wave, OCC waves per SIMD.
template <int MODE, int NQM, int RF, int OCC>
__global__ void __launch_bounds__(256, OCC) k_lap_rowstream(const double* __restrict__ K, int64_t n,
                                                            int64_t n_pad, int64_t mp,
                                                            int64_t chunk, LapPassArgs pa) {
  extern __shared__ __attribute__((aligned(16))) double s_part[];   // [4][mp]
  __shared__ double s_red[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nq = (int)(mp / 128);
  const int64_t ch = blockIdx.x;
  const int64_t i0 = ch * chunk;
  const int64_t i1 = (i0 + chunk < n_pad) ? i0 + chunk : n_pad;
  const double2* K2 = reinterpret_cast<const double2*>(K);
  const double2* x2 = reinterpret_cast<const double2*>(pa.x);
  const int64_t mp2 = mp / 2;
  double2 xr[NQM], acc[NQM];
#pragma unroll
  for (int q = 0; q < NQM; ++q) {
    xr[q] = (q < nq) ? x2[lane + 64 * q] : make_double2(0.0, 0.0);
    acc[q] = make_double2(0.0, 0.0);
  }
  double sc = 0.0;   // the pass's scalar sum over the rows this lane updated
  for (int64_t g0 = i0 + (int64_t)wv * RF; g0 < i1; g0 += 4 * RF) {
    double2 kr[RF][NQM];
#pragma unroll
    for (int r = 0; r < RF; ++r)
#pragma unroll
      for (int q = 0; q < NQM; ++q)
        kr[r][q] = (g0 + r < i1 && q < nq) ? K2[(g0 + r) * mp2 + lane + 64 * q]
                                           : make_double2(0.0, 0.0);
    double d[RF];
#pragma unroll
    for (int r = 0; r < RF; ++r) {
      double s0 = 0.0;
#pragma unroll
      for (int q = 0; q < NQM; ++q) {
        s0 = fma(kr[r][q].x, xr[q].x, s0);
        s0 = fma(kr[r][q].y, xr[q].y, s0);
      }
      d[r] = wave_sum(s0);
    }
    // the row updates: lane r < RF takes row g0 + r (one exp per row, not one per lane)
    double dme = d[0];
#pragma unroll
    for (int r = 1; r < RF; ++r) dme = (lane == r) ? d[r] : dme;
    double vme = 0.0;
    const int64_t im = g0 + lane;
    if (lane < RF && im < i1) {
      if constexpr (MODE == LAP_PASS_A) {   // k_lap_nr_a
        if (im < n) {
          const double fi = pa.f[im], yi = pa.y[im], mui = pa.mu[im], zi = pa.Z[im];
          const double iz = pa.zinv[im];
          const double ai = pa.av ? pa.av[im] : pa.expo;
          const double e = exp(fi);
          const double W = -ai * e;
          const double gi = -ai * e + yi;
          const double om = 1.0 - zi * W;
          const double gp = gi + (-iz * (fi - mui) + iz * dme);
          vme = (1.0 / om) * gp;
          pa.g[im] = gi;
          pa.omzw[im] = om;
          pa.gpsi[im] = gp;
          if (fabs(gp) > pa.tol) sc += 1.0;
        } else {
          pa.g[im] = 0.0;
          pa.omzw[im] = 1.0;
          pa.gpsi[im] = 0.0;
        }
        pa.y1[im] = dme;
        pa.v[im] = vme;
      } else {                              // k_lap_nr_b; tv = (f - mu)/Z at the new f
        if (im < n) {
          const double fi = pa.f[im], mui = pa.mu[im], zi = pa.Z[im], iz = pa.zinv[im];
          const double gi = pa.g_in[im], om = pa.omzw_in[im], y1i = pa.y1_in[im];
          const double a11 = (zi / om) * gi;
          const double a12 = (1.0 / om) * (fi - mui);
          const double a13 = y1i / om;
          const double a2 = dme / om;
          const double fn = fi + (a11 - a12 + a13 + a2);
          pa.f_out[im] = fn;
          const double rr = fn - mui;
          vme = iz * rr;
          sc = fma(vme, rr, sc);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < RF; ++r) {
      const double vi = __shfl(vme, r, 64);   // 0 for rows past i1
#pragma unroll
      for (int q = 0; q < NQM; ++q) {
        acc[q].x = fma(kr[r][q].x, vi, acc[q].x);
        acc[q].y = fma(kr[r][q].y, vi, acc[q].y);
      }
    }
  }
  sc = wave_sum(sc);   // lanes 0..RF-1 hold their rows' parts
#pragma unroll
  for (int q = 0; q < NQM; ++q)
    if (q < nq) reinterpret_cast<double2*>(s_part + wv * mp)[lane + 64 * q] = acc[q];
  if (lane == 0) s_red[wv] = sc;
  __syncthreads();
  for (int64_t j = tid; j < mp; j += 256)
    pa.part[ch * mp + j] = ((s_part[j] + s_part[mp + j]) + s_part[2 * mp + j]) + s_part[3 * mp + j];
  if (tid == 0) pa.sc[ch] = ((s_red[0] + s_red[1]) + s_red[2]) + s_red[3];
}

// part[ch][j] = sum_{i in chunk ch} K_ij^2
__global__ void __launch_bounds__(128) k_colnorm2(const double* __restrict__ K, int64_t n_pad,
                                                  int64_t mp, int64_t chunk,
                                                  double* __restrict__ part) {
  const int64_t j = (int64_t)blockIdx.x * 128 + threadIdx.x;
  const int64_t ch = blockIdx.y;
  const int64_t i0 = ch * chunk;
  const int64_t i1 = (i0 + chunk < n_pad) ? i0 + chunk : n_pad;
  double acc = 0.0;
  for (int64_t i = i0; i < i1; ++i) {
    const double k = K[i * mp + j];
    acc = fma(k, k, acc);
  }
  part[ch * mp + j] = acc;
}

// Bordered-system scalars of one candidate knot t (VI):
//   s_K = kxx - k22c^T K22^-1 k22c,  s_B = kxx + c/z - b^T Bm^-1 b  (b = k22c + P/z),
//   dq = k_c^T r - z b^T u,  trinc = w^T S w - 2 w^T p + c  (w = K22^-1 k22c, p = K^T k_c)
// out[t] = {s_K, s_B, dq, trinc}; base = {kxx, z}.  One block per candidate.
__global__ void __launch_bounds__(256) k_vi_cand_scalars(int64_t m, int64_t Tp,
                                                         const double* __restrict__ K22c,
                                                         const double* __restrict__ W,
                                                         const double* __restrict__ SW,
                                                         const double* __restrict__ P,
                                                         const double* __restrict__ Bt,
                                                         const double* __restrict__ BB,
                                                         const double* __restrict__ u,
                                                         const double* __restrict__ rk,
                                                         const double* __restrict__ cc,
                                                         const double* __restrict__ base,
                                                         double* __restrict__ out) {
  const int64_t t = blockIdx.x;
  double a[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  for (int64_t j = threadIdx.x; j < m; j += 256) {
    const int64_t o = j * Tp + t;
    const double w = W[o], b = Bt[o];
    a[0] = fma(K22c[o], w, a[0]);
    a[1] = fma(w, SW[o], a[1]);
    a[2] = fma(w, P[o], a[2]);
    a[3] = fma(b, BB[o], a[3]);
    a[4] = fma(b, u[j], a[4]);
  }
  __shared__ double sh[4][5];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const double v = wave_sum(a[k]);
    if (lane == 0) sh[wv][k] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double r[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) r[k] = sh[0][k] + sh[1][k] + sh[2][k] + sh[3][k];
    const double kxx = base[0], z = base[1], c = cc[t];
    out[t * 4 + 0] = kxx - r[0];
    out[t * 4 + 1] = (kxx + c / z) - r[3];
    out[t * 4 + 2] = rk[t] - z * r[4];
    out[t * 4 + 3] = r[1] - 2.0 * r[2] + c;
  }
}

constexpr int LAP_NB = 1024;   // blocks of the per-row kernels (slab rows)

int row_blocks(int64_t n_pad) {
  int64_t nb = (n_pad + 255) / 256;
  return (int)(nb > LAP_NB ? LAP_NB : (nb < 1 ? 1 : nb));
}

}  // namespace

int64_t lap_gemv_cols_chunks(int64_t n_pad, int64_t mp) {
  int64_t target = 4096 / (mp / 128);
  if (target < 1) target = 1;
  int64_t maxch = (n_pad + 15) / 16;
  return target < maxch ? target : maxch;
}

int64_t lap_gemv_cols_slab(int64_t n_pad, int64_t mp, int nv) {
  return lap_gemv_cols_chunks(n_pad, mp) * nv * mp;
}

hipError_t launch_gemv_rows(const double* K, int64_t n_pad, int64_t mp, const double* x1,
                            const double* x2, double* y1, double* y2, hipStream_t s) {
  int64_t nb = (n_pad + 3) / 4;
  if (nb > 4096) nb = 4096;
  hipLaunchKernelGGL(k_gemv_rows, dim3((unsigned)nb), dim3(256), 0, s, K, n_pad, mp, x1, x2, y1,
                     y2);
  return hipGetLastError();
}

hipError_t launch_gemv_cols(const double* K, int64_t n_pad, int64_t mp, const double* V,
                            int64_t ldv, int nv, double* part, int64_t part_cap, double* out,
                            hipStream_t s) {
  const int64_t nch = lap_gemv_cols_chunks(n_pad, mp);
  if (nch * nv * mp > part_cap || nv < 1 || nv > 4) return hipErrorInvalidValue;
  const int64_t chunk = (n_pad + nch - 1) / nch;
  dim3 grid((unsigned)(mp / 128), (unsigned)nch);
  switch (nv) {
    case 1: hipLaunchKernelGGL(k_gemv_cols<1>, grid, dim3(128), 0, s, K, n_pad, mp, V, ldv, chunk, part); break;
    case 2: hipLaunchKernelGGL(k_gemv_cols<2>, grid, dim3(128), 0, s, K, n_pad, mp, V, ldv, chunk, part); break;
    case 3: hipLaunchKernelGGL(k_gemv_cols<3>, grid, dim3(128), 0, s, K, n_pad, mp, V, ldv, chunk, part); break;
    default: hipLaunchKernelGGL(k_gemv_cols<4>, grid, dim3(128), 0, s, K, n_pad, mp, V, ldv, chunk, part); break;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_colsum(part, nch, nv * mp, out, s);
}

hipError_t launch_lap_z(const double* q, int64_t n, int64_t n_pad, double c0, double* Z,
                        double* zinv, hipStream_t s) {
  hipLaunchKernelGGL(k_lap_z, dim3(row_blocks(n_pad)), dim3(256), 0, s, q, n, n_pad, c0, Z, zinv);
  return hipGetLastError();
}

hipError_t launch_lap_obj(int64_t n, int64_t n_pad, const double* f, const double* y,
                          const double* mu, const double* Z, const double* zinv, double expo,
                          const double* av, double* B, double* rf, double* tv, double* slab,
                          int* nblocks, hipStream_t s) {
  const int nb = row_blocks(n_pad);
  *nblocks = nb;
  hipLaunchKernelGGL(k_lap_obj, dim3(nb), dim3(256), 0, s, n, n_pad, f, y, mu, Z, zinv, expo,
                     av ? 0.0 : log(expo), av, B, rf, tv, slab);
  return hipGetLastError();
}

hipError_t launch_lap_nr_a(int64_t n, int64_t n_pad, const double* f, const double* y,
                           const double* mu, const double* Z, const double* zinv, double expo,
                           const double* av, const double* y1, double tol, double* g,
                           double* omzw, double* v, double* gpsi, double* slab, int* nblocks,
                           hipStream_t s) {
  const int nb = row_blocks(n_pad);
  *nblocks = nb;
  hipLaunchKernelGGL(k_lap_nr_a, dim3(nb), dim3(256), 0, s, n, n_pad, f, y, mu, Z, zinv, expo, av,
                     y1, tol, g, omzw, v, gpsi, slab);
  return hipGetLastError();
}

int64_t lap_rowpass_chunks(int64_t n_pad, int64_t mp) {
  // 65536 / mp rows per workgroup (128 at mp = 512), at most LAP_NB x 4 workgroups
  const int64_t rows = 65536 / mp;
  int64_t nch = (n_pad + rows - 1) / rows;
  if (nch > 4 * LAP_NB) nch = 4 * LAP_NB;
  return nch < 1 ? 1 : nch;
}

int64_t lap_rowpass_slab(int64_t n_pad, int64_t mp) {
  const int64_t nch = lap_rowpass_chunks(n_pad, mp);
  return nch * mp + nch;
}

namespace {
template <int MODE>
hipError_t launch_rowpass(const double* K, int64_t n, int64_t n_pad, int64_t mp, LapPassArgs pa,
                          double* part, int64_t part_cap, double* out_t, double* out_sc,
                          hipStream_t s) {
  constexpr int NS = 1;
  if (mp < 128 || mp > 2048 || mp % 128 != 0) return hipErrorInvalidValue;
  const int64_t nch = lap_rowpass_chunks(n_pad, mp);
  if (nch * mp + NS * nch > part_cap) return hipErrorInvalidValue;
  const int64_t chunk = (n_pad + nch - 1) / nch;
  pa.part = part;
  pa.sc = part + nch * mp;
  {
    const size_t shm = sizeof(double) * 4 * (size_t)mp;
    const dim3 g((unsigned)nch), b(256);
    const int nq = (int)(mp / 128);
    // rows in flight per wave and waves per SIMD (SGP_LAP_RS_CFG: probe configurations)
    constexpr int C = SGP_LAP_RS_CFG;
    constexpr int F2 = C == 1 ? 4 : C == 2 ? 16 : 8, O2 = C == 1 ? 4 : C == 2 ? 2 : 3;
    constexpr int F4 = C == 1 ? 2 : C == 2 ? 8 : 4, O4 = O2;
    if (nq <= 2) hipLaunchKernelGGL((k_lap_rowstream<MODE, 2, F2, O2>), g, b, shm, s, K, n, n_pad, mp, chunk, pa);
    else if (nq <= 4) hipLaunchKernelGGL((k_lap_rowstream<MODE, 4, F4, O4>), g, b, shm, s, K, n, n_pad, mp, chunk, pa);
    else if (nq <= 8) hipLaunchKernelGGL((k_lap_rowstream<MODE, 8, 2, 2>), g, b, shm, s, K, n, n_pad, mp, chunk, pa);
    else hipLaunchKernelGGL((k_lap_rowstream<MODE, 16, 1, 2>), g, b, shm, s, K, n, n_pad, mp, chunk, pa);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = launch_colsum(part, nch, mp, out_t, s);
  if (e != hipSuccess) return e;
  return launch_colsum(pa.sc, nch, NS, out_sc, s);
}
}  // namespace

hipError_t launch_lap_nr_a_fused(const double* K, int64_t n, int64_t n_pad, int64_t mp,
                                 const double* x1, const double* f, const double* y,
                                 const double* mu, const double* Z, const double* zinv,
                                 double expo, const double* av, double tol, double* y1, double* g,
                                 double* omzw, double* v, double* gpsi, double* part,
                                 int64_t part_cap, double* out, double* out_cnt, hipStream_t s) {
  LapPassArgs pa{};
  pa.x = x1; pa.f = f; pa.y = y; pa.mu = mu; pa.Z = Z; pa.zinv = zinv;
  pa.expo = expo; pa.av = av; pa.tol = tol;
  pa.y1 = y1; pa.g = g; pa.omzw = omzw; pa.v = v; pa.gpsi = gpsi;
  return launch_rowpass<LAP_PASS_A>(K, n, n_pad, mp, pa, part, part_cap, out, out_cnt, s);
}

hipError_t launch_lap_nr_b_t_fused(const double* K, int64_t n, int64_t n_pad, int64_t mp,
                                   const double* x2, double* f, const double* y,
                                   const double* mu, const double* Z, const double* zinv,
                                   const double* g, const double* omzw, const double* y1,
                                   double* part, int64_t part_cap, double* out_t, double* out_rr,
                                   hipStream_t s) {
  LapPassArgs pa{};
  pa.x = x2; pa.f = f; pa.f_out = f; pa.y = y; pa.mu = mu; pa.Z = Z; pa.zinv = zinv;
  pa.g_in = g; pa.omzw_in = omzw; pa.y1_in = y1;
  double* out_sc = out_rr;
  return launch_rowpass<LAP_PASS_B>(K, n, n_pad, mp, pa, part, part_cap, out_t, out_sc, s);
}

hipError_t launch_lap_nr_b(int64_t n, int64_t n_pad, double* f, const double* mu, const double* Z,
                           const double* g, const double* omzw, const double* y1,
                           const double* y2, hipStream_t s) {
  hipLaunchKernelGGL(k_lap_nr_b, dim3(row_blocks(n_pad)), dim3(256), 0, s, n, n_pad, f, mu, Z, g,
                     omzw, y1, y2);
  return hipGetLastError();
}

hipError_t launch_lap_grad_a(int64_t n, int64_t n_pad, const double* f, const double* y,
                             const double* mu, const double* Z, const double* zinv, double expo,
                             const double* av, const double* y1, const double* p, double* c2,
                             double* g, double* B, double* dMt, double* sv, double* bsv,
                             hipStream_t s) {
  hipLaunchKernelGGL(k_lap_grad_a, dim3(row_blocks(n_pad)), dim3(256), 0, s, n, n_pad, f, y, mu,
                     Z, zinv, expo, av, y1, p, c2, g, B, dMt, sv, bsv);
  return hipGetLastError();
}

hipError_t launch_lap_grad_b(int64_t n, int64_t n_pad, const double* B, const double* sv,
                             const double* y3, const double* dMt, const double* c2,
                             const double* g, double* h, double* a, double* slab, int* nblocks,
                             hipStream_t s) {
  const int nb = row_blocks(n_pad);
  *nblocks = nb;
  hipLaunchKernelGGL(k_lap_grad_b, dim3(nb), dim3(256), 0, s, n, n_pad, B, sv, y3, dMt, c2, g, h,
                     a, slab);
  return hipGetLastError();
}

hipError_t launch_colnorm2(const double* K, int64_t n_pad, int64_t mp, double* part,
                           int64_t part_cap, double* out, hipStream_t s) {
  const int64_t nch = lap_gemv_cols_chunks(n_pad, mp);
  if (nch * mp > part_cap) return hipErrorInvalidValue;
  const int64_t chunk = (n_pad + nch - 1) / nch;
  hipLaunchKernelGGL(k_colnorm2, dim3((unsigned)(mp / 128), (unsigned)nch), dim3(128), 0, s, K,
                     n_pad, mp, chunk, part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_colsum(part, nch, mp, out, s);
}

hipError_t launch_vi_cand_scalars(int64_t m, int64_t mp, int64_t T, int64_t Tp,
                                  const double* K22c, const double* W, const double* SW,
                                  const double* P, const double* Bt, const double* BB,
                                  const double* u, const double* rk, const double* cc,
                                  const double* base, double* out, hipStream_t s) {
  (void)mp;
  hipLaunchKernelGGL(k_vi_cand_scalars, dim3((unsigned)T), dim3(256), 0, s, m, Tp, K22c, W, SW, P,
                     Bt, BB, u, rk, cc, base, out);
  return hipGetLastError();
}
