// Row-sharded multi-device contexts (multi.hip), behind the one-device entry points of capi.hip.
//
// A context made by sgp_ctx_create_multi is an sgp_ctx whose `multi` member points at a MultiCtx:
// N ordinary one-device contexts (the shards, contiguous row blocks as dist.shard_rows), one host
// worker thread per distinct device, and an RCCL communicator over those devices.  capi.hip's
// public functions forward to the multi_* functions below when c->multi is set.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sgp.h"

#define SGP_MAX_SHARDS 64

struct MultiCtx;

// capi.hip hooks used by multi.hip
void sgp_internal_set_err(const char* msg);
void sgp_internal_forget_eval(sgp_ctx* c);   // no posterior / grad psi after candidate scoring
hipStream_t sgp_internal_stream(sgp_ctx* c);  // the context's launch stream
int sgp_internal_share_streams(sgp_ctx* c, sgp_ctx* src);   // c uses src's three streams

int multi_create(MultiCtx** out, const int* devices, int nshards, const double* X, int64_t n,
                 int64_t ldx, int d, const double* y, const double* mu, int64_t m_max);
void multi_destroy(MultiCtx* mc);
int multi_shards(const MultiCtx* mc, int* nshards, int* ndevices);
sgp_ctx* multi_lead(MultiCtx* mc);   // shard 0: holds the replicated state of an evaluation
int multi_set_data(MultiCtx* mc, const double* y, const double* mu);
int multi_eval_vi(MultiCtx* mc, int kernel, const double* theta, const double* U, int64_t m,
                  int64_t ldu, double delta, unsigned flags, double* obj, double* grad);
int multi_eval_fitc(MultiCtx* mc, int kernel, const double* theta, const double* U, int64_t m,
                    int64_t ldu, double delta, unsigned flags, double* obj, double* grad);
// flags SGP_FLAG_OBJ_ONLY: newtrap_sparseGP alone (sgp_lap_nr)
int multi_eval_laplace(MultiCtx* mc, int kernel, const double* theta, const double* U,
                       int64_t m, int64_t ldu, double delta, double expo, double tol, int maxit,
                       unsigned flags, double* obj, double* grad, int* nr_iters);
int multi_lap_set_f(MultiCtx* mc, const double* f, double fill);
int multi_lap_set_expo(MultiCtx* mc, const double* a, double fill);
int multi_lap_get_f(MultiCtx* mc, double* f);
int multi_lap_get_grad_psi(MultiCtx* mc, double* out);
int multi_enable_knot_grad(MultiCtx* mc, int enable);
int multi_knot_gradient(MultiCtx* mc, const double* bounds, double* grad_knot);
int multi_row_bounds(MultiCtx* mc, double* lo, double* hi);
int multi_vi_candidates(MultiCtx* mc, int kernel, const double* theta, const double* U,
                        int64_t m, int64_t ldu, double delta, unsigned flags, const double* cand,
                        int64_t T, int64_t ldc, double* obj_out);
int multi_fitc_candidates(MultiCtx* mc, int kernel, const double* theta, const double* U,
                          int64_t m, int64_t ldu, double delta, unsigned flags,
                          const double* cand, int64_t T, int64_t ldc, double* obj_out);
int multi_lap_candidates(MultiCtx* mc, int kernel, const double* theta, const double* U,
                         int64_t m, int64_t ldu, double delta, double expo, double tol,
                         int maxit, const double* cand, int64_t T, int64_t ldc,
                         double* obj_out);
