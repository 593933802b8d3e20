// sgp_probe.h -- timing-probe hooks of the product kernels, compiled to nothing in the product.
//
// The micro-benchmarks under tools/micro/ include a product kernel source after defining one
// of the probe macros below (and SGP_PROBE_BUILD); libsgp.so defines none of them, so every
// hook is an empty statement there.  A probe that changes results (SGP_CON_NO_EPILOGUE drops
// the gradient epilogue) refuses to build without SGP_PROBE_BUILD.
//
//   SGP_CON_TRACE(k)       s_memtime stamp k of a k_contract workgroup   (tools/micro/con_trace.hip)
//   SGP_CON_NO_EPILOGUE    k_contract<.., EPI_GRAD> returns after the k-loop (timing only)
//   SGP_CON_PROBE_NO_EPI_MFMA  the epilogue's D products on the VALU, wrong (timing only)
//   SGP_CON_PROBE_NO_KDMA  the epilogue's K stages not loaded (timing only)
//   SGP_GJ_TRACE(k, p)     stamp p of the GJ look-ahead workgroup at pivot k (tools/micro/gj_trace.hip)
//
// Experiment knobs (schedule / staging alternatives measured in A/B runs).  The product values
// are fixed here; overriding one needs SGP_PROBE_BUILD, i.e. a variant library built by
// sparsergps_amd._build.build_variant() into tools/ab/ (the product build takes no -D flags):
//   SGP_IL_VMEM0        first MFMA slot of the k-step's global loads (mfma_interleave)
//   SGP_CON_IL_PAT      LDS-store placement of the contraction's k-step (mfma_interleave PAT)
//   SGP_SYRK_IL_PAT     the same for the SYRKs
//   SGP_CON_IL_SPREAD   contraction: LDS fragment reads spread over the step instead of up front
//   SGP_CON_SHMEM       dynamic LDS pad of the gradient-contraction launches
//   SGP_SYRK_BAL        0: no balanced S-only SYRK plan (syrk_plan_bal)
//   SGP_SDT_IL          0: the diagonal-tile SYRK step without the interleave request
//   SGP_SDT_W           syrk_plan_bal's cost of a diagonal-tile wave-step, in MFMAs (36 issued)
//   SGP_SDT_WW          ... plus this with per-fragment weights
//   SGP_SDT_WT          ... plus this with the t slice
//   SGP_SYRK_W3         0: signed-weight / t SYRKs keep per-fragment weights on the packed plan
//   SGP_CON_ROWQ_KU     1: the row-quadratic pass without u keeps the (unused) K u fold
//   SGP_LAP_RS_CFG      k_lap_rowstream at mp <= 512: 0 (16 / NQM rows per wave, 3 waves per
//                       SIMD), 1 (half the rows, 4 waves), 2 (twice the rows, 2 waves)
//   SGP_GJ_MM_UNROLL    unroll of gj_mm64's 16 k-substeps (16; 4 before round 4)
//   SGP_S256_IL         1: k_syrk_s256's step with an interleave request
//   SGP_VI_BUILD_NO_T   1: VI's builder without t (wrong results: builder timing only)
//   SGP_GJ_STEPS        1: the m x m inverses as one launch per pivot step (before round 5)
//   SGP_GJ_GMAX         workgroups of a persistent Gauss-Jordan chain (at most)
//   SGP_CON_EPI_PRIO    contraction: wave priority (s_setprio) of the epilogue (0: none)
//   SGP_BUILD_OCC_T2    workgroups per CU of the with-t K12 builder at d <= 8 (launch bound)
//   SGP_CHAIN_US_STEP   chain_shared_rb's model of a K22 chain beside the builder: us per
//   SGP_CHAIN_US_FIX    64-wide step, and fixed us
// Fault injection (environment, read by probe builds only; the product ignores it):
//   SGP_PROBE_GJ_WITHHOLD=<ticket>  the process's first persistent Gauss-Jordan launch skips the
//                       flag publish of that task ticket, so the chain's watchdog must fire
//                       (tests/test_gpu_gj.py)
#pragma once

#if (defined(SGP_CON_TRACE) || defined(SGP_CON_NO_EPILOGUE) || defined(SGP_GJ_TRACE) ||       \
     defined(SGP_IL_VMEM0) || defined(SGP_CON_IL_PAT) || defined(SGP_SYRK_IL_PAT) ||          \
     defined(SGP_CON_IL_SPREAD) || defined(SGP_CON_SHMEM) ||                                  \
     defined(SGP_SYRK_BAL) || defined(SGP_SDT_IL) || defined(SGP_S256_IL) ||                  \
     defined(SGP_SDT_W) || defined(SGP_SDT_WW) || defined(SGP_SDT_WT) ||                      \
     defined(SGP_SYRK_W3) || defined(SGP_CON_ROWQ_KU) ||                                      \
     defined(SGP_LAP_RS_CFG) || defined(SGP_GJ_MM_UNROLL) || defined(SGP_VI_BUILD_NO_T) ||        \
     defined(SGP_GJ_STEPS) || defined(SGP_GJ_GMAX) || defined(SGP_CHAIN_US_STEP) ||         \
     defined(SGP_CHAIN_US_FIX) || defined(SGP_HOST_PROBE) || defined(SGP_BUILD_OCC_T2) ||      \
     defined(SGP_CON_EPI_PRIO) || defined(SGP_CON_PROBE_NO_EPI_MFMA) ||                       \
     defined(SGP_CON_PROBE_NO_KDMA)) &&      \
    !defined(SGP_PROBE_BUILD)
#error "timing probes and experiment knobs are for variant builds only (SGP_PROBE_BUILD)"
#endif

#ifndef SGP_CON_EPI_PRIO
#define SGP_CON_EPI_PRIO 0
#endif
#ifndef SGP_BUILD_OCC_T2
#define SGP_BUILD_OCC_T2 4
#endif
#ifndef SGP_IL_VMEM0
#define SGP_IL_VMEM0 0
#endif
#ifndef SGP_CON_IL_PAT
#define SGP_CON_IL_PAT 2   // contraction: stores in the last MFMA slots (65.5 vs 64.5 TF/s)
#endif
#ifndef SGP_SYRK_IL_PAT
#define SGP_SYRK_IL_PAT 0
#endif
#ifndef SGP_CON_IL_SPREAD
#define SGP_CON_IL_SPREAD false   // reads up front: 66.5-66.9 vs 65.3 TF/s spread
#endif
#ifndef SGP_CON_SHMEM
#define SGP_CON_SHMEM 0
#endif
#ifndef SGP_SYRK_BAL
#define SGP_SYRK_BAL 1
#endif
#ifndef SGP_SDT_IL
#define SGP_SDT_IL 1
#endif
#ifndef SGP_SDT_W
#define SGP_SDT_W 38
#endif
#ifndef SGP_SDT_WW
#define SGP_SDT_WW 2
#endif
#ifndef SGP_SDT_WT
#define SGP_SDT_WT 6
#endif
#ifndef SGP_SYRK_W3
#define SGP_SYRK_W3 1
#endif
#ifndef SGP_CON_ROWQ_KU
#define SGP_CON_ROWQ_KU 0
#endif
#ifndef SGP_LAP_RS_CFG
#define SGP_LAP_RS_CFG 0
#endif
#ifndef SGP_GJ_MM_UNROLL
#define SGP_GJ_MM_UNROLL 16
#endif
#ifndef SGP_S256_IL
#define SGP_S256_IL 0
#endif
#ifndef SGP_GJ_STEPS
#define SGP_GJ_STEPS 0
#endif
#ifndef SGP_GJ_GMAX
#define SGP_GJ_GMAX 128
#endif
#ifndef SGP_CHAIN_US_STEP
#define SGP_CHAIN_US_STEP 60.0
#endif
#ifndef SGP_CHAIN_US_FIX
#define SGP_CHAIN_US_FIX 250.0
#endif
#ifndef SGP_VI_BUILD_NO_T
#define SGP_VI_BUILD_NO_T 0
#endif

// k_contract: stamp k from thread 0 of the workgroup
#ifdef SGP_CON_TRACE
#define SGP_PROBE_CON_STAMP(k_)        \
  do {                                 \
    if (tid == 0) SGP_CON_TRACE(k_);   \
  } while (0)
#else
#define SGP_PROBE_CON_STAMP(k_) \
  do {                          \
  } while (0)
#endif

// k_contract<.., EPI_GRAD>: leave after the k-loop, keeping the accumulators live
#ifdef SGP_CON_NO_EPILOGUE
#define SGP_PROBE_CON_SKIP_EPILOGUE()                                                   \
  if constexpr (EPI == EPI_GRAD) {                                                      \
    double v_ = 0.0;                                                                    \
    _Pragma("unroll") for (int fm_ = 0; fm_ < 4; ++fm_)                                 \
      _Pragma("unroll") for (int fn_ = 0; fn_ < 4; ++fn_)                               \
        v_ += acc[fm_][fn_][0] + acc[fm_][fn_][3];                                      \
    if (v_ == 1234.5) slab[tid] = v_;                                                   \
    return;                                                                             \
  }
#else
#define SGP_PROBE_CON_SKIP_EPILOGUE()
#endif

// k_gj_step: stamps of the workgroup that solves the next pivot
#ifdef SGP_GJ_TRACE
#define SGP_PROBE_GJ_DECL() const bool gj_tr_ = (i == k + 1) && (j == k + 1) && threadIdx.x == 0
#define SGP_PROBE_GJ_STAMP(p_)          \
  do {                                  \
    if (gj_tr_) SGP_GJ_TRACE(k, p_);    \
  } while (0)
#else
#define SGP_PROBE_GJ_DECL() \
  do {                      \
  } while (0)
#define SGP_PROBE_GJ_STAMP(p_) \
  do {                         \
  } while (0)
#endif
