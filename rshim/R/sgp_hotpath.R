## sgp_hotpath.R -- R-level drop-ins for sparseRGPs' per-iteration hot path on libsgp.so.
##
## Each function keeps the reference's name, formals and return list; the work runs in one
## fused HIP evaluation over a device-resident context (rshim/sparseRGPs_sgp.c, Part 2):
##   elbo_fun        R/vi_functions.R:64-121            sgp_eval_vi     (objective)
##   delbo_dcov_par  R/vi_functions.R:126-602           sgp_eval_vi     (+ knot gradient)
##   obj_fun_norm    R/laplace_approx_obj_funs.R:6-52   sgp_eval_fitc   (objective)
##   dlogp_dcov_par  R/laplace_approx_gradient.R:720-1135  sgp_eval_fitc (+ knot gradient)
##   newtrap_sparseGP R/newtrap_sparseGP.R:6-186        sgp_lap_nr      (Poisson likelihood)
##   dlogq_dcov_par  R/laplace_approx_gradient.R:25-553 sgp_eval_laplace (maxit = 0: at ff)
##
## elbo_fun / obj_fun_norm receive the already-built Sigma12 / Sigma22 in the reference; the
## fused path needs the inputs instead, so they take it only when the caller also passes
## xy = , xu = , cov_fun = through `...` (the two-line driver patch in INTEGRATION.md sec. 3)
## and otherwise run the package's own R function (saved by sgp_install()).  Inside a patched
## driver the objective call evaluates objective AND gradient once and the gradient call that
## follows at the same (cov_par, xu) reuses it: one GPU evaluation per optimizer iteration.
##
## R's det() overflow (quirk Q4): log(det(Sigma22)) is +-Inf in the reference when |Sigma22|
## leaves double range; sgp_options(r_det = TRUE) (the default) passes SGP_FLAG_R_DET so the
## objective is identical, FALSE uses the factorisation's finite log-determinant.

.sgp <- new.env(parent = emptyenv())
.sgp$opts <- list(r_det = TRUE)
.sgp$orig <- list()

SGP_FLAG_R_DET <- 1L
SGP_FLAG_OBJ_ONLY <- 2L

sgp_options <- function(...) {
  new <- list(...)
  .sgp$opts[names(new)] <- new
  invisible(.sgp$opts)
}

## replace the six hot functions inside the package namespace, keeping the originals for
## callers that pass matrices only (knot proposals, user code)
sgp_install <- function(ns = asNamespace("sparseRGPs")) {
  fns <- c("elbo_fun", "delbo_dcov_par", "obj_fun_norm", "dlogp_dcov_par",
           "newtrap_sparseGP", "dlogq_dcov_par")
  for (f in fns) {
    if (is.null(.sgp$orig[[f]])) .sgp$orig[[f]] <- get(f, envir = ns)
    utils::assignInNamespace(f, get(paste0("sgp_", f)), ns = ns)
  }
  invisible(fns)
}

## ---------------------------------------------------------------- context + theta layout

## one device context per data set (X, y, mu uploaded once); reused while xy, y, mu are
## identical() and m fits, recreated otherwise
.sgp_ctx <- function(xy, y, mu, m) {
  xy <- as.matrix(xy)
  y <- as.numeric(y)
  mu <- rep_len(as.numeric(mu), nrow(xy))
  e <- .sgp$ctx
  if (!is.null(e) && e$m_max >= m && identical(e$xy, xy) && identical(e$y, y) &&
      identical(e$mu, mu))
    return(e$ptr)
  m_max <- max(m, if (is.null(e)) 0L else e$m_max)
  if (!is.null(e)) .Call("sgp_R_ctx_destroy", e$ptr)
  .sgp$ctx <- NULL
  .sgp$last <- NULL
  ptr <- .Call("sgp_R_ctx_create", xy, y, mu, as.integer(m_max))
  .sgp$ctx <- list(ptr = ptr, xy = xy, y = y, mu = mu, m_max = m_max, knots = FALSE)
  ptr
}

.sgp_knots <- function(ptr, enable) {
  if (!identical(.sgp$ctx$knots, enable)) {
    .Call("sgp_R_enable_knot_grad", ptr, enable)
    .sgp$ctx$knots <- enable
  }
}

## [sigma, l | l1..ld, tau] (include/sgp.h) and the names of that layout
.sgp_theta <- function(cov_par, cov_fun, d) {
  ls <- if (cov_fun == "ard") paste("l", 1:d, sep = "") else "l"
  nm <- c("sigma", ls, "tau")
  stats::setNames(vapply(nm, function(k) as.numeric(cov_par[[k]]), 0.0), nm)
}

.sgp_flags <- function(obj_only = FALSE) {
  bitwOr(if (isTRUE(.sgp$opts$r_det)) SGP_FLAG_R_DET else 0L,
         if (obj_only) SGP_FLAG_OBJ_ONLY else 0L)
}

## knot_bounds of vi_functions.R:175-178: column range of xy widened by a tenth
.sgp_knot_bounds <- function(xy) {
  lo <- apply(X = xy, MARGIN = 2, FUN = min)
  hi <- apply(X = xy, MARGIN = 2, FUN = max)
  diffs <- hi - lo
  cbind(lo - diffs / 10, hi + diffs / 10)
}

## one fused evaluation (method 0 VI, 1 FITC) with its gradient; cached by its arguments
.sgp_eval <- function(method, cov_par, cov_fun, xu, xy, y, mu, delta, knots) {
  xu <- as.matrix(xu)
  xy <- as.matrix(xy)
  theta <- .sgp_theta(cov_par, cov_fun, ncol(xy))
  key <- list(method, theta, xu, delta, knots, .sgp$opts$r_det)
  last <- .sgp$last
  ptr <- .sgp_ctx(xy, y, mu, nrow(xu))
  if (!is.null(last) && identical(last$key, key)) return(last)
  .sgp_knots(ptr, knots)
  ev <- .Call("sgp_R_eval", ptr, as.integer(method), cov_fun, unname(theta), xu,
              as.numeric(delta), .sgp_flags())
  names(ev$gradient) <- names(theta)
  if (knots)
    ev$knot_gradient <- .Call("sgp_R_knot_gradient", ptr, .sgp_knot_bounds(xy),
                              nrow(xu), ncol(xu))
  ev$key <- key
  .sgp$last <- ev
  ev
}

## the return list of delbo_dcov_par (vi_functions.R:594-601) / dlogp_dcov_par
.sgp_grad_list <- function(ev, cov_par, dcov_fun_dtheta, knots, knot_opt, xu, xy) {
  grad <- if (is.list(dcov_fun_dtheta)) ev$gradient[names(cov_par)] else 0
  trans_par <- lapply(cov_par, log)
  if (!knots) return(list("gradient" = grad, "trans_par" = trans_par))
  xu <- as.matrix(xu)
  b <- .sgp_knot_bounds(as.matrix(xy))
  ## knots not in knot_opt get zero gradient (vi_functions.R:502-506; knot_opt = NA zeroes all)
  keep <- seq_len(nrow(xu)) %in% knot_opt
  gk <- ev$knot_gradient * rep(keep, each = ncol(xu))
  trans_knot <- log(t(t(xu) - b[, 1]) + 1e-4) - log(t(b[, 2] - t(xu)) + 1e-4)
  list("gradient" = grad, "knot_gradient" = gk, "trans_par" = trans_par,
       "trans_knot" = trans_knot)
}

.sgp_fused_args <- function(args) all(c("xy", "xu", "cov_fun") %in% names(args))

## ---------------------------------------------------------------- Gaussian paths

sgp_elbo_fun <- function(ff = NA, mu, Z, Sigma12, Sigma22, y,
                         trace_term_fun = trace_term_fun, cov_par, ...)
{
  args <- list(...)
  if (!.sgp_fused_args(args))
    return(.sgp$orig$elbo_fun(ff = ff, mu = mu, Z = Z, Sigma12 = Sigma12, Sigma22 = Sigma22,
                              y = y, trace_term_fun = trace_term_fun, cov_par = cov_par, ...))
  delta <- if (is.null(args$delta)) 1e-6 else args$delta
  .sgp_eval(0L, cov_par, args$cov_fun, args$xu, args$xy, y, mu, delta,
            isTRUE(args$knots))$objective
}

sgp_delbo_dcov_par <- function(cov_par, cov_fun, dcov_fun_dtheta, dcov_fun_dknot = NA,
                               knot_opt, xu, xy, y, ff = NA, mu, transform = TRUE,
                               delta = 1e-6, ...)
{
  knots <- is.function(dcov_fun_dknot)
  ev <- .sgp_eval(0L, cov_par, cov_fun, xu, xy, y, mu, delta, knots)
  .sgp_grad_list(ev, cov_par, dcov_fun_dtheta, knots,
                 knot_opt, xu, xy)
}

sgp_obj_fun_norm <- function(ff = NA, mu, Z, Sigma12, Sigma22, y, ...)
{
  args <- list(...)
  if (!.sgp_fused_args(args))
    return(.sgp$orig$obj_fun_norm(ff = ff, mu = mu, Z = Z, Sigma12 = Sigma12,
                                  Sigma22 = Sigma22, y = y, ...))
  delta <- if (is.null(args$delta)) 1e-6 else args$delta
  .sgp_eval(1L, args$cov_par, args$cov_fun, args$xu, args$xy, y, mu, delta,
            isTRUE(args$knots))$objective
}

sgp_dlogp_dcov_par <- function(cov_par, cov_fun, dcov_fun_dtheta, dcov_fun_dknot = NA,
                               knot_opt, xu, xy, y, ff = NA, mu, transform = TRUE,
                               delta = 1e-6, ...)
{
  knots <- is.function(dcov_fun_dknot)
  ev <- .sgp_eval(1L, cov_par, cov_fun, xu, xy, y, mu, delta, knots)
  .sgp_grad_list(ev, cov_par, dcov_fun_dtheta, knots,
                 knot_opt, xu, xy)
}

## ---------------------------------------------------------------- Poisson sparse Laplace

## the fused path implements the Poisson likelihood with a scalar exposure m
.sgp_poisson <- function(d2log_py_dff, args) {
  pois <- tryCatch(get("d2log_py_dff_pois", envir = asNamespace("sparseRGPs")),
                   error = function(e) NULL)
  m <- if (is.null(args$m)) 1 else args$m
  !is.null(pois) && identical(body(d2log_py_dff), body(pois)) &&
    length(unique(as.numeric(m))) == 1
}

sgp_newtrap_sparseGP <- function(start_vals, obj_fun, grad_loglik_fn, dlog_py_dff,
                                 d2log_py_dff, maxit = 1000, tol = 1e-6, cov_par, cov_fun,
                                 xy, xu, y, mu, muu, delta = 1e-6, ...)
{
  args <- list(...)
  if (!.sgp_poisson(d2log_py_dff, args))
    return(.sgp$orig$newtrap_sparseGP(start_vals = start_vals, obj_fun = obj_fun,
                                      grad_loglik_fn = grad_loglik_fn,
                                      dlog_py_dff = dlog_py_dff, d2log_py_dff = d2log_py_dff,
                                      maxit = maxit, tol = tol, cov_par = cov_par,
                                      cov_fun = cov_fun, xy = xy, xu = xu, y = y, mu = mu,
                                      muu = muu, delta = delta, ...))
  xu <- as.matrix(xu)
  ptr <- .sgp_ctx(xy, y, mu, nrow(xu))
  .sgp$last <- NULL
  .Call("sgp_R_lap_set_f", ptr, as.numeric(start_vals))
  theta <- .sgp_theta(cov_par, cov_fun, ncol(xu))
  expo <- as.numeric(if (is.null(args$m)) 1 else args$m)[1]
  ## newtrap_sparseGP.R:79-96 performs the first update whatever maxit is
  .Call("sgp_R_eval_laplace", ptr, cov_fun, unname(theta), xu, as.numeric(delta), expo,
        as.numeric(tol), as.integer(max(maxit, 1)), FALSE)
  out <- list("gp" = .Call("sgp_R_lap_get_f", ptr),
              "objective_function_values" = .Call("sgp_R_lap_objective_values", ptr),
              ## grad_psi at the returned mode is not materialised by the fused NR loop
              "gradient" = NA_real_)
  if (!missing(muu)) {
    post <- .Call("sgp_R_posterior_u", ptr, rep_len(as.numeric(muu), nrow(xu)))
    out$u_posterior_mean <- post$u_mean
    out$u_posterior_variance <- post$u_var
  }
  out
}

sgp_dlogq_dcov_par <- function(cov_par, cov_fun, dcov_fun_dtheta, dcov_fun_dknot = NA,
                               knot_opt, xu, xy, y, ff, dlog_py_dff, d2log_py_dff,
                               d3log_py_dff, mu, transform = TRUE, delta = 1e-6, ...)
{
  args <- list(...)
  if (!.sgp_poisson(d2log_py_dff, args))
    return(.sgp$orig$dlogq_dcov_par(cov_par = cov_par, cov_fun = cov_fun,
                                    dcov_fun_dtheta = dcov_fun_dtheta,
                                    dcov_fun_dknot = dcov_fun_dknot, knot_opt = knot_opt,
                                    xu = xu, xy = xy, y = y, ff = ff,
                                    dlog_py_dff = dlog_py_dff, d2log_py_dff = d2log_py_dff,
                                    d3log_py_dff = d3log_py_dff, mu = mu,
                                    transform = transform, delta = delta, ...))
  xu <- as.matrix(xu)
  xy <- as.matrix(xy)
  knots <- is.function(dcov_fun_dknot)
  ptr <- .sgp_ctx(xy, y, mu, nrow(xu))
  .sgp$last <- NULL
  .sgp_knots(ptr, knots)
  .Call("sgp_R_lap_set_f", ptr, as.numeric(ff))
  theta <- .sgp_theta(cov_par, cov_fun, ncol(xu))
  expo <- as.numeric(if (is.null(args$m)) 1 else args$m)[1]
  ## maxit = 0: objective and gradient at the given ff, no NR step
  ev <- .Call("sgp_R_eval_laplace", ptr, cov_fun, unname(theta), xu, as.numeric(delta), expo,
              0, 0L, TRUE)
  names(ev$gradient) <- names(theta)
  if (knots)
    ev$knot_gradient <- .Call("sgp_R_knot_gradient", ptr, .sgp_knot_bounds(xy),
                              nrow(xu), ncol(xu))
  .sgp_grad_list(ev, cov_par, dcov_fun_dtheta, knots,
                 knot_opt, xu, xy)
}
