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
## and the callers above them, so optimize_gp() / predict_gp() run unchanged on the GPU:
##   norm_grad_ascent_vi R/vi_functions.R:606-1218            one sgp_eval_vi per iteration
##   norm_grad_ascent    R/laplace_gradient_ascent.R:1111-1693 one sgp_eval_fitc per iteration
##   laplace_grad_ascent R/laplace_gradient_ascent.R:10-623    one sgp_eval_laplace per iteration
##   predict_gp          R/laplace_approx_prediction.R:408-542 sgp_predict
##
## The drivers keep the reference's formals, opt() defaults, adadelta / ga updates (sign-change
## damping, the bounded knot transform), stop rule, histories and return lists; each iteration
## body -- the two K builds, the objective and the gradient function (quirk Q17) -- is one
## fused evaluation on a device-resident context.  They run the package's original driver
## whenever the fused path does not apply: a user-supplied objective, non-package derivative
## closures, a knot derivative that does not match cov_fun, the "exp" kernel, a non-Poisson
## likelihood or an exposure that is not positive and finite.
##
## elbo_fun / obj_fun_norm receive the already-built Sigma12 / Sigma22 in the reference; called
## directly they take the fused path only when the caller also passes xy = , xu = , cov_fun =
## through `...`, and otherwise run the package's own R function (saved by sgp_install()).
##
## R's det() overflow (quirk Q4): log(det(Sigma22)) is +-Inf in the reference when |Sigma22|
## leaves double range; sgp_options(r_det = TRUE) (the default) passes SGP_FLAG_R_DET so the
## objective is identical, FALSE uses the factorisation's finite log-determinant.

## Multi-GPU (north star C4): the rows of a fit are split into contiguous blocks over the GPUs of
## the node and every evaluation's row sums are combined inside libsgp by an RCCL all-reduce
## (sgp_ctx_create_multi).  Multi-GPU is opt-in: ngpus = NULL (the default) is one GPU;
## sgp_options(ngpus = k) uses devices 0..k-1; ngpus = "auto" uses every visible GPU once each
## shard keeps >= 125 000 rows (one GPU below that: the replicated m x m work would dominate);
## sgp_options(devices = c(...)) names the device of each shard explicitly (repeats allowed).
.sgp <- new.env(parent = emptyenv())
.sgp$opts <- list(r_det = TRUE, ngpus = NULL, devices = NULL)
.sgp$orig <- list()

SGP_FLAG_R_DET <- 1L
SGP_FLAG_OBJ_ONLY <- 2L

sgp_options <- function(...) {
  new <- list(...)
  .sgp$opts[names(new)] <- new
  invisible(.sgp$opts)
}

## replace the hot functions and their drivers inside the package namespace (optimize_gp()
## and predict_gp() resolve them there), keeping the originals for the fall-back paths
sgp_install <- function(ns = asNamespace("sparseRGPs")) {
  fns <- c("elbo_fun", "delbo_dcov_par", "obj_fun_norm", "dlogp_dcov_par",
           "newtrap_sparseGP", "dlogq_dcov_par", "norm_grad_ascent_vi", "norm_grad_ascent",
           "laplace_grad_ascent", "predict_gp")
  for (f in fns) {
    if (is.null(.sgp$orig[[f]])) .sgp$orig[[f]] <- get(f, envir = ns)
    utils::assignInNamespace(f, get(paste0("sgp_", f)), ns = ns)
  }
  invisible(fns)
}

## ---------------------------------------------------------------- context + theta layout

## the device of each row shard (integer(0): one device, SGP_DEVICE)
.sgp_devices <- function(n) {
  dv <- .sgp$opts$devices
  if (!is.null(dv)) return(as.integer(dv))
  ng <- .sgp$opts$ngpus
  if (is.null(ng)) return(integer(0))
  if (identical(ng, "auto")) {
    nd <- .Call("sgp_R_device_count")
    ng <- max(1L, min(nd, n %/% 125000L))
  }
  ng <- as.integer(ng)
  if (ng <= 1L) integer(0) else seq_len(ng) - 1L
}

## one device context per data set (X, y, mu uploaded once); reused while xy, y, mu are
## identical() and m fits, recreated otherwise
.sgp_ctx <- function(xy, y, mu, m) {
  xy <- as.matrix(xy)
  y <- as.numeric(y)
  mu <- rep_len(as.numeric(mu), nrow(xy))
  e <- .sgp$ctx
  devices <- .sgp_devices(nrow(xy))
  if (!is.null(e) && e$m_max >= m && identical(e$xy, xy) && identical(e$y, y) &&
      identical(e$mu, mu) && identical(e$devices, devices))
    return(e$ptr)
  m_max <- max(m, if (is.null(e)) 0L else e$m_max)
  if (!is.null(e)) .Call("sgp_R_ctx_destroy", e$ptr)
  .sgp$ctx <- NULL
  .sgp$last <- NULL
  ptr <- .Call("sgp_R_ctx_create", xy, y, mu, as.integer(m_max), devices)
  .sgp$ctx <- list(ptr = ptr, xy = xy, y = y, mu = mu, m_max = m_max, knots = FALSE,
                   devices = devices)
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

## the fused path implements the Poisson likelihood with the exposure m a scalar or one value
## per row (a vector of cell areas, derivative_functions_of_data_likelihoods.R:38), each
## positive and finite (anything else runs the reference's own R code)
.sgp_poisson <- function(d2log_py_dff, args) {
  pois <- tryCatch(get("d2log_py_dff_pois", envir = asNamespace("sparseRGPs")),
                   error = function(e) NULL)
  m <- as.numeric(if (is.null(args$m)) 1 else args$m)
  !is.null(pois) && identical(body(d2log_py_dff), body(pois)) && length(m) >= 1 &&
    all(is.finite(m) & m > 0)
}

## the exposure as the shim takes it: one value, or one per row (R's recycling of -m * exp(ff))
.sgp_expo <- function(args, n) {
  m <- as.numeric(if (is.null(args$m)) 1 else args$m)
  if (length(m) == 1L || length(unique(m)) == 1L) m[1] else rep_len(m, n)
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
  expo <- .sgp_expo(args, nrow(as.matrix(xy)))
  ## newtrap_sparseGP.R:79-96 performs the first update whatever maxit is
  .Call("sgp_R_eval_laplace", ptr, cov_fun, unname(theta), xu, as.numeric(delta), expo,
        as.numeric(tol), as.integer(max(maxit, 1)), FALSE)
  out <- list("gp" = .Call("sgp_R_lap_get_f", ptr),
              "objective_function_values" = .Call("sgp_R_lap_objective_values", ptr),
              ## grad_psi of the last NR step (newtrap_sparseGP.R:183-184)
              "gradient" = .Call("sgp_R_lap_get_grad_psi", ptr))
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
  expo <- .sgp_expo(args, nrow(as.matrix(xy)))
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

## ---------------------------------------------------------------- drivers (optimize_gp's L3)

## opt_master of vi_functions.R:663-684 / laplace_gradient_ascent.R:77-99, 1163-1183:
## defaults, overridden by name; unknown names are skipped
.sgp_opts <- function(opt, extra = list()) {
  opt_master <- c(list("optim_method" = "adadelta", "decay" = 0.95, "epsilon" = 1e-6,
                       "learn_rate" = 1e-2, "eta" = 1e3, "maxit" = 1000, "obj_tol" = 1e-3,
                       "grad_tol" = Inf, "delta" = 1e-6), extra)
  if (length(opt) > 0)
    for (i in 1:length(opt)) {
      if (!any(names(opt_master) == names(opt)[i])) next
      opt_master[[which(names(opt_master) == names(opt)[i])]] <- opt[[i]]
    }
  opt_master
}

## the package closure a function's body matches (NULL if none)
.sgp_pkg_fun <- function(f, candidates) {
  if (!is.function(f)) return(NULL)
  ns <- asNamespace("sparseRGPs")
  for (nm in candidates) {
    g <- tryCatch(get(nm, envir = ns), error = function(e) NULL)
    orig <- .sgp$orig[[nm]]
    if ((!is.null(g) && identical(body(f), body(g))) ||
        (!is.null(orig) && identical(body(f), body(orig))))
      return(nm)
  }
  NULL
}

## the caller's objective, or the package's default when the formal was missing
.sgp_obj_or_default <- function(obj_fun, of, name) {
  if (is.null(of)) get(name, envir = asNamespace("sparseRGPs")) else obj_fun
}

## can the fused evaluation stand in for this driver call?
.sgp_fusable <- function(cov_fun, cov_par_start, dcov_fun_dtheta, dcov_fun_dknot, obj_fun,
                         obj_names) {
  if (!cov_fun %in% c("sqexp", "ard")) return(FALSE)
  if (!all(c("sigma", "tau") %in% names(cov_par_start))) return(FALSE)
  if (!is.null(obj_fun) && is.null(.sgp_pkg_fun(obj_fun, obj_names))) return(FALSE)
  if (is.list(dcov_fun_dtheta)) {
    ok <- vapply(dcov_fun_dtheta, function(f) !is.null(.sgp_pkg_fun(
      f, c("dsqexp_dsigma", "dsqexp_dsigma_ard", "dsqexp_dl", "dsqexp_dtau"))), TRUE)
    if (!all(ok)) return(FALSE)
  }
  if (is.function(dcov_fun_dknot)) {
    k <- .sgp_pkg_fun(dcov_fun_dknot, c("dsqexp_dx2", "dsqexp_dx2_ard"))
    if (is.null(k) || k != (if (cov_fun == "ard") "dsqexp_dx2_ard" else "dsqexp_dx2"))
      return(FALSE)
  }
  TRUE
}

## The adadelta / ga loop shared by the three drivers (vi_functions.R:806-1159,
## laplace_gradient_ascent.R:226-582, 1305-1634).  evaluate(cov_par, xu) returns
## list(obj, grad) with grad the gradient function's list (gradient, trans_par[, knot_gradient,
## trans_knot]).  Variable names follow the reference so rbind() gives the same dimnames.
.sgp_ascent <- function(evaluate, cov_par_start, cov_fun, dcov_fun_dtheta, dcov_fun_dknot, xu,
                        xy, o, verbose, print_after = FALSE)
{
  optim_method <- o$optim_method
  optim_par <- list("decay" = o$decay, "epsilon" = o$epsilon, "eta" = o$eta,
                    "learn_rate" = o$learn_rate)
  maxit <- o$maxit
  obj_tol <- o$obj_tol
  grad_tol <- o$grad_tol
  lnames <- if (cov_fun == "ard") paste("l", 1:ncol(xy), sep = "") else character()

  current_cov_par <- unlist(cov_par_start)
  cov_par_vals <- matrix(ncol = length(current_cov_par))
  cov_par <- as.list(current_cov_par)
  obj_fun_vals <- numeric()
  grad_vals <- matrix(ncol = length(current_cov_par))
  current_grad_val_theta <- if (is.list(dcov_fun_dtheta)) NA else 0
  grad_knot_vals <- matrix(ncol = nrow(xu) * ncol(xu))
  current_grad_val_knot <- NA

  ev <- evaluate(cov_par, xu)
  current_obj_fun <- ev$obj
  obj_fun_vals[1] <- current_obj_fun
  cov_par_vals[1, ] <- current_cov_par
  temp_grad_eval <- ev$grad
  if (is.list(dcov_fun_dtheta)) {
    current_grad_val_theta <- c(temp_grad_eval$gradient)
    grad_vals[1, ] <- current_grad_val_theta
  }
  current_cov_par_trans <- unlist(temp_grad_eval$trans_par)
  if (is.function(dcov_fun_dknot)) {
    current_grad_val_knot <- c(temp_grad_eval$knot_gradient)
    grad_knot_vals[1, ] <- current_grad_val_knot
    xu_vals <- xu
    knot_bounds <- .sgp_knot_bounds(xy)
    current_xu_trans <- temp_grad_eval$trans_knot
  } else {
    current_grad_val_knot <- 0
  }

  ## real -> bounded knot coordinates (dsqexp_dx2's trans_fun,
  ## covariance_function_derivatives.R:191-197), one knot per row
  to_bounded <- function(xt) {
    xu <- apply(X = xt, MARGIN = 1, FUN = function(x, bounds)
      bounds[, 2] * (1 / (1 + exp(-x))) + bounds[, 1] * (1 / (1 + exp(x))), bounds = knot_bounds)
    matrix(xu, ncol = ncol(xy), byrow = TRUE)
  }
  ## transformed -> positive: real_to_pos for the ARD length scales, the closures' trans_fun
  ## (exp) otherwise
  to_pos <- function() {
    for (j in 1:length(cov_par)) current_cov_par[j] <- exp(current_cov_par_trans[j])
    current_cov_par
  }
  say <- function() {
    print(paste("iteration ", iter, sep = ""))
    print(c(current_grad_val_theta, current_grad_val_knot))
  }

  iter <- 1
  adadelta <- optim_method == "adadelta"
  if (adadelta) {
    sg2_theta <- sd2_theta <- sign_change_theta <- rep(0, times = length(current_cov_par))
    sg2_knot <- sd2_knot <- sign_change_knot <- rep(0, times = nrow(xu) * ncol(xu))
  }
  while (iter < maxit &&
         (any(abs(c(current_grad_val_theta, current_grad_val_knot)) > grad_tol) ||
          ifelse(iter > 1, yes = abs(current_obj_fun - obj_fun_vals[iter - 1]) > obj_tol,
                 no = TRUE))) {
    iter <- iter + 1
    if (verbose == TRUE && !(adadelta && print_after)) say()
    if (is.list(dcov_fun_dtheta)) {
      if (adadelta) {
        sg2_theta <- optim_par$decay * sg2_theta +
          (1 - optim_par$decay) * current_grad_val_theta^2
        delta_theta <- ((1 / optim_par$eta)^(sign_change_theta)) *
          (sqrt(sd2_theta + rep(optim_par$epsilon, times = length(sd2_theta))) /
             sqrt(sg2_theta + rep(optim_par$epsilon, times = length(sd2_theta)))) *
          current_grad_val_theta
        sd2_theta <- optim_par$decay * sd2_theta + (1 - optim_par$decay) * delta_theta^2
        current_cov_par_trans <- current_cov_par_trans + delta_theta
      } else {
        current_cov_par_trans <- current_cov_par_trans +
          optim_par$learn_rate * current_grad_val_theta
      }
    }
    if (is.function(dcov_fun_dknot)) {
      if (adadelta) {
        sg2_knot <- optim_par$decay * sg2_knot + (1 - optim_par$decay) * current_grad_val_knot^2
        delta_knot <- ((1 / optim_par$eta)^(sign_change_knot)) *
          (sqrt(sd2_knot + rep(optim_par$epsilon, times = length(sd2_knot))) /
             sqrt(sg2_knot + rep(optim_par$epsilon, times = length(sd2_knot)))) *
          current_grad_val_knot
        sd2_knot <- optim_par$decay * sd2_knot + (1 - optim_par$decay) * delta_knot^2
      } else {
        delta_knot <- optim_par$learn_rate * current_grad_val_knot
      }
      ## the knot gradient vector is row-major: c(xu[1, ], xu[2, ], ...) (quirk Q16)
      current_xu_trans <- current_xu_trans + matrix(data = delta_knot, nrow = nrow(xu),
                                                    ncol = ncol(xu), byrow = TRUE)
      xu <- to_bounded(current_xu_trans)
      xu_vals <- abind::abind(xu_vals, xu, along = 3)
    }
    if (is.list(dcov_fun_dtheta)) {
      current_cov_par <- to_pos()
      cov_par <- as.list(current_cov_par)
    }

    ev <- evaluate(cov_par, xu)
    current_obj_fun <- ev$obj
    obj_fun_vals[iter] <- current_obj_fun
    cov_par_vals <- rbind(cov_par_vals, current_cov_par)
    temp_grad_eval <- ev$grad
    if (is.list(dcov_fun_dtheta)) {
      if (adadelta)
        sign_change_theta <- (optim_par$decay * sign_change_theta +
          (1 - optim_par$decay) * abs(sign(c(temp_grad_eval$gradient)) -
                                        sign(current_grad_val_theta)) / 2)
      current_grad_val_theta <- c(temp_grad_eval$gradient)
      current_cov_par_trans <- unlist(temp_grad_eval$trans_par)
      grad_vals <- rbind(grad_vals, current_grad_val_theta)
    }
    if (is.function(dcov_fun_dknot)) {
      ## (no halving for the knots, as in the reference)
      if (adadelta)
        sign_change_knot <- (optim_par$decay * sign_change_knot +
          (1 - optim_par$decay) * abs(sign(c(temp_grad_eval$knot_gradient)) -
                                        sign(current_grad_val_knot)))
      current_grad_val_knot <- c(temp_grad_eval$knot_gradient)
      grad_knot_vals <- rbind(grad_knot_vals, current_grad_val_knot)
    }
    if (verbose == TRUE && adadelta && print_after) say()
  }
  list(current_cov_par = current_cov_par, cov_par = cov_par, xu = xu, iter = iter,
       obj_fun_vals = obj_fun_vals, grad_vals = grad_vals, grad_knot_vals = grad_knot_vals,
       xu_vals = if (is.function(dcov_fun_dknot)) xu_vals else xu, cov_par_vals = cov_par_vals)
}

## return list of norm_grad_ascent_vi / norm_grad_ascent (vi_functions.R:1182-1215,
## laplace_gradient_ascent.R:1657-1690), knot posterior from the final evaluation
.sgp_gaussian_result <- function(a, ptr, cov_fun, xy, mu, muu, dcov_fun_dknot) {
  post <- .Call("sgp_R_posterior_u", ptr, as.numeric(muu))
  u_mean <- post$u_mean
  u_var <- post$u_var
  if (is.function(dcov_fun_dknot))
    return(list("cov_par" = as.list(a$current_cov_par), "cov_fun" = cov_fun, "xu" = a$xu,
                "xy" = xy, "mu" = mu, "muu" = muu, "u_mean" = u_mean, "u_var" = u_var,
                "iter" = a$iter, "obj_fun" = a$obj_fun_vals, "grad" = a$grad_vals,
                "knot_grad" = a$grad_knot_vals, "knot_history" = a$xu_vals,
                "cov_par_history" = a$cov_par_vals))
  list("cov_par" = as.list(a$current_cov_par), "cov_fun" = cov_fun, "xu" = a$xu, "xy" = xy,
       "mu" = mu, "muu" = muu, "u_mean" = u_mean, "u_var" = u_var, "cov_fun" = cov_fun,
       "iter" = a$iter, "obj_fun" = a$obj_fun_vals, "grad" = a$grad_vals, "knot_grad" = 0,
       "knot_history" = a$xu, "cov_par_history" = a$cov_par_vals)
}

.sgp_gaussian_driver <- function(method, cov_par_start, cov_fun, dcov_fun_dtheta, dcov_fun_dknot,
                                 knot_opt, xu, xy, y, mu, muu, opt, verbose)
{
  o <- .sgp_opts(opt)
  delta <- o$delta
  xy <- as.matrix(xy)
  xu <- as.matrix(xu)
  if (!is.numeric(mu)) mu <- rep(mean(y), times = length(y))          # quirk Q14
  if (!is.numeric(muu)) muu <- rep(mean(y), times = nrow(xu))
  y <- as.numeric(y)
  knots <- is.function(dcov_fun_dknot)
  evaluate <- function(cov_par, xu) {
    ev <- .sgp_eval(method, cov_par, cov_fun, xu, xy, y, mu, delta, knots)
    list(obj = ev$objective,
         grad = .sgp_grad_list(ev, cov_par, dcov_fun_dtheta, knots, knot_opt, xu, xy))
  }
  a <- .sgp_ascent(evaluate, cov_par_start, cov_fun, dcov_fun_dtheta, dcov_fun_dknot, xu, xy,
                   o, verbose)
  .sgp_gaussian_result(a, .sgp$ctx$ptr, cov_fun, xy, mu, muu, dcov_fun_dknot)
}

sgp_norm_grad_ascent_vi <- function(cov_par_start,
                                    cov_fun,
                                    dcov_fun_dtheta,
                                    dcov_fun_dknot,
                                    knot_opt,
                                    xu,
                                    xy,
                                    y,
                                    mu = NA,
                                    muu = NA,
                                    obj_fun = elbo_fun,
                                    opt = list(),
                                    verbose = FALSE,
                                    ...)
{
  of <- if (missing(obj_fun)) NULL else obj_fun
  if (!.sgp_fusable(cov_fun, cov_par_start, dcov_fun_dtheta, dcov_fun_dknot, of, "elbo_fun"))
    return(.sgp$orig$norm_grad_ascent_vi(cov_par_start = cov_par_start, cov_fun = cov_fun,
                                         dcov_fun_dtheta = dcov_fun_dtheta,
                                         dcov_fun_dknot = dcov_fun_dknot, knot_opt = knot_opt,
                                         xu = xu, xy = xy, y = y, mu = mu, muu = muu,
                                         obj_fun = .sgp_obj_or_default(obj_fun, of, "elbo_fun"),
                                         opt = opt, verbose = verbose, ...))
  .sgp_gaussian_driver(0L, cov_par_start, cov_fun, dcov_fun_dtheta, dcov_fun_dknot, knot_opt,
                       xu, xy, y, mu, muu, opt, verbose)
}

sgp_norm_grad_ascent <- function(cov_par_start,
                                 cov_fun,
                                 dcov_fun_dtheta,
                                 dcov_fun_dknot,
                                 knot_opt,
                                 xu,
                                 xy,
                                 y,
                                 mu = NA,
                                 muu = NA,
                                 transform = TRUE,
                                 obj_fun,
                                 opt = list(),
                                 verbose = FALSE,
                                 ...)
{
  of <- if (missing(obj_fun)) NULL else obj_fun
  if (!isTRUE(transform) ||
      !.sgp_fusable(cov_fun, cov_par_start, dcov_fun_dtheta, dcov_fun_dknot, of, "obj_fun_norm"))
    return(.sgp$orig$norm_grad_ascent(cov_par_start = cov_par_start, cov_fun = cov_fun,
                                      dcov_fun_dtheta = dcov_fun_dtheta,
                                      dcov_fun_dknot = dcov_fun_dknot, knot_opt = knot_opt,
                                      xu = xu, xy = xy, y = y, mu = mu, muu = muu,
                                      transform = transform, obj_fun = obj_fun, opt = opt,
                                      verbose = verbose, ...))
  .sgp_gaussian_driver(1L, cov_par_start, cov_fun, dcov_fun_dtheta, dcov_fun_dknot, knot_opt,
                       xu, xy, y, mu, muu, opt, verbose)
}

sgp_laplace_grad_ascent <- function(cov_par_start,
                                    cov_fun,
                                    dcov_fun_dtheta,
                                    dcov_fun_dknot,
                                    knot_opt,
                                    xu,
                                    xy,
                                    y,
                                    ff,
                                    grad_loglik_fn,
                                    dlog_py_dff,
                                    d2log_py_dff,
                                    d3log_py_dff,
                                    mu,
                                    muu,
                                    transform = TRUE,
                                    obj_fun,
                                    opt = list(),
                                    verbose = FALSE,
                                    ...)
{
  args <- list(...)
  of <- if (missing(obj_fun)) NULL else obj_fun
  if (!isTRUE(transform) || !.sgp_poisson(d2log_py_dff, args) ||
      !.sgp_fusable(cov_fun, cov_par_start, dcov_fun_dtheta, dcov_fun_dknot, of, "obj_fun_pois"))
    return(.sgp$orig$laplace_grad_ascent(cov_par_start = cov_par_start, cov_fun = cov_fun,
                                         dcov_fun_dtheta = dcov_fun_dtheta,
                                         dcov_fun_dknot = dcov_fun_dknot, knot_opt = knot_opt,
                                         xu = xu, xy = xy, y = y, ff = ff,
                                         grad_loglik_fn = grad_loglik_fn,
                                         dlog_py_dff = dlog_py_dff, d2log_py_dff = d2log_py_dff,
                                         d3log_py_dff = d3log_py_dff, mu = mu, muu = muu,
                                         transform = transform, obj_fun = obj_fun, opt = opt,
                                         verbose = verbose, ...))
  o <- .sgp_opts(opt, list("maxit_nr" = 1000, "tol_nr" = 1e-6))
  delta <- o$delta
  xy <- as.matrix(xy)
  xu <- as.matrix(xu)
  if (!is.numeric(mu)) mu <- rep(mean(y), times = length(y))
  if (!is.numeric(muu)) muu <- rep(mean(y), times = nrow(xu))
  y <- as.numeric(y)
  expo <- .sgp_expo(args, nrow(as.matrix(xy)))
  knots <- is.function(dcov_fun_dknot)
  ptr <- .sgp_ctx(xy, y, mu, nrow(xu))
  .sgp$last <- NULL
  .sgp_knots(ptr, knots)
  .Call("sgp_R_lap_set_f", ptr, as.numeric(ff))
  ## each iteration: newtrap_sparseGP warm-started from the resident mode (fmax,
  ## laplace_gradient_ascent.R:507-519) and dlogq_dcov_par at the new mode, fused
  evaluate <- function(cov_par, xu) {
    theta <- .sgp_theta(cov_par, cov_fun, ncol(xu))
    ev <- .Call("sgp_R_eval_laplace", ptr, cov_fun, unname(theta), xu, as.numeric(delta), expo,
                as.numeric(o$tol_nr), as.integer(max(o$maxit_nr, 1)), TRUE)
    names(ev$gradient) <- names(theta)
    if (knots)
      ev$knot_gradient <- .Call("sgp_R_knot_gradient", ptr, .sgp_knot_bounds(xy), nrow(xu),
                                ncol(xu))
    list(obj = ev$objective,
         grad = .sgp_grad_list(ev, cov_par, dcov_fun_dtheta, knots, knot_opt, xu, xy))
  }
  a <- .sgp_ascent(evaluate, cov_par_start, cov_fun, dcov_fun_dtheta, dcov_fun_dknot, xu, xy,
                   o, verbose, print_after = TRUE)
  fmax <- .Call("sgp_R_lap_get_f", ptr)
  post <- .Call("sgp_R_posterior_u", ptr, as.numeric(muu))
  out <- list("cov_par" = a$cov_par, "cov_fun" = cov_fun, "xu" = a$xu, "xy" = xy, "mu" = mu,
              "muu" = muu, "fmax" = fmax, "iter" = a$iter, "obj_fun" = a$obj_fun_vals,
              "fmax" = fmax, "u_mean" = post$u_mean, "u_var" = post$u_var,
              "grad" = a$grad_vals,
              "knot_grad" = if (knots) a$grad_knot_vals else 0,
              "knot_history" = a$xu_vals, "cov_par_history" = a$cov_par_vals)
  out
}

## ---------------------------------------------------------------- predict_gp (L5)

## R/laplace_approx_prediction.R:408-542: the sparse predictors (predict_vi / predict_laplace)
## and the full Gaussian GP's predict_gp_full through sgp_predict; full Poisson / Bernoulli
## fits (predict_laplace_full) run the package's original function
sgp_predict_gp <- function(mod, x_pred, mu_pred = NA, full_cov, vi = FALSE)
{
  family <- mod$family
  sparse <- mod$sparse
  m <- mod$results
  delta <- mod$delta
  if (vi == TRUE && family != "gaussian")
    return("Error: VI not supported for non-gaussian data.")
  if ((sparse == FALSE && family != "gaussian") || !m$cov_fun %in% c("sqexp", "ard"))
    return(.sgp$orig$predict_gp(mod = mod, x_pred = x_pred, mu_pred = mu_pred,
                                full_cov = full_cov, vi = vi))
  inv_link_fn <- NA
  if (family == "poisson") inv_link_fn <- function(x) { return(exp(x)) }
  if (family == "bernoulli") inv_link_fn <- function(x) { return(1 / (1 + exp(-x))) }
  if (!is.matrix(x_pred)) {
    print("Warning: x_pred must be a matrix. I'll try to make the conversion.")
    x_pred <- matrix(data = x_pred, ncol = 1)
  }
  if (any(is.na(mu_pred))) {
    print("Warnings: you did not define the mean of the GP at locations at which you wish to make predictions. Setting the mean to be zero.")
    mu_pred <- rep(0, times = nrow(x_pred))
  }
  theta <- unname(.sgp_theta(m$cov_par, m$cov_fun, ncol(x_pred)))
  if (sparse == FALSE) {
    ## predict_gp_full: U = xy, u_mean = y, muu = mu (include/sgp.h SGP_PRED_FULL)
    xy <- as.matrix(m$xy)
    pred <- .Call("sgp_R_predict", 2L, TRUE, m$cov_fun, theta, as.numeric(delta), xy,
                  as.numeric(m$y), rep_len(as.numeric(m$mu), nrow(xy)), NULL, x_pred,
                  as.numeric(mu_pred), full_cov)
  } else {
    xu <- as.matrix(m$xu)
    k <- nrow(xu)
    pred <- .Call("sgp_R_predict", if (vi == TRUE) 0L else 1L, family == "gaussian",
                  m$cov_fun, theta, as.numeric(delta), xu, as.numeric(m$u_mean[1:k]),
                  as.numeric(m$muu[1:k]), as.matrix(m$u_var), x_pred, as.numeric(mu_pred),
                  full_cov)
  }
  return(list("pred" = pred, "sparse" = sparse, "family" = family, "x_pred" = x_pred,
              "inverse_link" = inv_link_fn))
}
