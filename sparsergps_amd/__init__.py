"""sparsergps_amd -- MI355X-native sparse-GP objective + gradient (drop-in for sparseRGPs' hot path).

Product path: libsgp.so (HIP, gfx950) behind the C ABI in include/sgp.h; this package is the
host-side mirror of the reference's R/Rcpp interface for that path.
"""
from ._build import build
from ._lib import NotPositiveDefinite, SGPError
from .covariance import (cov_fun_expC, cov_fun_sqrd_exp_ardC, cov_fun_sqrd_expC, dsig_dtheta_ardC,
                         dsig_dthetaC, make_cov_mat_ardC, make_cov_matC)
from .drivers import laplace_grad_ascent, norm_grad_ascent, norm_grad_ascent_vi
from .full import (dlogp_dcov_par_full, full_eval, norm_grad_ascent_full, obj_fun_norm_full,
                   predict_gp_full)
from .predict import predict_gp, predict_laplace, predict_vi
from .laplace import dlogq_dcov_par, laplace_eval, newtrap_sparseGP, obj_fun_pois
from .vi import (SparseGPContext, delbo_dcov_par, dlogp_dcov_par, elbo_fun, fitc_eval, param_names,
                 vi_eval)

__all__ = [
    "build", "SGPError", "NotPositiveDefinite",
    "make_cov_matC", "make_cov_mat_ardC", "dsig_dthetaC", "dsig_dtheta_ardC",
    "cov_fun_sqrd_expC", "cov_fun_sqrd_exp_ardC", "cov_fun_expC",
    "SparseGPContext", "vi_eval", "elbo_fun", "delbo_dcov_par", "param_names",
    "fitc_eval", "dlogp_dcov_par",
    "laplace_eval", "newtrap_sparseGP", "dlogq_dcov_par", "obj_fun_pois",
    "predict_vi", "predict_laplace", "predict_gp",
    "norm_grad_ascent_vi", "norm_grad_ascent", "laplace_grad_ascent",
    "full_eval", "obj_fun_norm_full", "dlogp_dcov_par_full", "norm_grad_ascent_full",
    "predict_gp_full",
]
