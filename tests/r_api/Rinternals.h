/* Declarations-only subset of R's C API for a syntax check (see tests/r_api/R.h). */
#ifndef SGP_TEST_RINTERNALS_H
#define SGP_TEST_RINTERNALS_H
#include <stddef.h>
typedef struct SEXPREC* SEXP;
typedef int R_len_t;
typedef ptrdiff_t R_xlen_t;
typedef unsigned int SEXPTYPE;
typedef int Rboolean;
#define STRSXP 16
#define REALSXP 14
#define VECSXP 19
#define EXTPTRSXP 22
extern SEXP R_NilValue;
extern SEXP R_NamesSymbol;
SEXP Rf_protect(SEXP);
void Rf_unprotect(int);
#define PROTECT(s) Rf_protect(s)
#define UNPROTECT(n) Rf_unprotect(n)
int TYPEOF(SEXP);
double* REAL(SEXP);
R_xlen_t XLENGTH(SEXP);
SEXP STRING_ELT(SEXP, R_xlen_t);
void SET_STRING_ELT(SEXP, R_xlen_t, SEXP);
SEXP SET_VECTOR_ELT(SEXP, R_xlen_t, SEXP);
SEXP VECTOR_ELT(SEXP, R_xlen_t);
const char* CHAR(SEXP);
SEXP Rf_mkChar(const char*);
R_len_t Rf_length(SEXP);
Rboolean Rf_isNull(SEXP);
Rboolean Rf_isString(SEXP);
Rboolean Rf_isMatrix(SEXP);
int Rf_nrows(SEXP);
int Rf_ncols(SEXP);
double Rf_asReal(SEXP);
int Rf_asInteger(SEXP);
int Rf_asLogical(SEXP);
SEXP Rf_coerceVector(SEXP, SEXPTYPE);
SEXP Rf_allocVector(SEXPTYPE, R_xlen_t);
SEXP Rf_allocMatrix(SEXPTYPE, int, int);
SEXP Rf_ScalarReal(double);
SEXP Rf_ScalarInteger(int);
SEXP Rf_getAttrib(SEXP, SEXP);
SEXP Rf_setAttrib(SEXP, SEXP, SEXP);
void Rf_error(const char*, ...) __attribute__((noreturn));
typedef void (*R_CFinalizer_t)(SEXP);
SEXP R_MakeExternalPtr(void*, SEXP, SEXP);
void* R_ExternalPtrAddr(SEXP);
void R_ClearExternalPtr(SEXP);
void R_RegisterCFinalizerEx(SEXP, R_CFinalizer_t, Rboolean);
#endif
