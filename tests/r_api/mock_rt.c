/*
 * mock_rt.c -- a minimal executable R runtime for running rshim/sparseRGPs_sgp.c without R.
 *
 * TEST INFRASTRUCTURE ONLY (R is absent from this image).  It implements exactly
 * the subset of R's C API that the headers in tests/r_api declare, with R's documented semantics where
 * the shim depends on them:
 *   - SEXPs carry a type, a length, a payload and the names / dim attributes;
 *   - logical NA (matrix() is a 1x1 logical NA) coerces to a NaN double (NA_real_);
 *   - Rf_error formats the message and longjmps back to the .Call frame (mock_call), which
 *     restores the PROTECT stack as R's context unwinding does;
 *   - the PROTECT stack is checked after every successful call: a routine that returns with
 *     a different stack depth than it started with is reported (status 2);
 *   - REprintf is captured so tests can read the reference's Rcerr-style messages;
 *   - R_registerRoutines records the CallEntries table so calls go by registered name and the
 *     argument count is checked like R's .Call does;
 *   - external pointers keep their C finalizer, run by mock_gc().
 * Objects are never freed until mock_reset() (the tests are short-lived).
 *
 * Python drives it through ctypes (tests/test_rshim_exec.py): mock_* constructors and
 * accessors below plus mock_call(name, nargs, args, &out).
 */
#include <setjmp.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <R.h>
#include <R_ext/Rdynload.h>
#include <Rinternals.h>

#define NILSXP_ 0
#define CHARSXP_ 9
#define LGLSXP_ 10
#define INTSXP_ 13
#define NA_LOGICAL_ INT32_MIN

struct SEXPREC {
  SEXPTYPE type;
  R_xlen_t len;
  void* data; /* double* | int* | SEXP* | char* | extptr address */
  SEXP names;
  SEXP dim; /* INTSXP of length 2 or NULL */
  R_CFinalizer_t fin;
  SEXP next_all;
};

static struct SEXPREC nil_rec = {NILSXP_, 0, NULL, NULL, NULL, NULL, NULL};
static struct SEXPREC names_sym_rec = {NILSXP_, 0, NULL, NULL, NULL, NULL, NULL};
SEXP R_NilValue = &nil_rec;
SEXP R_NamesSymbol = &names_sym_rec;

static SEXP all_objs = NULL;
#define PSTACK 10000
static SEXP pstack[PSTACK];
static int ptop = 0;
static jmp_buf* err_jmp = NULL;
static char err_msg[4096];
static char eprint[8192];
static size_t eprint_len = 0;
static const R_CallMethodDef* reg = NULL;
static int reg_count = 0;
static int dyn_symbols = -1;

static SEXP new_obj(SEXPTYPE t, R_xlen_t len) {
  SEXP s = (SEXP)calloc(1, sizeof(struct SEXPREC));
  s->type = t;
  s->len = len;
  s->names = R_NilValue;
  s->dim = NULL;
  size_t esz = t == REALSXP ? sizeof(double)
               : (t == INTSXP_ || t == LGLSXP_) ? sizeof(int)
               : (t == STRSXP || t == VECSXP) ? sizeof(SEXP)
                                               : 0;
  if (esz) s->data = calloc(len > 0 ? (size_t)len : 1, esz);
  if (t == STRSXP || t == VECSXP)
    for (R_xlen_t i = 0; i < len; ++i) ((SEXP*)s->data)[i] = R_NilValue;
  s->next_all = all_objs;
  all_objs = s;
  return s;
}

/* ---------------------------------------------------------------- the declared R API */

void REprintf(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  int w = vsnprintf(eprint + eprint_len, sizeof(eprint) - eprint_len, fmt, ap);
  va_end(ap);
  if (w > 0) eprint_len += (size_t)w < sizeof(eprint) - eprint_len ? (size_t)w : sizeof(eprint) - eprint_len - 1;
}

void Rf_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(err_msg, sizeof(err_msg), fmt, ap);
  va_end(ap);
  if (!err_jmp) {
    fprintf(stderr, "mock_rt: Rf_error outside a .Call: %s\n", err_msg);
    abort();
  }
  longjmp(*err_jmp, 1);
}

SEXP Rf_protect(SEXP s) {
  if (ptop >= PSTACK) Rf_error("protect(): protection stack overflow");
  pstack[ptop++] = s;
  return s;
}

void Rf_unprotect(int n) {
  if (n > ptop) {
    fprintf(stderr, "mock_rt: unprotect(%d) with only %d protected\n", n, ptop);
    abort(); /* R: "unprotect(): only %d protected items" is a fatal error */
  }
  ptop -= n;
}

int TYPEOF(SEXP s) { return (int)s->type; }

double* REAL(SEXP s) {
  if (s->type != REALSXP) {
    fprintf(stderr, "mock_rt: REAL() on a non-double SEXP (type %u)\n", s->type);
    abort();
  }
  return (double*)s->data;
}

R_xlen_t XLENGTH(SEXP s) { return s->len; }
R_len_t Rf_length(SEXP s) { return s == R_NilValue ? 0 : (R_len_t)s->len; }

SEXP STRING_ELT(SEXP s, R_xlen_t i) {
  if (s->type != STRSXP || i < 0 || i >= s->len) abort();
  return ((SEXP*)s->data)[i];
}

void SET_STRING_ELT(SEXP s, R_xlen_t i, SEXP v) {
  if (s->type != STRSXP || i < 0 || i >= s->len || v->type != CHARSXP_) abort();
  ((SEXP*)s->data)[i] = v;
}

SEXP SET_VECTOR_ELT(SEXP s, R_xlen_t i, SEXP v) {
  if (s->type != VECSXP || i < 0 || i >= s->len) abort();
  ((SEXP*)s->data)[i] = v;
  return v;
}

SEXP VECTOR_ELT(SEXP s, R_xlen_t i) {
  if (s->type != VECSXP || i < 0 || i >= s->len) abort();
  return ((SEXP*)s->data)[i];
}

const char* CHAR(SEXP s) {
  if (s->type != CHARSXP_) abort();
  return (const char*)s->data;
}

SEXP Rf_mkChar(const char* c) {
  SEXP s = new_obj(CHARSXP_, (R_xlen_t)strlen(c));
  s->data = strdup(c);
  return s;
}

Rboolean Rf_isNull(SEXP s) { return s == R_NilValue || s->type == NILSXP_; }
Rboolean Rf_isString(SEXP s) { return s->type == STRSXP; }
Rboolean Rf_isMatrix(SEXP s) { return s->dim != NULL; }

int Rf_nrows(SEXP s) { return s->dim ? ((int*)s->dim->data)[0] : (int)s->len; }
int Rf_ncols(SEXP s) { return s->dim ? ((int*)s->dim->data)[1] : 1; }

static double elt_real(SEXP s, R_xlen_t i) {
  switch (s->type) {
    case REALSXP: return ((double*)s->data)[i];
    case INTSXP_:
    case LGLSXP_: {
      int v = ((int*)s->data)[i];
      return v == NA_LOGICAL_ ? NAN : (double)v;
    }
    default: Rf_error("cannot coerce type %u to double", s->type);
  }
  return NAN;
}

double Rf_asReal(SEXP s) {
  if (s->len < 1) return NAN;
  if (s->type == VECSXP) Rf_error("(list) object cannot be coerced to type 'double'");
  return elt_real(s, 0);
}

int Rf_asInteger(SEXP s) {
  if (s->len < 1) return NA_LOGICAL_;
  double v = elt_real(s, 0);
  return v != v ? NA_LOGICAL_ : (int)v;
}

int Rf_asLogical(SEXP s) {
  if (s->len < 1) return NA_LOGICAL_;
  double v = elt_real(s, 0);
  return v != v ? NA_LOGICAL_ : v != 0.0;
}

SEXP Rf_coerceVector(SEXP s, SEXPTYPE t) {
  if (s->type == t) return s;
  if (t != REALSXP) Rf_error("mock_rt: coercion to type %u not implemented", t);
  SEXP o = new_obj(REALSXP, s->len);
  for (R_xlen_t i = 0; i < s->len; ++i) ((double*)o->data)[i] = elt_real(s, i);
  o->dim = s->dim; /* R keeps dim and names on coerceVector of a vector */
  o->names = s->names;
  return o;
}

SEXP Rf_allocVector(SEXPTYPE t, R_xlen_t n) {
  if (t != REALSXP && t != STRSXP && t != VECSXP && t != INTSXP_ && t != LGLSXP_)
    Rf_error("mock_rt: allocVector of type %u", t);
  return new_obj(t, n);
}

static SEXP mk_dim(int nr, int nc) {
  SEXP d = new_obj(INTSXP_, 2);
  ((int*)d->data)[0] = nr;
  ((int*)d->data)[1] = nc;
  return d;
}

SEXP Rf_allocMatrix(SEXPTYPE t, int nr, int nc) {
  if (nr < 0 || nc < 0) Rf_error("negative extents to matrix");
  SEXP s = Rf_allocVector(t, (R_xlen_t)nr * nc);
  s->dim = mk_dim(nr, nc);
  return s;
}

SEXP Rf_ScalarReal(double v) {
  SEXP s = new_obj(REALSXP, 1);
  ((double*)s->data)[0] = v;
  return s;
}

SEXP Rf_ScalarInteger(int v) {
  SEXP s = new_obj(INTSXP_, 1);
  ((int*)s->data)[0] = v;
  return s;
}

SEXP Rf_getAttrib(SEXP s, SEXP sym) {
  if (sym != R_NamesSymbol) abort();
  return s->names ? s->names : R_NilValue;
}

SEXP Rf_setAttrib(SEXP s, SEXP sym, SEXP v) {
  if (sym != R_NamesSymbol) abort();
  if (!Rf_isNull(v) && (v->type != STRSXP || v->len != s->len))
    Rf_error("'names' attribute [%ld] must be the same length as the vector [%ld]",
             (long)v->len, (long)s->len);
  s->names = v;
  return v;
}

SEXP R_MakeExternalPtr(void* p, SEXP tag, SEXP prot) {
  (void)tag;
  (void)prot;
  SEXP s = new_obj(EXTPTRSXP, 1);
  s->data = p;
  return s;
}

void* R_ExternalPtrAddr(SEXP s) { return s->type == EXTPTRSXP ? s->data : NULL; }
void R_ClearExternalPtr(SEXP s) {
  if (s->type == EXTPTRSXP) s->data = NULL;
}
void R_RegisterCFinalizerEx(SEXP s, R_CFinalizer_t f, Rboolean onexit) {
  (void)onexit;
  s->fin = f;
}

int R_registerRoutines(DllInfo* dll, const void* c, const R_CallMethodDef* call, const void* f,
                       const void* e) {
  (void)dll;
  (void)c;
  (void)f;
  (void)e;
  reg = call;
  reg_count = 0;
  while (call[reg_count].name) ++reg_count;
  return 1;
}

int R_useDynamicSymbols(DllInfo* dll, int v) {
  (void)dll;
  dyn_symbols = v;
  return 1;
}

/* ---------------------------------------------------------------- test-side entry points */

void R_init_sparseRGPs(DllInfo* dll);

int mock_load(void) {
  R_init_sparseRGPs(NULL);
  return reg_count;
}

int mock_dynamic_symbols(void) { return dyn_symbols; }
const char* mock_routine_name(int i) { return i >= 0 && i < reg_count ? reg[i].name : NULL; }
int mock_routine_arity(int i) { return i >= 0 && i < reg_count ? reg[i].numArgs : -1; }

SEXP mock_real(const double* v, long n) {
  SEXP s = new_obj(REALSXP, n);
  if (n) memcpy(s->data, v, sizeof(double) * (size_t)n);
  return s;
}

/* column-major nr x nc double matrix */
SEXP mock_matrix(const double* v, int nr, int nc) {
  SEXP s = mock_real(v, (long)nr * nc);
  s->dim = mk_dim(nr, nc);
  return s;
}

SEXP mock_int(const int* v, long n) {
  SEXP s = new_obj(INTSXP_, n);
  if (n) memcpy(s->data, v, sizeof(int) * (size_t)n);
  return s;
}

SEXP mock_logical(int v) {
  SEXP s = new_obj(LGLSXP_, 1);
  ((int*)s->data)[0] = v;
  return s;
}

/* R's matrix(): a 1x1 logical NA */
SEXP mock_na_matrix(void) {
  SEXP s = new_obj(LGLSXP_, 1);
  ((int*)s->data)[0] = NA_LOGICAL_;
  s->dim = mk_dim(1, 1);
  return s;
}

SEXP mock_strings(const char** v, long n) {
  SEXP s = new_obj(STRSXP, n);
  for (long i = 0; i < n; ++i) ((SEXP*)s->data)[i] = Rf_mkChar(v[i]);
  return s;
}

SEXP mock_list(const char** names, SEXP* vals, long n) {
  SEXP s = new_obj(VECSXP, n);
  for (long i = 0; i < n; ++i) ((SEXP*)s->data)[i] = vals[i];
  if (names) s->names = mock_strings(names, n);
  return s;
}

SEXP mock_nil(void) { return R_NilValue; }
int mock_type(SEXP s) { return (int)s->type; }
long mock_length(SEXP s) { return (long)Rf_length(s); }
int mock_is_matrix(SEXP s) { return s->dim != NULL; }
int mock_nrow(SEXP s) { return Rf_nrows(s); }
int mock_ncol(SEXP s) { return Rf_ncols(s); }
const double* mock_real_ptr(SEXP s) { return s->type == REALSXP ? (const double*)s->data : NULL; }
const int* mock_int_ptr(SEXP s) {
  return (s->type == INTSXP_ || s->type == LGLSXP_) ? (const int*)s->data : NULL;
}
SEXP mock_elt(SEXP s, long i) { return VECTOR_ELT(s, i); }
const char* mock_name(SEXP s, long i) {
  return Rf_isNull(s->names) ? NULL : CHAR(STRING_ELT(s->names, i));
}
const char* mock_str(SEXP s, long i) { return CHAR(STRING_ELT(s, i)); }
const char* mock_error(void) { return err_msg; }
const char* mock_eprint(void) { return eprint; }
int mock_protect_depth(void) { return ptop; }

/* .Call(name, args...): 0 = returned (stack balanced), 1 = R error (message in mock_error),
 * 2 = returned with an unbalanced PROTECT stack, 3 = no such routine, 4 = wrong arity. */
int mock_call(const char* name, int nargs, SEXP* a, SEXP* out) {
  int idx = -1;
  for (int i = 0; i < reg_count; ++i)
    if (!strcmp(reg[i].name, name)) idx = i;
  if (idx < 0) return 3;
  if (reg[idx].numArgs != nargs) return 4;
  err_msg[0] = 0;
  eprint[0] = 0;
  eprint_len = 0;
  const int depth = ptop;
  jmp_buf jb;
  jmp_buf* prev = err_jmp;
  err_jmp = &jb;
  if (setjmp(jb)) {
    err_jmp = prev;
    ptop = depth; /* R unwinds the protect stack with the context */
    *out = R_NilValue;
    return 1;
  }
  DL_FUNC f = reg[idx].fun;
  SEXP r;
  switch (nargs) {
#define A(i) a[i]
    case 0: r = ((SEXP(*)(void))f)(); break;
    case 1: r = ((SEXP(*)(SEXP))f)(A(0)); break;
    case 2: r = ((SEXP(*)(SEXP, SEXP))f)(A(0), A(1)); break;
    case 3: r = ((SEXP(*)(SEXP, SEXP, SEXP))f)(A(0), A(1), A(2)); break;
    case 4: r = ((SEXP(*)(SEXP, SEXP, SEXP, SEXP))f)(A(0), A(1), A(2), A(3)); break;
    case 5: r = ((SEXP(*)(SEXP, SEXP, SEXP, SEXP, SEXP))f)(A(0), A(1), A(2), A(3), A(4)); break;
    case 6:
      r = ((SEXP(*)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP))f)(A(0), A(1), A(2), A(3), A(4), A(5));
      break;
    case 7:
      r = ((SEXP(*)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP))f)(A(0), A(1), A(2), A(3), A(4),
                                                                 A(5), A(6));
      break;
    case 9:
      r = ((SEXP(*)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP))f)(
          A(0), A(1), A(2), A(3), A(4), A(5), A(6), A(7), A(8));
      break;
    case 10:
      r = ((SEXP(*)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP))f)(
          A(0), A(1), A(2), A(3), A(4), A(5), A(6), A(7), A(8), A(9));
      break;
    case 12:
      r = ((SEXP(*)(SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP, SEXP))f)(
          A(0), A(1), A(2), A(3), A(4), A(5), A(6), A(7), A(8), A(9), A(10), A(11));
      break;
#undef A
    default:
      err_jmp = prev;
      return 4;
  }
  err_jmp = prev;
  *out = r;
  return ptop == depth ? 0 : 2;
}

/* run every registered external-pointer finalizer once (R's gc of unreachable contexts) */
int mock_gc(void) {
  int ran = 0;
  for (SEXP s = all_objs; s; s = s->next_all)
    if (s->type == EXTPTRSXP && s->fin) {
      R_CFinalizer_t f = s->fin;
      s->fin = NULL;
      f(s);
      ++ran;
    }
  return ran;
}

void mock_reset(void) {
  mock_gc();
  SEXP s = all_objs;
  while (s) {
    SEXP nx = s->next_all;
    if (s->type != EXTPTRSXP) free(s->data);
    free(s);
    s = nx;
  }
  all_objs = NULL;
  ptop = 0;
}
