/* Declarations-only subset of R's C API (as documented in "Writing R Extensions") used by
 * rshim/sparseRGPs_sgp.c -- for tests/test_rshim.py's `gcc -fsyntax-only` check in an image
 * without R.  Not a usable R runtime; the shim is built against R's real headers. */
#ifndef SGP_TEST_R_H
#define SGP_TEST_R_H
#include <math.h>
#include <stddef.h>
#define ISNAN(x) (isnan(x) != 0)
#ifndef TRUE
#define TRUE 1
#define FALSE 0
#endif
void REprintf(const char*, ...);
#endif
