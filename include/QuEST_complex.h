/* Native complex-number interop for QuEST's Complex struct (reference:
 * QuEST/src/QuEST_complex.h:30-87).  `qcomp` is the language's complex type of
 * precision qreal: std::complex<qreal> in C++, `qreal _Complex` in C99. */
#ifndef QUEST_COMPLEX_H
#define QUEST_COMPLEX_H

#include "QuEST_precision.h"

#ifdef __cplusplus

#include <complex>
typedef std::complex<qreal> qcomp;
#define fromComplex(comp) qcomp((comp).real, (comp).imag)

static inline Complex toComplex(qcomp z) {
    Complex c;
    c.real = z.real();
    c.imag = z.imag();
    return c;
}

#else

#include <complex.h>
#if QuEST_PREC == 1
typedef float complex qcomp;
#elif QuEST_PREC == 2
typedef double complex qcomp;
#else
typedef long double complex qcomp;
#endif
#define fromComplex(comp) ((comp).real + I * (comp).imag)
#define toComplex(scalar) ((Complex){.real = creal(scalar), .imag = cimag(scalar)})

#endif

#endif /* QUEST_COMPLEX_H */
