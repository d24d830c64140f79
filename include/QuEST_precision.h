/* QuEST-for-MI355X: compile-time floating point precision.
 *
 * The amplitude precision is fixed when the library is built, exactly as in the
 * reference (QuEST/include/QuEST_precision.h:17-62): QuEST_PREC = 1 (float),
 * 2 (double, the default) or 4 (long double; host plumbing build only - the HIP
 * build accepts 1 or 2).  Programs must be compiled with the same QuEST_PREC as
 * the library they link (quest_amd/lib/libQuEST_<backend>_f{32,64}.so).
 */
#ifndef QUEST_PRECISION_H
#define QUEST_PRECISION_H

#include <math.h>

#ifndef QuEST_PREC
#define QuEST_PREC 2
#endif

#if QuEST_PREC == 1
#define qreal float
/* largest amplitude count moved by one point-to-point message (kept for source
 * compatibility; the RCCL exchange slices by bytes, see src/comm) */
#define MPI_MAX_AMPS_IN_MSG (1LL << 29)
#define REAL_STRING_FORMAT "%.8f"
#define REAL_QASM_FORMAT "%.8g"
#define REAL_EPS 1e-5
#define absReal(X) fabs(X)

#elif QuEST_PREC == 2
#define qreal double
#define MPI_MAX_AMPS_IN_MSG (1LL << 28)
#define REAL_STRING_FORMAT "%.14f"
#define REAL_QASM_FORMAT "%.14g"
#define REAL_EPS 1e-13
#define absReal(X) fabs(X)

#elif QuEST_PREC == 4
#define qreal long double
#define MPI_MAX_AMPS_IN_MSG (1LL << 27)
#define REAL_STRING_FORMAT "%.17Lf"
#define REAL_QASM_FORMAT "%.17Lg"
#define REAL_EPS 1e-14
#define absReal(X) fabsl(X)

#else
#error "QuEST_PREC must be 1, 2 or 4"
#endif

#endif /* QUEST_PRECISION_H */
