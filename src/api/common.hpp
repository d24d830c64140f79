// Hardware-agnostic math used by the front-end and the QASM recorder
// (reference: QuEST/src/QuEST_common.c:25-121).
#pragma once

#include "QuEST.h"

namespace qa {

Complex conjScalar(Complex z);
ComplexMatrix2 conjMatrix(const ComplexMatrix2& m);
// alpha = cos(a/2) - i sin(a/2) n_z ; beta = sin(a/2) (n_y - i n_x)
void complexPairFromRotation(qreal angle, Vector axis, Complex* alpha, Complex* beta);
// U(alpha, beta) = Rz(rz2) Ry(ry) Rz(rz1) (up to global phase)
void zyzFromComplexPair(Complex alpha, Complex beta, qreal* rz2, qreal* ry, qreal* rz1);
// u = exp(i phase) U(alpha, beta)
void complexPairAndPhaseFromUnitary(const ComplexMatrix2& u, Complex* alpha, Complex* beta, qreal* phase);
// reference measurement draw (QuEST_common.c:103-121)
int generateMeasurementOutcome(qreal zeroProb, qreal* outcomeProb);

}  // namespace qa
