#include "common.hpp"

#include <cmath>

extern "C" double genrand_real1(void);

namespace qa {

Complex conjScalar(Complex z) {
    Complex c;
    c.real = z.real;
    c.imag = -z.imag;
    return c;
}

ComplexMatrix2 conjMatrix(const ComplexMatrix2& m) {
    ComplexMatrix2 c;
    c.r0c0 = conjScalar(m.r0c0);
    c.r0c1 = conjScalar(m.r0c1);
    c.r1c0 = conjScalar(m.r1c0);
    c.r1c1 = conjScalar(m.r1c1);
    return c;
}

void complexPairFromRotation(qreal angle, Vector axis, Complex* alpha, Complex* beta) {
    qreal mag = std::sqrt(axis.x * axis.x + axis.y * axis.y + axis.z * axis.z);
    qreal ux = axis.x / mag, uy = axis.y / mag, uz = axis.z / mag;
    qreal c = std::cos(angle / 2.0), s = std::sin(angle / 2.0);
    alpha->real = c;
    alpha->imag = -s * uz;
    beta->real = s * uy;
    beta->imag = -s * ux;
}

void zyzFromComplexPair(Complex alpha, Complex beta, qreal* rz2, qreal* ry, qreal* rz1) {
    qreal alphaMag = std::sqrt(alpha.real * alpha.real + alpha.imag * alpha.imag);
    *ry = 2.0 * std::acos(alphaMag);
    qreal alphaPhase = std::atan2(alpha.imag, alpha.real);
    qreal betaPhase = std::atan2(beta.imag, beta.real);
    *rz2 = -alphaPhase + betaPhase;
    *rz1 = -alphaPhase - betaPhase;
}

void complexPairAndPhaseFromUnitary(const ComplexMatrix2& u, Complex* alpha, Complex* beta, qreal* phase) {
    qreal p00 = std::atan2(u.r0c0.imag, u.r0c0.real);
    qreal p11 = std::atan2(u.r1c1.imag, u.r1c1.real);
    *phase = (p00 + p11) / 2.0;
    qreal c = std::cos(*phase), s = std::sin(*phase);
    alpha->real = u.r0c0.real * c + u.r0c0.imag * s;
    alpha->imag = u.r0c0.imag * c - u.r0c0.real * s;
    beta->real = u.r1c0.real * c + u.r1c0.imag * s;
    beta->imag = u.r1c0.imag * c - u.r1c0.real * s;
}

int generateMeasurementOutcome(qreal zeroProb, qreal* outcomeProb) {
    int outcome;
    if (zeroProb < REAL_EPS)
        outcome = 1;
    else if (1 - zeroProb < REAL_EPS)
        outcome = 0;
    else
        outcome = (genrand_real1() > zeroProb);
    *outcomeProb = (outcome == 0) ? zeroProb : 1 - zeroProb;
    return outcome;
}

}  // namespace qa
