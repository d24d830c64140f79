// OPENQASM 2.0 recorder: the reference's only tracing facility, reproduced
// text-for-text (QuEST/src/QuEST_qasm.c:55-471): same header, gate labels,
// parameter format (REAL_QASM_FORMAT), ZYZ decomposition of unitaries and the
// Rz global-phase fix-up lines after controlled phase / controlled unitary.
#pragma once

#include "QuEST.h"

namespace qa {
namespace qasm {

enum Gate {
    G_SIGMA_X, G_SIGMA_Y, G_SIGMA_Z, G_T, G_S, G_HADAMARD,
    G_ROTATE_X, G_ROTATE_Y, G_ROTATE_Z, G_ROTATE_AROUND_AXIS, G_UNITARY, G_PHASE_SHIFT
};

void setup(QASMLogger* log, int numQubits);
void release(QASMLogger* log);
void start(const Qureg& q);
void stop(const Qureg& q);
void clear(const Qureg& q);
void print(const Qureg& q);
int writeToFile(const Qureg& q, const char* filename);

void comment(const Qureg& q, const char* text);
void gate(const Qureg& q, Gate g, int target);
void paramGate(const Qureg& q, Gate g, int target, qreal param);
void compactUnitary(const Qureg& q, Complex a, Complex b, int target);
void unitary(const Qureg& q, const ComplexMatrix2& u, int target);
void axisRotation(const Qureg& q, qreal angle, Vector axis, int target);
void controlledGate(const Qureg& q, Gate g, int ctrl, int target);
void controlledParamGate(const Qureg& q, Gate g, int ctrl, int target, qreal param);
void controlledCompactUnitary(const Qureg& q, Complex a, Complex b, int ctrl, int target);
void controlledUnitary(const Qureg& q, const ComplexMatrix2& u, int ctrl, int target);
void controlledAxisRotation(const Qureg& q, qreal angle, Vector axis, int ctrl, int target);
void multiControlledGate(const Qureg& q, Gate g, const int* ctrls, int n, int target);
void multiControlledParamGate(const Qureg& q, Gate g, const int* ctrls, int n, int target, qreal param);
void multiControlledUnitary(const Qureg& q, const ComplexMatrix2& u, const int* ctrls, int n, int target);
void measurement(const Qureg& q, int target);
void initZero(const Qureg& q);
void initPlus(const Qureg& q);
void initClassical(const Qureg& q, long long stateInd);

}  // namespace qasm
}  // namespace qa
