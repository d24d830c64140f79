// Input validation with the reference's error codes and messages
// (QuEST/src/QuEST_validation.c:19-80).  Default behaviour is the
// reference's: print the message and exit(code).  A handler installed with
// setQuESTErrorHandler() (quest_amd.h) is called instead, and the API call
// then returns without touching the state - the Python binding turns that
// into a QuESTError exception.
#pragma once

#include "QuEST.h"

namespace qa {

enum ErrorCode {
    E_SUCCESS = 0,
    E_INVALID_NUM_QUBITS,
    E_INVALID_TARGET_QUBIT,
    E_INVALID_CONTROL_QUBIT,
    E_INVALID_STATE_INDEX,
    E_INVALID_NUM_AMPS,
    E_INVALID_OFFSET_NUM_AMPS,
    E_TARGET_IS_CONTROL,
    E_TARGET_IN_CONTROLS,
    E_TARGETS_NOT_UNIQUE,
    E_INVALID_NUM_CONTROLS,
    E_NON_UNITARY_MATRIX,
    E_NON_UNITARY_COMPLEX_PAIR,
    E_ZERO_VECTOR,
    E_SYS_TOO_BIG_TO_PRINT,
    E_COLLAPSE_STATE_ZERO_PROB,
    E_INVALID_QUBIT_OUTCOME,
    E_CANNOT_OPEN_FILE,
    E_SECOND_ARG_MUST_BE_STATEVEC,
    E_MISMATCHING_QUREG_DIMENSIONS,
    E_MISMATCHING_QUREG_TYPES,
    E_DEFINED_ONLY_FOR_STATEVECS,
    E_DEFINED_ONLY_FOR_DENSMATRS,
    E_INVALID_PROB,
    E_UNNORM_PROBS,
    E_INVALID_ONE_QUBIT_DEPHASE_PROB,
    E_INVALID_TWO_QUBIT_DEPHASE_PROB,
    E_INVALID_ONE_QUBIT_DEPOL_PROB,
    E_INVALID_TWO_QUBIT_DEPOL_PROB,
    // extensions (not in the reference)
    E_TOO_MANY_QUBITS_FOR_RANKS,
    E_OUT_OF_MEMORY,
    E_DEVICE_ERROR,
    E_CHECKPOINT_MISMATCH,
    E_NUM_ERROR_CODES
};

// Report an error; returns false when a handler swallowed it.
bool raiseError(ErrorCode code, const char* caller);
bool raiseErrorMsg(ErrorCode code, const char* caller, const char* detail);
const char* errorMessage(ErrorCode code);

namespace v {
bool createNumQubits(int n, int numRanks, const char* f);
bool stateIndex(const Qureg& q, long long i, const char* f);
bool numAmps(const Qureg& q, long long start, long long n, const char* f);
bool target(const Qureg& q, int t, const char* f);
bool control(const Qureg& q, int c, const char* f);
bool controlTarget(const Qureg& q, int c, int t, const char* f);
bool uniqueTargets(const Qureg& q, int a, int b, const char* f);
bool multiControls(const Qureg& q, const int* c, int n, const char* f);
bool multiControlsTarget(const Qureg& q, const int* c, int n, int t, const char* f);
bool unitaryMatrix(const ComplexMatrix2& u, const char* f);
bool unitaryPair(const Complex& a, const Complex& b, const char* f);
bool vector(const Vector& v, const char* f);
bool stateVec(const Qureg& q, const char* f);
bool densMatr(const Qureg& q, const char* f);
bool outcome(int o, const char* f);
bool measurementProb(qreal p, const char* f);
bool matchingDims(const Qureg& a, const Qureg& b, const char* f);
bool matchingTypes(const Qureg& a, const Qureg& b, const char* f);
bool secondStateVec(const Qureg& q, const char* f);
bool fileOpened(int ok, const char* f);
bool prob(qreal p, const char* f);
bool oneQubitDephaseProb(qreal p, const char* f);
bool twoQubitDephaseProb(qreal p, const char* f);
bool oneQubitDepolProb(qreal p, const char* f);
bool oneQubitDampingProb(qreal p, const char* f);
bool twoQubitDepolProb(qreal p, const char* f);
}  // namespace v

}  // namespace qa
