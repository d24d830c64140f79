// Validation layer: reference semantics (QuEST/src/QuEST_validation.c:82-263),
// including its quirks (damping reuses the depolarising error code; the
// unitarity tolerance is REAL_EPS).
#include <string>
#include "validation.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "quest_amd.h"

namespace qa {

static const char* kMessages[E_NUM_ERROR_CODES] = {
    "Success.",
    "Invalid number of qubits. Must create >0.",
    "Invalid target qubit. Note qubits are zero indexed.",
    "Invalid control qubit. Note qubits are zero indexed.",
    "Invalid state index. Must be >=0 and <2^numQubits.",
    "Invalid number of amplitudes. Must be >=0 and <=2^numQubits.",
    "More amplitudes given than exist in the statevector from the given starting index.",
    "Control qubit cannot equal target qubit.",
    "Control qubits cannot include target qubit.",
    "The two target qubits must be unique.",
    "Invalid number of control qubits. Must be >0 and <numQubits.",
    "Matrix is not unitary.",
    "Compact matrix formed by given complex numbers is not unitary.",
    "Invalid axis vector. Must be non-zero.",
    "Invalid system size. Cannot print output for systems greater than 5 qubits.",
    "Can't collapse to state with zero probability.",
    "Invalid measurement outcome -- must be either 0 or 1.",
    "Could not open file",
    "Second argument must be a state-vector.",
    "Dimensions of the qubit registers don't match.",
    "Registers must both be state-vectors or both be density matrices.",
    "Operation valid only for state-vectors.",
    "Operation valid only for density matrices.",
    "Probabilities must be in [0, 1].",
    "Probabilities must sum to ~1.",
    "The probability of a single qubit dephase error cannot exceed 1/2, which maximally mixes.",
    "The probability of a two-qubit qubit dephase error cannot exceed 3/4, which maximally mixes.",
    "The probability of a single qubit depolarising error cannot exceed 3/4, which maximally mixes.",
    "The probability of a two-qubit depolarising error cannot exceed 15/16, which maximally mixes.",
    "Too few qubits to distribute the register over this many ranks.",
    "Out of device memory while allocating the register.",
    "Device runtime error.",
    "Checkpoint does not match the register (number of qubits, register type or precision).",
};

static QuESTErrorHandler g_handler = nullptr;

const char* errorMessage(ErrorCode code) {
    if (code < 0 || code >= E_NUM_ERROR_CODES) return "Unknown error.";
    return kMessages[code];
}

bool raiseErrorMsg(ErrorCode code, const char* caller, const char* detail) {
    if (g_handler) {
        std::string msg = errorMessage(code);
        if (detail) msg += std::string(" (") + detail + ")";
        g_handler((int)code, msg.c_str(), caller);
        return false;
    }
    printf("!!!\n");
    printf("QuEST Error in function %s: %s", caller, errorMessage(code));
    if (detail) printf(" (%s)", detail);
    printf("\n!!!\n");
    printf("exiting..\n");
    fflush(stdout);
    exit((int)code);
}

bool raiseError(ErrorCode code, const char* caller) { return raiseErrorMsg(code, caller, nullptr); }

static inline bool check(bool ok, ErrorCode code, const char* f) { return ok ? true : raiseError(code, f); }

namespace v {

bool createNumQubits(int n, int numRanks, const char* f) {
    if (!check(n > 0, E_INVALID_NUM_QUBITS, f)) return false;
    int g = 0;
    while ((1 << g) < numRanks) g++;
    return check(n >= g + 1, E_TOO_MANY_QUBITS_FOR_RANKS, f);
}

bool stateIndex(const Qureg& q, long long i, const char* f) {
    long long mx = 1LL << q.numQubitsRepresented;
    return check(i >= 0 && i < mx, E_INVALID_STATE_INDEX, f);
}

bool numAmps(const Qureg& q, long long start, long long n, const char* f) {
    if (!stateIndex(q, start, f)) return false;
    if (!check(n >= 0 && n <= q.numAmpsTotal, E_INVALID_NUM_AMPS, f)) return false;
    return check(n + start <= q.numAmpsTotal, E_INVALID_OFFSET_NUM_AMPS, f);
}

bool target(const Qureg& q, int t, const char* f) {
    return check(t >= 0 && t < q.numQubitsRepresented, E_INVALID_TARGET_QUBIT, f);
}

bool control(const Qureg& q, int c, const char* f) {
    return check(c >= 0 && c < q.numQubitsRepresented, E_INVALID_CONTROL_QUBIT, f);
}

bool controlTarget(const Qureg& q, int c, int t, const char* f) {
    return target(q, t, f) && control(q, c, f) && check(c != t, E_TARGET_IS_CONTROL, f);
}

bool uniqueTargets(const Qureg& q, int a, int b, const char* f) {
    return target(q, a, f) && target(q, b, f) && check(a != b, E_TARGETS_NOT_UNIQUE, f);
}

bool multiControls(const Qureg& q, const int* c, int n, const char* f) {
    if (!check(n > 0 && n <= q.numQubitsRepresented, E_INVALID_NUM_CONTROLS, f)) return false;
    for (int i = 0; i < n; i++)
        if (!control(q, c[i], f)) return false;
    return true;
}

bool multiControlsTarget(const Qureg& q, const int* c, int n, int t, const char* f) {
    if (!target(q, t, f) || !multiControls(q, c, n, f)) return false;
    for (int i = 0; i < n; i++)
        if (!check(c[i] != t, E_TARGET_IN_CONTROLS, f)) return false;
    return true;
}

static bool isUnitary(const ComplexMatrix2& u) {
    if (absReal(u.r0c0.real * u.r0c0.real + u.r0c0.imag * u.r0c0.imag + u.r1c0.real * u.r1c0.real +
                u.r1c0.imag * u.r1c0.imag - 1) > REAL_EPS)
        return false;
    if (absReal(u.r0c1.real * u.r0c1.real + u.r0c1.imag * u.r0c1.imag + u.r1c1.real * u.r1c1.real +
                u.r1c1.imag * u.r1c1.imag - 1) > REAL_EPS)
        return false;
    if (absReal(u.r0c0.real * u.r0c1.real + u.r0c0.imag * u.r0c1.imag + u.r1c0.real * u.r1c1.real +
                u.r1c0.imag * u.r1c1.imag) > REAL_EPS)
        return false;
    if (absReal(u.r0c1.real * u.r0c0.imag - u.r0c0.real * u.r0c1.imag + u.r1c1.real * u.r1c0.imag -
                u.r1c0.real * u.r1c1.imag) > REAL_EPS)
        return false;
    return true;
}

bool unitaryMatrix(const ComplexMatrix2& u, const char* f) {
    return check(isUnitary(u), E_NON_UNITARY_MATRIX, f);
}

bool unitaryPair(const Complex& a, const Complex& b, const char* f) {
    qreal s = a.real * a.real + a.imag * a.imag + b.real * b.real + b.imag * b.imag;
    return check(absReal(s - 1) < REAL_EPS, E_NON_UNITARY_COMPLEX_PAIR, f);
}

bool vector(const Vector& vec, const char* f) {
    qreal mag = std::sqrt(vec.x * vec.x + vec.y * vec.y + vec.z * vec.z);
    return check(mag > REAL_EPS, E_ZERO_VECTOR, f);
}

bool stateVec(const Qureg& q, const char* f) { return check(!q.isDensityMatrix, E_DEFINED_ONLY_FOR_STATEVECS, f); }
bool densMatr(const Qureg& q, const char* f) { return check(q.isDensityMatrix, E_DEFINED_ONLY_FOR_DENSMATRS, f); }
bool outcome(int o, const char* f) { return check(o == 0 || o == 1, E_INVALID_QUBIT_OUTCOME, f); }
bool measurementProb(qreal p, const char* f) { return check(p > REAL_EPS, E_COLLAPSE_STATE_ZERO_PROB, f); }
bool matchingDims(const Qureg& a, const Qureg& b, const char* f) {
    return check(a.numQubitsRepresented == b.numQubitsRepresented, E_MISMATCHING_QUREG_DIMENSIONS, f);
}
bool matchingTypes(const Qureg& a, const Qureg& b, const char* f) {
    return check(a.isDensityMatrix == b.isDensityMatrix, E_MISMATCHING_QUREG_TYPES, f);
}
bool secondStateVec(const Qureg& q, const char* f) {
    return check(!q.isDensityMatrix, E_SECOND_ARG_MUST_BE_STATEVEC, f);
}
bool fileOpened(int ok, const char* f) { return check(ok != 0, E_CANNOT_OPEN_FILE, f); }
bool prob(qreal p, const char* f) { return check(p >= 0 && p <= 1, E_INVALID_PROB, f); }
bool oneQubitDephaseProb(qreal p, const char* f) {
    return prob(p, f) && check(p <= 1 / 2.0, E_INVALID_ONE_QUBIT_DEPHASE_PROB, f);
}
bool twoQubitDephaseProb(qreal p, const char* f) {
    return prob(p, f) && check(p <= 3 / 4.0, E_INVALID_TWO_QUBIT_DEPHASE_PROB, f);
}
bool oneQubitDepolProb(qreal p, const char* f) {
    return prob(p, f) && check(p <= 3 / 4.0, E_INVALID_ONE_QUBIT_DEPOL_PROB, f);
}
bool oneQubitDampingProb(qreal p, const char* f) {
    // reference quirk: reuses the depolarising code (QuEST_validation.c:255-258)
    return prob(p, f) && check(p <= 1.0, E_INVALID_ONE_QUBIT_DEPOL_PROB, f);
}
bool twoQubitDepolProb(qreal p, const char* f) {
    return prob(p, f) && check(p <= 15 / 16.0, E_INVALID_TWO_QUBIT_DEPOL_PROB, f);
}

}  // namespace v
}  // namespace qa

extern "C" void setQuESTErrorHandler(QuESTErrorHandler h) { qa::g_handler = h; }
