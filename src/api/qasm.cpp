#include "qasm.hpp"

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "common.hpp"

namespace qa {
namespace qasm {

namespace {

constexpr int kInitialBuffer = 1000;

const char* label(Gate g) {
    switch (g) {
        case G_SIGMA_X: return "x";
        case G_SIGMA_Y: return "y";
        case G_SIGMA_Z: return "z";
        case G_T: return "t";
        case G_S: return "s";
        case G_HADAMARD: return "h";
        case G_ROTATE_X: return "Rx";
        case G_ROTATE_Y: return "Ry";
        case G_ROTATE_Z: return "Rz";
        case G_UNITARY: return "U";
        case G_PHASE_SHIFT: return "Rz";  // needs a phase fix when controlled
        default: return "?";
    }
}

void append(QASMLogger* log, const std::string& s) {
    int need = log->bufferFill + (int)s.size() + 1;
    if (need > log->bufferSize) {
        int sz = log->bufferSize > 0 ? log->bufferSize : kInitialBuffer;
        while (sz < need) sz *= 2;
        char* nb = (char*)realloc(log->buffer, (size_t)sz);
        if (!nb) {
            printf("!!!\nINTERNAL ERROR: QASM line buffer filled!\n!!!");
            exit(1);
        }
        log->buffer = nb;
        log->bufferSize = sz;
    }
    memcpy(log->buffer + log->bufferFill, s.data(), s.size());
    log->bufferFill += (int)s.size();
    log->buffer[log->bufferFill] = '\0';
}

std::string fmt(const char* f, ...) {
    char buf[256];
    va_list ap;
    va_start(ap, f);
    vsnprintf(buf, sizeof buf, f, ap);
    va_end(ap);
    return buf;
}

bool on(const Qureg& q) { return q.qasmLog && q.qasmLog->isLogging; }

void addGate(const Qureg& q, Gate g, const int* ctrls, int nc, int target, const qreal* params, int np) {
    std::string line;
    for (int i = 0; i < nc; i++) line += "c";
    line += label(g);
    if (np > 0) {
        line += "(";
        for (int i = 0; i < np; i++) {
            line += fmt(REAL_QASM_FORMAT, params[i]);
            if (i != np - 1) line += ",";
        }
        line += ")";
    }
    line += " ";
    for (int i = 0; i < nc; i++) line += fmt("q[%d],", ctrls[i]);
    line += fmt("q[%d];\n", target);
    append(q.qasmLog, line);
}

void zyzParams(Complex a, Complex b, qreal p[3]) { zyzFromComplexPair(a, b, &p[0], &p[1], &p[2]); }

}  // namespace

void setup(QASMLogger* log, int numQubits) {
    log->isLogging = 0;
    log->bufferSize = kInitialBuffer;
    log->buffer = (char*)malloc(kInitialBuffer);
    log->bufferFill = 0;
    log->buffer[0] = '\0';
    append(log, fmt("OPENQASM 2.0;\nqreg q[%d];\ncreg c[%d];\n", numQubits, numQubits));
}

void release(QASMLogger* log) {
    free(log->buffer);
    log->buffer = nullptr;
    log->bufferSize = log->bufferFill = 0;
}

void start(const Qureg& q) { q.qasmLog->isLogging = 1; }
void stop(const Qureg& q) { q.qasmLog->isLogging = 0; }

void clear(const Qureg& q) {
    q.qasmLog->buffer[0] = '\0';
    q.qasmLog->bufferFill = 0;
}

void print(const Qureg& q) {
    printf("%s", q.qasmLog->buffer);
    fflush(stdout);
}

int writeToFile(const Qureg& q, const char* filename) {
    FILE* f = fopen(filename, "w");
    if (!f) return 0;
    fprintf(f, "%s", q.qasmLog->buffer);
    fclose(f);
    return 1;
}

void comment(const Qureg& q, const char* text) {
    if (!on(q)) return;
    append(q.qasmLog, fmt("// %s\n", text));
}

void gate(const Qureg& q, Gate g, int target) {
    if (!on(q)) return;
    addGate(q, g, nullptr, 0, target, nullptr, 0);
}

void paramGate(const Qureg& q, Gate g, int target, qreal param) {
    if (!on(q)) return;
    addGate(q, g, nullptr, 0, target, &param, 1);
}

void compactUnitary(const Qureg& q, Complex a, Complex b, int target) {
    if (!on(q)) return;
    qreal p[3];
    zyzParams(a, b, p);
    addGate(q, G_UNITARY, nullptr, 0, target, p, 3);
}

void unitary(const Qureg& q, const ComplexMatrix2& u, int target) {
    if (!on(q)) return;
    Complex a, b;
    qreal phase, p[3];
    complexPairAndPhaseFromUnitary(u, &a, &b, &phase);
    zyzParams(a, b, p);
    addGate(q, G_UNITARY, nullptr, 0, target, p, 3);
}

void axisRotation(const Qureg& q, qreal angle, Vector axis, int target) {
    if (!on(q)) return;
    Complex a, b;
    qreal p[3];
    complexPairFromRotation(angle, axis, &a, &b);
    zyzParams(a, b, p);
    addGate(q, G_UNITARY, nullptr, 0, target, p, 3);
}

void controlledGate(const Qureg& q, Gate g, int ctrl, int target) {
    if (!on(q)) return;
    addGate(q, g, &ctrl, 1, target, nullptr, 0);
}

void controlledParamGate(const Qureg& q, Gate g, int ctrl, int target, qreal param) {
    if (!on(q)) return;
    addGate(q, g, &ctrl, 1, target, &param, 1);
    if (g == G_PHASE_SHIFT) {
        comment(q, "Restoring the discarded global phase of the previous controlled phase gate");
        qreal fix = param / 2.0;
        addGate(q, G_ROTATE_Z, nullptr, 0, target, &fix, 1);
    }
}

void controlledCompactUnitary(const Qureg& q, Complex a, Complex b, int ctrl, int target) {
    if (!on(q)) return;
    qreal p[3];
    zyzParams(a, b, p);
    addGate(q, G_UNITARY, &ctrl, 1, target, p, 3);
}

void controlledUnitary(const Qureg& q, const ComplexMatrix2& u, int ctrl, int target) {
    if (!on(q)) return;
    Complex a, b;
    qreal phase, p[3];
    complexPairAndPhaseFromUnitary(u, &a, &b, &phase);
    zyzParams(a, b, p);
    addGate(q, G_UNITARY, &ctrl, 1, target, p, 3);
    comment(q, "Restoring the discarded global phase of the previous controlled unitary");
    addGate(q, G_ROTATE_Z, nullptr, 0, target, &phase, 1);
}

void controlledAxisRotation(const Qureg& q, qreal angle, Vector axis, int ctrl, int target) {
    if (!on(q)) return;
    Complex a, b;
    qreal p[3];
    complexPairFromRotation(angle, axis, &a, &b);
    zyzParams(a, b, p);
    addGate(q, G_UNITARY, &ctrl, 1, target, p, 3);
}

void multiControlledGate(const Qureg& q, Gate g, const int* ctrls, int n, int target) {
    if (!on(q)) return;
    addGate(q, g, ctrls, n, target, nullptr, 0);
}

void multiControlledParamGate(const Qureg& q, Gate g, const int* ctrls, int n, int target, qreal param) {
    if (!on(q)) return;
    addGate(q, g, ctrls, n, target, &param, 1);
    if (g == G_PHASE_SHIFT) {
        comment(q, "Restoring the discarded global phase of the previous multicontrolled phase gate");
        qreal fix = param / 2.0;
        addGate(q, G_ROTATE_Z, nullptr, 0, target, &fix, 1);
    }
}

void multiControlledUnitary(const Qureg& q, const ComplexMatrix2& u, const int* ctrls, int n, int target) {
    if (!on(q)) return;
    Complex a, b;
    qreal phase, p[3];
    complexPairAndPhaseFromUnitary(u, &a, &b, &phase);
    zyzParams(a, b, p);
    addGate(q, G_UNITARY, ctrls, n, target, p, 3);
    addGate(q, G_ROTATE_Z, nullptr, 0, target, &phase, 1);
}

void measurement(const Qureg& q, int target) {
    if (!on(q)) return;
    append(q.qasmLog, fmt("measure q[%d] -> c[%d];\n", target, target));
}

void initZero(const Qureg& q) {
    if (!on(q)) return;
    append(q.qasmLog, "reset q;\n");
}

void initPlus(const Qureg& q) {
    if (!on(q)) return;
    comment(q, "Initialising state |+>");
    initZero(q);
    append(q.qasmLog, "h q;\n");
}

void initClassical(const Qureg& q, long long stateInd) {
    if (!on(q)) return;
    comment(q, fmt("Initialising state |%lld>", stateInd).c_str());
    initZero(q);
    for (int t = 0; t < q.numQubitsRepresented; t++)
        if ((stateInd >> t) & 1) gate(q, G_SIGMA_X, t);
}

}  // namespace qasm
}  // namespace qa
