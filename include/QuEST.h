/* QuEST-for-MI355X public C API.
 *
 * Source- and ABI-compatible with the QuEST v2 API (reference:
 * QuEST/include/QuEST.h:26-1571): the same structs with the same field order,
 * and the same 79 functions with the same semantics.  The implementation
 * behind it is new: host C++17 front-end + hand-written CDNA4 (gfx950) HIP
 * kernels + RCCL over xGMI for multi-GPU state-vectors (one process per GPU).
 *
 * Conventions shared with the reference:
 *  - qubit q is bit q of the amplitude index (little endian);
 *  - a density matrix of N qubits is stored as a 2N-qubit state-vector with
 *    element (row r, column c) at flat index r + c * 2^N;
 *  - every function validates its input and, on error, prints a message and
 *    exits with the error code (see src/api/validation.cpp).
 *
 * MI355X-specific extensions (gate-fusion control, profiling, torch interop,
 * explicit multi-GPU bootstrap) live in quest_amd.h.
 */
#ifndef QUEST_H
#define QUEST_H

#include "QuEST_precision.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Codes for Z-axis phase gate variations (kept for source compatibility). */
enum phaseGateType { SIGMA_Z = 0, S_GATE = 1, T_GATE = 2 };

/* Growable QASM text buffer attached to every Qureg. */
typedef struct {
    char* buffer;     /* generated QASM string */
    int bufferSize;   /* capacity in chars */
    int bufferFill;   /* chars currently used */
    int isLogging;    /* whether operations are being recorded */
} QASMLogger;

/* Struct-of-arrays amplitude storage. */
typedef struct ComplexArray {
    qreal* real;
    qreal* imag;
} ComplexArray;

typedef struct Complex {
    qreal real;
    qreal imag;
} Complex;

/* 2x2 complex matrix, row-major element names. */
typedef struct ComplexMatrix2 {
    Complex r0c0, r0c1;
    Complex r1c0, r1c1;
} ComplexMatrix2;

typedef struct Vector {
    qreal x, y, z;
} Vector;

/* A register of qubits: a pure state-vector or a density matrix.
 *
 * On the HIP build the amplitudes live only in device memory
 * (deviceStateVec); stateVec is a host staging buffer that is NULL until a
 * host-side operation (reportState, initStateFromSingleFile) needs it.  With
 * several ranks, each process holds numAmpsPerChunk contiguous amplitudes. */
typedef struct Qureg {
    int isDensityMatrix;
    int numQubitsRepresented;
    int numQubitsInStateVec;
    long long int numAmpsPerChunk;
    long long int numAmpsTotal;
    int chunkId;
    int numChunks;
    ComplexArray stateVec;
    ComplexArray pairStateVec;
    ComplexArray deviceStateVec;
    qreal *firstLevelReduction, *secondLevelReduction;
    QASMLogger* qasmLog;
} Qureg;

/* Execution environment: this process's rank and the number of ranks. */
typedef struct QuESTEnv {
    int rank;
    int numRanks;
} QuESTEnv;

/* ------------------------------------------------------------------------ */
/* registers                                                                */
/* ------------------------------------------------------------------------ */

/* Create an N-qubit state-vector initialised to |0...0>. */
Qureg createQureg(int numQubits, QuESTEnv env);
/* Create an N-qubit density matrix initialised to |0...0><0...0|. */
Qureg createDensityQureg(int numQubits, QuESTEnv env);
void destroyQureg(Qureg qureg, QuESTEnv env);

/* Write this rank's amplitudes to state_rank_<chunkId>.csv. */
void reportState(Qureg qureg);
/* Print the amplitudes (registers of at most 5 state-vector qubits). */
void reportStateToScreen(Qureg qureg, QuESTEnv env, int reportRank);
void reportQuregParams(Qureg qureg);
int getNumQubits(Qureg qureg);
/* Number of amplitudes of a state-vector (rejects density matrices). */
int getNumAmps(Qureg qureg);

/* ------------------------------------------------------------------------ */
/* state initialisation                                                     */
/* ------------------------------------------------------------------------ */

void initZeroState(Qureg qureg);
/* |+>^N (state-vector) or the uniform density matrix with all entries 1/2^N. */
void initPlusState(Qureg qureg);
void initClassicalState(Qureg qureg, long long int stateInd);
/* qureg := pure (state-vector) or |pure><pure| (density matrix). */
void initPureState(Qureg qureg, Qureg pure);
void initStateFromAmps(Qureg qureg, qreal* reals, qreal* imags);
void setAmps(Qureg qureg, long long int startInd, qreal* reals, qreal* imags, long long int numAmps);
void cloneQureg(Qureg targetQureg, Qureg copyQureg);

/* ------------------------------------------------------------------------ */
/* unitaries                                                                */
/* ------------------------------------------------------------------------ */

/* Multiply the |1> amplitudes of the target by exp(i angle). */
void phaseShift(Qureg qureg, const int targetQubit, qreal angle);
void controlledPhaseShift(Qureg qureg, const int idQubit1, const int idQubit2, qreal angle);
void multiControlledPhaseShift(Qureg qureg, int* controlQubits, int numControlQubits, qreal angle);
void controlledPhaseFlip(Qureg qureg, const int idQubit1, const int idQubit2);
void multiControlledPhaseFlip(Qureg qureg, int* controlQubits, int numControlQubits);
void sGate(Qureg qureg, const int targetQubit);
void tGate(Qureg qureg, const int targetQubit);

/* ------------------------------------------------------------------------ */
/* environment                                                              */
/* ------------------------------------------------------------------------ */

/* Initialise the device (and, when launched with WORLD_SIZE > 1, the RCCL
 * communicator of this rank) and seed the RNG with time and pid. */
QuESTEnv createQuESTEnv(void);
void destroyQuESTEnv(QuESTEnv env);
/* Block until every queued operation of every rank has completed. */
void syncQuESTEnv(QuESTEnv env);
/* Logical AND of successCode over all ranks. */
int syncQuESTSuccess(int successCode);
void reportQuESTEnv(QuESTEnv env);
void getEnvironmentString(QuESTEnv env, Qureg qureg, char str[200]);

/* ------------------------------------------------------------------------ */
/* amplitude access and calculations                                        */
/* ------------------------------------------------------------------------ */

Complex getAmp(Qureg qureg, long long int index);
qreal getRealAmp(Qureg qureg, long long int index);
qreal getImagAmp(Qureg qureg, long long int index);
qreal getProbAmp(Qureg qureg, long long int index);
Complex getDensityAmp(Qureg qureg, long long int row, long long int col);
/* Sum of |amp|^2 (state-vector) or the trace (density matrix). */
qreal calcTotalProb(Qureg qureg);

/* ------------------------------------------------------------------------ */
/* more unitaries                                                           */
/* ------------------------------------------------------------------------ */

/* U = [[alpha, -conj(beta)], [beta, conj(alpha)]], |alpha|^2+|beta|^2 = 1. */
void compactUnitary(Qureg qureg, const int targetQubit, Complex alpha, Complex beta);
void unitary(Qureg qureg, const int targetQubit, ComplexMatrix2 u);
void rotateX(Qureg qureg, const int rotQubit, qreal angle);
void rotateY(Qureg qureg, const int rotQubit, qreal angle);
void rotateZ(Qureg qureg, const int rotQubit, qreal angle);
void rotateAroundAxis(Qureg qureg, const int rotQubit, qreal angle, Vector axis);
void controlledRotateX(Qureg qureg, const int controlQubit, const int targetQubit, qreal angle);
void controlledRotateY(Qureg qureg, const int controlQubit, const int targetQubit, qreal angle);
void controlledRotateZ(Qureg qureg, const int controlQubit, const int targetQubit, qreal angle);
void controlledRotateAroundAxis(Qureg qureg, const int controlQubit, const int targetQubit, qreal angle, Vector axis);
void controlledCompactUnitary(Qureg qureg, const int controlQubit, const int targetQubit, Complex alpha, Complex beta);
void controlledUnitary(Qureg qureg, const int controlQubit, const int targetQubit, ComplexMatrix2 u);
void multiControlledUnitary(Qureg qureg, int* controlQubits, const int numControlQubits, const int targetQubit, ComplexMatrix2 u);
void pauliX(Qureg qureg, const int targetQubit);
void pauliY(Qureg qureg, const int targetQubit);
void pauliZ(Qureg qureg, const int targetQubit);
void hadamard(Qureg qureg, const int targetQubit);
void controlledNot(Qureg qureg, const int controlQubit, const int targetQubit);
void controlledPauliY(Qureg qureg, const int controlQubit, const int targetQubit);

/* ------------------------------------------------------------------------ */
/* measurement                                                              */
/* ------------------------------------------------------------------------ */

/* Probability of outcome (0 or 1); outcome 1 is computed as 1 - P(0). */
qreal calcProbOfOutcome(Qureg qureg, const int measureQubit, int outcome);
/* Force the outcome, renormalise, return its probability. */
qreal collapseToOutcome(Qureg qureg, const int measureQubit, int outcome);
int measure(Qureg qureg, int measureQubit);
int measureWithStats(Qureg qureg, int measureQubit, qreal* outcomeProb);
/* <bra|ket> of two state-vectors. */
Complex calcInnerProduct(Qureg bra, Qureg ket);

/* ------------------------------------------------------------------------ */
/* random numbers (MT19937, bit-compatible with the reference)              */
/* ------------------------------------------------------------------------ */

void seedQuESTDefault(void);
void seedQuEST(unsigned long int* seedArray, int numSeeds);

/* ------------------------------------------------------------------------ */
/* QASM recording                                                           */
/* ------------------------------------------------------------------------ */

void startRecordingQASM(Qureg qureg);
void stopRecordingQASM(Qureg qureg);
void clearRecordedQASM(Qureg qureg);
void printRecordedQASM(Qureg qureg);
void writeRecordedQASMToFile(Qureg qureg, char* filename);

/* ------------------------------------------------------------------------ */
/* decoherence (density matrices only)                                      */
/* ------------------------------------------------------------------------ */

void applyOneQubitDephaseError(Qureg qureg, const int targetQubit, qreal prob);
void applyTwoQubitDephaseError(Qureg qureg, const int qubit1, const int qubit2, qreal prob);
void applyOneQubitDepolariseError(Qureg qureg, const int targetQubit, qreal prob);
void applyOneQubitDampingError(Qureg qureg, const int targetQubit, qreal prob);
void applyTwoQubitDepolariseError(Qureg qureg, const int qubit1, const int qubit2, qreal prob);
/* combineQureg := (1-prob) combineQureg + prob otherQureg */
void addDensityMatrix(Qureg combineQureg, qreal prob, Qureg otherQureg);
/* Tr(rho^2) */
qreal calcPurity(Qureg qureg);
/* |<psi|qureg>|^2 (state-vector) or <psi|rho|psi> (density matrix). */
qreal calcFidelity(Qureg qureg, Qureg pureState);

#ifdef __cplusplus
}
#endif

#endif /* QUEST_H */
