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
 *    element (row r, column c) at flat index r + c * 2^N; a unitary U on
 *    qubit t acts as U on bit t and conj(U) on bit t + N;
 *  - every function validates its input and, on error, prints
 *    "QuEST Error in function <name>: <message>" and exits with the error
 *    code (src/api/validation.cpp; setQuESTErrorHandler in quest_amd.h
 *    replaces the exit).  The codes used below:
 *      E_INVALID_NUM_QUBITS (1)      E_INVALID_TARGET_QUBIT (2)
 *      E_INVALID_CONTROL_QUBIT (3)   E_INVALID_STATE_INDEX (4)
 *      E_INVALID_NUM_AMPS (5)        E_INVALID_OFFSET_NUM_AMPS (6)
 *      E_TARGET_IS_CONTROL (7)       E_TARGET_IN_CONTROLS (8)
 *      E_TARGETS_NOT_UNIQUE (9)      E_INVALID_NUM_CONTROLS (10)
 *      E_NON_UNITARY_MATRIX (11)     E_NON_UNITARY_COMPLEX_PAIR (12)
 *      E_ZERO_VECTOR (13)            E_SYS_TOO_BIG_TO_PRINT (14)
 *      E_COLLAPSE_STATE_ZERO_PROB (15) E_INVALID_QUBIT_OUTCOME (16)
 *      E_CANNOT_OPEN_FILE (17)       E_SECOND_ARG_MUST_BE_STATEVEC (18)
 *      E_MISMATCHING_QUREG_DIMENSIONS (19) E_MISMATCHING_QUREG_TYPES (20)
 *      E_DEFINED_ONLY_FOR_STATEVECS (21) E_DEFINED_ONLY_FOR_DENSMATRS (22)
 *      E_INVALID_PROB (23)           E_UNNORM_PROBS (24)
 *      E_INVALID_ONE_QUBIT_DEPHASE_PROB (25) E_INVALID_TWO_QUBIT_DEPHASE_PROB (26)
 *      E_INVALID_ONE_QUBIT_DEPOL_PROB (27)   E_INVALID_TWO_QUBIT_DEPOL_PROB (28)
 *    plus the extensions E_TOO_MANY_QUBITS_FOR_RANKS (29), E_OUT_OF_MEMORY
 *    (30), E_DEVICE_ERROR (31) and E_CHECKPOINT_MISMATCH (32).
 *    Unitarity is checked to REAL_EPS (QuEST_precision.h).
 *
 * Execution model (differs from the reference only in timing, never in
 * results): gates and channels are queued per register and executed as
 * fused passes over the state (src/core/tiles.cpp, the wave-tile kernel);
 * anything that reads the state flushes the queue first, so every function
 * below returns exactly what an op-by-op execution would.  Functions marked
 * "collective" must be called by every rank of a multi-process run (they
 * exchange data or reduce over ranks).
 *
 * MI355X-specific extensions (gate-fusion control, profiling, torch interop,
 * checkpoints, explicit multi-GPU bootstrap) live in quest_amd.h.
 */
#ifndef QUEST_H
#define QUEST_H

#include "QuEST_precision.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Codes for Z-axis phase gate variations (kept for source compatibility;
 * the QASM recorder names these gates z, s and t). */
enum phaseGateType { SIGMA_Z = 0, S_GATE = 1, T_GATE = 2 };

/* Growable QASM text buffer attached to every Qureg.  On this
 * implementation Qureg.qasmLog points at the library-side register object,
 * whose first member is this logger; read it only through the QASM
 * functions below. */
typedef struct {
    char* buffer;     /* generated QASM string */
    int bufferSize;   /* capacity in chars */
    int bufferFill;   /* chars currently used */
    int isLogging;    /* whether operations are being recorded */
} QASMLogger;

/* Struct-of-arrays amplitude storage: real and imaginary parts in two
 * arrays of numAmpsPerChunk qreals each. */
typedef struct ComplexArray {
    qreal* real;
    qreal* imag;
} ComplexArray;

/* A complex scalar. */
typedef struct Complex {
    qreal real;
    qreal imag;
} Complex;

/* 2x2 complex matrix, element r<i>c<j> = row i, column j. */
typedef struct ComplexMatrix2 {
    Complex r0c0, r0c1;
    Complex r1c0, r1c1;
} ComplexMatrix2;

/* A 3-vector (rotation axis; need not be normalised, must be non-zero). */
typedef struct Vector {
    qreal x, y, z;
} Vector;

/* A register of qubits: a pure state-vector or a density matrix.
 *
 *  isDensityMatrix        1 for a density matrix
 *  numQubitsRepresented   N, the number of qubits the user sees
 *  numQubitsInStateVec    N (state-vector) or 2N (density matrix)
 *  numAmpsPerChunk        amplitudes held by this rank (2^numQubitsInStateVec
 *                         / numChunks)
 *  numAmpsTotal           2^numQubitsInStateVec
 *  chunkId, numChunks     this rank's chunk and the number of chunks (= ranks)
 *  stateVec               host amplitudes on the CPU build; on the HIP build a
 *                         host staging buffer, NULL unless QUEST_HOST_MIRROR=1
 *                         (copyStateToGPU / copyStateFromGPU in quest_amd.h)
 *  pairStateVec           unused (the distributed exchange uses its own
 *                         device buffers)
 *  deviceStateVec         device amplitudes on the HIP build (NULL on CPU)
 *  first/secondLevelReduction  unused (reductions keep their own scratch)
 *  qasmLog                the library-side register (see QASMLogger)
 *
 * On the distributed build the chunk layout may be permuted internally (qubit
 * relabelling); amplitude-level functions always present the canonical
 * layout. */
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

/* Create a state-vector of numQubits qubits in |0...0>.  2^numQubits
 * amplitudes are allocated (in device memory on the HIP build), split over
 * the ranks of env.  Collective.
 * Errors: E_INVALID_NUM_QUBITS (numQubits < 1), E_TOO_MANY_QUBITS_FOR_RANKS
 * (fewer amplitudes than ranks), E_OUT_OF_MEMORY (state + exchange buffers
 * exceed the device's free memory; getQuregMemoryPlan in quest_amd.h). */
Qureg createQureg(int numQubits, QuESTEnv env);

/* Create a density matrix of numQubits qubits in |0...0><0...0| (stored as
 * a 2 numQubits-qubit state-vector).  Collective.  Errors as createQureg. */
Qureg createDensityQureg(int numQubits, QuESTEnv env);

/* Free a register's memory (waits for its queued work).  The Qureg value
 * must not be used afterwards.  Collective. */
void destroyQureg(Qureg qureg, QuESTEnv env);

/* Write this rank's amplitudes, one "real, imag" line each (chunk 0 starts
 * with the header line "real, imag"), to state_rank_<chunkId>.csv in the
 * working directory (the format initStateFromSingleFile reads).
 * Collective. */
void reportState(Qureg qureg);

/* Print the amplitudes of a register of at most 5 state-vector qubits
 * (rank reportRank prints).  Errors: E_SYS_TOO_BIG_TO_PRINT.  Collective. */
void reportStateToScreen(Qureg qureg, QuESTEnv env, int reportRank);

/* Print the register's qubit count, amplitude count and chunking (rank 0). */
void reportQuregParams(Qureg qureg);

/* The number of qubits the register represents (N for an N-qubit density
 * matrix). */
int getNumQubits(Qureg qureg);

/* 2^N for an N-qubit state-vector.  Errors: E_DEFINED_ONLY_FOR_STATEVECS. */
int getNumAmps(Qureg qureg);

/* ------------------------------------------------------------------------ */
/* state initialisation                                                     */
/* ------------------------------------------------------------------------ */

/* |0...0> (state-vector) or |0...0><0...0| (density matrix).  Discards any
 * queued operations' effect by overwriting the state. */
void initZeroState(Qureg qureg);

/* |+>^N = 2^(-N/2) sum_i |i> (state-vector) or the uniform density matrix
 * with every element 1/2^N. */
void initPlusState(Qureg qureg);

/* The computational basis state |stateInd> (or |stateInd><stateInd|).
 * Errors: E_INVALID_STATE_INDEX (stateInd outside [0, 2^N)). */
void initClassicalState(Qureg qureg, long long int stateInd);

/* qureg := pure (state-vector) or |pure><pure| (density matrix); pure must
 * be a state-vector with the same number of qubits.  Collective.
 * Errors: E_SECOND_ARG_MUST_BE_STATEVEC, E_MISMATCHING_QUREG_DIMENSIONS. */
void initPureState(Qureg qureg, Qureg pure);

/* Overwrite the whole state-vector from host arrays of 2^N reals and
 * imaginaries (on every rank: each rank copies its own chunk).  No
 * normalisation is checked.  Errors: E_DEFINED_ONLY_FOR_STATEVECS. */
void initStateFromAmps(Qureg qureg, qreal* reals, qreal* imags);

/* Overwrite numAmps amplitudes starting at flat index startInd from host
 * arrays (all ranks pass the same arrays).
 * Errors: E_DEFINED_ONLY_FOR_STATEVECS, E_INVALID_STATE_INDEX,
 * E_INVALID_NUM_AMPS, E_INVALID_OFFSET_NUM_AMPS. */
void setAmps(Qureg qureg, long long int startInd, qreal* reals, qreal* imags, long long int numAmps);

/* targetQureg := copyQureg (device-to-device copy, both of the same type
 * and size).  Errors: E_MISMATCHING_QUREG_TYPES,
 * E_MISMATCHING_QUREG_DIMENSIONS. */
void cloneQureg(Qureg targetQureg, Qureg copyQureg);

/* ------------------------------------------------------------------------ */
/* phase gates (diagonal: never move data between ranks)                   */
/* ------------------------------------------------------------------------ */

/* Multiply the amplitudes whose targetQubit is 1 by exp(i angle).
 * Errors: E_INVALID_TARGET_QUBIT. */
void phaseShift(Qureg qureg, const int targetQubit, qreal angle);

/* Multiply the amplitudes where both qubits are 1 by exp(i angle) (the gate
 * is symmetric in its two qubits).  Errors: E_INVALID_TARGET_QUBIT,
 * E_INVALID_CONTROL_QUBIT, E_TARGET_IS_CONTROL. */
void controlledPhaseShift(Qureg qureg, const int idQubit1, const int idQubit2, qreal angle);

/* Multiply the amplitudes where every listed qubit is 1 by exp(i angle).
 * Errors: E_INVALID_NUM_CONTROLS (numControlQubits < 1 or > N),
 * E_INVALID_CONTROL_QUBIT. */
void multiControlledPhaseShift(Qureg qureg, int* controlQubits, int numControlQubits, qreal angle);

/* Controlled-Z: negate the amplitudes where both qubits are 1.  Errors as
 * controlledPhaseShift. */
void controlledPhaseFlip(Qureg qureg, const int idQubit1, const int idQubit2);

/* Negate the amplitudes where every listed qubit is 1.  Errors as
 * multiControlledPhaseShift. */
void multiControlledPhaseFlip(Qureg qureg, int* controlQubits, int numControlQubits);

/* S = diag(1, i) on targetQubit.  Errors: E_INVALID_TARGET_QUBIT. */
void sGate(Qureg qureg, const int targetQubit);

/* T = diag(1, exp(i pi/4)) on targetQubit.  Errors: E_INVALID_TARGET_QUBIT. */
void tGate(Qureg qureg, const int targetQubit);

/* ------------------------------------------------------------------------ */
/* environment                                                              */
/* ------------------------------------------------------------------------ */

/* Initialise this process: select the GPU (LOCAL_RANK modulo the visible
 * devices), and when launched with WORLD_SIZE > 1 (torchrun-style RANK /
 * WORLD_SIZE / MASTER_ADDR / MASTER_PORT) bring up the RCCL communicator;
 * seed the RNG from time and pid, broadcast from rank 0 so every rank draws
 * the same measurement outcomes.  Call once, before any register.
 * Collective. */
QuESTEnv createQuESTEnv(void);

/* Wait for all device work and tear down the communicator and device
 * state.  Collective. */
void destroyQuESTEnv(QuESTEnv env);

/* Block until every queued operation of every register has completed on
 * this rank, then barrier over ranks.  Collective. */
void syncQuESTEnv(QuESTEnv env);

/* Logical AND of successCode over all ranks (1 if every rank passed a
 * non-zero code).  Collective. */
int syncQuESTSuccess(int successCode);

/* Print the backend (HIP device, CU count, HBM; or host build), the number
 * of ranks, the transport and the precision (rank 0). */
void reportQuESTEnv(QuESTEnv env);

/* Write "<N>qubits_<backend>_<ranks>ranks" (at most 200 chars) into str. */
void getEnvironmentString(QuESTEnv env, Qureg qureg, char str[200]);

/* ------------------------------------------------------------------------ */
/* amplitude access and calculations                                        */
/* ------------------------------------------------------------------------ */

/* Amplitude <index|psi> of a state-vector (read on its owner rank and
 * broadcast; collective).  Errors: E_DEFINED_ONLY_FOR_STATEVECS,
 * E_INVALID_STATE_INDEX. */
Complex getAmp(Qureg qureg, long long int index);

/* Real part of getAmp.  Same errors. */
qreal getRealAmp(Qureg qureg, long long int index);

/* Imaginary part of getAmp.  Same errors. */
qreal getImagAmp(Qureg qureg, long long int index);

/* |getAmp|^2.  Same errors. */
qreal getProbAmp(Qureg qureg, long long int index);

/* Element rho(row, col) of a density matrix (collective).
 * Errors: E_DEFINED_ONLY_FOR_DENSMATRS, E_INVALID_STATE_INDEX. */
Complex getDensityAmp(Qureg qureg, long long int row, long long int col);

/* Sum of |amp|^2 (state-vector) or the real part of the trace (density
 * matrix), accumulated in fp64 on the device.  Collective. */
qreal calcTotalProb(Qureg qureg);

/* ------------------------------------------------------------------------ */
/* single-qubit and controlled unitaries                                    */
/* ------------------------------------------------------------------------ */

/* U = [[alpha, -conj(beta)], [beta, conj(alpha)]] on targetQubit.
 * Errors: E_INVALID_TARGET_QUBIT, E_NON_UNITARY_COMPLEX_PAIR
 * (|alpha|^2 + |beta|^2 != 1 beyond REAL_EPS). */
void compactUnitary(Qureg qureg, const int targetQubit, Complex alpha, Complex beta);

/* Any 2x2 unitary u on targetQubit.
 * Errors: E_INVALID_TARGET_QUBIT, E_NON_UNITARY_MATRIX. */
void unitary(Qureg qureg, const int targetQubit, ComplexMatrix2 u);

/* Rx(angle) = exp(-i angle X / 2) = [[cos a/2, -i sin a/2], [-i sin a/2, cos a/2]].
 * Errors: E_INVALID_TARGET_QUBIT. */
void rotateX(Qureg qureg, const int rotQubit, qreal angle);

/* Ry(angle) = exp(-i angle Y / 2) = [[cos a/2, -sin a/2], [sin a/2, cos a/2]].
 * Errors: E_INVALID_TARGET_QUBIT. */
void rotateY(Qureg qureg, const int rotQubit, qreal angle);

/* Rz(angle) = exp(-i angle Z / 2) = diag(exp(-i a/2), exp(i a/2)).
 * Errors: E_INVALID_TARGET_QUBIT. */
void rotateZ(Qureg qureg, const int rotQubit, qreal angle);

/* exp(-i angle (n . sigma) / 2) about the normalised axis n.
 * Errors: E_INVALID_TARGET_QUBIT, E_ZERO_VECTOR. */
void rotateAroundAxis(Qureg qureg, const int rotQubit, qreal angle, Vector axis);

/* rotateX on targetQubit where controlQubit is 1.  Errors:
 * E_INVALID_TARGET_QUBIT, E_INVALID_CONTROL_QUBIT, E_TARGET_IS_CONTROL. */
void controlledRotateX(Qureg qureg, const int controlQubit, const int targetQubit, qreal angle);

/* rotateY where controlQubit is 1.  Errors as controlledRotateX. */
void controlledRotateY(Qureg qureg, const int controlQubit, const int targetQubit, qreal angle);

/* rotateZ where controlQubit is 1.  Errors as controlledRotateX. */
void controlledRotateZ(Qureg qureg, const int controlQubit, const int targetQubit, qreal angle);

/* rotateAroundAxis where controlQubit is 1.  Errors as controlledRotateX and
 * E_ZERO_VECTOR. */
void controlledRotateAroundAxis(Qureg qureg, const int controlQubit, const int targetQubit, qreal angle, Vector axis);

/* compactUnitary where controlQubit is 1.  Errors as controlledRotateX and
 * E_NON_UNITARY_COMPLEX_PAIR. */
void controlledCompactUnitary(Qureg qureg, const int controlQubit, const int targetQubit, Complex alpha, Complex beta);

/* unitary where controlQubit is 1.  Errors as controlledRotateX and
 * E_NON_UNITARY_MATRIX. */
void controlledUnitary(Qureg qureg, const int controlQubit, const int targetQubit, ComplexMatrix2 u);

/* unitary on targetQubit where every control qubit is 1.  Errors:
 * E_INVALID_NUM_CONTROLS (< 1 or > N), E_INVALID_CONTROL_QUBIT,
 * E_INVALID_TARGET_QUBIT, E_TARGET_IN_CONTROLS, E_NON_UNITARY_MATRIX. */
void multiControlledUnitary(Qureg qureg, int* controlQubits, const int numControlQubits, const int targetQubit, ComplexMatrix2 u);

/* Pauli X (NOT).  On a rank-held (global) qubit this relabels chunks
 * instead of moving data.  Errors: E_INVALID_TARGET_QUBIT. */
void pauliX(Qureg qureg, const int targetQubit);

/* Pauli Y = [[0, -i], [i, 0]] (density matrices: conj(Y) on the column
 * qubit).  Errors: E_INVALID_TARGET_QUBIT. */
void pauliY(Qureg qureg, const int targetQubit);

/* Pauli Z = diag(1, -1).  Errors: E_INVALID_TARGET_QUBIT. */
void pauliZ(Qureg qureg, const int targetQubit);

/* Hadamard (|0> + |1>)/sqrt2, (|0> - |1>)/sqrt2.  Errors:
 * E_INVALID_TARGET_QUBIT. */
void hadamard(Qureg qureg, const int targetQubit);

/* CNOT: flip targetQubit where controlQubit is 1.  Errors:
 * E_INVALID_TARGET_QUBIT, E_INVALID_CONTROL_QUBIT, E_TARGET_IS_CONTROL. */
void controlledNot(Qureg qureg, const int controlQubit, const int targetQubit);

/* Pauli Y on targetQubit where controlQubit is 1.  Errors as controlledNot. */
void controlledPauliY(Qureg qureg, const int controlQubit, const int targetQubit);

/* ------------------------------------------------------------------------ */
/* measurement                                                              */
/* ------------------------------------------------------------------------ */

/* Probability that measuring measureQubit gives outcome: the sum of |amp|^2
 * over amplitudes with that bit (state-vector) or of the diagonal elements
 * (density matrix); outcome 1 is computed as total - P(0), as in the
 * reference.  A second query of the same state computes every qubit's
 * marginal in one pass and caches them until the state changes.
 * Collective.  Errors: E_INVALID_TARGET_QUBIT, E_INVALID_QUBIT_OUTCOME. */
qreal calcProbOfOutcome(Qureg qureg, const int measureQubit, int outcome);

/* Project measureQubit onto outcome and renormalise (state-vector: divide
 * by sqrt(p); density matrix: by p); returns p.  Collective.
 * Errors: E_INVALID_TARGET_QUBIT, E_INVALID_QUBIT_OUTCOME,
 * E_COLLAPSE_STATE_ZERO_PROB (p < REAL_EPS). */
qreal collapseToOutcome(Qureg qureg, const int measureQubit, int outcome);

/* Measure measureQubit: draw the outcome from the seeded MT19937 stream
 * with P(0) = calcProbOfOutcome(.., 0), collapse, return the outcome.
 * Every rank draws the same outcome.  Collective.
 * Errors: E_INVALID_TARGET_QUBIT. */
int measure(Qureg qureg, int measureQubit);

/* measure, also returning the outcome's probability in *outcomeProb. */
int measureWithStats(Qureg qureg, int measureQubit, qreal* outcomeProb);

/* <bra|ket> = sum conj(bra_i) ket_i of two state-vectors of equal size
 * (fp64 accumulation, one pass).  Collective.
 * Errors: E_DEFINED_ONLY_FOR_STATEVECS, E_MISMATCHING_QUREG_DIMENSIONS. */
Complex calcInnerProduct(Qureg bra, Qureg ket);

/* ------------------------------------------------------------------------ */
/* random numbers (MT19937, bit-compatible with the reference)              */
/* ------------------------------------------------------------------------ */

/* Seed from the current time (ms) and the process id; rank 0's seed is
 * broadcast to every rank.  Collective. */
void seedQuESTDefault(void);

/* Seed with init_by_array(seedArray, numSeeds): the same outcome sequence
 * as the reference for the same seeds. */
void seedQuEST(unsigned long int* seedArray, int numSeeds);

/* ------------------------------------------------------------------------ */
/* QASM recording                                                           */
/* ------------------------------------------------------------------------ */

/* Start appending OPENQASM 2.0 lines for every subsequent operation on the
 * register (header "OPENQASM 2.0;", qreg / creg declarations). */
void startRecordingQASM(Qureg qureg);

/* Stop recording (the text recorded so far is kept). */
void stopRecordingQASM(Qureg qureg);

/* Discard the recorded text, keeping the header. */
void clearRecordedQASM(Qureg qureg);

/* Print the recorded text to stdout (rank 0). */
void printRecordedQASM(Qureg qureg);

/* Write the recorded text to filename (rank 0).
 * Errors: E_CANNOT_OPEN_FILE. */
void writeRecordedQASMToFile(Qureg qureg, char* filename);

/* ------------------------------------------------------------------------ */
/* decoherence (density matrices only)                                      */
/* ------------------------------------------------------------------------ */

/* Dephasing: rho -> (1-prob) rho + prob Z rho Z on targetQubit, i.e. the
 * off-diagonal blocks scale by 1 - 2 prob.  prob in [0, 1/2].
 * Errors: E_DEFINED_ONLY_FOR_DENSMATRS, E_INVALID_TARGET_QUBIT,
 * E_INVALID_PROB, E_INVALID_ONE_QUBIT_DEPHASE_PROB. */
void applyOneQubitDephaseError(Qureg qureg, const int targetQubit, qreal prob);

/* Two-qubit dephasing: rho -> (1-prob) rho + prob/3 (Z1 rho Z1 + Z2 rho Z2 +
 * Z1Z2 rho Z1Z2): elements whose (row, column) bits differ on either qubit
 * scale by 1 - 4 prob / 3.  prob in [0, 3/4].  Errors as above with
 * E_TARGETS_NOT_UNIQUE and E_INVALID_TWO_QUBIT_DEPHASE_PROB. */
void applyTwoQubitDephaseError(Qureg qureg, const int qubit1, const int qubit2, qreal prob);

/* Depolarising: rho -> (1-prob) rho + prob/3 (X rho X + Y rho Y + Z rho Z).
 * prob in [0, 3/4] (3/4 maximally mixes).  Errors as
 * applyOneQubitDephaseError with E_INVALID_ONE_QUBIT_DEPOL_PROB. */
void applyOneQubitDepolariseError(Qureg qureg, const int targetQubit, qreal prob);

/* Amplitude damping with decay probability prob in [0, 1]: Kraus operators
 * [[1, 0], [0, sqrt(1-prob)]] and [[0, sqrt(prob)], [0, 0]].  (The
 * reference reports a prob > 1 with the depolarising error code; so does
 * this implementation.) */
void applyOneQubitDampingError(Qureg qureg, const int targetQubit, qreal prob);

/* Two-qubit depolarising: rho -> (1-prob) rho + prob/15 sum over the 15
 * non-identity two-qubit Paulis P rho P.  prob in [0, 15/16].  Errors as
 * applyTwoQubitDephaseError with E_INVALID_TWO_QUBIT_DEPOL_PROB. */
void applyTwoQubitDepolariseError(Qureg qureg, const int qubit1, const int qubit2, qreal prob);

/* combineQureg := (1-prob) combineQureg + prob otherQureg (density matrices
 * of equal size, one streaming pass).  Errors: E_DEFINED_ONLY_FOR_DENSMATRS,
 * E_MISMATCHING_QUREG_DIMENSIONS, E_INVALID_PROB. */
void addDensityMatrix(Qureg combineQureg, qreal prob, Qureg otherQureg);

/* Purity Tr(rho^2) = sum |rho_ij|^2.  Collective.
 * Errors: E_DEFINED_ONLY_FOR_DENSMATRS. */
qreal calcPurity(Qureg qureg);

/* |<pureState|qureg>|^2 (state-vector) or <pureState|rho|pureState>
 * (density matrix; the pure state is gathered onto every rank).  Collective.
 * Errors: E_SECOND_ARG_MUST_BE_STATEVEC, E_MISMATCHING_QUREG_DIMENSIONS. */
qreal calcFidelity(Qureg qureg, Qureg pureState);

#ifdef __cplusplus
}
#endif

#endif /* QUEST_H */
