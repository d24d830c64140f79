// QuEST.h front-end: validate -> route -> record QASM.
//
// Semantics follow the reference front-end (QuEST/src/QuEST.c:28-726) and
// its hardware-agnostic layer (QuEST/src/QuEST_common.c:153-326): a density
// matrix rho of N qubits is a 2N-qubit vector and U rho U^dag is applied as U
// on the row qubit t and conj(U) on the column qubit t+N.  Every unitary is
// lowered to one of four backend op kinds (src/core/core.hpp) instead of the
// reference's ~40 per-gate backend entry points.
#include <sys/time.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
#include <string>
#include <vector>

#include "QuEST.h"
#include "QuEST_debug.h"
#include "quest_amd.h"

#include "../comm/comm.hpp"
#include "../core/backend.hpp"
#include "../core/router.hpp"
#include "../core/tiles.hpp"
#include "../core/wave.hpp"
#include "common.hpp"
#include "qasm.hpp"
#include "validation.hpp"

extern "C" void init_by_array(unsigned long init_key[], int key_length);

using namespace qa;

namespace qa {
Runtime& rt() {
    static Runtime r;
    return r;
}
}  // namespace qa

namespace {

std::set<QuregImpl*>& liveQuregs() {
    static std::set<QuregImpl*> s;
    return s;
}

unsigned long g_seeds[64];
int g_numSeeds = 0;

inline QuregImpl& Q(const Qureg& q) { return *impl(q); }

inline cplx C(Complex z) { return {z.real, z.imag}; }

void fillQuregStruct(Qureg& q, QuregImpl& m) {
    memset(&q, 0, sizeof q);
    q.isDensityMatrix = m.isDensity ? 1 : 0;
    q.numQubitsRepresented = m.nRep;
    q.numQubitsInStateVec = m.nSV;
    q.numAmpsPerChunk = m.numAmpsPerChunk;
    q.numAmpsTotal = m.numAmpsTotal;
    q.chunkId = m.chunkId;
    q.numChunks = m.numChunks;
    if (be::stateOnHost()) {
        q.stateVec.real = m.re;
        q.stateVec.imag = m.im;
    } else {
        q.deviceStateVec.real = m.re;
        q.deviceStateVec.imag = m.im;
        q.stateVec.real = m.hostRe;
        q.stateVec.imag = m.hostIm;
    }
    q.qasmLog = &m.log;
}

// The per-rank memory a register needs (router::memoryPlan) against what
// the device has free: fail with the breakdown rather than die in hipMalloc
// or, for distributed registers, at the first swap's buffer allocation.
bool memoryBudget(int nSV, const char* caller) {
    const router::MemoryPlan m = router::memoryPlan(nSV, rt().numRanks);
    size_t freeB = 0, totalB = 0;
    bool known = be::memoryInfo(&freeB, &totalB);
    if (const char* e = getenv("QUEST_DEVICE_MEM_MB")) {
        freeB = (size_t)atoll(e) << 20;
        known = true;
    }
    int fits = !known || (long long)freeB >= m.total;
    // every rank takes the same decision (ranks sharing one GPU see
    // different free amounts): one rank returning an empty Qureg while the
    // others go on into collectives would hang the job
    if (comm::active()) fits = comm::allreduceAnd(fits);
    if (fits) return true;
    char detail[256];
    const double G = 1024.0 * 1024 * 1024;
    snprintf(detail, sizeof detail,
             "%d qubits on %d rank(s) need %.2f GiB per rank: state %.2f + exchange buffers %.2f + scratch %.2f; "
             "%.2f GiB free",
             nSV, rt().numRanks, m.total / G, m.state / G, m.exchange / G, m.scratch / G, freeB / G);
    return raiseErrorMsg(E_OUT_OF_MEMORY, caller, detail);
}

Qureg makeQureg(int nSV, bool density, int nRep) {
    QuregImpl* m = new QuregImpl();
    m->magic = kQuregMagic;
    router::create(*m, nSV, density);
    qasm::setup(&m->log, nRep);
    if (!be::stateOnHost()) {
        const char* mirror = getenv("QUEST_HOST_MIRROR");
        if (mirror && atoi(mirror)) {
            m->hostRe = (real*)calloc((size_t)m->numAmpsPerChunk, sizeof(real));
            m->hostIm = (real*)calloc((size_t)m->numAmpsPerChunk, sizeof(real));
        }
    }
    liveQuregs().insert(m);
    Qureg q;
    fillQuregStruct(q, *m);
    return q;
}

const cplx kX[4] = {{0, 0}, {1, 0}, {1, 0}, {0, 0}};
const cplx kY[4] = {{0, 0}, {0, -1}, {0, 1}, {0, 0}};
const cplx kYConj[4] = {{0, 0}, {0, 1}, {0, -1}, {0, 0}};

void conj4(const cplx in[4], cplx out[4]) {
    for (int i = 0; i < 4; i++) out[i] = cconj(in[i]);
}

void compactMatrix(Complex a, Complex b, cplx m[4]) {
    m[0] = {a.real, a.imag};
    m[1] = {-b.real, b.imag};  // -conj(beta)
    m[2] = {b.real, b.imag};
    m[3] = {a.real, -a.imag};  // conj(alpha)
}

void unitaryMatrix(const ComplexMatrix2& u, cplx m[4]) {
    m[0] = C(u.r0c0);
    m[1] = C(u.r0c1);
    m[2] = C(u.r1c0);
    m[3] = C(u.r1c1);
}

// apply a (multi-)controlled 2x2 matrix; density: also conj(m) on shifted qubits
void applyMat2(const Qureg& qu, int target, const int* ctrls, int nc, const cplx m[4], const cplx* mConj = nullptr) {
    QuregImpl& q = Q(qu);
    router::mat2(q, target, ctrls, nc, m);
    if (q.isDensity) {
        int sh = q.nRep;
        std::vector<int> c2(ctrls, ctrls + nc);
        for (int& c : c2) c += sh;
        cplx mc[4];
        if (mConj)
            for (int i = 0; i < 4; i++) mc[i] = mConj[i];
        else
            conj4(m, mc);
        router::mat2(q, target + sh, c2.data(), nc, mc);
    }
}

void applyDiag(const Qureg& qu, const int* qubits, int nq, cplx term) {
    QuregImpl& q = Q(qu);
    router::diag(q, qubits, nq, term);
    if (q.isDensity) {
        std::vector<int> s(qubits, qubits + nq);
        for (int& x : s) x += q.nRep;
        router::diag(q, s.data(), nq, cconj(term));
    }
}

void rotationMatrix(qreal angle, Vector axis, cplx m[4]) {
    Complex a, b;
    complexPairFromRotation(angle, axis, &a, &b);
    compactMatrix(a, b, m);
}

void realMat4(QuregImpl& q, int t, const real r[16]) {
    cplx m[16];
    for (int i = 0; i < 16; i++) m[i] = {r[i], 0};
    router::mat4(q, t, t + q.nRep, m);
}

int seedFromEnvOrTime(unsigned long key[2]) {
    struct timeval tv;
    gettimeofday(&tv, nullptr);
    double ms = (double)tv.tv_sec * 1000 + (double)(tv.tv_usec / 1000);
    key[0] = (unsigned long)ms;
    key[1] = (unsigned long)getpid();
    return 2;
}

void readEnvConfig() {
    if (const char* f = getenv("QUEST_FUSION")) rt().fusion = atoi(f) != 0;
    if (const char* k = getenv("QUEST_FUSE_QUBITS")) rt().fuseMaxQubits = atoi(k);
    if (const char* v = getenv("QUEST_VERIFY")) rt().verify = atoi(v) != 0;
    if (const char* v = getenv("QUEST_WAVE_SHADOW")) rt().waveShadow = atoi(v) != 0;
    if (const char* t = getenv("QUEST_VERIFY_TOL")) rt().verifyTol = atof(t);
    if (const char* s = getenv("QUEST_EXCHANGE_SLICE_MB")) {
        long long mb = atoll(s);
        if (mb > 0) rt().exchangeSliceBytes = mb << 20;
    }
    if (const char* s = getenv("QUEST_EXCHANGE_SLICE_KB")) {  // tests: many slices on small registers
        long long kb = atoll(s);
        if (kb > 0) rt().exchangeSliceBytes = kb << 10;
    }
}

}  // namespace

extern "C" {

// ===========================================================================
// environment
// ===========================================================================

QuESTEnv createQuESTEnv(void) {
    QuESTEnv env;
    if (!rt().initialised) {
        int rank, size, local;
        comm::discover(&rank, &size, &local);
        rt().rank = rank;
        rt().numRanks = size;
        rt().localRank = local;
        readEnvConfig();
        be::envInit(rank, size, local);
        comm::init(rank, size);
        rt().initialised = true;
        seedQuESTDefault();
    }
    env.rank = rt().rank;
    env.numRanks = rt().numRanks;
    return env;
}

void destroyQuESTEnv(QuESTEnv env) {
    (void)env;
    if (!rt().initialised) return;
    for (QuregImpl* q : liveQuregs()) be::flush(*q);
    be::deviceSync();
    comm::finalize();
    be::envFinalize();
    rt().initialised = false;
}

void syncQuESTEnv(QuESTEnv env) {
    (void)env;
    for (QuregImpl* q : liveQuregs()) be::flush(*q);
    be::deviceSync();
    if (comm::active()) comm::barrier();
}

int syncQuESTSuccess(int successCode) {
    if (!comm::active()) return successCode;
    return comm::allreduceAnd(successCode);
}

void reportQuESTEnv(QuESTEnv env) {
    if (env.rank != 0) return;
    printf("EXECUTION ENVIRONMENT:\n");
    printf("Running %s backend: %s\n", be::shortName(), be::describe().c_str());
    printf("Number of ranks is %d\n", env.numRanks);
    printf("Communication: %s\n", comm::describe().c_str());
    printf("Precision: %d (%s)\n", QuEST_PREC, QuEST_PREC == 1 ? "single" : QuEST_PREC == 2 ? "double" : "quad");
    printf("Gate fusion %s\n", rt().fusion ? "enabled" : "disabled");
    fflush(stdout);
}

void getEnvironmentString(QuESTEnv env, Qureg qureg, char str[200]) {
    snprintf(str, 200, "%dqubits_%s_%dranks", qureg.numQubitsInStateVec, be::shortName(), env.numRanks);
}

void seedQuESTDefault(void) {
    unsigned long key[2];
    seedFromEnvOrTime(key);
    if (comm::active()) comm::bcastHost(key, sizeof key, 0);
    g_seeds[0] = key[0];
    g_seeds[1] = key[1];
    g_numSeeds = 2;
    init_by_array(key, 2);
}

void seedQuEST(unsigned long int* seedArray, int numSeeds) {
    g_numSeeds = std::min(numSeeds, 64);
    for (int i = 0; i < g_numSeeds; i++) g_seeds[i] = seedArray[i];
    init_by_array(seedArray, numSeeds);
}

// ===========================================================================
// registers
// ===========================================================================

Qureg createQureg(int numQubits, QuESTEnv env) {
    (void)env;
    Qureg q;
    memset(&q, 0, sizeof q);
    if (!v::createNumQubits(numQubits, rt().numRanks, __func__)) return q;
    if (!memoryBudget(numQubits, __func__)) return q;
    q = makeQureg(numQubits, false, numQubits);
    initZeroState(q);
    return q;
}

Qureg createDensityQureg(int numQubits, QuESTEnv env) {
    (void)env;
    Qureg q;
    memset(&q, 0, sizeof q);
    if (!v::createNumQubits(numQubits, 1, __func__)) return q;
    if (!v::createNumQubits(2 * numQubits, rt().numRanks, __func__)) return q;
    if (!memoryBudget(2 * numQubits, __func__)) return q;
    q = makeQureg(2 * numQubits, true, numQubits);
    initZeroState(q);
    return q;
}

void destroyQureg(Qureg qureg, QuESTEnv env) {
    (void)env;
    QuregImpl* m = impl(qureg);
    router::destroy(*m);
    qasm::release(&m->log);
    free(m->hostRe);
    free(m->hostIm);
    liveQuregs().erase(m);
    m->magic = 0;
    delete m;
}

void cloneQureg(Qureg targetQureg, Qureg copyQureg) {
    if (!v::matchingTypes(targetQureg, copyQureg, __func__)) return;
    if (!v::matchingDims(targetQureg, copyQureg, __func__)) return;
    router::clone(Q(targetQureg), Q(copyQureg));
}

int getNumQubits(Qureg qureg) { return qureg.numQubitsRepresented; }

int getNumAmps(Qureg qureg) {
    if (!v::stateVec(qureg, __func__)) return 0;
    return (int)qureg.numAmpsTotal;
}

// ===========================================================================
// reporting
// ===========================================================================

void reportState(Qureg qureg) {
    QuregImpl& q = Q(qureg);
    router::canonicalise(q);
    char name[100];
    snprintf(name, sizeof name, "state_rank_%d.csv", q.chunkId);
    FILE* f = fopen(name, "w");
    if (!f) return;
    if (q.chunkId == 0) fprintf(f, "real, imag\n");
    const i64 piece = 1 << 20;
    std::vector<real> re((size_t)std::min(piece, q.numAmpsPerChunk)), im(re.size());
    for (i64 off = 0; off < q.numAmpsPerChunk; off += piece) {
        i64 n = std::min(piece, q.numAmpsPerChunk - off);
        be::readAmps(q, off, re.data(), im.data(), n);
        for (i64 i = 0; i < n; i++) fprintf(f, "%.12f, %.12f\n", (double)re[i], (double)im[i]);
    }
    fclose(f);
}

void reportStateToScreen(Qureg qureg, QuESTEnv env, int reportRank) {
    QuregImpl& q = Q(qureg);
    if (q.nSV > 5) {
        // as the reference's host build (QuEST_cpu.c:1275); E_SYS_TOO_BIG_TO_PRINT is never raised there
        if (q.chunkId == 0) printf("Error: reportStateToScreen will not print output for systems of more than 5 qubits.\n");
        fflush(stdout);
        return;
    }
    std::vector<real> re((size_t)q.numAmpsPerChunk), im(re.size());
    router::readChunk(q, re.data(), im.data());
    for (int r = 0; r < q.numChunks; r++) {
        if (q.chunkId == r) {
            if (reportRank) {
                printf("Reporting state from rank %d [\n", q.chunkId);
                printf("real, imag\n");
            } else if (r == 0) {
                printf("Reporting state [\n");
                printf("real, imag\n");
            }
            for (i64 i = 0; i < q.numAmpsPerChunk; i++)
                printf(REAL_STRING_FORMAT ", " REAL_STRING_FORMAT "\n", re[i], im[i]);
            if (reportRank || r == q.numChunks - 1) printf("]\n");
            fflush(stdout);
        }
        syncQuESTEnv(env);
    }
}

void reportQuregParams(Qureg qureg) {
    long long numAmps = 1LL << qureg.numQubitsInStateVec;
    if (qureg.chunkId == 0) {
        printf("QUBITS:\n");
        printf("Number of qubits is %d.\n", qureg.numQubitsInStateVec);
        printf("Number of amps is %lld.\n", numAmps);
        printf("Number of amps per rank is %lld.\n", numAmps / qureg.numChunks);
        fflush(stdout);
    }
}

// ===========================================================================
// initialisation
// ===========================================================================

void initZeroState(Qureg qureg) {
    router::initClassical(Q(qureg), 0);
    qasm::initZero(qureg);
}

void initPlusState(Qureg qureg) {
    QuregImpl& q = Q(qureg);
    if (q.isDensity)
        router::initUniform(q, (real)1.0 / (real)(1LL << q.nRep));
    else
        router::initUniform(q, (real)1.0 / std::sqrt((real)q.numAmpsTotal));
    qasm::initPlus(qureg);
}

void initClassicalState(Qureg qureg, long long int stateInd) {
    if (!v::stateIndex(qureg, stateInd, __func__)) return;
    QuregImpl& q = Q(qureg);
    i64 flat = q.isDensity ? (((i64)1 << q.nRep) + 1) * stateInd : stateInd;
    router::initClassical(q, flat);
    qasm::initClassical(qureg, stateInd);
}

void initPureState(Qureg qureg, Qureg pure) {
    if (!v::secondStateVec(pure, __func__)) return;
    if (!v::matchingDims(qureg, pure, __func__)) return;
    QuregImpl& q = Q(qureg);
    if (q.isDensity)
        router::densInitPure(q, Q(pure));
    else
        router::clone(q, Q(pure));
    qasm::comment(qureg, "Here, the register was initialised to an undisclosed given pure state.");
}

void initStateFromAmps(Qureg qureg, qreal* reals, qreal* imags) {
    if (!v::stateVec(qureg, __func__)) return;
    router::setAmps(Q(qureg), 0, reals, imags, qureg.numAmpsTotal);
    qasm::comment(qureg, "Here, the register was initialised to an undisclosed given pure state.");
}

void setAmps(Qureg qureg, long long int startInd, qreal* reals, qreal* imags, long long int numAmps) {
    if (!v::stateVec(qureg, __func__)) return;
    if (!v::numAmps(qureg, startInd, numAmps, __func__)) return;
    router::setAmps(Q(qureg), startInd, reals, imags, numAmps);
    qasm::comment(qureg, "Here, some amplitudes in the statevector were manually edited.");
}

void setDensityAmps(Qureg qureg, qreal* reals, qreal* imags) {
    router::setAmps(Q(qureg), 0, reals, imags, qureg.numAmpsTotal);
    qasm::comment(qureg, "Here, some amplitudes in the density matrix were manually edited.");
}

// ===========================================================================
// unitaries
// ===========================================================================

void hadamard(Qureg qureg, const int targetQubit) {
    if (!v::target(qureg, targetQubit, __func__)) return;
    const real s = (real)(1.0 / std::sqrt(2.0));
    cplx m[4] = {{s, 0}, {s, 0}, {s, 0}, {-s, 0}};
    applyMat2(qureg, targetQubit, nullptr, 0, m);
    qasm::gate(qureg, qasm::G_HADAMARD, targetQubit);
}

void rotateX(Qureg qureg, const int targetQubit, qreal angle) {
    if (!v::target(qureg, targetQubit, __func__)) return;
    cplx m[4];
    rotationMatrix(angle, Vector{1, 0, 0}, m);
    applyMat2(qureg, targetQubit, nullptr, 0, m);
    qasm::paramGate(qureg, qasm::G_ROTATE_X, targetQubit, angle);
}

void rotateY(Qureg qureg, const int targetQubit, qreal angle) {
    if (!v::target(qureg, targetQubit, __func__)) return;
    cplx m[4];
    rotationMatrix(angle, Vector{0, 1, 0}, m);
    applyMat2(qureg, targetQubit, nullptr, 0, m);
    qasm::paramGate(qureg, qasm::G_ROTATE_Y, targetQubit, angle);
}

void rotateZ(Qureg qureg, const int targetQubit, qreal angle) {
    if (!v::target(qureg, targetQubit, __func__)) return;
    cplx m[4];
    rotationMatrix(angle, Vector{0, 0, 1}, m);
    applyMat2(qureg, targetQubit, nullptr, 0, m);
    qasm::paramGate(qureg, qasm::G_ROTATE_Z, targetQubit, angle);
}

void rotateAroundAxis(Qureg qureg, const int rotQubit, qreal angle, Vector axis) {
    if (!v::target(qureg, rotQubit, __func__)) return;
    if (!v::vector(axis, __func__)) return;
    cplx m[4];
    rotationMatrix(angle, axis, m);
    applyMat2(qureg, rotQubit, nullptr, 0, m);
    qasm::axisRotation(qureg, angle, axis, rotQubit);
}

static void controlledRotation(Qureg qureg, int c, int t, qreal angle, Vector axis) {
    cplx m[4];
    rotationMatrix(angle, axis, m);
    applyMat2(qureg, t, &c, 1, m);
}

void controlledRotateX(Qureg qureg, const int controlQubit, const int targetQubit, qreal angle) {
    if (!v::controlTarget(qureg, controlQubit, targetQubit, __func__)) return;
    controlledRotation(qureg, controlQubit, targetQubit, angle, Vector{1, 0, 0});
    qasm::controlledParamGate(qureg, qasm::G_ROTATE_X, controlQubit, targetQubit, angle);
}

void controlledRotateY(Qureg qureg, const int controlQubit, const int targetQubit, qreal angle) {
    if (!v::controlTarget(qureg, controlQubit, targetQubit, __func__)) return;
    controlledRotation(qureg, controlQubit, targetQubit, angle, Vector{0, 1, 0});
    qasm::controlledParamGate(qureg, qasm::G_ROTATE_Y, controlQubit, targetQubit, angle);
}

void controlledRotateZ(Qureg qureg, const int controlQubit, const int targetQubit, qreal angle) {
    if (!v::controlTarget(qureg, controlQubit, targetQubit, __func__)) return;
    controlledRotation(qureg, controlQubit, targetQubit, angle, Vector{0, 0, 1});
    qasm::controlledParamGate(qureg, qasm::G_ROTATE_Z, controlQubit, targetQubit, angle);
}

void controlledRotateAroundAxis(Qureg qureg, const int controlQubit, const int targetQubit, qreal angle,
                                Vector axis) {
    if (!v::controlTarget(qureg, controlQubit, targetQubit, __func__)) return;
    if (!v::vector(axis, __func__)) return;
    controlledRotation(qureg, controlQubit, targetQubit, angle, axis);
    qasm::controlledAxisRotation(qureg, angle, axis, controlQubit, targetQubit);
}

void unitary(Qureg qureg, const int targetQubit, ComplexMatrix2 u) {
    if (!v::target(qureg, targetQubit, __func__)) return;
    if (!v::unitaryMatrix(u, __func__)) return;
    cplx m[4];
    unitaryMatrix(u, m);
    applyMat2(qureg, targetQubit, nullptr, 0, m);
    qasm::unitary(qureg, u, targetQubit);
}

void controlledUnitary(Qureg qureg, const int controlQubit, const int targetQubit, ComplexMatrix2 u) {
    if (!v::controlTarget(qureg, controlQubit, targetQubit, __func__)) return;
    if (!v::unitaryMatrix(u, __func__)) return;
    cplx m[4];
    unitaryMatrix(u, m);
    int c = controlQubit;
    applyMat2(qureg, targetQubit, &c, 1, m);
    qasm::controlledUnitary(qureg, u, controlQubit, targetQubit);
}

void multiControlledUnitary(Qureg qureg, int* controlQubits, const int numControlQubits, const int targetQubit,
                            ComplexMatrix2 u) {
    if (!v::multiControlsTarget(qureg, controlQubits, numControlQubits, targetQubit, __func__)) return;
    if (!v::unitaryMatrix(u, __func__)) return;
    cplx m[4];
    unitaryMatrix(u, m);
    applyMat2(qureg, targetQubit, controlQubits, numControlQubits, m);
    qasm::multiControlledUnitary(qureg, u, controlQubits, numControlQubits, targetQubit);
}

void compactUnitary(Qureg qureg, const int targetQubit, Complex alpha, Complex beta) {
    if (!v::target(qureg, targetQubit, __func__)) return;
    if (!v::unitaryPair(alpha, beta, __func__)) return;
    cplx m[4];
    compactMatrix(alpha, beta, m);
    applyMat2(qureg, targetQubit, nullptr, 0, m);
    qasm::compactUnitary(qureg, alpha, beta, targetQubit);
}

void controlledCompactUnitary(Qureg qureg, const int controlQubit, const int targetQubit, Complex alpha,
                              Complex beta) {
    if (!v::controlTarget(qureg, controlQubit, targetQubit, __func__)) return;
    if (!v::unitaryPair(alpha, beta, __func__)) return;
    cplx m[4];
    compactMatrix(alpha, beta, m);
    int c = controlQubit;
    applyMat2(qureg, targetQubit, &c, 1, m);
    qasm::controlledCompactUnitary(qureg, alpha, beta, controlQubit, targetQubit);
}

void pauliX(Qureg qureg, const int targetQubit) {
    if (!v::target(qureg, targetQubit, __func__)) return;
    applyMat2(qureg, targetQubit, nullptr, 0, kX);
    qasm::gate(qureg, qasm::G_SIGMA_X, targetQubit);
}

void pauliY(Qureg qureg, const int targetQubit) {
    if (!v::target(qureg, targetQubit, __func__)) return;
    applyMat2(qureg, targetQubit, nullptr, 0, kY, kYConj);
    qasm::gate(qureg, qasm::G_SIGMA_Y, targetQubit);
}

void pauliZ(Qureg qureg, const int targetQubit) {
    if (!v::target(qureg, targetQubit, __func__)) return;
    int t = targetQubit;
    applyDiag(qureg, &t, 1, cplx{-1, 0});
    qasm::gate(qureg, qasm::G_SIGMA_Z, targetQubit);
}

void sGate(Qureg qureg, const int targetQubit) {
    if (!v::target(qureg, targetQubit, __func__)) return;
    int t = targetQubit;
    applyDiag(qureg, &t, 1, cplx{0, 1});
    qasm::gate(qureg, qasm::G_S, targetQubit);
}

void tGate(Qureg qureg, const int targetQubit) {
    if (!v::target(qureg, targetQubit, __func__)) return;
    int t = targetQubit;
    const real s = (real)(1.0 / std::sqrt(2.0));
    applyDiag(qureg, &t, 1, cplx{s, s});
    qasm::gate(qureg, qasm::G_T, targetQubit);
}

void phaseShift(Qureg qureg, const int targetQubit, qreal angle) {
    if (!v::target(qureg, targetQubit, __func__)) return;
    int t = targetQubit;
    applyDiag(qureg, &t, 1, cplx{(real)std::cos(angle), (real)std::sin(angle)});
    qasm::paramGate(qureg, qasm::G_PHASE_SHIFT, targetQubit, angle);
}

void controlledPhaseShift(Qureg qureg, const int idQubit1, const int idQubit2, qreal angle) {
    if (!v::controlTarget(qureg, idQubit1, idQubit2, __func__)) return;
    int qs[2] = {idQubit1, idQubit2};
    applyDiag(qureg, qs, 2, cplx{(real)std::cos(angle), (real)std::sin(angle)});
    qasm::controlledParamGate(qureg, qasm::G_PHASE_SHIFT, idQubit1, idQubit2, angle);
}

void multiControlledPhaseShift(Qureg qureg, int* controlQubits, int numControlQubits, qreal angle) {
    if (!v::multiControls(qureg, controlQubits, numControlQubits, __func__)) return;
    applyDiag(qureg, controlQubits, numControlQubits, cplx{(real)std::cos(angle), (real)std::sin(angle)});
    qasm::multiControlledParamGate(qureg, qasm::G_PHASE_SHIFT, controlQubits, numControlQubits - 1,
                                   controlQubits[numControlQubits - 1], angle);
}

void controlledNot(Qureg qureg, const int controlQubit, const int targetQubit) {
    if (!v::controlTarget(qureg, controlQubit, targetQubit, __func__)) return;
    int c = controlQubit;
    applyMat2(qureg, targetQubit, &c, 1, kX);
    qasm::controlledGate(qureg, qasm::G_SIGMA_X, controlQubit, targetQubit);
}

void controlledPauliY(Qureg qureg, const int controlQubit, const int targetQubit) {
    if (!v::controlTarget(qureg, controlQubit, targetQubit, __func__)) return;
    int c = controlQubit;
    applyMat2(qureg, targetQubit, &c, 1, kY, kYConj);
    qasm::controlledGate(qureg, qasm::G_SIGMA_Y, controlQubit, targetQubit);
}

void controlledPhaseFlip(Qureg qureg, const int idQubit1, const int idQubit2) {
    if (!v::controlTarget(qureg, idQubit1, idQubit2, __func__)) return;
    int qs[2] = {idQubit1, idQubit2};
    applyDiag(qureg, qs, 2, cplx{-1, 0});
    qasm::controlledGate(qureg, qasm::G_SIGMA_Z, idQubit1, idQubit2);
}

void multiControlledPhaseFlip(Qureg qureg, int* controlQubits, int numControlQubits) {
    if (!v::multiControls(qureg, controlQubits, numControlQubits, __func__)) return;
    applyDiag(qureg, controlQubits, numControlQubits, cplx{-1, 0});
    qasm::multiControlledGate(qureg, qasm::G_SIGMA_Z, controlQubits, numControlQubits - 1,
                              controlQubits[numControlQubits - 1]);
}

// ===========================================================================
// amplitudes and calculations
// ===========================================================================

qreal getRealAmp(Qureg qureg, long long int index) {
    if (!v::stateVec(qureg, __func__) || !v::stateIndex(qureg, index, __func__)) return 0;
    return router::getAmp(Q(qureg), index).re;
}

qreal getImagAmp(Qureg qureg, long long int index) {
    if (!v::stateVec(qureg, __func__) || !v::stateIndex(qureg, index, __func__)) return 0;
    return router::getAmp(Q(qureg), index).im;
}

qreal getProbAmp(Qureg qureg, long long int index) {
    if (!v::stateVec(qureg, __func__) || !v::stateIndex(qureg, index, __func__)) return 0;
    cplx a = router::getAmp(Q(qureg), index);
    return a.re * a.re + a.im * a.im;
}

Complex getAmp(Qureg qureg, long long int index) {
    Complex c = {0, 0};
    if (!v::stateVec(qureg, __func__) || !v::stateIndex(qureg, index, __func__)) return c;
    cplx a = router::getAmp(Q(qureg), index);
    c.real = a.re;
    c.imag = a.im;
    return c;
}

Complex getDensityAmp(Qureg qureg, long long int row, long long int col) {
    Complex c = {0, 0};
    if (!v::densMatr(qureg, __func__) || !v::stateIndex(qureg, row, __func__) ||
        !v::stateIndex(qureg, col, __func__))
        return c;
    long long ind = row + col * (1LL << qureg.numQubitsRepresented);
    cplx a = router::getAmp(Q(qureg), ind);
    c.real = a.re;
    c.imag = a.im;
    return c;
}

qreal calcTotalProb(Qureg qureg) {
    QuregImpl& q = Q(qureg);
    return q.isDensity ? (qreal)router::densTrace(q) : (qreal)router::sumSqAll(q);
}

Complex calcInnerProduct(Qureg bra, Qureg ket) {
    Complex c = {0, 0};
    if (!v::stateVec(bra, __func__) || !v::stateVec(ket, __func__) || !v::matchingDims(bra, ket, __func__))
        return c;
    cplx r = router::inner(Q(bra), Q(ket));
    c.real = r.re;
    c.imag = r.im;
    return c;
}

static qreal probOfOutcome(QuregImpl& q, int t, int outcome) {
    qreal p0 = q.isDensity ? (qreal)router::densProbZero(q, t) : (qreal)router::probZero(q, t);
    return outcome == 1 ? 1 - p0 : p0;
}

qreal calcProbOfOutcome(Qureg qureg, const int measureQubit, int outcome) {
    if (!v::target(qureg, measureQubit, __func__) || !v::outcome(outcome, __func__)) return 0;
    return probOfOutcome(Q(qureg), measureQubit, outcome);
}

static void collapseKnown(QuregImpl& q, int t, int outcome, qreal prob) {
    if (q.isDensity)
        router::densCollapse(q, t, outcome, prob);
    else
        router::collapse(q, t, outcome, (real)(1 / std::sqrt(prob)));
}

qreal collapseToOutcome(Qureg qureg, const int measureQubit, int outcome) {
    if (!v::target(qureg, measureQubit, __func__) || !v::outcome(outcome, __func__)) return 0;
    QuregImpl& q = Q(qureg);
    qreal p = probOfOutcome(q, measureQubit, outcome);
    if (!v::measurementProb(p, __func__)) return 0;
    collapseKnown(q, measureQubit, outcome, p);
    qasm::measurement(qureg, measureQubit);
    return p;
}

int measureWithStats(Qureg qureg, int measureQubit, qreal* outcomeProb) {
    if (!v::target(qureg, measureQubit, __func__)) return 0;
    QuregImpl& q = Q(qureg);
    qreal zeroProb = probOfOutcome(q, measureQubit, 0);
    int outcome = generateMeasurementOutcome(zeroProb, outcomeProb);
    collapseKnown(q, measureQubit, outcome, *outcomeProb);
    qasm::measurement(qureg, measureQubit);
    return outcome;
}

int measure(Qureg qureg, int measureQubit) {
    qreal discarded;
    return measureWithStats(qureg, measureQubit, &discarded);
}

qreal calcPurity(Qureg qureg) {
    if (!v::densMatr(qureg, __func__)) return 0;
    return (qreal)router::sumSqAll(Q(qureg));
}

qreal calcFidelity(Qureg qureg, Qureg pureState) {
    if (!v::secondStateVec(pureState, __func__) || !v::matchingDims(qureg, pureState, __func__)) return 0;
    QuregImpl& q = Q(qureg);
    if (q.isDensity) return (qreal)router::densFidelity(q, Q(pureState));
    cplx ip = router::inner(q, Q(pureState));
    return ip.re * ip.re + ip.im * ip.im;
}

void addDensityMatrix(Qureg combineQureg, qreal otherProb, Qureg otherQureg) {
    if (!v::densMatr(combineQureg, __func__) || !v::densMatr(otherQureg, __func__) ||
        !v::matchingDims(combineQureg, otherQureg, __func__) || !v::prob(otherProb, __func__))
        return;
    router::axpby(Q(combineQureg), 1 - otherProb, Q(otherQureg), otherProb);
}

// ===========================================================================
// decoherence
// ===========================================================================

// Dephasing strengths whose factor is at least this large run as diagonal
// ops (their inverse powers stay well inside the range of qreal); stronger
// dephasing keeps the channel form.
// QUEST_DEPHASE_DIAG=0 keeps the channel forms (A/B).
// fp64 / long double only: the diagonal form multiplies the populations by factors whose
// product is 1 only up to rounding (two factors for one qubit, fifteen up to
// g^-4 for two), about 1e-16 relative in fp64 but 1e-7 in fp32, where the
// channel forms (which never touch the populations) are kept.
constexpr double kDiagDephaseMin = 1e-3;
bool dephaseDiag() {
    static const bool on = sizeof(real) >= 8 &&
                           (!getenv("QUEST_DEPHASE_DIAG") || atoi(getenv("QUEST_DEPHASE_DIAG")) != 0);
    return on;
}

// Two-qubit channels as one-qubit ops (QUEST_CHAN2_GATES=0: the 16-element
// channel op of the LDS kernel instead).  In the "differs" frame -- c1 ^= r1,
// c2 ^= r2 by CNOTs, so c1 / c2 tell whether row and column bits differ --
// the channels become a phase-free diagonal on the coherences and real 2x2
// mixes of the populations controlled on c1 = c2 = 0; every op is a wave-
// engine op (CNOTs, Xs that the wave planner defers to its exchange frame,
// diagonal factors, controlled real 2x2), so the channels fuse with the gates
// around them in register-resident passes, and the populations are never
// multiplied by anything but the channel's own coefficients.
bool twoQubitChannelsAsGates() {
    static const bool on = !getenv("QUEST_CHAN2_GATES") || atoi(getenv("QUEST_CHAN2_GATES")) != 0;
    return on;
}

// Enter (undo = false) or leave the differs frame.  Entering leaves c1 and c2
// flipped (X), so that c1 = c2 = 1 marks the populations.
void differsFrame(QuregImpl& q, int r1, int r2, int c1, int c2, bool undo) {
    if (!undo) {
        router::mat2(q, c1, &r1, 1, kX);
        router::mat2(q, c2, &r2, 1, kX);
        router::mat2(q, c1, nullptr, 0, kX);
        router::mat2(q, c2, nullptr, 0, kX);
    } else {
        router::mat2(q, c1, nullptr, 0, kX);
        router::mat2(q, c2, nullptr, 0, kX);
        router::mat2(q, c2, &r2, 1, kX);
        router::mat2(q, c1, &r1, 1, kX);
    }
}

// Factor g on the elements with (r1, r2) != (c1, c2): in the differs frame
// g on c1 = 0 (row and column of qubit 1 differ), then g on c1 = 1, c2 = 0.
// leave = true returns to the plain frame; false stays in it (c1, c2 flipped).
void twoQubitDephaseAsGates(QuregImpl& q, int r1, int r2, int c1, int c2, real g, bool leave) {
    router::mat2(q, c1, &r1, 1, kX);
    router::mat2(q, c2, &r2, 1, kX);
    router::diag(q, &c1, 1, {g, 0});                 // qubit 1 differs
    router::mat2(q, c1, nullptr, 0, kX);
    const int both[2] = {c1, c2};
    router::diag(q, both, 2, {g, 0});                // qubit 1 agrees, qubit 2 differs
    router::mat2(q, c2, nullptr, 0, kX);            // c1 = c2 = 1: populations
    if (leave) differsFrame(q, r1, r2, c1, c2, true);
}

void applyOneQubitDephaseError(Qureg qureg, const int targetQubit, qreal prob) {
    if (!v::densMatr(qureg, __func__) || !v::target(qureg, targetQubit, __func__) ||
        !v::oneQubitDephaseProb(prob, __func__))
        return;
    real dephase = 2 * prob;
    if (dephase == 0) return;
    real f = 1 - dephase;
    QuregImpl& q = Q(qureg);
    if (dephaseDiag() && std::fabs(f) >= kDiagDephaseMin) {
        // f on the elements whose row and column bits differ, as three
        // diagonal ops (factors on all-ones masks: f^r f^c f^(-2rc)); they
        // need no tile bits, so they fuse into any pass instead of forming a
        // (row, column) channel that needs both bits in one tile
        const int r = targetQubit, c = targetQubit + q.nRep, rc[2] = {r, c};
        router::diag(q, &r, 1, {f, 0});
        router::diag(q, &c, 1, {f, 0});
        router::diag(q, rc, 2, {1 / (f * f), 0});
        return;
    }
    const real m[16] = {1, 0, 0, 0, 0, f, 0, 0, 0, 0, f, 0, 0, 0, 0, 1};
    realMat4(q, targetQubit, m);
}

void applyTwoQubitDephaseError(Qureg qureg, int qubit1, int qubit2, qreal prob) {
    if (!v::densMatr(qureg, __func__) || !v::uniqueTargets(qureg, qubit1, qubit2, __func__) ||
        !v::twoQubitDephaseProb(prob, __func__))
        return;
    if (qubit1 > qubit2) std::swap(qubit1, qubit2);
    real d = (4 * prob) / 3.0;
    if (d == 0) return;
    QuregImpl& q = Q(qureg);
    const real g = 1 - d;
    if (dephaseDiag() && std::fabs(g) >= kDiagDephaseMin) {
        // g on the elements with (r1, r2) != (c1, c2): g^(1 - [r1==c1][r2==c2])
        // expanded over the bits into factors g^e on all-ones masks (15
        // diagonal ops that fuse into any pass, as for one qubit)
        const int r1 = qubit1, r2 = qubit2, c1 = qubit1 + q.nRep, c2 = qubit2 + q.nRep;
        struct Term {
            int n, e;
            int b[4];
        };
        const Term terms[15] = {{1, 1, {r1}},           {1, 1, {c1}},           {2, -2, {r1, c1}},
                                {1, 1, {r2}},           {1, 1, {c2}},           {2, -2, {r2, c2}},
                                {2, -1, {r1, r2}},      {2, -1, {r1, c2}},      {2, -1, {c1, r2}},
                                {2, -1, {c1, c2}},      {3, 2, {r1, r2, c2}},   {3, 2, {c1, r2, c2}},
                                {3, 2, {r1, c1, r2}},   {3, 2, {r1, c1, c2}},   {4, -4, {r1, c1, r2, c2}}};
        for (const Term& t : terms) router::diag(q, t.b, t.n, {(real)std::pow((double)g, t.e), 0});
        return;
    }
    if (twoQubitChannelsAsGates()) {
        twoQubitDephaseAsGates(q, qubit1, qubit2, qubit1 + q.nRep, qubit2 + q.nRep, g, true);
        return;
    }
    router::densChan2(q, qubit1, qubit2, qubit1 + q.nRep, qubit2 + q.nRep, 1 - d, 1, 0);
}

void applyOneQubitDepolariseError(Qureg qureg, const int targetQubit, qreal prob) {
    if (!v::densMatr(qureg, __func__) || !v::target(qureg, targetQubit, __func__) ||
        !v::oneQubitDepolProb(prob, __func__))
        return;
    real d = (4 * prob) / 3.0;
    if (d == 0) return;
    real a = 1 - d / 2, b = d / 2, f = 1 - d;
    const real m[16] = {a, 0, 0, b, 0, f, 0, 0, 0, 0, f, 0, b, 0, 0, a};
    realMat4(Q(qureg), targetQubit, m);
}

void applyOneQubitDampingError(Qureg qureg, const int targetQubit, qreal prob) {
    if (!v::densMatr(qureg, __func__) || !v::target(qureg, targetQubit, __func__) ||
        !v::oneQubitDampingProb(prob, __func__))
        return;
    if (prob == 0) return;
    real f = std::sqrt(1 - prob);
    const real m[16] = {1, 0, 0, prob, 0, f, 0, 0, 0, 0, f, 0, 0, 0, 0, 1 - prob};
    realMat4(Q(qureg), targetQubit, m);
}

void applyTwoQubitDepolariseError(Qureg qureg, int qubit1, int qubit2, qreal prob) {
    if (!v::densMatr(qureg, __func__) || !v::uniqueTargets(qureg, qubit1, qubit2, __func__) ||
        !v::twoQubitDepolProb(prob, __func__))
        return;
    if (qubit1 > qubit2) std::swap(qubit1, qubit2);
    real d = (16 * prob) / 15.0;
    if (d == 0) return;
    QuregImpl& q = Q(qureg);
    if (twoQubitChannelsAsGates()) {
        // dephasing of the coherences by 1 - d, then the populations of the
        // pair depolarised: (1 - d) x + d mean = gamma (I + delta X1)(I +
        // delta X2)(I + delta X1 X2) x with eta = 2 / d, delta = eta - 1 -
        // sqrt((eta - 1)^2 - 1) (delta / (1 + delta)^2 = d / 4), gamma =
        // (1 + delta)^-3 -- the reference's
        // three-step form (QuEST_cpu_local.c:40-51, QuEST_cpu.c:379-480), here
        // as one-qubit ops in the "differs" frame (see twoQubitDephaseAsGates)
        // delta as 1 / (a + sqrt(a^2 - 1)), a = eta - 1 (the two roots multiply
        // to 1): no cancellation for weak channels, where the reference's
        // difference form loses digits (its "TODO -- test delta too small")
        const double a = 2 / (double)d - 1;
        const double delta = 1 / (a + std::sqrt(std::max(0.0, a * a - 1)));
        const double gamma = 1 / ((1 + delta) * (1 + delta) * (1 + delta));
        const int r1 = qubit1, r2 = qubit2, c1 = qubit1 + q.nRep, c2 = qubit2 + q.nRep;
        twoQubitDephaseAsGates(q, r1, r2, c1, c2, 1 - d, false);
        // populations: c1 = c2 = 1 after the X on both (r1 == c1, r2 == c2)
        const int ctl[2] = {c1, c2};
        const cplx mix[4] = {{1, 0}, {(real)delta, 0}, {(real)delta, 0}, {1, 0}};
        const cplx mixG[4] = {{(real)gamma, 0}, {(real)(gamma * delta), 0}, {(real)(gamma * delta), 0},
                              {(real)gamma, 0}};
        router::mat2(q, r1, ctl, 2, mix);     // I + delta X1
        router::mat2(q, r2, ctl, 2, mix);     // I + delta X2
        router::mat2(q, r2, &r1, 1, kX);      // X1 X2 -> X1
        router::mat2(q, r1, ctl, 2, mixG);    // gamma (I + delta X1 X2)
        router::mat2(q, r2, &r1, 1, kX);
        differsFrame(q, r1, r2, c1, c2, true);
        return;
    }
    router::densChan2(q, qubit1, qubit2, qubit1 + q.nRep, qubit2 + q.nRep, 1 - d, 1 - d, d);
}

// ===========================================================================
// QASM
// ===========================================================================

void startRecordingQASM(Qureg qureg) { qasm::start(qureg); }
void stopRecordingQASM(Qureg qureg) { qasm::stop(qureg); }
void clearRecordedQASM(Qureg qureg) { qasm::clear(qureg); }
void printRecordedQASM(Qureg qureg) { qasm::print(qureg); }
void writeRecordedQASMToFile(Qureg qureg, char* filename) {
    int ok = qasm::writeToFile(qureg, filename);
    v::fileOpened(ok, __func__);
}

// ===========================================================================
// debug API (QuEST_debug.h)
// ===========================================================================

void initStateDebug(Qureg qureg) { router::initDebug(Q(qureg)); }

void initStateOfSingleQubit(Qureg* qureg, int qubitId, int outcome) {
    if (!v::stateVec(*qureg, __func__) || !v::target(*qureg, qubitId, __func__) || !v::outcome(outcome, __func__))
        return;
    QuregImpl& q = Q(*qureg);
    real val = (real)(1.0 / std::sqrt((double)q.numAmpsTotal / 2));
    router::initSingleQubit(q, qubitId, outcome, val);
}

void initStateFromSingleFile(Qureg* qureg, char filename[200], QuESTEnv env) {
    (void)env;
    QuregImpl& q = Q(*qureg);
    FILE* fp = fopen(filename, "r");
    if (!v::fileOpened(fp != nullptr, __func__)) return;
    router::prepareOverwrite(q);  // rank r reads the lines of chunk r
    std::vector<real> re((size_t)q.numAmpsPerChunk, 0), im(re.size(), 0);
    char line[200];
    i64 total = 0, mine = 0;
    while (fgets(line, sizeof line, fp) != nullptr && total < q.numAmpsTotal) {
        if (line[0] == '#') continue;
        if ((int)(total / q.numAmpsPerChunk) == q.chunkId) {
            double a = 0, b = 0;
            sscanf(line, "%lf, %lf", &a, &b);
            re[(size_t)mine] = (real)a;
            im[(size_t)mine] = (real)b;
            mine++;
        }
        total++;
    }
    fclose(fp);
    router::writeChunk(q, re.data(), im.data());
}

int compareStates(Qureg qureg1, Qureg qureg2, qreal precision) {
    if (!v::matchingDims(qureg1, qureg2, __func__)) return 0;
    QuregImpl &a = Q(qureg1), &b = Q(qureg2);
    router::canonicalise(a);
    router::canonicalise(b);
    const i64 piece = 1 << 20;
    i64 n = std::min(a.numAmpsPerChunk, b.numAmpsPerChunk);
    std::vector<real> ar((size_t)std::min(piece, n)), ai(ar.size()), br(ar.size()), bi(ar.size());
    int ok = 1;
    for (i64 off = 0; off < n && ok; off += piece) {
        i64 k = std::min(piece, n - off);
        be::readAmps(a, off, ar.data(), ai.data(), k);
        be::readAmps(b, off, br.data(), bi.data(), k);
        for (i64 i = 0; i < k; i++)
            if (absReal(ar[i] - br[i]) > precision || absReal(ai[i] - bi[i]) > precision) {
                ok = 0;
                break;
            }
    }
    return syncQuESTSuccess(ok);
}

int getQuEST_PREC(void) { return (int)(sizeof(qreal) / 4); }

// ===========================================================================
// MI355X extensions (quest_amd.h)
// ===========================================================================

void setGateFusion(int enabled) {
    for (QuregImpl* q : liveQuregs()) be::flush(*q);
    rt().fusion = enabled != 0;
}
int getGateFusion(void) { return rt().fusion ? 1 : 0; }
void setFusionMaxQubits(int numQubits) {
    for (QuregImpl* q : liveQuregs()) be::flush(*q);
    rt().fuseMaxQubits = numQubits;
}

int setQuESTTuning(const char* key, int value) {
    for (QuregImpl* q : liveQuregs()) router::flush(*q);
    if (key && !strcmp(key, "fuse_blocks")) {
        fuseBlocks() = value != 0;
        return 1;
    }
    if (key && !strcmp(key, "verify")) {
        rt().verify = value != 0;
        return 1;
    }
    if (key && !strcmp(key, "plan_max_ops")) {
        planMaxOps() = value;
        return 1;
    }
    if (key && !strcmp(key, "wave_relabel")) {
        waveRelabel() = value != 0;
        return 1;
    }
    if (key && !strcmp(key, "wave_lane_order")) {
        waveLaneOrder() = value;
        return 1;
    }
    if (key && !strcmp(key, "wave_shadow")) {
        rt().waveShadow = value != 0;
        return 1;
    }
    if (key && !strcmp(key, "verify_inject")) {  // fault injection for the verify test
        rt().verifyInject = value != 0;
        return 1;
    }
    return be::setTuning(key, value) ? 1 : 0;
}

int getQuESTTuning(const char* key, int* value) {
    int v = 0;
    bool known = true;
    if (key && !strcmp(key, "fuse_blocks"))
        v = fuseBlocks() ? 1 : 0;
    else if (key && !strcmp(key, "verify"))
        v = rt().verify ? 1 : 0;
    else if (key && !strcmp(key, "plan_max_ops"))
        v = planMaxOps();
    else if (key && !strcmp(key, "wave_relabel"))
        v = waveRelabel() ? 1 : 0;
    else if (key && !strcmp(key, "wave_lane_order"))
        v = waveLaneOrder();
    else if (key && !strcmp(key, "wave_shadow"))
        v = rt().waveShadow ? 1 : 0;
    else
        known = be::getTuning(key, &v);
    if (known && value) *value = v;
    return known ? 1 : 0;
}

void flushQureg(Qureg qureg) { router::flush(Q(qureg)); }
void syncQureg(Qureg qureg) { router::sync(Q(qureg)); }

void copyStateToGPU(Qureg qureg) {
    QuregImpl& q = Q(qureg);
    // the reference idiom "write qureg.stateVec, then copyStateToGPU": on the
    // host build stateVec IS the state, so only the cached norm / marginals
    // (router.cpp) must learn that it changed
    router::touch(q);
    if (be::stateOnHost() || !q.hostRe) return;
    router::writeChunk(q, q.hostRe, q.hostIm);
}

void copyStateFromGPU(Qureg qureg) {
    QuregImpl& q = Q(qureg);
    if (be::stateOnHost() || !q.hostRe) return;
    router::readChunk(q, q.hostRe, q.hostIm);
}

void copyChunkToBuffers(Qureg qureg, qreal* re, qreal* im) {
    QuregImpl& q = Q(qureg);
    router::canonicalise(q);
    be::toBuffer(q, 0, q.numAmpsPerChunk, re, im);
    be::deviceSync();
}

void copyChunkFromBuffers(Qureg qureg, const qreal* re, const qreal* im) {
    QuregImpl& q = Q(qureg);
    be::flush(q);
    router::canonicalise(q);
    be::fromBuffer(q, 0, q.numAmpsPerChunk, re, im);
    router::touch(q);
    be::deviceSync();
}

void getAmps(Qureg qureg, long long int startInd, qreal* reals, qreal* imags, long long int numAmps) {
    if (startInd < 0 || numAmps < 0 || startInd + numAmps > qureg.numAmpsTotal) {
        raiseError(E_INVALID_NUM_AMPS, __func__);
        return;
    }
    router::readRange(Q(qureg), startInd, reals, imags, numAmps);
}

int runCommSelfTest(char* report, int reportLen) {
    std::string r;
    const bool ok = comm::selfTest(r);
    if (report && reportLen > 0) snprintf(report, (size_t)reportLen, "%s", r.c_str());
    return ok ? 1 : 0;
}

int runFootprintCheck(int numQubitsInStateVec, int numRanks, char* report, int reportLen) {
    std::string r;
    const bool ok = router::footprintCheck(numQubitsInStateVec, numRanks, r);
    if (report && reportLen > 0) snprintf(report, (size_t)reportLen, "%s", r.c_str());
    return ok ? 1 : 0;
}

void getQuregMemoryPlan(int numQubitsInStateVec, int numRanks, long long out[4]) {
    const router::MemoryPlan m = router::memoryPlan(numQubitsInStateVec, numRanks > 0 ? numRanks : rt().numRanks);
    out[0] = m.state;
    out[1] = m.exchange;
    out[2] = m.scratch;
    out[3] = m.total;
}

void canonicaliseQureg(Qureg qureg) { router::canonicalise(Q(qureg)); }

void getQubitLayout(Qureg qureg, int* physicalOfLogical) {
    QuregImpl& q = Q(qureg);
    for (int i = 0; i < q.nSV; i++) physicalOfLogical[i] = q.l2p[i];
}

void getQuESTStats(QuESTStats* s) {
    s->opsQueued = stats().opsQueued;
    s->passes = stats().passes;
    s->fusedOps = stats().fusedOps;
    s->swaps = stats().swaps;
    s->bytesExchanged = stats().bytesExchanged;
    s->reductions = stats().reductions;
    s->verifiedFlushes = stats().verifiedFlushes;
    s->wavePasses = stats().wavePasses;
    s->waveOps = stats().waveOps;
    s->waveTransposes = stats().waveTransposes;
    s->relabels = stats().relabels;
    s->globalDiags = stats().globalDiags;
    s->flushes = stats().flushes;
    s->marginalPasses = stats().marginalPasses;
    s->waveShadowChecks = stats().waveShadowChecks;
    s->waveShadowMismatches = stats().waveShadowMismatches;
    s->permutedOps = stats().permutedOps;
    s->relayouts = stats().relayouts;
    s->restoreRounds = stats().restoreRounds;
    s->swapMicros = be::swapMicros(true);
    s->overlappedSwaps = stats().overlappedSwaps;
    s->overlappedPasses = stats().overlappedPasses;
    s->layoutAligns = stats().layoutAligns;
    s->placementProbes = stats().placementProbes;
}

void resetQuESTStats(void) {
    stats() = Stats();
    be::swapMicrosReset();
}

const char* getQuESTTransport(void) {
    static std::string d;
    d = comm::describe();
    return d.c_str();
}

const char* getQuESTBackend(void) { return be::shortName(); }

void getQuESTSeeds(unsigned long* seeds, int* numSeeds) {
    for (int i = 0; i < g_numSeeds; i++) seeds[i] = g_seeds[i];
    *numSeeds = g_numSeeds;
}

}  // extern "C"
