// Internal core types shared by the API front-end, the distributed router, the
// fusion planner and the two compile-time backends (HIP for gfx950, host C++).
//
// Design (see docs/ARCHITECTURE.md):
//   API (logical qubits)  ->  router (logical->physical map, RCCL swaps,
//   chunk predicates)  ->  backend queue (physical local ops, fused into LDS
//   tile passes on the GPU)  ->  kernels.
//
// The reference's equivalent boundary is QuEST/src/QuEST_internal.h:22-188
// (statevec_* / densmatr_* per backend); here the backend surface is much
// smaller because every unitary reduces to four op kinds (Op below).
#pragma once

#include "QuEST.h"

#include <cstddef>
#include <cstdint>
#include <string>
#include <future>
#include <vector>

namespace qa {

using real = qreal;
using i64 = long long;
using u64 = unsigned long long;

struct cplx {
    real re, im;
};

inline cplx cmul(cplx a, cplx b) { return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
inline cplx cadd(cplx a, cplx b) { return {a.re + b.re, a.im + b.im}; }
inline cplx cconj(cplx a) { return {a.re, -a.im}; }

// Elementary operation on this rank's chunk, in PHYSICAL LOCAL qubit positions.
enum class OpKind : int {
    Mat2 = 0,       // 2x2 complex matrix on t[0]; amplitudes whose ctrl bits are all 1
    Diag = 1,       // multiply amplitudes with (index & ctrl) == ctrl by m[0]
    Mat4 = 2,       // 4x4 complex on (t[0], t[1]); group index = bit(t0) + 2 bit(t1)
    DensChan2 = 3,  // two-qubit dephase/depolarise superoperator, see below
};

// Rank predicates of distributed registers (router issue): an op controlled by
// a rank qubit, a phase on one and a collapse of one used to be queued only on
// the ranks where they apply -- so the ranks' planners saw different op lists
// and could relabel local qubits differently (round 5 patched that with a
// layout broadcast before every swap).  Now every rank queues the SAME op,
// tagged in ctrl bits 48..62 (above every local position, at least two bits:
// never fused into a two-qubit block) -- an out-of-tile control to every
// planner, so all ranks plan the same passes -- and the rank's verdict sits in
// QuregImpl::rankSkip[tag].  Backends resolve tags where they execute ops
// (resolveRankTag): the tag bits cleared where the op runs; left in place
// where it does not, where no local index matches them (the op is skipped).
constexpr int kRankTagShift = 48;
constexpr int kRankTagCount = 1 << 14;                     // tag ids 1 .. 16383 (bits 48..61) + marker bit 62
constexpr unsigned long long kRankTagMask = 0x7fffull << kRankTagShift;

// DensChan2 acts on the 16 elements spanned by t = {row q1, row q2, col q1, col q2}.
// With a = bit(t0) + 2 bit(t1) and b = bit(t2) + 2 bit(t3):
//   a != b : x *= m[0].re                          (off-diagonal dephasing)
//   a == b : x_aa = m[1].re x_aa + m[2].re/4 * sum_a' x_a'a'  (depolarising mix)
struct Op {
    OpKind kind = OpKind::Mat2;
    int nt = 1;          // number of valid targets in t[]
    int t[4] = {0, 0, 0, 0};
    u64 ctrl = 0;        // local control mask (Diag: the phase mask)
    cplx m[16];          // row-major matrix / parameters
};

// Library-side state of a register.  Qureg.qasmLog points at `log`, which is
// the first member, so the impl is recovered from any Qureg passed by value
// without changing the reference's struct layout.
struct QuregImpl {
    QASMLogger log;
    unsigned magic;
    bool isDensity;
    int nRep;            // qubits represented
    int nSV;             // qubits in the state-vector (2 nRep for density)
    int L;               // physical qubits held locally (nSV - log2 numChunks)
    i64 numAmpsPerChunk;
    i64 numAmpsTotal;
    int chunkId;         // LOGICAL chunk held by this rank (rank qubits' values)
    int numChunks;
    // logical chunk -> rank holding it.  Identity unless an X-like gate on a
    // rank qubit relabelled chunks instead of moving their data (router).
    std::vector<int> chunkRank;
    real* re;            // this chunk's amplitudes (device memory on the HIP build)
    real* im;
    int l2p[64];         // logical qubit -> physical bit position
    int p2l[64];         // physical bit position -> logical qubit
    i64 useClock = 0;    // LRU bookkeeping for choosing swap victims
    i64 lastUse[64];
    std::vector<Op> pending;  // ops queued for fusion (backend-owned semantics)
    std::vector<Op> lpending; // distributed registers: ops in LOGICAL qubits awaiting routing
    bool jointAlloc = false;  // HIP: re and im share one allocation (freed through allocBase)
    void* allocBase = nullptr;  // HIP: that allocation (re may start inside it)
    void* be = nullptr;       // backend-private state
    // Router-level change counter of the LOGICAL state (bumped identically on
    // every rank by every op / overwrite) and the one-qubit marginals cached
    // at margGen: margP0[lg] = sum |a|^2 over amplitudes with logical qubit lg
    // = 0 (all ranks), margP0[nSV] = the norm.
    u64 stateGen = 0;
    u64 margGen = ~0ull;
    u64 probGen = ~0ull;      // state generation of the last single-qubit query
    double margP0[65];
    u64 normGen = ~0ull;      // state generation of normCache (sumSqAll)
    double normCache = 0;
    real* hostRe = nullptr;   // optional host mirror (Qureg.stateVec)
    real* hostIm = nullptr;
    // wave planner: always-resident low positions chosen for the ops queued
    // now (chooseWaveCmin), kept until the queue has drained (-1: not chosen)
    int waveCmin = -1;
    // wave planner strategy for this queue's front flushes (searchWaveStrategy,
    // run in the background after the window's first front flush; -1: the
    // default), kept until the queue has drained
    int planStrategy = -1;
    std::future<int> strategySearch;
    // local positions the planner keeps out of tile padding (router planSwap:
    // the victims of the swap being prepared; 0 otherwise)
    u64 tileAvoid = 0;
    // logical qubits a swap about to run moves out (router planSwap, before
    // its flush; -1 none): the backend can split the passes that avoid them
    int swapVictims[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
    int nSwapVictims = 0;
    // rank predicates (kRankTagMask): this rank's verdict per tag id (1: the
    // op does not apply here), tags handed out round robin
    std::vector<unsigned char> rankSkip;
    int rankTagNext = 0;
    // local positions the first passes planned after a swap keep out of
    // their tiles, targets included (router multiSwap: the swap's receive
    // ranges, so those passes can run range by range as they land), and how
    // many passes still do (consumed by the flushes that plan them)
    u64 firstPassAvoid = 0;
    int firstAvoidLeft = 0;
    bool permIdentity() const {
        for (int i = 0; i < nSV; i++)
            if (l2p[i] != i) return false;
        return true;
    }
};

constexpr unsigned kQuregMagic = 0x51A3D355u;

// The rank-tag verdicts of the register being flushed (set by the backends'
// flush for its duration; RankSkipScope) and the resolution of a predicate
// mask against them: tag bits cleared when the op applies on this rank.
const unsigned char*& rankSkipTable();
[[noreturn]] void rankTagFatal();
inline u64 resolveRankTag(u64 m) {
    if (!(m & kRankTagMask)) return m;
    const unsigned char* s = rankSkipTable();
    if (!s) rankTagFatal();
    return s[(m >> kRankTagShift) & (kRankTagCount - 1)] ? m : (m & ~kRankTagMask);
}
struct RankSkipScope {
    const unsigned char* prev;
    explicit RankSkipScope(const QuregImpl& q) : prev(rankSkipTable()) {
        rankSkipTable() = q.rankSkip.empty() ? nullptr : q.rankSkip.data();
    }
    ~RankSkipScope() { rankSkipTable() = prev; }
};

// A flush planned `passes` passes: the swap-range constraint holds for that
// many fewer (QuregImpl::firstAvoidLeft)
inline void consumeFirstAvoid(QuregImpl& q, int passes) {
    if (q.firstAvoidLeft <= 0) return;
    q.firstAvoidLeft -= passes;
    if (q.firstAvoidLeft <= 0) {
        q.firstAvoidLeft = 0;
        q.firstPassAvoid = 0;
    }
}

QuregImpl* impl(const Qureg& q);

// Global runtime state (one per process).
struct Runtime {
    int rank = 0;
    int numRanks = 1;
    int localRank = 0;
    bool initialised = false;
    bool fusion = true;        // QUEST_FUSION=0 disables gate fusion
    int fuseMaxQubits = 0;     // 0 = backend default
    i64 exchangeSliceBytes = 256ll << 20;  // QUEST_EXCHANGE_SLICE_MB
    // QUEST_VERIFY=1: every fused flush is re-run op by op on a shadow copy
    // of the state and compared (debug mode; doubles memory and time)
    bool verify = false;
    double verifyTol = 0;  // QUEST_VERIFY_TOL; 0 = 1e-10 (fp64) / 1e-4 (fp32)
    bool verifyInject = false;  // test hook: corrupt the next verified flush once
    // QUEST_WAVE_SHADOW=1 / tuning "wave_shadow" (HIP build, debug): every
    // wave pass is also run by the host emulation (src/core/wave_emu.cpp) on a
    // host copy of the state and the two compared; a mismatch is reported with
    // the pass's ops and layout, counted (QuESTStats.waveShadowMismatches) and
    // the emulated state written back, so later passes are checked on their own
    bool waveShadow = false;
};
Runtime& rt();

}  // namespace qa
