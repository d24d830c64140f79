// Distributed router: takes operations on LOGICAL qubits from the API
// front-end and turns them into backend ops on PHYSICAL, chunk-local qubits.
//
// Replaces the reference's per-gate local/remote branching
// (QuEST/src/CPU/QuEST_cpu_distributed.c:816-1214) with one mechanism:
//  * each register keeps a logical->physical qubit map;
//  * on a distributed register ops wait in a logical queue; routing issues,
//    in commutation-respecting order, every op whose targets are local, and
//    when blocked swaps in the rank qubits the queue needs, all at once, with
//    ONE all-to-all among the 2^k ranks concerned (every peer's xGMI link at
//    once; the reference exchanges a whole chunk pairwise, per gate); the map
//    is updated instead of swapping back, so later gates stay local;
//  * controls and diagonal bits on global qubits become per-rank predicates
//    (no communication, and a rank whose control bit is 0 does nothing);
//  * reductions are chunk partials + one allreduce.
#pragma once

#include <string>

#include "core.hpp"

namespace qa {
namespace router {

// Device memory one rank needs for a register of nSV qubits over numRanks
// ranks: its chunk (re + im), the largest set of exchange slice buffers a
// distributed swap allocates (send + recv, double-buffered, per peer) and a
// fixed allowance for reduction scratch / program upload.
struct MemoryPlan {
    long long state = 0, exchange = 0, scratch = 0, total = 0;
};
MemoryPlan memoryPlan(int nSV, int numRanks);
// The per-rank footprint of an nSV-qubit register on numRanks ranks, on this
// (single-process) job's device next to whatever it already holds: the
// exchange buffers of the plan's largest all-to-all swap allocated as
// multiSwap would, a transport communicator brought up and the pipelined
// exchange run through them (comm::selfTest).  Free device memory before,
// with the buffers and with the communicator up goes to report.
bool footprintCheck(int nSV, int numRanks, std::string& report);

void create(QuregImpl& q, int nSV, bool density);
void destroy(QuregImpl& q);
void flush(QuregImpl& q);
void sync(QuregImpl& q);

// ---- unitary / non-unitary ops on logical qubits ----------------------------
void mat2(QuregImpl& q, int target, const int* ctrls, int nc, const cplx m[4]);
// amplitudes whose `qubits` are all 1 are multiplied by term
void diag(QuregImpl& q, const int* qubits, int nq, cplx term);
// 4x4 on (q0, q1), group index bit(q0) + 2 bit(q1)
void mat4(QuregImpl& q, int q0, int q1, const cplx m[16]);
void densChan2(QuregImpl& q, int r1, int r2, int c1, int c2, real offFac, real keep, real mix);
// projective collapse of one qubit (state-vector: renorm = 1/sqrt(p))
void collapse(QuregImpl& q, int qubit, int outcome, real renorm);
// density matrix: keep rows and cols with the outcome, scale by 1/prob
void densCollapse(QuregImpl& q, int qubit, int outcome, real prob);

// ---- state preparation -------------------------------------------------------
void initClassical(QuregImpl& q, i64 index);  // one amplitude = 1 (flat index)
void initUniform(QuregImpl& q, real val);
void initDebug(QuregImpl& q);
void initSingleQubit(QuregImpl& q, int qubit, int outcome, real val);
void setAmps(QuregImpl& q, i64 start, const real* re, const real* im, i64 n);
void clone(QuregImpl& dst, QuregImpl& src);
void densInitPure(QuregImpl& rho, QuregImpl& psi);
void axpby(QuregImpl& a, real alpha, QuregImpl& b, real beta);
void canonicalise(QuregImpl& q);

// ---- reads and reductions (collective over ranks) -------------------------------
cplx getAmp(QuregImpl& q, i64 flatIndex);
double probZero(QuregImpl& q, int qubit);
// the state was changed outside the router (e.g. copyChunkFromBuffers)
void touch(QuregImpl& q);
double sumSqAll(QuregImpl& q);
double densProbZero(QuregImpl& q, int qubit);
double densTrace(QuregImpl& q);
cplx inner(QuregImpl& bra, QuregImpl& ket);
double densFidelity(QuregImpl& rho, QuregImpl& psi);
// read this rank's chunk in canonical order (host arrays of numAmpsPerChunk)
void readChunk(QuregImpl& q, real* re, real* im);
void writeChunk(QuregImpl& q, const real* re, const real* im);
// route and flush everything queued, then reset the layout to canonical
// without moving data: the caller overwrites the whole chunk next
void prepareOverwrite(QuregImpl& q);
// collective read of global amplitudes [start, start+n) onto every rank
void readRange(QuregImpl& q, i64 start, real* re, real* im, i64 n);

}  // namespace router

// runtime statistics (quest_amd.h: QuESTStats)
struct Stats {
    long long opsQueued = 0, passes = 0, fusedOps = 0, swaps = 0, bytesExchanged = 0, reductions = 0;
    long long verifiedFlushes = 0;
    long long wavePasses = 0;     // passes run by the wave-tile engine
    long long waveOps = 0, waveTransposes = 0;  // their ops / cross-lane transpositions
    long long relabels = 0;       // anti-diagonal gates on rank qubits done by relabelling chunks
    long long globalDiags = 0;    // diagonal gates on rank qubits done as per-rank scalings
    long long flushes = 0;        // backend queue flushes (each planned into passes)
    long long marginalPasses = 0; // one-pass all-qubit marginals (probZero cache fills)
    long long waveShadowChecks = 0, waveShadowMismatches = 0;  // rt().waveShadow
    long long permutedOps = 0;    // inner products / axpby of registers in different layouts, no relayout
    long long relayouts = 0;      // canonicalisations that moved data
    long long layoutAligns = 0;   // swaps / chunk restores before which this rank moved its local qubits to rank 0's positions
    long long restoreRounds = 0;  // concurrent rounds of whole-chunk exchanges restoring chunk placement
    long long overlappedSwaps = 0;   // swaps issued on their own stream (be::swapOverlapBegin)
    long long overlappedPasses = 0;  // passes started on the part a swap in flight leaves in place
    long long placementProbes = 0;   // re / im placements measured by the allocation probe
};
Stats& stats();

// QUEST_VERIFY: compare the fused result of a flush with its op-by-op
// re-execution; exits with a report when they differ by more than the
// tolerance (src/core/router.cpp)
void verifyFlush(int qubits, size_t ops, size_t passes, double maxDiff);

}  // namespace qa
