#include "router.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../comm/comm.hpp"
#include "backend.hpp"

namespace qa {

Stats& stats() {
    static Stats s;
    return s;
}

QuregImpl* impl(const Qureg& q) {
    QuregImpl* p = reinterpret_cast<QuregImpl*>(q.qasmLog);
    if (!p || p->magic != kQuregMagic) {
        fprintf(stderr, "QuEST: invalid or destroyed Qureg passed to the API\n");
        exit(EXIT_FAILURE);
    }
    return p;
}

namespace router {

namespace {

// Reusable comm buffers for sliced exchanges: [re | im] for send and recv.
struct XBuf {
    real* send = nullptr;
    real* recv = nullptr;
    i64 amps = 0;  // capacity in amplitudes (per re/im half)
} g_x;

void ensureXBuf(i64 amps) {
    if (g_x.amps >= amps) return;
    if (g_x.send) be::freeComm(g_x.send);
    if (g_x.recv) be::freeComm(g_x.recv);
    g_x.send = (real*)be::allocComm(sizeof(real) * 2 * amps);
    g_x.recv = (real*)be::allocComm(sizeof(real) * 2 * amps);
    g_x.amps = amps;
}

inline int chunkBit(const QuregImpl& q, int phys) { return (q.chunkId >> (phys - q.L)) & 1; }

void touch(QuregImpl& q, int phys) { q.lastUse[phys] = ++q.useClock; }

// Swap the qubit at global position g with the one at local position l.
// Pairs of ranks differing in rank bit (g - L) exchange the half of their
// chunk whose local bit l differs from their own rank bit, in slices.
void swapGlobalLocal(QuregImpl& q, int g, int l) {
    be::flush(q);
    const int rbit = g - q.L;
    const int partner = q.chunkId ^ (1 << rbit);
    const int b = (q.chunkId >> rbit) & 1;
    const i64 half = q.numAmpsPerChunk / 2;
    i64 slice = rt().exchangeSliceBytes / (i64)(2 * sizeof(real));
    if (slice < 1) slice = 1;
    slice = std::min(slice, half);
    ensureXBuf(slice);
    for (i64 off = 0; off < half; off += slice) {
        i64 n = std::min(slice, half - off);
        be::packBit(q, l, 1 - b, off, n, g_x.send, g_x.send + n);
        comm::sendrecv(partner, g_x.send, g_x.recv, sizeof(real) * 2 * (size_t)n);
        be::unpackBit(q, l, 1 - b, off, n, g_x.recv, g_x.recv + n);
        stats().bytesExchanged += (long long)(sizeof(real) * 2 * n);
    }
    int lg = q.p2l[g], ll = q.p2l[l];
    q.l2p[lg] = l;
    q.l2p[ll] = g;
    q.p2l[g] = ll;
    q.p2l[l] = lg;
    std::swap(q.lastUse[g], q.lastUse[l]);
    stats().swaps++;
}

// Make the given logical qubits local, never evicting a protected one.
void ensureLocal(QuregImpl& q, const int* lq, int n, const int* protect, int np) {
    if (q.L == q.nSV) return;
    for (int i = 0; i < n; i++) {
        int p = q.l2p[lq[i]];
        if (p < q.L) continue;
        // least-recently-used local position not holding a protected qubit
        int victim = -1;
        for (int v = q.L - 1; v >= 0; v--) {
            int logical = q.p2l[v];
            bool prot = false;
            for (int k = 0; k < n && !prot; k++) prot = (lq[k] == logical);
            for (int k = 0; k < np && !prot; k++) prot = (protect[k] == logical);
            if (prot) continue;
            if (victim < 0 || q.lastUse[v] < q.lastUse[victim]) victim = v;
        }
        if (victim < 0) {
            fprintf(stderr, "QuEST: no local qubit available for a distributed swap\n");
            exit(EXIT_FAILURE);
        }
        swapGlobalLocal(q, p, victim);
    }
}

void resetLayout(QuregImpl& q) {
    for (int i = 0; i < 64; i++) {
        q.l2p[i] = q.p2l[i] = i;
        q.lastUse[i] = 0;
    }
}

void enqueue(QuregImpl& q, const Op& op) {
    be::enqueue(q, op);
    stats().opsQueued++;
}

i64 logicalToPhysicalIndex(const QuregImpl& q, i64 idx) {
    if (q.numChunks == 1 && q.permIdentity()) return idx;
    i64 p = 0;
    for (int j = 0; j < q.nSV; j++)
        if ((idx >> j) & 1) p |= (i64)1 << q.l2p[j];
    return p;
}

}  // namespace

void create(QuregImpl& q, int nSV, bool density) {
    int g = 0;
    while ((1 << g) < rt().numRanks) g++;
    q.nSV = nSV;
    q.isDensity = density;
    q.nRep = density ? nSV / 2 : nSV;
    q.L = nSV - g;
    q.numChunks = rt().numRanks;
    q.chunkId = rt().rank;
    q.numAmpsTotal = (i64)1 << nSV;
    q.numAmpsPerChunk = (i64)1 << q.L;
    resetLayout(q);
    be::allocState(q);
}

void destroy(QuregImpl& q) {
    be::flush(q);
    be::freeState(q);
}

void flush(QuregImpl& q) { be::flush(q); }

void sync(QuregImpl& q) {
    be::flush(q);
    be::deviceSync();
}

// ---------------------------------------------------------------------------
// ops
// ---------------------------------------------------------------------------

void mat2(QuregImpl& q, int target, const int* ctrls, int nc, const cplx m[4]) {
    ensureLocal(q, &target, 1, ctrls, nc);
    Op op;
    op.kind = OpKind::Mat2;
    op.nt = 1;
    op.t[0] = q.l2p[target];
    touch(q, op.t[0]);
    for (int i = 0; i < nc; i++) {
        int p = q.l2p[ctrls[i]];
        if (p >= q.L) {
            if (!chunkBit(q, p)) return;  // this rank's amplitudes all fail the control
        } else {
            op.ctrl |= 1ull << p;
        }
    }
    for (int i = 0; i < 4; i++) op.m[i] = m[i];
    enqueue(q, op);
}

void diag(QuregImpl& q, const int* qubits, int nq, cplx term) {
    Op op;
    op.kind = OpKind::Diag;
    op.nt = 0;
    for (int i = 0; i < nq; i++) {
        int p = q.l2p[qubits[i]];
        if (p >= q.L) {
            if (!chunkBit(q, p)) return;
        } else {
            op.ctrl |= 1ull << p;
        }
    }
    op.m[0] = term;
    enqueue(q, op);
}

void mat4(QuregImpl& q, int q0, int q1, const cplx m[16]) {
    int t[2] = {q0, q1};
    ensureLocal(q, t, 2, nullptr, 0);
    Op op;
    op.kind = OpKind::Mat4;
    op.nt = 2;
    op.t[0] = q.l2p[q0];
    op.t[1] = q.l2p[q1];
    touch(q, op.t[0]);
    touch(q, op.t[1]);
    for (int i = 0; i < 16; i++) op.m[i] = m[i];
    enqueue(q, op);
}

void densChan2(QuregImpl& q, int r1, int r2, int c1, int c2, real offFac, real keep, real mix) {
    int t[4] = {r1, r2, c1, c2};
    ensureLocal(q, t, 4, nullptr, 0);
    Op op;
    op.kind = OpKind::DensChan2;
    op.nt = 4;
    for (int i = 0; i < 4; i++) {
        op.t[i] = q.l2p[t[i]];
        touch(q, op.t[i]);
    }
    op.m[0] = {offFac, 0};
    op.m[1] = {keep, 0};
    op.m[2] = {mix, 0};
    enqueue(q, op);
}

void collapse(QuregImpl& q, int qubit, int outcome, real renorm) {
    int p = q.l2p[qubit];
    if (p >= q.L) {
        Op op;
        op.kind = OpKind::Diag;
        op.nt = 0;
        op.ctrl = 0;
        op.m[0] = {chunkBit(q, p) == outcome ? renorm : (real)0, 0};
        enqueue(q, op);
        return;
    }
    Op op;
    op.kind = OpKind::Mat2;
    op.nt = 1;
    op.t[0] = p;
    op.m[0] = {outcome == 0 ? renorm : (real)0, 0};
    op.m[1] = {0, 0};
    op.m[2] = {0, 0};
    op.m[3] = {outcome == 1 ? renorm : (real)0, 0};
    enqueue(q, op);
}

void densCollapse(QuregImpl& q, int qubit, int outcome, real prob) {
    // keep elements whose row bit (qubit) and column bit (qubit + n) both equal
    // the outcome; scale them by 1/prob (reference divides by p, not sqrt(p))
    real s = (real)1 / prob;
    int r = q.l2p[qubit], c = q.l2p[qubit + q.nRep];
    bool rGlobal = r >= q.L, cGlobal = c >= q.L;
    if (rGlobal && cGlobal) {
        bool keepChunk = chunkBit(q, r) == outcome && chunkBit(q, c) == outcome;
        Op op;
        op.kind = OpKind::Diag;
        op.nt = 0;
        op.m[0] = {keepChunk ? s : (real)0, 0};
        enqueue(q, op);
        return;
    }
    if (rGlobal || cGlobal) {
        int gpos = rGlobal ? r : c, lpos = rGlobal ? c : r;
        Op op;
        if (chunkBit(q, gpos) != outcome) {
            op.kind = OpKind::Diag;
            op.nt = 0;
            op.m[0] = {0, 0};
        } else {
            op.kind = OpKind::Mat2;
            op.nt = 1;
            op.t[0] = lpos;
            op.m[0] = {outcome == 0 ? s : (real)0, 0};
            op.m[1] = {0, 0};
            op.m[2] = {0, 0};
            op.m[3] = {outcome == 1 ? s : (real)0, 0};
        }
        enqueue(q, op);
        return;
    }
    Op op;
    op.kind = OpKind::Mat4;
    op.nt = 2;
    op.t[0] = r;
    op.t[1] = c;
    for (int i = 0; i < 16; i++) op.m[i] = {0, 0};
    if (outcome == 0)
        op.m[0] = {s, 0};
    else
        op.m[15] = {s, 0};
    enqueue(q, op);
}

// ---------------------------------------------------------------------------
// state preparation
// ---------------------------------------------------------------------------

void initClassical(QuregImpl& q, i64 index) {
    be::flush(q);
    resetLayout(q);
    be::fill(q, 0, 0);
    i64 start = (i64)q.chunkId * q.numAmpsPerChunk;
    if (index >= start && index < start + q.numAmpsPerChunk) be::setAmp(q, index - start, 1, 0);
}

void initUniform(QuregImpl& q, real val) {
    be::flush(q);
    resetLayout(q);
    be::fill(q, val, 0);
}

void initDebug(QuregImpl& q) {
    be::flush(q);
    resetLayout(q);
    be::initDebug(q, (i64)q.chunkId * q.numAmpsPerChunk);
}

void initSingleQubit(QuregImpl& q, int qubit, int outcome, real val) {
    be::flush(q);
    resetLayout(q);
    if (qubit >= q.L) {
        be::fill(q, chunkBit(q, qubit) == outcome ? val : (real)0, 0);
    } else {
        be::fillWhereBit(q, qubit, outcome, val);
    }
}

void setAmps(QuregImpl& q, i64 start, const real* re, const real* im, i64 n) {
    if (n == q.numAmpsTotal && start == 0) {
        be::flush(q);
        resetLayout(q);
    } else {
        canonicalise(q);
    }
    i64 c0 = (i64)q.chunkId * q.numAmpsPerChunk, c1 = c0 + q.numAmpsPerChunk;
    i64 lo = std::max(start, c0), hi = std::min(start + n, c1);
    if (lo < hi) be::writeAmps(q, lo - c0, re + (lo - start), im + (lo - start), hi - lo);
}

void clone(QuregImpl& dst, QuregImpl& src) {
    be::flush(src);
    be::flush(dst);
    be::copyState(dst, src);
    memcpy(dst.l2p, src.l2p, sizeof dst.l2p);
    memcpy(dst.p2l, src.p2l, sizeof dst.p2l);
    memcpy(dst.lastUse, src.lastUse, sizeof dst.lastUse);
    dst.useClock = src.useClock;
}

// Gather the full canonical pure state (2^n amps) onto every rank.
static void gatherPure(QuregImpl& psi, real** fullRe, real** fullIm) {
    canonicalise(psi);
    be::flush(psi);
    i64 total = psi.numAmpsTotal, chunk = psi.numAmpsPerChunk;
    *fullRe = (real*)be::allocComm(sizeof(real) * total);
    *fullIm = (real*)be::allocComm(sizeof(real) * total);
    if (psi.numChunks == 1) {
        be::toBuffer(psi, 0, chunk, *fullRe, *fullIm);
        return;
    }
    real* mine = (real*)be::allocComm(sizeof(real) * 2 * chunk);
    be::toBuffer(psi, 0, chunk, mine, mine + chunk);
    comm::allgather(mine, *fullRe, sizeof(real) * chunk);
    comm::allgather(mine + chunk, *fullIm, sizeof(real) * chunk);
    be::freeComm(mine);
}

void densInitPure(QuregImpl& rho, QuregImpl& psi) {
    real *fr, *fi;
    gatherPure(psi, &fr, &fi);
    be::flush(rho);
    resetLayout(rho);
    be::densInitPure(rho, fr, fi, rho.nRep, (i64)rho.chunkId * rho.numAmpsPerChunk);
    be::freeComm(fr);
    be::freeComm(fi);
}

void axpby(QuregImpl& a, real alpha, QuregImpl& b, real beta) {
    if (memcmp(a.l2p, b.l2p, sizeof(int) * a.nSV) != 0) {
        canonicalise(a);
        canonicalise(b);
    }
    be::flush(a);
    be::flush(b);
    be::axpby(a, alpha, b, beta);
}

void canonicalise(QuregImpl& q) {
    be::flush(q);
    if (q.permIdentity()) return;
    // 1. put the right logical qubit on every global position
    for (int g = q.L; g < q.nSV; g++) {
        if (q.p2l[g] == g) continue;
        int x = q.l2p[g];
        if (x < q.L) {
            swapGlobalLocal(q, g, x);
        } else {
            int v = q.L - 1;
            swapGlobalLocal(q, x, v);          // logical g -> local v
            swapGlobalLocal(q, g, q.l2p[g]);   // logical g -> position g
        }
    }
    // 2. permute local qubits with local SWAP ops
    static const cplx kSwap[16] = {{1, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {1, 0}, {0, 0},
                                   {0, 0}, {1, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {1, 0}};
    for (int i = 0; i < q.L; i++) {
        if (q.p2l[i] == i) continue;
        int x = q.l2p[i];  // where logical i currently sits (local, > i)
        Op op;
        op.kind = OpKind::Mat4;
        op.nt = 2;
        op.t[0] = i;
        op.t[1] = x;
        for (int k = 0; k < 16; k++) op.m[k] = kSwap[k];
        enqueue(q, op);
        int li = q.p2l[i];
        q.l2p[li] = x;
        q.l2p[i] = i;
        q.p2l[x] = li;
        q.p2l[i] = i;
    }
    be::flush(q);
}

// ---------------------------------------------------------------------------
// reads and reductions
// ---------------------------------------------------------------------------

cplx getAmp(QuregImpl& q, i64 flatIndex) {
    be::flush(q);
    i64 p = logicalToPhysicalIndex(q, flatIndex);
    int owner = (int)(p >> q.L);
    real v[2] = {0, 0};
    if (owner == q.chunkId) be::readAmps(q, p & (q.numAmpsPerChunk - 1), &v[0], &v[1], 1);
    if (q.numChunks > 1) comm::bcastHost(v, sizeof v, owner);
    return {v[0], v[1]};
}

static double allSum(double x) {
    if (comm::active()) comm::allreduceSum(&x, 1);
    return x;
}

double probZero(QuregImpl& q, int qubit) {
    be::flush(q);
    stats().reductions++;
    int p = q.l2p[qubit];
    double part;
    if (p >= q.L)
        part = chunkBit(q, p) == 0 ? be::sumSq(q, -1, 0) : 0.0;
    else
        part = be::sumSq(q, p, 0);
    return allSum(part);
}

double sumSqAll(QuregImpl& q) {
    be::flush(q);
    stats().reductions++;
    return allSum(be::sumSq(q, -1, 0));
}

static double densDiag(QuregImpl& q, int skipBit) {
    be::flush(q);
    stats().reductions++;
    u64 offs[64];
    for (int j = 0; j < q.nRep; j++) offs[j] = (1ull << q.l2p[j]) | (1ull << q.l2p[j + q.nRep]);
    double part = be::densDiagSum(q, offs, q.nRep, skipBit, (i64)q.chunkId * q.numAmpsPerChunk);
    return allSum(part);
}

double densProbZero(QuregImpl& q, int qubit) { return densDiag(q, qubit); }
double densTrace(QuregImpl& q) { return densDiag(q, -1); }

cplx inner(QuregImpl& bra, QuregImpl& ket) {
    if (memcmp(bra.l2p, ket.l2p, sizeof(int) * bra.nSV) != 0) {
        canonicalise(bra);
        canonicalise(ket);
    }
    be::flush(bra);
    be::flush(ket);
    stats().reductions++;
    double v[2];
    be::innerProduct(bra, ket, v);
    if (comm::active()) comm::allreduceSum(v, 2);
    return {(real)v[0], (real)v[1]};
}

double densFidelity(QuregImpl& rho, QuregImpl& psi) {
    real *fr, *fi;
    gatherPure(psi, &fr, &fi);
    canonicalise(rho);
    stats().reductions++;
    double part = be::densFidelity(rho, fr, fi, rho.nRep, (i64)rho.chunkId * rho.numAmpsPerChunk);
    be::freeComm(fr);
    be::freeComm(fi);
    return allSum(part);
}

void readChunk(QuregImpl& q, real* re, real* im) {
    canonicalise(q);
    be::readAmps(q, 0, re, im, q.numAmpsPerChunk);
}

void readRange(QuregImpl& q, i64 start, real* re, real* im, i64 n) {
    canonicalise(q);
    for (int r = 0; r < q.numChunks; r++) {
        i64 c0 = (i64)r * q.numAmpsPerChunk, c1 = c0 + q.numAmpsPerChunk;
        i64 lo = std::max(start, c0), hi = std::min(start + n, c1);
        if (lo >= hi) continue;
        if (r == q.chunkId) be::readAmps(q, lo - c0, re + (lo - start), im + (lo - start), hi - lo);
        if (q.numChunks > 1) {
            comm::bcastHost(re + (lo - start), sizeof(real) * (size_t)(hi - lo), r);
            comm::bcastHost(im + (lo - start), sizeof(real) * (size_t)(hi - lo), r);
        }
    }
}

void writeChunk(QuregImpl& q, const real* re, const real* im) {
    be::flush(q);
    resetLayout(q);
    be::writeAmps(q, 0, re, im, q.numAmpsPerChunk);
}

}  // namespace router
}  // namespace qa
