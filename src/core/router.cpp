#include "router.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../comm/comm.hpp"
#include "backend.hpp"
#include "trace.hpp"

namespace qa {

Stats& stats() {
    static Stats s;
    return s;
}

void verifyFlush(int qubits, size_t ops, size_t passes, double maxDiff) {
    const double tol = rt().verifyTol > 0 ? rt().verifyTol : (sizeof(real) >= 8 ? 1e-10 : 1e-4);
    stats().verifiedFlushes++;
    if (trace::on())
        trace::event("verify", "\"qubits\": %d, \"ops\": %zu, \"passes\": %zu, \"max_diff\": %.3e", qubits, ops,
                     passes, maxDiff);
    if (maxDiff <= tol) return;
    fprintf(stderr,
            "QuEST verify: rank %d: a fused flush of %zu ops (%zu passes) on %d local qubits differs from op-by-op "
            "execution by %.3e (tolerance %.1e)\n",
            rt().rank, ops, passes, qubits, maxDiff, tol);
    fflush(stderr);
    exit(EXIT_FAILURE);
}

const unsigned char*& rankSkipTable() {
    static thread_local const unsigned char* t = nullptr;
    return t;
}

void rankTagFatal() {
    fprintf(stderr, "QuEST: an op carries a rank tag outside a register flush\n");
    exit(EXIT_FAILURE);
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

// Reusable comm buffers for sliced exchanges: per peer [re | im], send and recv.
struct XBuf {
    std::vector<real*> send, recv;
    i64 amps = 0;  // capacity per buffer in amplitudes (per re/im half)
    bool hasSend = false;
} g_x;

// withSend = false: receive buffers only (RCCL sends straight from the state)
void ensureXBuf(int peers, i64 amps, bool withSend = true) {
    if ((int)g_x.recv.size() >= peers && g_x.amps >= amps && (g_x.hasSend || !withSend)) return;
    be::deviceSync();  // the communication stream may still read the old buffers
    for (real* p : g_x.send) if (p) be::freeComm(p);
    for (real* p : g_x.recv) be::freeComm(p);
    g_x.send.assign(peers, nullptr);
    g_x.recv.assign(peers, nullptr);
    for (int i = 0; i < peers; i++) {
        if (withSend) g_x.send[i] = (real*)be::allocComm(sizeof(real) * 2 * amps);
        g_x.recv[i] = (real*)be::allocComm(sizeof(real) * 2 * amps);
    }
    g_x.amps = amps;
    g_x.hasSend = withSend;
}

inline int chunkBit(const QuregImpl& q, int phys) { return (q.chunkId >> (phys - q.L)) & 1; }

inline bool distributed(const QuregImpl& q) { return q.L < q.nSV; }


// Rank predicates as tags (core.hpp kRankTagMask; QUEST_RANK_TAGS=0: the
// round-5 behaviour, ops queued only where they apply + layout alignment).
bool rankTagsOn(const QuregImpl& q) {
    static const bool on = !getenv("QUEST_RANK_TAGS") || atoi(getenv("QUEST_RANK_TAGS")) != 0;
    return on && distributed(q) && q.L < kRankTagShift;
}

// A fresh tag whose verdict on this rank is `skip` (the same tag id on every
// rank: tags are handed out in op order, which is the same everywhere).  A tag
// is reused after kRankTagCount - 1 newer ones, long after the backend queue
// (at most 1024 ops) has run the op that carried it.
u64 rankTag(QuregImpl& q, bool skip) {
    if (q.rankSkip.empty()) q.rankSkip.assign((size_t)kRankTagCount, 1);
    q.rankTagNext = q.rankTagNext % (kRankTagCount - 1) + 1;
    q.rankSkip[(size_t)q.rankTagNext] = skip ? 1 : 0;
    return (1ull << 62) | ((u64)q.rankTagNext << kRankTagShift);
}

// Rank holding logical chunk c (see QuregImpl::chunkRank).
inline int rankOf(const QuregImpl& q, int c) { return q.chunkRank.empty() ? c : q.chunkRank[(size_t)c]; }

void resetChunks(QuregImpl& q) {
    q.chunkId = rt().rank;
    q.chunkRank.resize((size_t)q.numChunks);
    for (int c = 0; c < q.numChunks; c++) q.chunkRank[(size_t)c] = c;
}

bool chunksIdentity(const QuregImpl& q) {
    for (int c = 0; c < (int)q.chunkRank.size(); c++)
        if (q.chunkRank[(size_t)c] != c) return false;
    return true;
}

inline bool isZero(cplx a) { return a.re == 0 && a.im == 0; }
inline bool isOne(cplx a) { return a.re == 1 && a.im == 0; }

// How a logical op can run given the set of local logical qubits.  A
// one-qubit gate on a RANK qubit needs no data movement when its matrix is
// diagonal (each rank scales its chunk by m[b][b], b = its rank bit) or
// anti-diagonal with only rank-qubit controls (X, Y, controlled-X between
// rank qubits: the chunks trade labels, then each scales by m[b][1-b]).
// The reference exchanges half chunks for every such gate
// (QuEST_cpu_distributed.c:1009-1115, statevec_pauliXDistributed / pauliY).
enum class Place { Local, RankDiag, RankAnti, Blocked };

bool rankGatesOn() {
    static const bool off = getenv("QUEST_RANK_GATES") && atoi(getenv("QUEST_RANK_GATES")) == 0;
    return !off;
}

Place placement(const Op& op, u64 tg, u64 local) {
    if (!(tg & ~local)) return Place::Local;
    if (!rankGatesOn() || op.kind != OpKind::Mat2 || op.nt != 1) return Place::Blocked;
    if (isZero(op.m[1]) && isZero(op.m[2])) return Place::RankDiag;
    if (isZero(op.m[0]) && isZero(op.m[3]) && !(op.ctrl & local)) return Place::RankAnti;
    return Place::Blocked;
}

// Whether the op's targets must be local wherever its controls sit (the swap
// planner only counts such uses).
bool targetsNeedLocal(const Op& op) {
    if (!rankGatesOn() || op.kind != OpKind::Mat2 || op.nt != 1) return true;
    if (isZero(op.m[1]) && isZero(op.m[2])) return false;
    return !(isZero(op.m[0]) && isZero(op.m[3]) && op.ctrl == 0);
}

void enqueue(QuregImpl& q, const Op& op) {
    be::enqueue(q, op);
    stats().opsQueued++;
}

// Exchange the qubits at global positions gpos[m] with those at local
// positions lpos[m] (m < k) in ONE all-to-all among the 2^k ranks that
// differ in those rank bits.  Part j of a chunk (its k local bits = j) goes to
// the peer whose k rank bits = j and comes back from it into the same place,
// so every rank sends (1 - 2^-k) of its chunk, 2^-k of it to each of 2^k - 1
// peers at once -- over as many xGMI links.  A one-qubit swap (k = 1) is the
// reference's pairwise half-chunk exchange; swapping all rank qubits at once
// uses every link (QuEST_cpu_distributed.c:41-512 exchanges whole chunks,
// pairwise, once per gate).
// The swap's pairs ordered by rank bit (peers then come in increasing
// (peer ^ rank) order) and this rank's part: local bits lpos = myG stay here.
void swapOrder(const QuregImpl& q, const int* gposIn, const int* lposIn, int k, int* gpos, int* lpos, int* myG) {
    int idx[8];
    for (int m = 0; m < k; m++) idx[m] = m;
    std::sort(idx, idx + k, [&](int a, int b) { return gposIn[a] < gposIn[b]; });
    for (int m = 0; m < k; m++) {
        gpos[m] = gposIn[idx[m]];
        lpos[m] = lposIn[idx[m]];
    }
    *myG = 0;
    for (int m = 0; m < k; m++) *myG |= chunkBit(q, gpos[m]) << m;
}

// Put every rank's local qubits on rank 0's positions.  The ranks' op lists
// differ -- an op controlled by a rank qubit runs only where that bit is 1, a
// rank-qubit phase only where it is not 1 -- so their planners may relabel
// differently, while a swap cuts its parts by position on both sides (the
// in-place IPC swap even indexes the peer's state with this rank's layout:
// 8 ranks x 22 qubits, bench seeds 13 / 17 lost norm 1e-5 .. 3e-3 before).
// One host broadcast per swap; ranks that differ move their qubits with
// op-free relabelling passes.  Collective.
void alignLayouts(QuregImpl& q) {
    static const bool on = !getenv("QUEST_ALIGN_LAYOUTS") || atoi(getenv("QUEST_ALIGN_LAYOUTS")) != 0;   // (0: study)
    if (!on || !distributed(q)) return;
    if (rankTagsOn(q)) {
        // Round 6: every rank plans the same op list (rank predicates are
        // tags, core.hpp), so the layouts agree by construction.  Checked with
        // a 64-bit hash through the bootstrap's host rendezvous -- no device
        // sync, unlike the layout broadcast -- and aligned below only if they
        // do not (counted in layoutAligns: the tests assert it stays 0).
        u64 h = 1469598103934665603ull;
        for (int p = 0; p < q.L; p++) h = (h ^ (u64)(unsigned)q.p2l[p]) * 1099511628211ull;
        std::vector<u64> all((size_t)rt().numRanks);
        boot::allgather(rt().rank, rt().numRanks, &h, all.data(), sizeof h);
        bool same = true;
        for (u64 x : all) same = same && x == all[0];
        if (same) return;
    }
    int ref[64];
    for (int p = 0; p < 64; p++) ref[p] = p < q.nSV ? q.p2l[p] : -1;
    comm::bcastHost(ref, sizeof ref, 0);
    bool same = true;
    for (int p = 0; p < q.L; p++) same = same && ref[p] == q.p2l[p];
    if (same) return;
    int want[64];   // rank 0's position of each local logical qubit
    for (int x = 0; x < 64; x++) want[x] = -1;
    for (int p = 0; p < q.L; p++) want[ref[p]] = p;
    int dest[64];
    for (int p = 0; p < q.L; p++) {
        dest[p] = want[q.p2l[p]];
        if (dest[p] < 0) {
            fprintf(stderr, "QuEST: rank %d holds local qubit %d, rank 0 does not\n", rt().rank, q.p2l[p]);
            exit(EXIT_FAILURE);
        }
    }
    stats().layoutAligns++;
    trace::event("align_layout", "\"qubits\": %d", q.nSV);
    if (be::permuteLocal(q, dest)) {
        int p2l[64];
        for (int p = 0; p < q.L; p++) p2l[dest[p]] = q.p2l[p];
        for (int p = 0; p < q.L; p++) {
            q.p2l[p] = p2l[p];
            q.l2p[p2l[p]] = p;
        }
        return;
    }
    // no relabelling passes on this backend: SWAP ops, position by position
    static const cplx kSwap[16] = {{1, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {1, 0}, {0, 0},
                                   {0, 0}, {1, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {1, 0}};
    for (int i = 0; i < q.L; i++) {
        if (q.p2l[i] == ref[i]) continue;
        const int x = q.l2p[ref[i]];   // where rank 0's qubit for position i sits here (local, > i)
        Op op;
        op.kind = OpKind::Mat4;
        op.nt = 2;
        op.t[0] = i;
        op.t[1] = x;
        for (int kk = 0; kk < 16; kk++) op.m[kk] = kSwap[kk];
        enqueue(q, op);
        const int li = q.p2l[i];
        q.l2p[li] = x;
        q.p2l[x] = li;
        q.l2p[ref[i]] = i;
        q.p2l[i] = ref[i];
    }
    be::flush(q);
}

void multiSwap(QuregImpl& q, const int* gposIn, const int* lposIn0, int k) {
    if (k <= 0) return;
    be::flush(q);
    // (the victims are logical qubits: their positions after the alignment)
    int victims[8], lposIn[8];
    for (int m = 0; m < k; m++) victims[m] = q.p2l[lposIn0[m]];
    alignLayouts(q);
    for (int m = 0; m < k; m++) lposIn[m] = q.l2p[victims[m]];
    trace::Range range("quest.swap");
    be::swapMark(true);
    const double t0 = trace::now();
    const long long bytes0 = stats().bytesExchanged;
    int gpos[8], lpos[8], myG;
    swapOrder(q, gposIn, lposIn, k, gpos, lpos, &myG);
    const int parts = 1 << k;
    const i64 partSize = q.numAmpsPerChunk >> k;
    i64 slice = (rt().exchangeSliceBytes >> (k - 1)) / (i64)(2 * sizeof(real));
    slice = std::max<i64>(slice, 16);
    slice = std::min(slice, partSize);
    // two buffer sets: slice s is packed into set s & 1 and exchanged on the
    // communication stream while slice s - 1 is unpacked and s + 1 packed
    const int np = parts - 1;
    // the swapped local bits are the top k local positions: part j of the
    // chunk is one contiguous range (its first amplitude index is setMask[j]),
    // sent straight from the state -- no pack, one HBM round trip of 7/8 of
    // the chunk fewer (transports that send from any device memory; RCCL)
    bool direct = false;   // parts sent straight from the state
    if (!comm::swapsInPlace()) {
        bool top = comm::sendsFromState();
        for (int m = 0; m < k; m++) top = top && lpos[m] >= q.L - k;
        static const bool directOn = !getenv("QUEST_SWAP_DIRECT") || atoi(getenv("QUEST_SWAP_DIRECT")) != 0;
        direct = top && directOn;
        ensureXBuf(2 * np, slice, !direct);
    }
    // Overlapped swap (stream-ordered transports, backend.hpp): the exchange
    // runs on a stream of its own next to the passes on the part of the chunk
    // it leaves in place (local bits lpos = myG) -- those planned before it
    // (be::preSwap) and after it; the reference's exchange blocks
    // (QuEST_cpu_distributed.c:451-479)
    const bool overlap = !comm::swapsInPlace() && comm::exchangeStreamOrdered() && be::swapOverlapBegin(q, lpos, k, myG);
    std::vector<comm::Xfer> xs[2] = {std::vector<comm::Xfer>(np), std::vector<comm::Xfer>(np)};
    std::vector<u64> setMask(parts);
    for (int j = 0; j < parts; j++) {
        u64 msk = 0;
        for (int m = 0; m < k; m++)
            if ((j >> m) & 1) msk |= 1ull << lpos[m];
        setMask[j] = msk;
    }
    if (comm::swapsInPlace()) {
        // IPC: the two parts of each rank pair are swapped in place through
        // the peer's mapped state (no buffers; every amplitude read and
        // written once), each rank of the pair taking half of the range so
        // that all ranks move the same bytes (between GPUs both directions of
        // each link carry traffic)
        std::vector<int> peers((size_t)np);
        for (int d = 1; d < parts; d++) {
            int peerChunk = q.chunkId;
            for (int m = 0; m < k; m++)
                if ((d >> m) & 1) peerChunk ^= 1 << (gpos[m] - q.L);
            peers[(size_t)(d - 1)] = rankOf(q, peerChunk);
        }
        std::vector<void*> pp((size_t)(2 * np));
        void* arrays[2] = {q.re, q.im};
        comm::mapPeerArrays(peers.data(), np, arrays, 2, pp.data());
        const i64 half = (partSize / 2) & ~(i64)15;
        for (int d = 1; d < parts; d++) {
            const bool low = rt().rank < peers[(size_t)(d - 1)];
            be::swapPartsWithPeer(q, static_cast<real*>(pp[(size_t)(2 * (d - 1))]),
                                  static_cast<real*>(pp[(size_t)(2 * (d - 1) + 1)]), lpos, k, setMask[myG ^ d],
                                  setMask[myG], low ? 0 : half, low ? half : partSize - half);
        }
        comm::peersDone(peers.data(), np);
        stats().bytesExchanged += (long long)(sizeof(real) * 2 * partSize) * np;
    } else {
        const i64 nSlices = (partSize + slice - 1) / slice;
        if (direct)
            for (int b = 0; b < 2; b++) xs[b].resize((size_t)(2 * np));
        // Receive-side overlap (round 6, be::swapRanges): the slices run in
        // the natural order of the part, i.e. by the chunk's top local
        // positions other than the swapped ones -- the first post-swap passes
        // (whose tiles hold the incoming qubits) run range by range as the
        // ranges land, next to the transfer of the later ones.
        int nRange = 0, rangePos[3];
        i64 perRange = nSlices;
        // (QUEST_SWAP_RANGES_STUDY=1: the ranges' planning constraint on any
        // backend, for host plan studies of its pass count)
        static const bool study = getenv("QUEST_SWAP_RANGES_STUDY") && atoi(getenv("QUEST_SWAP_RANGES_STUDY")) != 0;
        if ((overlap || study) && partSize % slice == 0) {
            for (int p = q.L - 1; p >= 0 && nRange < 3 && (nSlices >> (nRange + 1)) >= 1; p--) {
                bool swapped = false;
                for (int m = 0; m < k; m++) swapped = swapped || lpos[m] == p;
                if (!swapped) rangePos[nRange++] = p;
            }
            if (nRange) {
                // (ascending: bit m of a range index is rangePos[m], the top
                // nRange bits of the packed part index)
                std::reverse(rangePos, rangePos + nRange);
                perRange = nSlices >> nRange;
                be::swapRanges(q, rangePos, nRange);
                // the first pass after the swap holds the incoming qubits: it
                // keeps the ranges' positions out of its tile (their ops wait
                // for the next pass), so it can run range by range
                // (QUEST_SWAP_RANGES_FIRST: how many passes after the swap do,
                // 0 none; the backend runs such passes range-major -- every one
                // of them on range v as soon as v landed)
                // (default: 3 for swaps of 1 or 2 qubits, 2 for 3 -- a link
                // carries 2^-k of the chunk, so the transfer hides fewer passes
                // the larger k; host plan study, 2 ranks x 28 local qubits, five
                // bench seeds' windows: 64 / 66 / 68 passes with 1 / 2 / 3
                // chained, profiles/r6/range_chain.txt)
                static const int firstAvoidEnv = getenv("QUEST_SWAP_RANGES_FIRST") ? atoi(getenv("QUEST_SWAP_RANGES_FIRST"))
                                                                                    : -1;
                const int firstAvoid = firstAvoidEnv >= 0 ? firstAvoidEnv : (k <= 2 ? 3 : 2);
                if (firstAvoid > 0) {
                    for (int i = 0; i < nRange; i++) q.firstPassAvoid |= 1ull << rangePos[i];
                    q.firstAvoidLeft = firstAvoid;
                }
                if (!overlap) nRange = 0;   // (study: no range events)
            }
        }
        auto unpack = [&](i64 s) {
            const int b = (int)(s & 1);
            const i64 off = s * slice, n = std::min(slice, partSize - off);
            for (int d = 1; d < parts; d++) {
                real* r = g_x.recv[(size_t)(b * np + d - 1)];
                be::unpackBits(q, lpos, k, setMask[myG ^ d], off, n, r, r + n);
            }
            if (nRange && (s + 1) % perRange == 0) be::swapRangeLanded(q, (int)(s / perRange));
        };
        for (i64 s = 0; s < nSlices; s++) {
            const int b = (int)(s & 1);
            const i64 off = s * slice, n = std::min(slice, partSize - off);
            for (int d = 1; d < parts; d++) {
                // peers are paired by logical chunk (step d matches chunk c with
                // c ^ D(d) on every rank), then mapped to the rank holding it
                int peerChunk = q.chunkId;
                for (int m = 0; m < k; m++)
                    if ((d >> m) & 1) peerChunk ^= 1 << (gpos[m] - q.L);
                real* rb = g_x.recv[(size_t)(b * np + d - 1)];
                if (direct) {
                    const i64 at = (i64)setMask[myG ^ d] + off;
                    xs[b][(size_t)(2 * (d - 1))] = {rankOf(q, peerChunk), q.re + at, rb, sizeof(real) * (size_t)n};
                    xs[b][(size_t)(2 * (d - 1) + 1)] = {rankOf(q, peerChunk), q.im + at, rb + n, sizeof(real) * (size_t)n};
                    continue;
                }
                real* sb = g_x.send[(size_t)(b * np + d - 1)];
                be::packBits(q, lpos, k, setMask[myG ^ d], off, n, sb, sb + n);
                xs[b][(size_t)(d - 1)] = {rankOf(q, peerChunk), sb, rb, sizeof(real) * 2 * (size_t)n};
            }
            comm::exchangeAsync(xs[b].data(), (int)xs[b].size(), b);
            if (s > 0) {
                comm::exchangeWait(1 - b);
                unpack(s - 1);
            }
            stats().bytesExchanged += (long long)(sizeof(real) * 2 * n) * np;
        }
        comm::exchangeWait((int)((nSlices - 1) & 1));
        unpack(nSlices - 1);
    }
    be::swapMark(false);
    if (overlap) be::swapOverlapEnd(q);
    char moved[128];
    int at = 0;
    moved[0] = 0;
    for (int m = 0; m < k && at < 100; m++)
        at += snprintf(moved + at, sizeof moved - (size_t)at, "%s[%d, %d]", m ? ", " : "", q.p2l[gpos[m]], q.p2l[lpos[m]]);
    for (int m = 0; m < k; m++) {
        const int g = gpos[m], l = lpos[m];
        const int lg = q.p2l[g], ll = q.p2l[l];
        q.l2p[lg] = l;
        q.l2p[ll] = g;
        q.p2l[g] = ll;
        q.p2l[l] = lg;
    }
    stats().swaps += k;
    if (trace::on()) {
        char lp[64];
        int la = 0;
        lp[0] = 0;
        for (int m = 0; m < k && la < 56; m++) la += snprintf(lp + la, sizeof lp - (size_t)la, m ? ", %d" : "%d", lpos[m]);
        trace::event("swap", "\"k\": %d, \"bytes_sent\": %lld, \"host_ms\": %.3f, \"in_out\": [%s], \"lpos\": [%s], "
                     "\"direct\": %d", k, stats().bytesExchanged - bytes0, 1e3 * (trace::now() - t0), moved, lp,
                     (int)direct);
    }
}

u64 logicalTargets(const Op& op) {
    u64 m = 0;
    for (int i = 0; i < op.nt; i++) m |= 1ull << op.t[i];
    return m;
}

// Per-rank scalar (times a local-control mask): Diag op over the chunk.
void scaleChunk(QuregImpl& q, u64 localCtrl, cplx s) {
    if (isOne(s)) return;
    Op op;
    op.kind = OpKind::Diag;
    op.nt = 0;
    op.ctrl = localCtrl;
    op.m[0] = s;
    enqueue(q, op);
}

// Logical op -> physical op for the backend.  Controls (and the phase mask
// of a diagonal op) on rank bits are decided per rank: either this rank's
// whole chunk satisfies them (dropped from the mask) or none of it does (the
// op is skipped here) -- no communication.
void issue(QuregImpl& q, const Op& lop) {
    Op op = lop;
    op.ctrl = 0;
    for (int i = 0; i < lop.nt; i++) op.t[i] = q.l2p[lop.t[i]];
    bool rankCtl = false, skip = false;
    for (u64 c = lop.ctrl; c; c &= c - 1) {
        const int p = q.l2p[__builtin_ctzll(c)];
        if (p >= q.L) {
            rankCtl = true;
            skip = skip || !chunkBit(q, p);
        } else {
            op.ctrl |= 1ull << p;
        }
    }
    if (rankCtl) {
        if (!rankTagsOn(q)) {
            if (skip) return;
        } else {
            op.ctrl |= rankTag(q, skip);
        }
    }
    enqueue(q, op);
}

// A diagonal whose value depends on this rank's chunk: v[b] on the chunks
// whose rank bits `bitsOf` take the value b (b = 0, 1), on amplitudes with the
// local controls; `skipCtl`: the rank controls of the op fail here.  With rank
// tags every rank queues both values (the same ops everywhere); else the
// round-5 per-rank scaling.
void rankDiagPair(QuregImpl& q, u64 localCtrl, bool skipCtl, int b, cplx v0, cplx v1) {
    if (!rankTagsOn(q)) {
        if (!skipCtl) scaleChunk(q, localCtrl, b ? v1 : v0);
        return;
    }
    for (int v = 0; v < 2; v++) {
        const cplx s = v ? v1 : v0;
        if (isOne(s)) continue;   // (the same decision on every rank)
        Op op;
        op.kind = OpKind::Diag;
        op.nt = 0;
        op.ctrl = localCtrl | rankTag(q, skipCtl || b != v);
        op.m[0] = s;
        enqueue(q, op);
    }
}

// Diagonal one-qubit gate on a rank qubit: scale by m[b][b].
void issueRankDiag(QuregImpl& q, const Op& lop) {
    const int b = chunkBit(q, q.l2p[lop.t[0]]);
    u64 ctrl = 0;
    bool skip = false;
    for (u64 c = lop.ctrl; c; c &= c - 1) {
        const int p = q.l2p[__builtin_ctzll(c)];
        if (p >= q.L) {
            skip = skip || !chunkBit(q, p);
        } else {
            ctrl |= 1ull << p;
        }
    }
    if (skip && !rankTagsOn(q)) return;
    stats().globalDiags++;
    rankDiagPair(q, ctrl, skip, b, lop.m[0], lop.m[3]);
}

// Anti-diagonal one-qubit gate on a rank qubit, controls on rank qubits
// only: every chunk satisfying the controls trades its label with the chunk
// differing in the target bit (the same table update on every rank), then the
// new amplitude at bit b is m[b][1-b] times the old one at 1-b.
void issueRankAnti(QuregImpl& q, const Op& lop) {
    const int tb = 1 << (q.l2p[lop.t[0]] - q.L);
    int cm = 0;
    for (u64 c = lop.ctrl; c; c &= c - 1) cm |= 1 << (q.l2p[__builtin_ctzll(c)] - q.L);
    std::vector<int> nr(q.chunkRank);
    for (int c = 0; c < q.numChunks; c++)
        if ((c & cm) == cm) nr[(size_t)(c ^ tb)] = q.chunkRank[(size_t)c];
    q.chunkRank.swap(nr);
    stats().relabels++;
    const bool skip = (q.chunkId & cm) != cm;
    if (skip && !rankTagsOn(q)) return;
    if (!skip) q.chunkId ^= tb;
    const int b = (q.chunkId & tb) ? 1 : 0;
    rankDiagPair(q, 0, skip, b, lop.m[1], lop.m[2]);
}

// Exchange this rank's whole chunk with `peer`'s (every pair of a round calls
// this at once), pipelined in slices through two buffer sets as in multiSwap:
// slice s is copied out and exchanged on the communication stream while
// slice s - 1 is copied in.
void swapWholeChunk(QuregImpl& q, int peer, i64 slice) {
    if (comm::swapsInPlace()) {
        std::vector<void*> pp(2);
        void* arrays[2] = {q.re, q.im};
        comm::mapPeerArrays(&peer, 1, arrays, 2, pp.data());
        const i64 half = (q.numAmpsPerChunk / 2) & ~(i64)15;
        const bool low = rt().rank < peer;
        be::swapPartsWithPeer(q, static_cast<real*>(pp[0]), static_cast<real*>(pp[1]), nullptr, 0, 0, 0,
                              low ? 0 : half, low ? half : q.numAmpsPerChunk - half);
        comm::peersDone(&peer, 1);
        stats().bytesExchanged += (long long)(sizeof(real) * 2 * q.numAmpsPerChunk);
        return;
    }
    const i64 nSlices = (q.numAmpsPerChunk + slice - 1) / slice;
    comm::Xfer xs[2];
    for (i64 s = 0; s < nSlices; s++) {
        const int b = (int)(s & 1);
        const i64 off = s * slice, n = std::min(slice, q.numAmpsPerChunk - off);
        be::toBuffer(q, off, n, g_x.send[(size_t)b], g_x.send[(size_t)b] + n);
        xs[b] = {peer, g_x.send[(size_t)b], g_x.recv[(size_t)b], sizeof(real) * 2 * (size_t)n};
        comm::exchangeAsync(&xs[b], 1, b);
        if (s > 0) {
            comm::exchangeWait(1 - b);
            const i64 po = (s - 1) * slice, pn = std::min(slice, q.numAmpsPerChunk - po);
            be::fromBuffer(q, po, pn, g_x.recv[(size_t)(1 - b)], g_x.recv[(size_t)(1 - b)] + pn);
        }
        stats().bytesExchanged += (long long)(sizeof(real) * 2 * n);
    }
    const int b = (int)((nSlices - 1) & 1);
    comm::exchangeWait(b);
    const i64 po = (nSlices - 1) * slice, pn = std::min(slice, q.numAmpsPerChunk - po);
    be::fromBuffer(q, po, pn, g_x.recv[(size_t)b], g_x.recv[(size_t)b] + pn);
}

// Move the data so that rank r holds logical chunk r again.  The chunk at
// rank r belongs at rank f(r) (its logical id); f is a product of two
// involutions (per cycle c0 -> c1 -> ... of f: the reflections c_i <-> c_(L-1-i)
// and then c_j <-> c_(L-j)), so at most two rounds of disjoint pairwise
// whole-chunk exchanges restore the placement, all pairs of a round at once
// over their own links.  The X gates on rank qubits that cause such
// placements make f an involution: one round.  (The round-3 code walked the
// pairs one after another.)
void restoreChunks(QuregImpl& q) {
    if (chunksIdentity(q)) return;
    be::flush(q);
    alignLayouts(q);   // whole chunks are exchanged by position
    const int R = q.numChunks, me = rt().rank;
    std::vector<int> f((size_t)R), rounds[2] = {std::vector<int>((size_t)R), std::vector<int>((size_t)R)};
    for (int c = 0; c < R; c++) f[(size_t)q.chunkRank[(size_t)c]] = c;
    for (int r = 0; r < R; r++) rounds[0][(size_t)r] = rounds[1][(size_t)r] = r;
    std::vector<char> seen((size_t)R, 0);
    for (int r = 0; r < R; r++) {
        if (seen[(size_t)r]) continue;
        std::vector<int> cyc;
        for (int x = r; !seen[(size_t)x]; x = f[(size_t)x]) {
            seen[(size_t)x] = 1;
            cyc.push_back(x);
        }
        const int L = (int)cyc.size();
        for (int i = 0; i < L; i++) {
            rounds[0][(size_t)cyc[(size_t)i]] = cyc[(size_t)(L - 1 - i)];
            rounds[1][(size_t)cyc[(size_t)i]] = cyc[(size_t)((L - i) % L)];
        }
    }
    const i64 slice = std::min<i64>(q.numAmpsPerChunk, std::max<i64>(rt().exchangeSliceBytes / (i64)(2 * sizeof(real)), 1));
    if (!comm::swapsInPlace()) ensureXBuf(2, slice);
    for (const std::vector<int>& pairOf : rounds) {
        bool any = false;
        for (int r = 0; r < R; r++) any = any || pairOf[(size_t)r] != r;
        if (!any) continue;
        stats().restoreRounds++;
        if (pairOf[(size_t)me] != me) swapWholeChunk(q, pairOf[(size_t)me], slice);
    }
    if (trace::on()) {
        int nr = 0;
        for (const std::vector<int>& pairOf : rounds)
            for (int r = 0; r < R; r++)
                if (pairOf[(size_t)r] != r) {
                    nr++;
                    break;
                }
        trace::event("restore_chunks", "\"rounds\": %d", nr);
    }
    for (int c = 0; c < R; c++) q.chunkRank[(size_t)c] = c;
    q.chunkId = me;
}

// Choose the qubits to bring onto local positions for the queued ops (the
// first one must become runnable) and swap them in with one all-to-all:
// every rank qubit the queue still targets comes in, in order of first use,
// displacing the local qubits whose first use lies furthest ahead (Belady),
// as long as that is later than the incoming qubit's.
// victims (local qubits to move out) for the qubits in[] the queue needs:
// furthest next locality-requiring use first; 0 if one of them sits on a
// position in `busy`; gp / lp as multiSwap takes them
int chooseVictims(QuregImpl& q, const std::vector<Op>& lq, u64 busy, int* gp, int* lp);

void planSwap(QuregImpl& q, const std::vector<Op>& lq) {
    // Victims chosen BEFORE the backend's queue is planned (QUEST_SWAP_EARLY,
    // default on) when none of them sits on a position a queued op targets
    // (nor on the low positions every tile holds).  The planner keeps those
    // positions out of its tiles (q.tileAvoid), so its relabelling passes
    // cannot move the victims, and the backend can split the pre-swap passes
    // around the swap (be::preSwap): the parts the swap sends first, the part
    // it keeps next to the transfer.  Without a victim outside the queue's
    // targets: run what the backend holds first, then choose (its passes may
    // relabel local qubits, and the positions must be the ones the swap moves
    // -- multiSwap's own flush would otherwise move whatever qubit a relabel
    // put at the victim's old position, a needless later swap).
    static const bool early = !getenv("QUEST_SWAP_EARLY") || atoi(getenv("QUEST_SWAP_EARLY")) != 0;
    int gp[8], lp[8], k = 0;
    int vlog[8];   // early victims as logical qubits: the flush below may still relabel them
    if (early) {
        k = chooseVictims(q, lq, be::queuedTargets(q), gp, lp);
        for (int m = 0; m < k; m++) vlog[m] = q.p2l[lp[m]];
        static const bool dbg = getenv("QUEST_SWAP_DEBUG") != nullptr;
        if (dbg)
            fprintf(stderr, "rank %d swap: victims chosen %s the flush (%zu ops queued)\n", rt().rank,
                    k ? "before" : "after", q.pending.size());
        if (k > 0) {
            u64 avoid = 0;
            for (int m = 0; m < k; m++) avoid |= 1ull << lp[m];
            q.tileAvoid = avoid;
            int gs[8], ls[8], myG;
            swapOrder(q, gp, lp, k, gs, ls, &myG);
            if (!comm::swapsInPlace() && comm::exchangeStreamOrdered()) be::preSwap(q, ls, k, myG);
        }
    }
    if (k == 0) {   // the victims as logical qubits (the same choice after the flush)
        int g2[8], l2[8];
        const int k2 = chooseVictims(q, lq, 0, g2, l2);
        q.nSwapVictims = k2;
        for (int m = 0; m < k2; m++) q.swapVictims[m] = q.p2l[l2[m]];
        // (their positions stay out of tile padding: a pass that does not
        // target them leaves them out)
        static const bool avoidPad = !getenv("QUEST_SWAP_AVOID") || atoi(getenv("QUEST_SWAP_AVOID")) != 0;
        if (avoidPad)
            for (int m = 0; m < k2; m++) q.tileAvoid |= 1ull << l2[m];
    }
    be::flush(q);
    q.nSwapVictims = 0;
    // (queuedTargets keeps the victims off the positions every tile holds for
    // the default planner only -- cmin <= 8; a larger QUEST_WAVE_CMIN or a
    // search strategy with one more resident position can relabel them: the
    // swap takes the logical victims wherever the flush left them, the same
    // qubits on every rank)
    for (int m = 0; m < k; m++) lp[m] = q.l2p[vlog[m]];
    if (k == 0) k = chooseVictims(q, lq, 0, gp, lp);
    if (k == 0) {
        fprintf(stderr, "QuEST: no local qubit available for a distributed swap\n");
        exit(EXIT_FAILURE);
    }
    multiSwap(q, gp, lp, k);
    q.tileAvoid = 0;
}

int chooseVictims(QuregImpl& q, const std::vector<Op>& lq, u64 busy, int* gp, int* lp) {
    const int INF = 1 << 30;
    int first[64];
    for (int i = 0; i < 64; i++) first[i] = INF;
    for (int i = 0; i < (int)lq.size(); i++) {
        if (i > 0 && !targetsNeedLocal(lq[i])) continue;
        for (int t = 0; t < lq[i].nt; t++)
            if (first[lq[i].t[t]] == INF) first[lq[i].t[t]] = i;
    }
    const u64 need0 = logicalTargets(lq[0]);
    // On a fully connected xGMI node an all-to-all moving k qubits sends
    // chunk / 2^k over each of 2^k - 1 links at once, so its time FALLS with
    // k: every rank qubit is swapped whenever one must be, qubits nothing
    // needs filling the spare positions (a k = 1 swap would push half the
    // chunk through a single link).
    std::vector<int> in, out;
    for (int lg = 0; lg < q.nSV; lg++)
        if (q.l2p[lg] >= q.L) in.push_back(lg);
    std::sort(in.begin(), in.end(), [&](int a, int b) { return first[a] < first[b]; });
    for (int lg = 0; lg < q.nSV; lg++)
        if (q.l2p[lg] < q.L && !((need0 >> lg) & 1)) out.push_back(lg);
    // (ties keep the logical order: breaking them by position -- to put
    // victims on the top positions for direct sends -- moved which qubit the
    // next window needs back and added a swap, host-build study)
    std::stable_sort(out.begin(), out.end(), [&](int a, int b) { return first[a] > first[b]; });
    int k = 0;
    for (size_t i = 0; i < in.size() && i < out.size() && k < 8; i++) {
        const bool required = (need0 >> in[i]) & 1;
        if (!required && first[out[i]] < first[in[i]]) break;
        gp[k] = q.l2p[in[i]];
        lp[k] = q.l2p[out[i]];
        k++;
    }
    // (busy: the victims must all sit outside it -- they are the same logical
    // qubits the choice after the flush would take, so the swap count does
    // not change; else the caller chooses again after its flush: a filtered
    // choice took victims needed sooner, 4 ranks x 26 qubits 2 -> 3-5 swaps
    // per window on three of five bench seeds)
    for (int m = 0; m < k; m++)
        if ((busy >> lp[m]) & 1) return 0;
    return k;
}

// Route the logical queue of a distributed register: issue, in commutation-
// respecting order, every op whose targets are local; when blocked, swap in
// the qubits the remaining ops need; repeat.
void flushLogical(QuregImpl& q) {
    std::vector<Op>& lq = q.lpending;
    while (!lq.empty()) {
        u64 local = 0;
        for (int lg = 0; lg < q.nSV; lg++)
            if (q.l2p[lg] < q.L) local |= 1ull << lg;
        std::vector<Op> rest;
        rest.reserve(lq.size());
        u64 blockedTg = 0, blockedTouch = 0;
        for (const Op& op : lq) {
            const u64 tg = logicalTargets(op), touch = tg | op.ctrl;
            const Place pl = placement(op, tg, local);
            if (!(tg & blockedTouch) && !(touch & blockedTg) && pl != Place::Blocked) {
                if (pl == Place::Local)
                    issue(q, op);
                else if (pl == Place::RankDiag)
                    issueRankDiag(q, op);
                else
                    issueRankAnti(q, op);
            } else {
                rest.push_back(op);
                blockedTg |= tg;
                blockedTouch |= touch;
            }
        }
        lq.swap(rest);
        if (!lq.empty()) planSwap(q, lq);
    }
}

constexpr size_t kLogicalWindow = 1024;

// Accept a logical op: single-rank registers go straight to the backend.
void submit(QuregImpl& q, const Op& lop) {
    q.stateGen++;
    if (!distributed(q)) {
        issue(q, lop);
        return;
    }
    q.lpending.push_back(lop);
    if (q.lpending.size() >= kLogicalWindow) flushLogical(q);
}

// Everything routed and handed to the backend (queue flushed, async).
void drain(QuregImpl& q) {
    flushLogical(q);
    be::flush(q);
}

// Identity qubit layout and chunk placement (callers overwrite the state).
void resetLayout(QuregImpl& q) {
    q.stateGen++;
    for (int i = 0; i < 64; i++) {
        q.l2p[i] = q.p2l[i] = i;
        q.lastUse[i] = 0;
    }
    resetChunks(q);
}

i64 logicalToPhysicalIndex(const QuregImpl& q, i64 idx) {
    if (q.numChunks == 1 && q.permIdentity()) return idx;
    i64 p = 0;
    for (int j = 0; j < q.nSV; j++)
        if ((idx >> j) & 1) p |= (i64)1 << q.l2p[j];
    return p;
}

}  // namespace

MemoryPlan memoryPlan(int nSV, int numRanks) {
    int g = 0;
    while ((1 << g) < numRanks) g++;
    const int L = nSV - g;
    MemoryPlan m;
    m.state = 2ll * (long long)sizeof(real) << L;
    // multiSwap with k rank qubits: 2 (send, recv) x 2 (double buffer) x
    // (2^k - 1) peers x slice amps x [re | im]; restoreChunks: one peer.
    // An upper bound: RCCL swaps of top-position parts allocate the receive
    // buffers only, and in-place IPC swaps none.
    const i64 partMax = (i64)1 << L;
    for (int k = 1; k <= g; k++) {
        i64 slice = (rt().exchangeSliceBytes >> (k - 1)) / (i64)(2 * sizeof(real));
        slice = std::min(std::max<i64>(slice, 16), partMax >> k);
        const long long b = 2ll * 2 * ((1ll << k) - 1) * slice * 2 * (long long)sizeof(real);
        m.exchange = std::max(m.exchange, b);
    }
    if (g > 0) {   // restoreChunks: two buffer sets of send + recv
        const i64 slice = std::min<i64>(partMax, std::max<i64>(rt().exchangeSliceBytes / (i64)(2 * sizeof(real)), 1));
        m.exchange = std::max(m.exchange, 2ll * 2 * slice * 2 * (long long)sizeof(real));
    }
    m.scratch = 64ll << 20;
    m.total = m.state + m.exchange + m.scratch;
    return m;
}

bool footprintCheck(int nSV, int numRanks, std::string& report) {
    int g = 0;
    while ((1 << g) < numRanks) g++;
    if (g == 0 || (1 << g) != numRanks || rt().numRanks != 1) {
        report = "footprintCheck: a single-process job and a power-of-two rank count > 1";
        return false;
    }
    const MemoryPlan m = memoryPlan(nSV, numRanks);
    // the buffers of the largest exchange: a k = g all-to-all (multiSwap)
    const int L = nSV - g, np = (1 << g) - 1;
    i64 slice = (rt().exchangeSliceBytes >> (g - 1)) / (i64)(2 * sizeof(real));
    slice = std::min(std::max<i64>(slice, 16), ((i64)1 << L) >> g);
    const size_t bytes = sizeof(real) * 2 * (size_t)slice;
    size_t f0 = 0, f1 = 0, tot = 0;
    be::deviceSync();
    const bool known = be::memoryInfo(&f0, &tot);
    std::vector<void*> send((size_t)(2 * np)), recv((size_t)(2 * np));
    for (int i = 0; i < 2 * np; i++) {
        send[(size_t)i] = be::allocComm(bytes);
        recv[(size_t)i] = be::allocComm(bytes);
    }
    be::memoryInfo(&f1, &tot);
    std::string r;
    const bool ok = comm::selfTest(r, send.data(), recv.data(), 2 * np, bytes);
    for (int i = 0; i < 2 * np; i++) {
        be::freeComm(send[(size_t)i]);
        be::freeComm(recv[(size_t)i]);
    }
    const double G = 1024.0 * 1024 * 1024;
    char head[512];
    snprintf(head, sizeof head,
             "%d qubits on %d ranks: per rank state %.2f GiB + exchange %.3f GiB (%d x 2 buffers of %.0f MiB, the "
             "k = %d all-to-all) + scratch %.2f GiB = %.2f GiB; device %.2f GiB, free %.2f GiB before the buffers, "
             "%.2f GiB with them%s; ",
             nSV, numRanks, m.state / G, 2.0 * 2 * np * bytes / G, 2 * np, bytes / 1048576.0, g, m.scratch / G,
             m.total / G, tot / G, f0 / G, f1 / G, known ? "" : " (unknown)");
    report = std::string(head) + r;
    // The plan's exchange term is the largest of the k = 1 .. g all-to-alls'
    // and the chunk restore's buffer sets (direct / in-place swaps allocate
    // less): recomputed here from the slice rule, it must equal the plan
    // exactly, and the k = g buffers just allocated must fit in it.
    long long bound = 0;
    for (int k = 1; k <= g; k++) {
        i64 sk = (rt().exchangeSliceBytes >> (k - 1)) / (i64)(2 * sizeof(real));
        sk = std::min(std::max<i64>(sk, 16), ((i64)1 << L) >> k);
        bound = std::max(bound, 2ll * 2 * ((1ll << k) - 1) * (long long)sizeof(real) * 2 * sk);
    }
    const i64 sr = std::min<i64>((i64)1 << L, std::max<i64>(rt().exchangeSliceBytes / (i64)(2 * sizeof(real)), 1));
    bound = std::max(bound, 2ll * 2 * (long long)sizeof(real) * 2 * sr);
    return ok && bound == m.exchange && (long long)(2 * 2 * np * bytes) <= m.exchange;
}

void create(QuregImpl& q, int nSV, bool density) {
    int g = 0;
    while ((1 << g) < rt().numRanks) g++;
    q.nSV = nSV;
    q.isDensity = density;
    q.nRep = density ? nSV / 2 : nSV;
    q.L = nSV - g;
    q.numChunks = rt().numRanks;
    q.numAmpsTotal = (i64)1 << nSV;
    q.numAmpsPerChunk = (i64)1 << q.L;
    resetLayout(q);
    be::allocState(q);
    if (trace::on())
        trace::event("create", "\"qubits\": %d, \"density\": %d, \"local_qubits\": %d, \"ranks\": %d", nSV,
                     density ? 1 : 0, q.L, q.numChunks);
}

void destroy(QuregImpl& q) {
    drain(q);
    if (trace::on()) trace::event("destroy", "\"qubits\": %d", q.nSV);
    be::freeState(q);
}

void flush(QuregImpl& q) { drain(q); }

void sync(QuregImpl& q) {
    drain(q);
    be::deviceSync();
}

// ---------------------------------------------------------------------------
// ops
// ---------------------------------------------------------------------------

void mat2(QuregImpl& q, int target, const int* ctrls, int nc, const cplx m[4]) {
    Op op;
    op.kind = OpKind::Mat2;
    op.nt = 1;
    op.t[0] = target;
    for (int i = 0; i < nc; i++) op.ctrl |= 1ull << ctrls[i];
    for (int i = 0; i < 4; i++) op.m[i] = m[i];
    submit(q, op);
}

void diag(QuregImpl& q, const int* qubits, int nq, cplx term) {
    Op op;
    op.kind = OpKind::Diag;
    op.nt = 0;
    for (int i = 0; i < nq; i++) op.ctrl |= 1ull << qubits[i];
    op.m[0] = term;
    submit(q, op);
}

void mat4(QuregImpl& q, int q0, int q1, const cplx m[16]) {
    Op op;
    op.kind = OpKind::Mat4;
    op.nt = 2;
    op.t[0] = q0;
    op.t[1] = q1;
    for (int i = 0; i < 16; i++) op.m[i] = m[i];
    submit(q, op);
}

void densChan2(QuregImpl& q, int r1, int r2, int c1, int c2, real offFac, real keep, real mix) {
    Op op;
    op.kind = OpKind::DensChan2;
    op.nt = 4;
    op.t[0] = r1;
    op.t[1] = r2;
    op.t[2] = c1;
    op.t[3] = c2;
    op.m[0] = {offFac, 0};
    op.m[1] = {keep, 0};
    op.m[2] = {mix, 0};
    submit(q, op);
}

void collapse(QuregImpl& q, int qubit, int outcome, real renorm) {
    q.stateGen++;
    flushLogical(q);
    int p = q.l2p[qubit];
    if (p >= q.L) {
        const cplx keep = {renorm, 0}, drop = {0, 0};
        if (rankTagsOn(q)) {   // (the same two ops on every rank)
            rankDiagPair(q, 0, false, chunkBit(q, p), outcome ? drop : keep, outcome ? keep : drop);
            return;
        }
        Op op;
        op.kind = OpKind::Diag;
        op.nt = 0;
        op.ctrl = 0;
        op.m[0] = chunkBit(q, p) == outcome ? keep : drop;
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
    q.stateGen++;
    // keep elements whose row bit (qubit) and column bit (qubit + n) both equal
    // the outcome; scale them by 1/prob (reference divides by p, not sqrt(p))
    flushLogical(q);
    real s = (real)1 / prob;
    int r = q.l2p[qubit], c = q.l2p[qubit + q.nRep];
    bool rGlobal = r >= q.L, cGlobal = c >= q.L;
    if (rGlobal && cGlobal) {
        bool keepChunk = chunkBit(q, r) == outcome && chunkBit(q, c) == outcome;
        if (rankTagsOn(q)) {   // (the same two ops on every rank)
            rankDiagPair(q, 0, false, keepChunk ? 1 : 0, {0, 0}, {s, 0});
            return;
        }
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
        if (rankTagsOn(q)) {
            // (the same two ops on every rank: the projector where the
            // chunk's bit is the outcome, zero elsewhere)
            const bool match = chunkBit(q, gpos) == outcome;
            op.kind = OpKind::Mat2;
            op.nt = 1;
            op.t[0] = lpos;
            op.ctrl = rankTag(q, !match);
            op.m[0] = {outcome == 0 ? s : (real)0, 0};
            op.m[1] = {0, 0};
            op.m[2] = {0, 0};
            op.m[3] = {outcome == 1 ? s : (real)0, 0};
            enqueue(q, op);
            Op z;
            z.kind = OpKind::Diag;
            z.nt = 0;
            z.ctrl = rankTag(q, match);
            z.m[0] = {0, 0};
            enqueue(q, z);
            return;
        }
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
    drain(q);
    resetLayout(q);
    be::fill(q, 0, 0);
    i64 start = (i64)q.chunkId * q.numAmpsPerChunk;
    if (index >= start && index < start + q.numAmpsPerChunk) be::setAmp(q, index - start, 1, 0);
}

void initUniform(QuregImpl& q, real val) {
    drain(q);
    resetLayout(q);
    be::fill(q, val, 0);
}

void initDebug(QuregImpl& q) {
    drain(q);
    resetLayout(q);
    be::initDebug(q, (i64)q.chunkId * q.numAmpsPerChunk);
}

void initSingleQubit(QuregImpl& q, int qubit, int outcome, real val) {
    drain(q);
    resetLayout(q);
    if (qubit >= q.L) {
        be::fill(q, chunkBit(q, qubit) == outcome ? val : (real)0, 0);
    } else {
        be::fillWhereBit(q, qubit, outcome, val);
    }
}

void setAmps(QuregImpl& q, i64 start, const real* re, const real* im, i64 n) {
    q.stateGen++;
    if (n == q.numAmpsTotal && start == 0) {
        drain(q);
        resetLayout(q);
    } else {
        canonicalise(q);
    }
    i64 c0 = (i64)q.chunkId * q.numAmpsPerChunk, c1 = c0 + q.numAmpsPerChunk;
    i64 lo = std::max(start, c0), hi = std::min(start + n, c1);
    if (lo < hi) be::writeAmps(q, lo - c0, re + (lo - start), im + (lo - start), hi - lo);
}

void clone(QuregImpl& dst, QuregImpl& src) {
    drain(src);
    drain(dst);
    be::copyState(dst, src);
    dst.stateGen++;
    memcpy(dst.l2p, src.l2p, sizeof dst.l2p);
    memcpy(dst.p2l, src.p2l, sizeof dst.p2l);
    memcpy(dst.lastUse, src.lastUse, sizeof dst.lastUse);
    dst.chunkId = src.chunkId;  // each rank copied its own (logical) chunk
    dst.chunkRank = src.chunkRank;
    dst.useClock = src.useClock;
}

// Gather the full canonical pure state (2^n amps) onto every rank.
static void gatherPure(QuregImpl& psi, real** fullRe, real** fullIm) {
    canonicalise(psi);
    drain(psi);
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
    drain(rho);
    resetLayout(rho);
    be::densInitPure(rho, fr, fi, rho.nRep, (i64)rho.chunkId * rho.numAmpsPerChunk);
    be::freeComm(fr);
    be::freeComm(fi);
}

// Two registers of the same shape whose rank qubits and chunk placement agree
// but whose local qubits may sit on different positions: sig[p] = b's
// position of the qubit a holds at local position p.  False when their
// global layouts differ (then both go to the canonical layout).
static bool localPermutation(const QuregImpl& a, const QuregImpl& b, int* sig) {
    if (a.L != b.L || a.nSV != b.nSV || a.chunkRank != b.chunkRank || a.chunkId != b.chunkId) return false;
    for (int j = 0; j < a.nSV; j++) {
        const int pa = a.l2p[j], pb = b.l2p[j];
        if ((pa >= a.L || pb >= b.L) && pa != pb) return false;
        if (pa < a.L) sig[pa] = pb;
    }
    return true;
}

// QUEST_PERM_KERNELS=0: relayout both registers as before round 4
static bool permKernels() {
    static const bool on = !getenv("QUEST_PERM_KERNELS") || atoi(getenv("QUEST_PERM_KERNELS")) != 0;
    return on;
}

void axpby(QuregImpl& a, real alpha, QuregImpl& b, real beta) {
    drain(a);  // routing may move qubits: compare layouts afterwards
    drain(b);
    int sig[64];
    if (memcmp(a.l2p, b.l2p, sizeof(int) * a.nSV) == 0 && a.chunkRank == b.chunkRank) {
        be::axpby(a, alpha, b, beta);
    } else if (permKernels() && localPermutation(a, b, sig)) {
        // b read in a's layout by the permuted kernel: no relayout of either
        stats().permutedOps++;
        be::axpbyPerm(a, alpha, b, beta, sig);
    } else {
        canonicalise(a);
        canonicalise(b);
        be::axpby(a, alpha, b, beta);
    }
    a.stateGen++;
}

void canonicalise(QuregImpl& q) {
    drain(q);
    if (q.permIdentity() && chunksIdentity(q)) return;
    stats().relayouts++;
    // 1. the right logical qubit on every global position, in all-to-all
    //    rounds: first every global position whose qubit is local comes in;
    //    qubits stuck on the wrong global position are first moved out to
    //    local positions that hold no rank qubit
    for (int round = 0; round < 4; round++) {
        int gp[8], lp[8], k = 0;
        for (int g = q.L; g < q.nSV; g++)
            if (q.p2l[g] != g && q.l2p[g] < q.L) {
                gp[k] = g;
                lp[k] = q.l2p[g];
                k++;
            }
        if (k == 0) {
            for (int g = q.L; g < q.nSV; g++) {
                if (q.p2l[g] == g) continue;
                for (int v = 0; v < q.L; v++) {
                    bool used = q.p2l[v] >= q.L;
                    for (int m = 0; m < k && !used; m++) used = lp[m] == v;
                    if (used) continue;
                    gp[k] = g;
                    lp[k] = v;
                    k++;
                    break;
                }
            }
        }
        if (k == 0) break;
        multiSwap(q, gp, lp, k);
    }
    // 2. every rank holds its own chunk again (undo X-gate relabellings)
    restoreChunks(q);
    // 3. permute local qubits: op-free relabelling passes of the wave engine
    //    (a permuted store, up to 12 qubits per HBM round trip), else SWAP ops
    {
        int dest[64];
        bool moved = false;
        for (int p = 0; p < q.L; p++) {
            dest[p] = q.p2l[p];
            moved = moved || dest[p] != p;
        }
        static const bool relayout = !getenv("QUEST_RELAYOUT_PASSES") || atoi(getenv("QUEST_RELAYOUT_PASSES")) != 0;
        if (moved && relayout && be::permuteLocal(q, dest)) {
            for (int p = 0; p < q.L; p++) q.l2p[p] = q.p2l[p] = p;
            return;
        }
    }
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
    drain(q);
}

// ---------------------------------------------------------------------------
// reads and reductions
// ---------------------------------------------------------------------------

cplx getAmp(QuregImpl& q, i64 flatIndex) {
    drain(q);
    i64 p = logicalToPhysicalIndex(q, flatIndex);
    int owner = (int)(p >> q.L);
    real v[2] = {0, 0};
    if (owner == q.chunkId) be::readAmps(q, p & (q.numAmpsPerChunk - 1), &v[0], &v[1], 1);
    if (q.numChunks > 1) comm::bcastHost(v, sizeof v, rankOf(q, owner));
    return {v[0], v[1]};
}

static double allSum(double x) {
    if (comm::active()) comm::allreduceSum(&x, 1);
    return x;
}

// P(qubit = 0) times the norm.  The first query after a state change reads
// the half of the state it needs; a second query of the same state computes
// every qubit's marginal in one pass (be::marginals, one allreduce of nSV + 1
// values) and later queries are answered from that cache until the next
// change.  Programs that read all marginals back to back (the fork's
// tutorial_example.c:521-525) stream the state 1.5 times instead of n / 2.
// The decisions depend only on stateGen, which changes identically on every
// rank, so all ranks take the same collective path.
static bool marginalCacheOn() {
    static const bool off = getenv("QUEST_MARGINAL_CACHE") && atoi(getenv("QUEST_MARGINAL_CACHE")) == 0;
    return !off;
}

double probZero(QuregImpl& q, int qubit) {
    drain(q);
    if (marginalCacheOn() && q.margGen == q.stateGen) return q.margP0[qubit];
    stats().reductions++;
    // a qubit on one of the lowest local positions shares every 128-byte
    // line between its two halves: its own reduction streams the whole
    // chunk anyway, so compute every marginal in that pass
    const int pq = q.l2p[qubit];
    const bool wholeLines = pq < q.L && ((i64)sizeof(real) << pq) < 128;
    if (marginalCacheOn() && (q.probGen == q.stateGen || wholeLines)) {
        double z[65], tot;
        be::marginals(q, z, &tot);
        double v[65];
        for (int lg = 0; lg < q.nSV; lg++) {
            const int p = q.l2p[lg];
            v[lg] = p < q.L ? z[p] : (chunkBit(q, p) == 0 ? tot : 0.0);
        }
        v[q.nSV] = tot;
        if (comm::active()) comm::allreduceSum(v, q.nSV + 1);
        memcpy(q.margP0, v, sizeof(double) * (size_t)(q.nSV + 1));
        q.margGen = q.stateGen;
        stats().marginalPasses++;
        return q.margP0[qubit];
    }
    q.probGen = q.stateGen;
    int p = q.l2p[qubit];
    double part;
    if (p >= q.L)
        part = chunkBit(q, p) == 0 ? be::sumSq(q, -1, 0) : 0.0;
    else
        part = be::sumSq(q, p, 0);
    return allSum(part);
}

// The norm, cached like the marginals: a normalisation check after every
// measurement round or a repeated calcTotalProb reads the state once.
double sumSqAll(QuregImpl& q) {
    drain(q);
    if (marginalCacheOn() && q.margGen == q.stateGen) return q.margP0[q.nSV];
    if (marginalCacheOn() && q.normGen == q.stateGen) return q.normCache;
    stats().reductions++;
    q.normCache = allSum(be::sumSq(q, -1, 0));
    q.normGen = q.stateGen;
    return q.normCache;
}

static double densDiag(QuregImpl& q, int skipBit) {
    drain(q);
    stats().reductions++;
    u64 offs[64];
    for (int j = 0; j < q.nRep; j++) offs[j] = (1ull << q.l2p[j]) | (1ull << q.l2p[j + q.nRep]);
    double part = be::densDiagSum(q, offs, q.nRep, skipBit, (i64)q.chunkId * q.numAmpsPerChunk);
    return allSum(part);
}

double densProbZero(QuregImpl& q, int qubit) { return densDiag(q, qubit); }
double densTrace(QuregImpl& q) { return densDiag(q, -1); }

cplx inner(QuregImpl& bra, QuregImpl& ket) {
    drain(bra);  // routing may move qubits: compare layouts afterwards
    drain(ket);
    stats().reductions++;
    double v[2];
    int sig[64];
    if (memcmp(bra.l2p, ket.l2p, sizeof(int) * bra.nSV) == 0 && bra.chunkRank == ket.chunkRank) {
        be::innerProduct(bra, ket, v);
    } else if (permKernels() && localPermutation(bra, ket, sig)) {
        // the reference sums locally and allreduces (QuEST_cpu_distributed.c:41-51);
        // so does this, with ket read in bra's layout -- no relayout
        stats().permutedOps++;
        be::innerProductPerm(bra, ket, sig, v);
    } else {
        canonicalise(bra);
        canonicalise(ket);
        be::innerProduct(bra, ket, v);
    }
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

void prepareOverwrite(QuregImpl& q) {
    drain(q);
    resetLayout(q);
}

void touch(QuregImpl& q) { q.stateGen++; }

void writeChunk(QuregImpl& q, const real* re, const real* im) {
    drain(q);
    resetLayout(q);
    be::writeAmps(q, 0, re, im, q.numAmpsPerChunk);
}

}  // namespace router
}  // namespace qa
