#include "tiles.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <mutex>
#include <cmath>
#include <complex>
#include <cstdlib>
#include <cstring>

namespace qa {

namespace {

u64 targetMask(const Op& op) {
    u64 m = 0;
    for (int i = 0; i < op.nt; i++) m |= 1ull << op.t[i];
    return m;
}

int popcount64(u64 x) { return __builtin_popcountll(x); }

void emitPass(const std::vector<Op>& ops, int b, int e, u64 tmask, int L, int k, int cmin, TileProgram& out,
              u64 avoid = 0) {
    TilePass ps;
    ps.k = k;
    // Q = low cmin bits + targets, padded with the lowest remaining bits
    // (not the avoided ones, unless nothing else is left)
    u64 q = tmask | ((cmin >= 64) ? ~0ull : ((1ull << cmin) - 1));
    for (int bit = 0; popcount64(q) < k && bit < L; bit++)
        if (!((avoid >> bit) & 1)) q |= 1ull << bit;
    for (int bit = 0; popcount64(q) < k && bit < L; bit++) q |= 1ull << bit;
    ps.qmask = q;
    int n = 0;
    int tileOf[64];
    for (int bit = 0; bit < L; bit++) {
        tileOf[bit] = -1;
        if ((q >> bit) & 1) {
            tileOf[bit] = n;
            ps.stPos[n] = bit;
            ps.pos[n++] = bit;
        }
    }
    ps.k = n;
    ps.opBegin = (int)out.ops.size();
    for (int i = b; i < e; i++) {
        const Op& op = ops[i];
        TileOp t;
        memset(&t, 0, sizeof t);
        t.kind = (int)op.kind;
        for (int j = 0; j < op.nt; j++) t.t[j] = tileOf[op.t[j]];
        for (int bit = 0; bit < L; bit++) {
            if (!((op.ctrl >> bit) & 1)) continue;
            if (tileOf[bit] >= 0)
                t.ctrlIn |= 1u << tileOf[bit];
            else
                t.ctrlOut |= 1ull << bit;
        }
        t.ctrlOut |= op.ctrl & kRankTagMask;   // a rank predicate: out of every tile (core.hpp)
        int nm = op.kind == OpKind::Mat2 ? 4 : op.kind == OpKind::Mat4 ? 16 : op.kind == OpKind::Diag ? 1 : 3;
        for (int j = 0; j < nm; j++) {
            t.m[2 * j] = op.m[j].re;
            t.m[2 * j + 1] = op.m[j].im;
        }
        laneSwaps(t, n);
        out.ops.push_back(t);
    }
    ps.opEnd = (int)out.ops.size();
    out.passes.push_back(ps);
}

}  // namespace

namespace {
unsigned insertZero(unsigned x, int b) { return ((x >> b) << (b + 1)) | (x & ((1u << b) - 1u)); }

void fillUniformParts(TileOp& op, int k) {
    const unsigned th = tileThreads(k);
    const int nt = op.kind == (int)OpKind::Mat2 ? 1 : op.kind == (int)OpKind::Mat4 ? 2 : 0;
    int lo = op.t[0], hi = op.t[0];
    if (nt == 2) {
        lo = std::min(op.t[0], op.t[1]);
        hi = std::max(op.t[0], op.t[1]);
    }
    for (int u = 0; u < 16; u++) {
        unsigned p = th * (unsigned)u;
        if (nt >= 1) p = insertZero(p, lo);
        if (nt == 2) p = insertZero(p, hi);
        for (int s = 0; s < op.nsw; s++) {
            const unsigned a = op.swA[s], b = op.swB[s];
            const unsigned x = ((p >> a) ^ (p >> b)) & 1u;
            p ^= (x << a) | (x << b);
        }
        op.du[u] = p;
        op.sdu[u] = ldsSwizzle(p);
    }
}
}  // namespace

namespace {
// swaps for (target mask, k): computed once per distinct pair
struct SwapPlan {
    int nsw = 0;
    unsigned char a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
};

SwapPlan computeSwaps(unsigned tmask, int k) {
    SwapPlan plan;
    int map[32], nf = 0;  // work-item bit i -> element bit map[i]
    for (int bit = 0; bit < k; bit++)
        if (!((tmask >> bit) & 1)) map[nf++] = bit;
    // GF(2) bases in echelon form: slot[l] holds the vector with leading bit l
    unsigned bR[8] = {0}, bW[8] = {0};
    auto reduce = [](const unsigned* basis, unsigned v) {
        for (int l = 7; l >= 0; l--)
            if (((v >> l) & 1) && basis[l]) v ^= basis[l];
        return v;
    };
    auto insert = [&](unsigned* basis, unsigned v) {
        v = reduce(basis, v);
        if (!v) return;
        int l = 31 - __builtin_clz(v);
        basis[l] = v;
    };
    for (int i = 0; i < 5 && i < nf; i++) {
        auto fits = [&](int e) {
            const unsigned v = ldsSwizzle(1u << e);
            return reduce(bR, v & 31u) != 0 && (i >= 4 || reduce(bW, v & 15u) != 0);
        };
        if (!fits(map[i])) {
            int j = -1;
            for (int c = i + 1; c < nf; c++)
                if (fits(map[c])) {
                    j = c;
                    break;
                }
            if (j < 0 || plan.nsw == 4) continue;  // best effort
            plan.a[plan.nsw] = (unsigned char)map[i];
            plan.b[plan.nsw] = (unsigned char)map[j];
            plan.nsw++;
            std::swap(map[i], map[j]);
        }
        const unsigned v = ldsSwizzle(1u << map[i]);
        insert(bR, v & 31u);
        if (i < 4) insert(bW, v & 15u);
    }
    return plan;
}
}  // namespace

void laneSwaps(TileOp& op, int k) {
    op.nsw = 0;
    if (op.kind != (int)OpKind::Mat2 && op.kind != (int)OpKind::Mat4) {
        fillUniformParts(op, k);
        return;
    }
    const int nt = op.kind == (int)OpKind::Mat2 ? 1 : 2;
    unsigned tmask = 0;
    for (int i = 0; i < nt; i++) tmask |= 1u << op.t[i];
    // memo: 1 + 2 targets among at most 16 tile bits, per tile size
    static thread_local std::vector<std::pair<unsigned long long, SwapPlan>> memo;
    const unsigned long long key = ((unsigned long long)k << 32) | tmask;
    const SwapPlan* plan = nullptr;
    for (auto& kv : memo)
        if (kv.first == key) {
            plan = &kv.second;
            break;
        }
    if (!plan) {
        memo.emplace_back(key, computeSwaps(tmask, k));
        plan = &memo.back().second;
    }
    op.nsw = plan->nsw;
    for (int s = 0; s < plan->nsw; s++) {
        op.swA[s] = plan->a[s];
        op.swB[s] = plan->b[s];
    }
    fillUniformParts(op, k);
}

namespace {

using zc = std::complex<double>;

// A run of gates on at most two qubits, multiplied into one matrix on the
// host: 4x4 in the basis (bit 0 <-> s[0], bit 1 <-> s[1]); a one-qubit block
// uses the top-left 2x2 as a matrix on s[0].
struct Block {
    int ns = 0;
    int s[2] = {-1, -1};
    zc m[4][4];
    int first = -1;      // index of its first op in the input
    int count = 0;       // ops absorbed
    bool allDiag = true;
};

// The op as a 4x4 matrix in the basis of block b (whose support contains the
// op's qubits).
void embed(const Op& op, const Block& b, zc e[4][4]) {
    auto bitOf = [&](int q) { return q == b.s[0] ? 0 : 1; };
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) e[r][c] = r == c ? 1.0 : 0.0;
    const int dim = b.ns == 2 ? 4 : 2;
    if (op.kind == OpKind::Diag) {
        unsigned mask = 0;
        for (u64 c = op.ctrl; c; c &= c - 1) mask |= 1u << bitOf(__builtin_ctzll(c));
        for (int i = 0; i < dim; i++)
            if ((i & mask) == mask) e[i][i] = zc(op.m[0].re, op.m[0].im);
        return;
    }
    if (op.kind == OpKind::Mat2) {
        const int tb = bitOf(op.t[0]);
        unsigned cmask = 0;
        for (u64 c = op.ctrl; c; c &= c - 1) cmask |= 1u << bitOf(__builtin_ctzll(c));
        for (int i = 0; i < dim; i++) {
            if ((i & cmask) != cmask || ((i >> tb) & 1)) continue;
            const int j = i | (1 << tb);
            e[i][i] = zc(op.m[0].re, op.m[0].im);
            e[i][j] = zc(op.m[1].re, op.m[1].im);
            e[j][i] = zc(op.m[2].re, op.m[2].im);
            e[j][j] = zc(op.m[3].re, op.m[3].im);
        }
        return;
    }
    // Mat4 on (t0, t1): op index g = bit(t0) + 2 bit(t1)
    const int b0 = bitOf(op.t[0]), b1 = bitOf(op.t[1]);
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) {
            const int gr = ((r >> b0) & 1) | (((r >> b1) & 1) << 1);
            const int gc = ((c >> b0) & 1) | (((c >> b1) & 1) << 1);
            e[r][c] = zc(op.m[4 * gr + gc].re, op.m[4 * gr + gc].im);
        }
}

void leftMultiply(Block& b, const zc e[4][4]) {
    zc out[4][4];
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) {
            zc acc = 0;
            for (int k = 0; k < 4; k++) acc += e[r][k] * b.m[k][c];
            out[r][c] = acc;
        }
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) b.m[r][c] = out[r][c];
}

// qubits an op touches, if it can join a two-qubit block (else -1)
int support(const Op& op, int q[2]) {
    int n = 0;
    auto add = [&](int x) {
        for (int i = 0; i < n; i++)
            if (q[i] == x) return true;
        if (n == 2) return false;
        q[n++] = x;
        return true;
    };
    if (op.kind == OpKind::DensChan2) return -1;
    if (op.kind == OpKind::Mat4 && op.ctrl) return -1;
    if (op.ctrl & kRankTagMask) return -1;   // rank-predicated ops stay single (core.hpp)
    for (int i = 0; i < op.nt; i++)
        if (!add(op.t[i])) return -1;
    for (u64 c = op.ctrl; c; c &= c - 1)
        if (!add(__builtin_ctzll(c))) return -1;
    return n;
}

}  // namespace

bool& fuseBlocks() {
    static bool on = [] {
        const char* e = getenv("QUEST_FUSE_BLOCKS");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

int& planMaxOps() {
    static int m = [] {
        const char* e = getenv("QUEST_PLAN_MAX_OPS");
        return e ? atoi(e) : 0;
    }();
    return m;
}

int& fuseBlockQubits() {
    static thread_local int q = 2;   // per thread: planner worker threads set their own
    return q;
}

void fuseGates(std::vector<Op>& ops) {
    const int n = (int)ops.size();
    if (n < 2) return;
    std::vector<Block> blocks;
    std::vector<int> opBlock(n, -1);  // block of each op (-1: kept as is)
    int last[64];                      // block last touching each qubit; -2 barrier, -1 none
    for (int i = 0; i < 64; i++) last[i] = -1;
    for (int i = 0; i < n; i++) {
        const Op& op = ops[i];
        int q[2];
        int ns = support(op, q);
        if (ns > fuseBlockQubits()) ns = -1;
        if (ns < 0) {  // barrier on every qubit it touches
            for (int t = 0; t < op.nt; t++) last[op.t[t]] = -2;
            for (u64 c = op.ctrl; c; c &= c - 1) last[__builtin_ctzll(c)] = -2;
            continue;
        }
        if (ns == 0) continue;  // global phase on the whole chunk: leave in place
        // joinable block: every qubit of the op last touched by the same block
        // (or by nothing), and the union support stays within two qubits
        int bid = -1;
        bool ok = true;
        for (int k = 0; k < ns && ok; k++) {
            const int l = last[q[k]];
            if (l == -2) ok = false;
            else if (l >= 0) {
                if (bid >= 0 && bid != l) ok = false;
                bid = l;
            }
        }
        if (ok && bid >= 0) {
            Block& b = blocks[bid];
            int extra = 0, ex = -1;
            for (int k = 0; k < ns; k++)
                if (q[k] != b.s[0] && q[k] != b.s[1]) extra++, ex = q[k];
            if (b.ns + extra > 2) ok = false;
            else if (extra == 1) {  // grow a one-qubit block: M -> I (x) M on the new qubit
                b.s[1] = ex;
                b.ns = 2;
                zc g[4][4];
                for (int r = 0; r < 4; r++)
                    for (int c = 0; c < 4; c++) g[r][c] = ((r >> 1) == (c >> 1)) ? b.m[r & 1][c & 1] : zc(0);
                for (int r = 0; r < 4; r++)
                    for (int c = 0; c < 4; c++) b.m[r][c] = g[r][c];
            }
        } else if (ok) {
            bid = -1;
        }
        if (!ok) bid = -1;
        if (bid < 0) {
            // blocked by another block: start a new one (the op's qubits'
            // previous blocks are closed for it)
            Block b;
            b.ns = ns;
            b.s[0] = q[0];
            b.s[1] = ns == 2 ? q[1] : -1;
            for (int r = 0; r < 4; r++)
                for (int c = 0; c < 4; c++) b.m[r][c] = r == c ? 1.0 : 0.0;
            b.first = i;
            blocks.push_back(b);
            bid = (int)blocks.size() - 1;
        }
        Block& b = blocks[bid];
        zc e[4][4];
        embed(op, b, e);
        leftMultiply(b, e);
        b.count++;
        b.allDiag = b.allDiag && op.kind == OpKind::Diag;
        opBlock[i] = bid;
        for (int k = 0; k < ns; k++) last[q[k]] = bid;
    }
    // emit: a block at the position of its first op; blocks of one op, or of
    // diagonal ops only, keep their original ops
    std::vector<Op> out;
    out.reserve(n);
    for (int i = 0; i < n; i++) {
        const int bid = opBlock[i];
        if (bid < 0 || blocks[bid].count == 1 || blocks[bid].allDiag) {
            out.push_back(ops[i]);
            continue;
        }
        const Block& b = blocks[bid];
        if (b.first != i) continue;
        Op f;
        f.ctrl = 0;
        if (b.ns == 1) {
            f.kind = OpKind::Mat2;
            f.nt = 1;
            f.t[0] = b.s[0];
            for (int r = 0; r < 2; r++)
                for (int c = 0; c < 2; c++) f.m[2 * r + c] = {(real)b.m[r][c].real(), (real)b.m[r][c].imag()};
        } else {
            f.kind = OpKind::Mat4;
            f.nt = 2;
            f.t[0] = b.s[0];
            f.t[1] = b.s[1];
            for (int r = 0; r < 4; r++)
                for (int c = 0; c < 4; c++) f.m[4 * r + c] = {(real)b.m[r][c].real(), (real)b.m[r][c].imag()};
        }
        out.push_back(f);
    }
    ops.swap(out);
}

thread_local int t_planCommute = -1;

bool programRelabels(const TileProgram& prog) {
    for (const TilePass& ps : prog.passes)
        for (int i = 0; i < ps.k; i++)
            if (ps.stPos[i] != ps.pos[i]) return true;
    return false;
}

namespace {

// Permute physical positions of an op by pi (positions not in pi unchanged).
void remapOp(Op& op, const int* pi) {
    for (int j = 0; j < op.nt; j++) op.t[j] = pi[op.t[j]];
    u64 c = 0;
    for (u64 m = op.ctrl; m; m &= m - 1) c |= 1ull << pi[__builtin_ctzll(m)];
    op.ctrl = c;
}

// Propose a store permutation for the pass just emitted (ps): the tile's
// positions >= from hold some logical qubits; the ones the queue needs soonest
// take the low positions [from, c), which every later tile contains, and the
// qubits they displace take the vacated high positions.  `mode` ranks the
// qubits: 0 by their first use in the queue, 1 by their uses among the next
// 64 ops.  pi (a product of disjoint swaps, so its own inverse) is the
// identity when nothing would move.
bool proposePerm(const std::vector<Op>& ops, const std::vector<char>& done, int first, int from, int c,
                 const TilePass& ps, int mode, int* pi) {
    const int INF = 1 << 30;
    int need[64];
    for (int p = 0; p < 64; p++) {
        need[p] = INF;
        pi[p] = p;
    }
    u64 open = 0;
    for (int i = 0; i < ps.k; i++) open |= 1ull << ps.pos[i];
    if (mode == 1) {
        int cnt[64] = {0};
        for (int i = first, seen = 0; i < (int)ops.size() && seen < 64; i++) {
            if (done[i]) continue;
            seen++;
            for (u64 tg = targetMask(ops[i]) & open; tg; tg &= tg - 1) cnt[__builtin_ctzll(tg)]++;
        }
        for (int p = 0; p < 64; p++) need[p] = cnt[p] ? 64 - cnt[p] : INF;
    } else {
        for (int i = first, rank = 0; i < (int)ops.size() && open; i++) {
            if (done[i]) continue;
            for (u64 tg = targetMask(ops[i]) & open; tg; tg &= tg - 1) {
                const int p = __builtin_ctzll(tg);
                need[p] = rank;
                open &= ~(1ull << p);
            }
            rank++;
        }
    }
    std::vector<int> cand;
    for (int i = 0; i < ps.k; i++)
        if (ps.pos[i] >= from) cand.push_back(ps.pos[i]);
    // soonest first; among equals keep the qubits already low
    std::stable_sort(cand.begin(), cand.end(), [&](int a, int b) {
        if (need[a] != need[b]) return need[a] < need[b];
        return (a < c) > (b < c);
    });
    const int slots = c - from;
    std::vector<int> in, freeLow;
    std::vector<char> chosenLow(64, 0);
    for (int x = 0; x < slots && x < (int)cand.size(); x++) {
        if (need[cand[x]] == INF) break;
        if (cand[x] < c)
            chosenLow[cand[x]] = 1;
        else
            in.push_back(cand[x]);
    }
    for (int p = from; p < c; p++)
        if (!chosenLow[p]) freeLow.push_back(p);
    // the low qubits needed latest make room first
    std::stable_sort(freeLow.begin(), freeLow.end(), [&](int a, int b) { return need[a] > need[b]; });
    bool any = false;
    for (size_t x = 0; x < in.size() && x < freeLow.size(); x++) {
        const int hi = in[x], lo = freeLow[x];
        if (need[lo] <= need[hi]) continue;
        pi[hi] = lo;
        pi[lo] = hi;
        any = true;
    }
    return any;
}

// A diagonal Mat2 with unit-modulus entries (Z, S, T, Rz, phase shifts and
// their controlled forms) as Diag ops: d1 / d0 on its controls + target, and
// d0 on its controls alone (dropped when 1).  A Diag op needs no tile bit, so
// the target qubit no longer has to be in the pass's tile.
void phasesFromDiagonals(std::vector<Op>& ops) {
    std::vector<Op> out;
    out.reserve(ops.size() + ops.size() / 4);
    for (const Op& op : ops) {
        const bool diag = op.kind == OpKind::Mat2 && op.m[1].re == 0 && op.m[1].im == 0 && op.m[2].re == 0 &&
                          op.m[2].im == 0;
        const double a0 = diag ? std::hypot((double)op.m[0].re, (double)op.m[0].im) : 0;
        const double a1 = diag ? std::hypot((double)op.m[3].re, (double)op.m[3].im) : 0;
        const double tol = sizeof(real) >= 8 ? 1e-14 : 1e-6;
        if (!diag || std::fabs(a0 - 1) > tol || std::fabs(a1 - 1) > tol) {
            out.push_back(op);
            continue;
        }
        const cplx d0 = op.m[0], d1 = op.m[3];
        // d1 / d0 = d1 * conj(d0) for |d0| = 1
        const cplx q = {d1.re * d0.re + d1.im * d0.im, d1.im * d0.re - d1.re * d0.im};
        Op a;
        a.kind = OpKind::Diag;
        a.nt = 0;
        a.ctrl = op.ctrl | (1ull << op.t[0]);
        a.m[0] = q;
        if (!(d0.re == 1 && d0.im == 0)) {
            Op b = a;
            b.ctrl = op.ctrl;
            b.m[0] = d0;
            out.push_back(b);
        }
        out.push_back(a);
    }
    ops.swap(out);
}

// QUEST_DIAG_PHASES: 0 never, 1 always, 2 (default) for queues of at most
// 4 ops per qubit
int& diagAsPhases() {
    static int v = getenv("QUEST_DIAG_PHASES") ? atoi(getenv("QUEST_DIAG_PHASES")) : 2;
    return v;
}

// QUEST_PLAN_COMMUTE=1: class-aware commutation in the pass scheduler; 0
// (default) the round-4 rule: ops touching a common bit never pass each other
// unless both touch it diagonally as controls / phase masks.  Over 15 bench
// seeds the greedy planner made 254 passes with it and 251 without (per seed
// -4 .. +4): more freedom per pass does not make the greedy plan better.
bool planCommute() {
    static const bool v = getenv("QUEST_PLAN_COMMUTE") && atoi(getenv("QUEST_PLAN_COMMUTE")) != 0;
    return t_planCommute >= 0 ? t_planCommute != 0 : v;
}

// 0: diagonal 2x2, 1: a I + b X, 2: anything else (multi-target ops too)
int commuteClass(const Op& op) {
    if (op.kind != OpKind::Mat2) return op.kind == OpKind::Diag ? 0 : 2;
    auto zero = [](cplx z) { return z.re == 0 && z.im == 0; };
    auto same = [](cplx a, cplx b) { return a.re == b.re && a.im == b.im; };
    if (zero(op.m[1]) && zero(op.m[2])) return 0;
    if (same(op.m[0], op.m[3]) && same(op.m[1], op.m[2])) return 1;
    return 2;
}

void applyPerm(std::vector<Op>& ops, const std::vector<char>& done, int first, const int* pi) {
    for (int i = first; i < (int)ops.size(); i++)
        if (!done[i]) remapOp(ops[i], pi);
}

}  // namespace

namespace {
// QUEST_PLAN_PROFILE=1: host time of planTiles by section, printed at exit
// (where a small register's planning goes: tools/experiments/plan_profile.sh)
struct PlanProfile {
    static constexpr int N = 8;
    const char* names[N] = {"prep", "candidates", "trim", "emit", "relabel-choice", "relabel-ok", "low-perm",
                            "pass-ready"};
    double ms[N] = {0};
    long calls = 0, passes = 0;
    std::mutex mu;
    bool on = getenv("QUEST_PLAN_PROFILE") && atoi(getenv("QUEST_PLAN_PROFILE")) != 0;
    ~PlanProfile() {
        if (!on || !calls) return;
        double tot = 0;
        for (double x : ms) tot += x;
        fprintf(stderr, "plan profile: %ld planTiles calls, %ld passes, %.3f ms (%.1f us / pass):", calls, passes, tot,
                passes ? 1e3 * tot / passes : 0.0);
        for (int i = 0; i < N; i++) fprintf(stderr, " %s %.3f", names[i], ms[i]);
        fprintf(stderr, "\n");
    }
};
PlanProfile& planProfile() {
    static PlanProfile p;
    return p;
}
struct PlanClock {
    bool on;
    double acc[PlanProfile::N] = {0};
    std::chrono::steady_clock::time_point t;
    PlanClock() : on(planProfile().on) {
        if (on) t = std::chrono::steady_clock::now();
    }
    void lap(int k) {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        acc[k] += std::chrono::duration<double, std::milli>(n - t).count();
        t = n;
    }
    void flush(long passes) {
        if (!on) return;
        PlanProfile& p = planProfile();
        std::lock_guard<std::mutex> g(p.mu);
        for (int i = 0; i < PlanProfile::N; i++) p.ms[i] += acc[i];
        p.calls++;
        p.passes += passes;
    }
};
}  // namespace

void planTiles(std::vector<Op>& ops, int L, int kmax, int cmin, bool fuse, TileProgram& out, int relabelFrom,
               const PlanHooks* hooks) {
    PlanClock clk;
    out.passes.clear();
    out.ops.clear();
    out.perm.resize(L);
    for (int x = 0; x < L; x++) out.perm[x] = x;
    if (ops.empty()) return;
    const int k = std::min(kmax, L);
    const int c = std::min(cmin, k);
    const u64 low = (c >= 64) ? ~0ull : ((1ull << c) - 1);
    // high targets allowed per pass besides the always-present low bits
    const int highSlots = k - c;
    int n = (int)ops.size();

    const bool ready = hooks && hooks->passReady;
    const u64 avoid = hooks ? hooks->avoidMask : 0;
    if (!fuse) {
        for (int i = 0; i < n; i++) {
            emitPass(ops, i, i + 1, targetMask(ops[i]), L, k, c, out, avoid);
            if (ready) hooks->passReady(out, i, ops);
        }
        return;
    }
    if (fuseBlocks()) {
        fuseGates(ops);
        n = (int)ops.size();
    }
    // short queues (a program that reads the state every layer or two): the
    // targets of lone diagonal gates are a binding constraint of the few
    // passes such a flush gets (window1: 194 -> 182 passes over 3 seeds);
    // over long windows the planner places them anyway (91 vs 93 passes)
    if (diagAsPhases() == 1 || (diagAsPhases() == 2 && n <= 4 * L)) {
        phasesFromDiagonals(ops);
        n = (int)ops.size();
    }

    clk.lap(0);
    // List scheduling with commutation: a pass greedily collects every queued
    // op whose targets fit the pass's tile bits and that commutes with all the
    // earlier ops left for later passes.  Two ops commute when neither's
    // targets meet the other's touched bits (controls and diagonal phase masks
    // act diagonally, so they commute among themselves).  Diagonal ops need
    // no tile bits at all.
    std::vector<Op> order;
    order.reserve(n);
    std::vector<char> done(n, 0);
    int first = 0;
    std::vector<int> take, best;
    const int maxOps = planMaxOps();
    // Commutation classes of one-target ops (QUEST_PLAN_COMMUTE=1): a
    // diagonal 2x2 (Z, S, T, Rz, phase shifts) commutes with controls and with
    // other diagonals on its target; an "X-class" 2x2 (a I + b X: X, Rx, the X
    // of CNOT / Toffoli) commutes with other X-class ops on its target, whatever
    // their controls (on every control configuration both act as commuting
    // 2x2s or not at all).  Anything else, and multi-target ops, conflicts with
    // every deferred op touching its targets.
    std::vector<unsigned char> cls(n, 2);   // 0 diagonal, 1 X-class, 2 general
    const bool commute = planCommute();
    if (commute)
        for (int i = 0; i < n; i++) cls[i] = (unsigned char)commuteClass(ops[i]);
    // one greedy scan from `first` with the high bits `preset` claimed up front
    const u64 firstAvoid = hooks ? hooks->firstPassAvoid : 0;
    const int firstAvoidN = hooks ? hooks->firstAvoidPasses : 0;
    auto scan = [&](u64 preset, std::vector<int>& picked) {
        picked.clear();
        u64 high = preset;
        const u64 hardAvoid = (int)out.passes.size() < firstAvoidN ? firstAvoid : 0;
        u64 blockedTg = 0;      // targets of ops deferred past this pass
        u64 blockedTouch = 0;   // targets | controls of deferred ops
        // (class-aware) deferred targets of diagonal / X-class / general ops,
        // and deferred controls and phase masks
        u64 bD = 0, bX = 0, bG = 0, bC = 0;
        for (int i = first; i < n; i++) {
            if (done[i]) continue;
            const u64 tg = targetMask(ops[i]);
            const u64 touch = tg | ops[i].ctrl;
            bool free;
            if (commute) {
                const int k2 = cls[i];
                const u64 hitT = k2 == 0 ? (bX | bG) : k2 == 1 ? (bD | bC | bG) : (bD | bX | bG | bC);
                free = !(tg & hitT) && !(ops[i].ctrl & (bX | bG));
            } else {
                free = !(tg & blockedTouch) && !(touch & blockedTg);
            }
            const u64 need = high | (tg & ~low);
            if (free && !(tg & hardAvoid) && popcount64(need) <= highSlots &&
                (maxOps <= 0 || (int)picked.size() < maxOps)) {
                high = need;
                picked.push_back(i);
            } else {
                blockedTg |= tg;
                blockedTouch |= touch;
                if (commute) {
                    (cls[i] == 0 ? bD : cls[i] == 1 ? bX : bG) |= tg;
                    bC |= ops[i].ctrl;
                }
            }
        }
        return high;
    };
    // Compute-aware passes (PlanHooks::passCost): drop ops from the end of a
    // pass predicted to be compute-bound, as long as each dropped op could run
    // in any later pass at no extra tile bits (a phase, or targets among the
    // always-resident low positions), no op kept after it in the pass depends
    // on it, and some op outside the pass remains anyway (there will be a
    // later pass to take them).
    auto trimPass = [&](std::vector<int>& v, u64 high) {
        auto cost = [&](const std::vector<int>& sel) {
            std::vector<Op> tmp;
            tmp.reserve(sel.size());
            for (int i : sel) tmp.push_back(ops[i]);
            TileProgram scratch;
            emitPass(tmp, 0, (int)tmp.size(), high, L, k, c, scratch, avoid);
            const TilePass& ps = scratch.passes.back();
            return hooks->passCost(ps, scratch.ops.data() + ps.opBegin);
        };
        const double C = cost(v);
        const double bound = hooks->memCost * (1 + hooks->costMargin);
        if (C <= bound) return;
        // another op stays queued after this pass?
        std::vector<char> inPass(n, 0);
        for (int i : v) inPass[i] = 1;
        bool rest = false;
        for (int i = first; i < n && !rest; i++) rest = !done[i] && !inPass[i];
        if (!rest) return;
        const double perOp = C / (double)v.size();
        double excess = C - bound;
        std::vector<char> drop(v.size(), 0);
        u64 keptTg = 0, keptTouch = 0;   // of the kept ops after the candidate
        for (int x = (int)v.size() - 1; x >= 0 && excess > 0; x--) {
            const Op& op = ops[v[(size_t)x]];
            const u64 tg = targetMask(op), touch = tg | op.ctrl;
            const bool movable = op.kind == OpKind::Diag || (op.kind == OpKind::Mat2 && !(tg & ~low));
            if (movable && !(tg & keptTouch) && !(touch & keptTg)) {
                drop[(size_t)x] = 1;
                excess -= perOp;
                continue;
            }
            keptTg |= tg;
            keptTouch |= touch;
        }
        std::vector<int> kept;
        for (size_t x = 0; x < v.size(); x++)
            if (!drop[x]) kept.push_back(v[x]);
        static const bool dbg = getenv("QUEST_PLAN_TRIM_DEBUG") != nullptr;
        if (dbg) {
            int movable = 0;
            for (int i : v) {
                const u64 tg = targetMask(ops[i]);
                movable += ops[i].kind == OpKind::Diag || (ops[i].kind == OpKind::Mat2 && !(tg & ~low));
            }
            fprintf(stderr, "trim: C %.0f bound %.0f ops %zu movable %d dropped %zu\n", C, bound, v.size(), movable,
                    v.size() - kept.size());
        }
        if (kept.size() < v.size() && !kept.empty()) v.swap(kept);
    };
    // Rollout scoring (QUEST_PLAN_ROLLOUT=1, experiment): a candidate
    // pass is judged by how many passes the plain greedy planner (with
    // first-use relabelling) then needs for the rest of the queue --
    // fewer first, more ops taken now on ties
    static const int rolloutEnv = getenv("QUEST_PLAN_ROLLOUT") ? atoi(getenv("QUEST_PLAN_ROLLOUT")) : 0;
    const int rollout = hooks && hooks->rollout >= 0 ? hooks->rollout : rolloutEnv;
    auto tileFor = [&](u64 high) {
        TilePass ps;
        u64 q = high | low;
        for (int bit = 0; popcount64(q) < k && bit < L; bit++)
            if (!((avoid >> bit) & 1)) q |= 1ull << bit;
        for (int bit = 0; popcount64(q) < k && bit < L; bit++) q |= 1ull << bit;
        int m = 0;
        for (int bit = 0; bit < L; bit++)
            if ((q >> bit) & 1) ps.pos[m++] = bit;
        ps.k = m;
        return ps;
    };
    auto rolloutPasses = [&](const std::vector<int>& cand, u64 candHigh) {
        const std::vector<Op> keepOps(ops.begin() + first, ops.end());
        const int keepFirst = first;
        std::vector<int> marked(cand);
        for (int i : cand) done[i] = 1;
        int passes = 0;
        u64 high = candHigh;
        std::vector<int> pick;
        while (true) {
            while (first < n && done[first]) first++;
            if (first >= n) break;
            if (relabelFrom >= 0 && rollout >= 1) {
                int pi[64];
                if (proposePerm(ops, done, first, relabelFrom, c, tileFor(high), 0, pi)) applyPerm(ops, done, first, pi);
            }
            high = scan(0, pick);
            if (pick.empty()) break;
            for (int i : pick) {
                done[i] = 1;
                marked.push_back(i);
            }
            passes++;
        }
        for (int i : marked) done[i] = 0;
        first = keepFirst;
        std::copy(keepOps.begin(), keepOps.end(), ops.begin() + first);
        return passes;
    };
    while ((int)order.size() < n) {
        while (done[first]) first++;
        const int begin = (int)order.size();
        // candidates: plain in-order greedy, and greedy seeded with the high
        // targets of one of the next few ops; keep the pass holding most ops
        u64 bestHigh = scan(0, best);
        // candidate score: ops taken, plus a bonus for ops from the front of
        // the queue (deferring them blocks everything behind them)
        static const double alpha = getenv("QUEST_PLAN_ALPHA") ? atof(getenv("QUEST_PLAN_ALPHA")) : 0.0;
        static const int frontN = getenv("QUEST_PLAN_FRONT") ? atoi(getenv("QUEST_PLAN_FRONT")) : 32;
        int frontEnd = first;
        for (int c = 0; frontEnd < n && c < frontN; frontEnd++)
            if (!done[frontEnd]) c++;
        // (0.3 since round 6 with the pass-time-model score of the search:
        // profiles/r6/plan_seeds.txt; 0 before)
        static const double betaEnv = getenv("QUEST_PLAN_LOOKAHEAD") ? atof(getenv("QUEST_PLAN_LOOKAHEAD"))
                                                                       : (sizeof(real) == 8 ? 0.3 : 0.0);
        const double beta = hooks && hooks->lookahead >= 0 ? hooks->lookahead : betaEnv;
        std::vector<int> nextTake;
        auto score = [&](const std::vector<int>& v) {
            int f = 0;
            for (int i : v) f += i < frontEnd;
            double sc = (double)v.size() + alpha * f;
            if (beta > 0) {
                // one-pass lookahead: how much the plain greedy pass after it takes
                for (int i : v) done[i] = 1;
                const int keepFirst = first;
                while (first < n && done[first]) first++;
                if (first < n) scan(0, nextTake); else nextTake.clear();
                first = keepFirst;
                for (int i : v) done[i] = 0;
                sc += beta * (double)nextTake.size();
            }
            return sc;
        };
        double bestScore = rollout ? -1e6 * rolloutPasses(best, bestHigh) + (double)best.size() : score(best);
        // (48 seeds, 32 distinct target sets: round 6's host study priced by the
        // measured pass-time model, profiles/r6/plan_seeds.txt -- 24 / 16 before)
        static const int maxSeedsEnv = [] {
            const char* e = getenv("QUEST_PLAN_SEEDS");
            return e ? atoi(e) : (sizeof(real) == 8 ? 48 : 24);   // (fp32: not tuned with the model, round 5's)
        }();
        const int maxSeeds = hooks && hooks->seeds > 0 ? hooks->seeds : maxSeedsEnv;
        int seeds = 0;
        // distinct seed target sets tried per pass (QUEST_PLAN_TRIED, at most 64)
        static const int maxTried = [] {
            const char* e = getenv("QUEST_PLAN_TRIED");
            return e ? std::max(1, std::min(64, atoi(e))) : (sizeof(real) == 8 ? 32 : 16);
        }();
        u64 tried[64];
        int nTried = 0;
        for (int i = first; i < n && seeds < maxSeeds; i++) {
            if (done[i]) continue;
            const u64 h = targetMask(ops[i]) & ~low;
            if (!h || ((int)out.passes.size() < firstAvoidN && (h & firstAvoid))) continue;
            seeds++;
            bool dup = false;
            for (int t = 0; t < nTried; t++) dup |= tried[t] == h;
            if (dup || nTried == maxTried) continue;
            tried[nTried++] = h;
            const u64 hh = scan(h, take);
            const double sc = rollout ? -1e6 * rolloutPasses(take, hh) + (double)take.size() : score(take);
            if (sc > bestScore) {
                best.swap(take);
                bestHigh = hh;
                bestScore = sc;
            }
        }
        clk.lap(1);
        if (hooks && hooks->passCost && hooks->memCost > 0 && best.size() > 1) trimPass(best, bestHigh);
        clk.lap(2);
        for (int i : best) {
            order.push_back(ops[i]);
            done[i] = 1;
        }
        emitPass(order, begin, (int)order.size(), bestHigh, L, k, c, out,
                 (int)out.passes.size() < firstAvoidN ? (avoid | firstAvoid) : avoid);
        clk.lap(3);
        if (relabelFrom >= 0 && (int)best.size() >= 2 && (int)order.size() < n) {
            // candidate store permutations (none, by first use, by use count),
            // each judged by how many ops the greedy plan of the NEXT pass
            // then takes (QUEST_RELABEL_MODE=0/1 forces one candidate)
            static const int forced = getenv("QUEST_RELABEL_MODE") ? atoi(getenv("QUEST_RELABEL_MODE")) : -1;
            const TilePass ps = out.passes.back();
            while (first < n && done[first]) first++;
            auto nextPassOps = [&]() {
                std::vector<int> pick;
                size_t most = 0;
                scan(0, pick);
                most = pick.size();
                static const int maxTries = getenv("QUEST_RELABEL_TRIES") ? atoi(getenv("QUEST_RELABEL_TRIES")) : 8;
                int tries = 0;
                for (int i = first; i < n && tries < maxTries; i++) {
                    if (done[i]) continue;
                    const u64 h = targetMask(ops[i]) & ~low;
                    if (!h) continue;
                    tries++;
                    scan(h, pick);
                    most = std::max(most, pick.size());
                }
                return most;
            };
            int pis[2][64];
            bool has[2];
            for (int m = 0; m < 2; m++) has[m] = proposePerm(ops, done, first, relabelFrom, c, ps, m, pis[m]);
            int choice = -1;
            if (forced >= 0) {
                if (forced < 2 && has[forced]) choice = forced;
            } else if (rollout >= 2) {
                // (rollout 2: the store permutation judged by the passes the
                // rest of the queue then needs, next-pass ops on ties)
                static const std::vector<int> none;
                auto judge = [&]() { return -1e6 * rolloutPasses(none, bestHigh) + (double)nextPassOps(); };
                double bestV = judge();
                for (int m = 0; m < 2; m++) {
                    if (!has[m] || (m == 1 && has[0] && !memcmp(pis[0], pis[1], sizeof pis[0]))) continue;
                    applyPerm(ops, done, first, pis[m]);
                    const double v = judge();
                    applyPerm(ops, done, first, pis[m]);   // involution: undo
                    if (v > bestV) {
                        bestV = v;
                        choice = m;
                    }
                }
            } else {
                size_t bestNext = nextPassOps();
                for (int m = 0; m < 2; m++) {
                    if (!has[m] || (m == 1 && has[0] && !memcmp(pis[0], pis[1], sizeof pis[0]))) continue;
                    applyPerm(ops, done, first, pis[m]);
                    const size_t v = nextPassOps();
                    applyPerm(ops, done, first, pis[m]);   // involution: undo
                    if (v > bestNext || (v == bestNext && choice < 0 && m == 0)) {
                        bestNext = v;
                        choice = m;
                    }
                }
            }
            clk.lap(4);
            if (choice >= 0 && hooks && hooks->relabelOk) {
                TilePass cand = ps;
                for (int i = 0; i < cand.k; i++) cand.stPos[i] = pis[choice][cand.pos[i]];
                if (!hooks->relabelOk(cand, out.ops.data() + cand.opBegin)) choice = -1;
            }
            clk.lap(5);
            if (choice >= 0) {
                const int* pi = pis[choice];
                TilePass& last = out.passes.back();
                for (int i = 0; i < last.k; i++) last.stPos[i] = pi[last.pos[i]];
                applyPerm(ops, done, first, pi);
                for (int x = 0; x < L; x++) out.perm[x] = pi[out.perm[x]];
            }
        }
        if (relabelFrom >= 0 && (int)best.size() >= 2 && hooks && hooks->lowPerm) {
            TilePass& last = out.passes.back();
            int sigma[64];
            if (hooks->lowPerm(last, out.ops.data() + last.opBegin, c, sigma)) {
                for (int i = 0; i < last.k; i++) last.stPos[i] = sigma[last.stPos[i]];
                while (first < n && done[first]) first++;
                applyPerm(ops, done, first, sigma);
                for (int x = 0; x < L; x++) out.perm[x] = sigma[out.perm[x]];
            }
        }
        clk.lap(6);
        if (ready) hooks->passReady(out, (int)out.passes.size() - 1, order);
        clk.lap(7);
        if (hooks && hooks->maxPasses > 0 && (int)out.passes.size() >= hooks->maxPasses && (int)order.size() < n) {
            if (hooks->leftover) {
                hooks->leftover->clear();
                for (int i = first; i < n; i++)
                    if (!done[i]) hooks->leftover->push_back(ops[i]);
            }
            break;
        }
    }
    ops.swap(order);
    clk.flush((long)out.passes.size());
}

namespace {

struct PhaseBuilder {
    int R;
    int k;
    std::vector<int> regs;   // ordered register tile bits (fixed prefix first)
    int fixed = 0;           // leading regs whose order is pinned (Mat4 pair / quad)
    int begin = 0;
    bool open = false;

    bool has(int b) const {
        for (int r : regs)
            if (r == b) return true;
        return false;
    }
};

// LDS slot (8-byte word mod 32) contribution of tile bit b under ldsSwizzle.
unsigned slotVector(int b) { return ldsSwizzle(1u << b) & 31u; }

int gf2Rank(const std::vector<unsigned>& vs) {
    std::vector<unsigned> basis;
    for (unsigned v : vs) {
        for (unsigned x : basis) v = std::min(v, v ^ x);
        if (v) basis.push_back(v);
    }
    return (int)basis.size();
}

// Lanes 0-31 of a half-wave vary the first 5 lane bits: pick non-register
// tile bits whose slot vectors are independent (conflict-free), lowest first,
// then the rest in ascending order.
void assignLanes(TilePhase& ph, int k, int R) {
    std::vector<int> nonreg;
    for (int b = 0; b < k; b++) {
        bool isReg = false;
        for (int r = 0; r < R; r++) isReg |= (ph.reg[r] == b);
        if (!isReg) nonreg.push_back(b);
    }
    std::vector<int> order;
    std::vector<unsigned> vecs;
    std::vector<bool> used(nonreg.size(), false);
    for (size_t i = 0; i < nonreg.size() && order.size() < 5; i++) {
        std::vector<unsigned> trial = vecs;
        trial.push_back(slotVector(nonreg[i]));
        if (gf2Rank(trial) == (int)trial.size()) {
            vecs = trial;
            order.push_back(nonreg[i]);
            used[i] = true;
        }
    }
    for (size_t i = 0; i < nonreg.size(); i++)
        if (!used[i]) order.push_back(nonreg[i]);
    for (size_t i = 0; i < order.size() && i < 16; i++) ph.lane[i] = order[i];
}

void closePhase(PhaseBuilder& pb, int end, TileProgram& prog) {
    if (!pb.open || end <= pb.begin) {
        pb.open = false;
        pb.regs.clear();
        pb.fixed = 0;
        return;
    }
    TilePhase ph;
    ph.opBegin = pb.begin;
    ph.opEnd = end;
    ph.lds = 0;
    // pad with unused tile bits, lowest first
    std::vector<int> regs = pb.regs;
    for (int b = 0; (int)regs.size() < pb.R && b < pb.k; b++) {
        bool used = false;
        for (int r : regs) used |= (r == b);
        if (!used) regs.push_back(b);
    }
    for (int r = 0; r < pb.R; r++) ph.reg[r] = regs[r];
    assignLanes(ph, pb.k, pb.R);
    for (int o = pb.begin; o < end; o++) {
        TileOp& op = prog.ops[o];
        int nt = op.kind == (int)OpKind::Mat2 ? 1 : op.kind == (int)OpKind::Mat4 ? 2
                 : op.kind == (int)OpKind::DensChan2 ? 4 : 0;
        for (int j = 0; j < nt; j++)
            for (int r = 0; r < pb.R; r++)
                if (ph.reg[r] == op.t[j]) op.rt[j] = r;
    }
    prog.phases.push_back(ph);
    pb.open = false;
    pb.regs.clear();
    pb.fixed = 0;
}

void startPhase(PhaseBuilder& pb, int at) {
    pb.open = true;
    pb.begin = at;
    pb.regs.clear();
    pb.fixed = 0;
}

}  // namespace

namespace {

// qubits (tile bits) an op touches: targets + in-tile controls / phase bits
unsigned opQubits(const TileOp& op) {
    unsigned m = op.ctrlIn;
    const int nt = op.kind == (int)OpKind::Mat2 ? 1 : op.kind == (int)OpKind::Mat4 ? 2
                   : op.kind == (int)OpKind::DensChan2 ? 4 : 0;
    for (int j = 0; j < nt; j++) m |= 1u << op.t[j];
    return m;
}

// apply one op to a 2^R block vector; loc[b] = block slot of tile bit b
void applyToBlock(const TileOp& op, const int* loc, int R, std::vector<cplx>& v) {
    const int M = 1 << R;
    unsigned cmask = 0;
    for (int b = 0; b < 32; b++)
        if ((op.ctrlIn >> b) & 1u) cmask |= 1u << loc[b];
    auto cm = [&](int r, int c) -> cplx { return {op.m[2 * (r * (op.kind == (int)OpKind::Mat2 ? 2 : 4) + c)],
                                                  op.m[2 * (r * (op.kind == (int)OpKind::Mat2 ? 2 : 4) + c) + 1]}; };
    if (op.kind == (int)OpKind::Diag) {
        const cplx t = {op.m[0], op.m[1]};
        for (int j = 0; j < M; j++)
            if (((unsigned)j & cmask) == cmask) v[j] = cmul(t, v[j]);
        return;
    }
    if (op.kind == (int)OpKind::Mat2) {
        const int a = loc[op.t[0]];
        for (int j = 0; j < M; j++) {
            if ((j >> a) & 1) continue;
            if (((unsigned)j & cmask) != cmask) continue;
            const int f = j | (1 << a);
            const cplx x = v[j], y = v[f];
            v[j] = cadd(cmul(cm(0, 0), x), cmul(cm(0, 1), y));
            v[f] = cadd(cmul(cm(1, 0), x), cmul(cm(1, 1), y));
        }
        return;
    }
    // Mat4
    const int a = loc[op.t[0]], b = loc[op.t[1]];
    for (int j = 0; j < M; j++) {
        if (((j >> a) & 1) || ((j >> b) & 1)) continue;
        if (((unsigned)j & cmask) != cmask) continue;
        int idx[4];
        cplx x[4];
        for (int g = 0; g < 4; g++) {
            idx[g] = j | ((g & 1) << a) | ((g >> 1) << b);
            x[g] = v[idx[g]];
        }
        for (int r = 0; r < 4; r++) {
            cplx s = {0, 0};
            for (int c = 0; c < 4; c++) s = cadd(s, cmul(cm(r, c), x[c]));
            v[idx[r]] = s;
        }
    }
}

void emitDenseBlock(TileProgram& prog, int k, int R, unsigned bmask, int b, int e) {
    TilePhase ph;
    ph.opBegin = b;
    ph.opEnd = e;
    ph.lds = 0;
    int n = 0;
    for (int bit = 0; bit < k && n < R; bit++)
        if ((bmask >> bit) & 1u) ph.reg[n++] = bit;
    for (int bit = 0; bit < k && n < R; bit++)
        if (!((bmask >> bit) & 1u)) ph.reg[n++] = bit;
    int loc[32];
    for (int i = 0; i < 32; i++) loc[i] = 0;
    for (int r = 0; r < R; r++) loc[ph.reg[r]] = r;
    const int M = 1 << R;
    ph.mat = (int)(prog.mats.size() / (2 * M * M));
    const size_t base = prog.mats.size();
    prog.mats.resize(base + 2 * M * M);
    std::vector<cplx> v(M);
    for (int c = 0; c < M; c++) {
        for (int j = 0; j < M; j++) v[j] = {j == c ? (real)1 : (real)0, 0};
        for (int o = b; o < e; o++) applyToBlock(prog.ops[o], loc, R, v);
        for (int r = 0; r < M; r++) {
            prog.mats[base + 2 * (r * M + c)] = v[r].re;
            prog.mats[base + 2 * (r * M + c) + 1] = v[r].im;
        }
    }
    assignLanes(ph, k, R);
    prog.phases.push_back(ph);
}

}  // namespace

void planDenseBlocks(TileProgram& prog, int k, int R) {
    prog.phases.clear();
    prog.mats.clear();
    for (TilePass& ps : prog.passes) {
        ps.phaseBegin = ps.phaseEnd = (int)prog.phases.size();
        if (k >= 0 ? ps.k != k : ps.k <= R) continue;
        unsigned cur = 0;
        int begin = ps.opBegin;
        for (int o = ps.opBegin; o < ps.opEnd; o++) {
            const TileOp& op = prog.ops[o];
            const unsigned s = opQubits(op);
            const bool fusable = op.ctrlOut == 0 && op.kind != (int)OpKind::DensChan2 && __builtin_popcount(s) <= R;
            if (fusable && __builtin_popcount(cur | s) <= R) {
                cur |= s;
                continue;
            }
            if (o > begin) emitDenseBlock(prog, ps.k, R, cur, begin, o);
            if (!fusable) {
                TilePhase ph;
                ph.opBegin = o;
                ph.opEnd = o + 1;
                ph.lds = 1;
                prog.phases.push_back(ph);
                begin = o + 1;
                cur = 0;
            } else {
                begin = o;
                cur = s;
            }
        }
        if (ps.opEnd > begin) emitDenseBlock(prog, ps.k, R, cur, begin, ps.opEnd);
        ps.phaseEnd = (int)prog.phases.size();
    }
}

void planPhases(TileProgram& prog, int k, int R) {
    prog.phases.clear();
    for (TilePass& ps : prog.passes) {
        ps.phaseBegin = ps.phaseEnd = (int)prog.phases.size();
        if (k >= 0 ? ps.k != k : ps.k <= R) continue;
        PhaseBuilder pb;
        pb.R = R;
        pb.k = ps.k;
        for (int o = ps.opBegin; o < ps.opEnd; o++) {
            TileOp& op = prog.ops[o];
            const OpKind kind = (OpKind)op.kind;
            if (!pb.open) startPhase(pb, o);
            if (kind == OpKind::Diag) continue;  // no register constraint
            if (kind == OpKind::Mat2) {
                const int t = op.t[0];
                if (pb.has(t)) continue;
                if ((int)pb.regs.size() < R) {
                    pb.regs.push_back(t);
                    continue;
                }
                closePhase(pb, o, prog);
                startPhase(pb, o);
                pb.regs.push_back(t);
                continue;
            }
            if (kind == OpKind::Mat4 && R >= 2) {
                const int a = op.t[0], b = op.t[1];
                bool samePair = pb.fixed == 2 && pb.regs[0] == a && pb.regs[1] == b;
                if (samePair) continue;
                if (pb.fixed == 0) {
                    // pin (a, b) in slots 0, 1 if everything fits
                    std::vector<int> nr = {a, b};
                    for (int r : pb.regs)
                        if (r != a && r != b) nr.push_back(r);
                    if ((int)nr.size() <= R) {
                        pb.regs = nr;
                        pb.fixed = 2;
                        continue;
                    }
                }
                closePhase(pb, o, prog);
                startPhase(pb, o);
                pb.regs = {a, b};
                pb.fixed = 2;
                continue;
            }
            if (kind == OpKind::DensChan2 && R >= 4) {
                closePhase(pb, o, prog);
                startPhase(pb, o);
                pb.regs = {op.t[0], op.t[1], op.t[2], op.t[3]};
                pb.fixed = 4;
                closePhase(pb, o + 1, prog);
                continue;
            }
            // fallback: op applied directly on the LDS tile
            closePhase(pb, o, prog);
            TilePhase ph;
            ph.opBegin = o;
            ph.opEnd = o + 1;
            ph.lds = 1;
            prog.phases.push_back(ph);
        }
        closePhase(pb, ps.opEnd, prog);
        ps.phaseEnd = (int)prog.phases.size();
    }
}

}  // namespace qa
