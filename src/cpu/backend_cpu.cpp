// Host backend: the compile-time alternative to src/hip/ for machines without
// a GPU (the reference's QuEST_cpu_local.c role), and the
// in-tree oracle for the HIP kernels.  Deliberately simple scalar C++: its job
// is to execute the same tile programs (src/core/tiles.hpp) as the GPU with
// obviously-correct loops, so every layer above the kernels (front-end,
// router, RCCL-style swaps, fusion planner) is testable on CPU.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <omp.h>
#include <sys/mman.h>

#include "../core/backend.hpp"
#include "../core/router.hpp"
#include "../core/tiles.hpp"
#include "../core/wave.hpp"
#include "../core/trace.hpp"

namespace qa {
namespace be {

namespace {

inline i64 insertZero(i64 x, int bit) {
    i64 low = x & (((i64)1 << bit) - 1);
    return ((x >> bit) << (bit + 1)) | low;
}

void applyTileOp(const TileOp& op, int k, real* re, real* im) {
    const unsigned n = 1u << k;
    switch ((OpKind)op.kind) {
        case OpKind::Mat2: {
            const int a = op.t[0];
            const real* m = op.m;
            for (unsigned j = 0; j < n / 2; j++) {
                unsigned p0 = (unsigned)insertZero(j, a), p1 = p0 | (1u << a);
                if ((p0 & op.ctrlIn) != op.ctrlIn) continue;
                real r0 = re[p0], i0 = im[p0], r1 = re[p1], i1 = im[p1];
                re[p0] = m[0] * r0 - m[1] * i0 + m[2] * r1 - m[3] * i1;
                im[p0] = m[0] * i0 + m[1] * r0 + m[2] * i1 + m[3] * r1;
                re[p1] = m[4] * r0 - m[5] * i0 + m[6] * r1 - m[7] * i1;
                im[p1] = m[4] * i0 + m[5] * r0 + m[6] * i1 + m[7] * r1;
            }
            break;
        }
        case OpKind::Diag: {
            const real tr = op.m[0], ti = op.m[1];
            for (unsigned p = 0; p < n; p++) {
                if ((p & op.ctrlIn) != op.ctrlIn) continue;
                real r = re[p], i = im[p];
                re[p] = tr * r - ti * i;
                im[p] = tr * i + ti * r;
            }
            break;
        }
        case OpKind::Mat4: {
            const int a = op.t[0], b = op.t[1];
            const int lo = std::min(a, b), hi = std::max(a, b);
            for (unsigned j = 0; j < n / 4; j++) {
                unsigned p = (unsigned)insertZero(insertZero(j, lo), hi);
                if ((p & op.ctrlIn) != op.ctrlIn) continue;
                unsigned idx[4];
                real vr[4], vi[4];
                for (int g = 0; g < 4; g++) {
                    idx[g] = p | ((unsigned)(g & 1) << a) | ((unsigned)(g >> 1) << b);
                    vr[g] = re[idx[g]];
                    vi[g] = im[idx[g]];
                }
                for (int r = 0; r < 4; r++) {
                    real sr = 0, si = 0;
                    for (int c = 0; c < 4; c++) {
                        const real mr = op.m[2 * (4 * r + c)], mi = op.m[2 * (4 * r + c) + 1];
                        sr += mr * vr[c] - mi * vi[c];
                        si += mr * vi[c] + mi * vr[c];
                    }
                    re[idx[r]] = sr;
                    im[idx[r]] = si;
                }
            }
            break;
        }
        case OpKind::DensChan2: {
            int s[4] = {op.t[0], op.t[1], op.t[2], op.t[3]};
            std::sort(s, s + 4);
            const real off = op.m[0], keep = op.m[2], mix = op.m[4];
            for (unsigned j = 0; j < n / 16; j++) {
                unsigned p = (unsigned)j;
                for (int x = 0; x < 4; x++) p = (unsigned)insertZero(p, s[x]);
                unsigned idx[16];
                for (int e = 0; e < 16; e++) {
                    idx[e] = p;
                    for (int x = 0; x < 4; x++)
                        if ((e >> x) & 1) idx[e] |= 1u << op.t[x];
                }
                real sr = 0, si = 0;
                for (int a = 0; a < 4; a++) {
                    sr += re[idx[a + 4 * a]];
                    si += im[idx[a + 4 * a]];
                }
                for (int e = 0; e < 16; e++) {
                    int a = e & 3, b = e >> 2;
                    if (a != b) {
                        re[idx[e]] *= off;
                        im[idx[e]] *= off;
                    } else {
                        re[idx[e]] = keep * re[idx[e]] + mix * sr / 4;
                        im[idx[e]] = keep * im[idx[e]] + mix * si / 4;
                    }
                }
            }
            break;
        }
    }
}

// Register-phase emulation: exactly the per-thread decomposition of the GPU
// kernel (src/hip/kernels_gates.hip), so the planner's register assignment is
// validated on CPU.  "Thread" tau owns the 2^R tile elements tb | regOff[j].
constexpr int kMaxRegSlots = 4;
int regSlots() {
    static int r = [] {
        const char* e = getenv("QUEST_CPU_REG_SLOTS");
        int v = e ? atoi(e) : 3;
        return v < 2 ? 2 : v > kMaxRegSlots ? kMaxRegSlots : v;
    }();
    return r;
}

void applyRegOp(const TileOp& op, int R, real* vr, real* vi, unsigned tb, const unsigned* regOff) {
    const int M = 1 << R;
    switch ((OpKind)op.kind) {
        case OpKind::Mat2: {
            const int a = op.rt[0];
            const real* m = op.m;
            for (int j = 0; j < M; j++) {
                if ((j >> a) & 1) continue;
                if (((tb | regOff[j]) & op.ctrlIn) != op.ctrlIn) continue;
                const int f = j | (1 << a);
                real r0 = vr[j], i0 = vi[j], r1 = vr[f], i1 = vi[f];
                vr[j] = m[0] * r0 - m[1] * i0 + m[2] * r1 - m[3] * i1;
                vi[j] = m[0] * i0 + m[1] * r0 + m[2] * i1 + m[3] * r1;
                vr[f] = m[4] * r0 - m[5] * i0 + m[6] * r1 - m[7] * i1;
                vi[f] = m[4] * i0 + m[5] * r0 + m[6] * i1 + m[7] * r1;
            }
            break;
        }
        case OpKind::Diag:
            for (int j = 0; j < M; j++) {
                if (((tb | regOff[j]) & op.ctrlIn) != op.ctrlIn) continue;
                real r = vr[j], i = vi[j];
                vr[j] = op.m[0] * r - op.m[1] * i;
                vi[j] = op.m[0] * i + op.m[1] * r;
            }
            break;
        case OpKind::Mat4: {
            const int a = op.rt[0], b = op.rt[1];
            for (int j = 0; j < M; j++) {
                if (((j >> a) & 1) || ((j >> b) & 1)) continue;
                if (((tb | regOff[j]) & op.ctrlIn) != op.ctrlIn) continue;
                int idx[4];
                real xr[4], xi[4];
                for (int g = 0; g < 4; g++) {
                    idx[g] = j | ((g & 1) << a) | ((g >> 1) << b);
                    xr[g] = vr[idx[g]];
                    xi[g] = vi[idx[g]];
                }
                for (int r = 0; r < 4; r++) {
                    real sr = 0, si = 0;
                    for (int c = 0; c < 4; c++) {
                        const real mr = op.m[2 * (4 * r + c)], mi = op.m[2 * (4 * r + c) + 1];
                        sr += mr * xr[c] - mi * xi[c];
                        si += mr * xi[c] + mi * xr[c];
                    }
                    vr[idx[r]] = sr;
                    vi[idx[r]] = si;
                }
            }
            break;
        }
        case OpKind::DensChan2: {
            const int* s = op.rt;
            for (int j = 0; j < M; j++) {
                bool base = true;
                for (int x = 0; x < 4; x++) base &= !((j >> s[x]) & 1);
                if (!base) continue;
                int idx[16];
                for (int e = 0; e < 16; e++) {
                    idx[e] = j;
                    for (int x = 0; x < 4; x++)
                        if ((e >> x) & 1) idx[e] |= 1 << s[x];
                }
                real sr = 0, si = 0;
                for (int a = 0; a < 4; a++) {
                    sr += vr[idx[a + 4 * a]];
                    si += vi[idx[a + 4 * a]];
                }
                for (int e = 0; e < 16; e++) {
                    if ((e & 3) != (e >> 2)) {
                        vr[idx[e]] *= op.m[0];
                        vi[idx[e]] *= op.m[0];
                    } else {
                        vr[idx[e]] = op.m[2] * vr[idx[e]] + op.m[4] * sr / 4;
                        vi[idx[e]] = op.m[2] * vi[idx[e]] + op.m[4] * si / 4;
                    }
                }
            }
            break;
        }
    }
}

void runPhase(const TilePhase& ph, const TileProgram& prog, int k, i64 base, real* br, real* bi) {
    if (ph.lds) {
        for (int o = ph.opBegin; o < ph.opEnd; o++) {
            const TileOp& op = prog.ops[o];
            if (((u64)base & op.ctrlOut) == op.ctrlOut) applyTileOp(op, k, br, bi);
        }
        return;
    }
    const int R = regSlots(), M = 1 << R;
    unsigned regMask = 0, regOff[1 << kMaxRegSlots];
    for (int r = 0; r < R; r++) regMask |= 1u << ph.reg[r];
    for (int j = 0; j < M; j++) {
        regOff[j] = 0;
        for (int r = 0; r < R; r++)
            if ((j >> r) & 1) regOff[j] |= 1u << ph.reg[r];
    }
    real vr[1 << kMaxRegSlots], vi[1 << kMaxRegSlots];
    for (unsigned tau = 0; tau < (1u << (k - R)); tau++) {
        unsigned tb = 0, x = tau;
        for (int b = 0; b < k; b++) {
            if ((regMask >> b) & 1) continue;
            tb |= (x & 1u) << b;
            x >>= 1;
        }
        for (int j = 0; j < M; j++) {
            vr[j] = br[tb | regOff[j]];
            vi[j] = bi[tb | regOff[j]];
        }
        if (ph.mat >= 0) {
            // dense block: y = U x with the host-composed 2^R x 2^R matrix
            const real* U = prog.mats.data() + (size_t)ph.mat * 2 * M * M;
            real yr[1 << kMaxRegSlots], yi[1 << kMaxRegSlots];
            for (int r = 0; r < M; r++) {
                real sr = 0, si = 0;
                for (int c = 0; c < M; c++) {
                    const real ur = U[2 * (r * M + c)], ui = U[2 * (r * M + c) + 1];
                    sr += ur * vr[c] - ui * vi[c];
                    si += ur * vi[c] + ui * vr[c];
                }
                yr[r] = sr;
                yi[r] = si;
            }
            for (int j = 0; j < M; j++) {
                vr[j] = yr[j];
                vi[j] = yi[j];
            }
        } else {
            for (int o = ph.opBegin; o < ph.opEnd; o++) {
                const TileOp& op = prog.ops[o];
                if (((u64)base & op.ctrlOut) != op.ctrlOut) continue;
                applyRegOp(op, R, vr, vi, tb, regOff);
            }
        }
        for (int j = 0; j < M; j++) {
            br[tb | regOff[j]] = vr[j];
            bi[tb | regOff[j]] = vi[j];
        }
    }
}

// OpenMP over tiles (each thread stages its own tile), as the reference's
// CPU kernels parallelise their pair loops (QuEST_cpu.c, `#pragma omp
// parallel for`); small registers stay on one thread.
constexpr i64 kOmpMin = (i64)1 << 22;  // below ~4M amplitudes thread wake-up costs more than it saves

void runTilePass(real* re, real* im, int L, const TileProgram& prog, const TilePass& ps) {
    const unsigned n = 1u << ps.k;
    std::vector<i64> offs(n);
    for (unsigned p = 0; p < n; p++) offs[p] = tileOffset(ps, p);
    const i64 tiles = (i64)1 << (L - ps.k);
#pragma omp parallel if (((i64)1 << L) >= kOmpMin)
    {
        std::vector<real> br(n), bi(n);
#pragma omp for schedule(static)
        for (i64 T = 0; T < tiles; T++) {
            const i64 base = tileBase(ps, T, L);
            for (unsigned p = 0; p < n; p++) {
                br[p] = re[base + offs[p]];
                bi[p] = im[base + offs[p]];
            }
            if (ps.phaseEnd > ps.phaseBegin) {
                for (int h = ps.phaseBegin; h < ps.phaseEnd; h++)
                    runPhase(prog.phases[h], prog, ps.k, base, br.data(), bi.data());
            } else {
                for (int o = ps.opBegin; o < ps.opEnd; o++) {
                    const TileOp& op = prog.ops[o];
                    if (((u64)base & op.ctrlOut) != op.ctrlOut) continue;
                    applyTileOp(op, ps.k, br.data(), bi.data());
                }
            }
            for (unsigned p = 0; p < n; p++) {
                re[base + offs[p]] = br[p];
                im[base + offs[p]] = bi[p];
            }
        }
    }
}

void runProgram(real* re, real* im, int L, const TileProgram& prog0, bool wave = false) {
    // rank predicates (core.hpp): the ops are planned as queued, identically on
    // every rank, then resolved against this rank's verdicts for execution
    bool tagged = false;
    for (const TileOp& op : prog0.ops) tagged = tagged || (op.ctrlOut & kRankTagMask);
    TileProgram resolved;
    if (tagged) {
        resolved = prog0;
        for (TileOp& op : resolved.ops) op.ctrlOut = resolveRankTag(op.ctrlOut);
    }
    const TileProgram& prog = tagged ? resolved : prog0;
    for (const TilePass& ps : prog.passes) {
        WaveProgram wp;
        if (wave && planWavePass(ps, prog0.ops.data() + ps.opBegin, ps.opEnd - ps.opBegin, wp)) {
            for (WaveOp& w : wp.ops) w.ctrlOut = resolveRankTag(w.ctrlOut);
            emulateWavePass(re, im, L, wp, wp.passes[0]);
            stats().wavePasses++;
        } else {
            if (wave && getenv("QUEST_WAVE_DUMP")) {
                fprintf(stderr, "not a wave pass: k %d, %d ops, pos", ps.k, ps.opEnd - ps.opBegin);
                for (int i = 0; i < ps.k; i++) fprintf(stderr, " %d->%d", ps.pos[i], ps.stPos[i]);
                fprintf(stderr, ", kinds");
                for (int o = ps.opBegin; o < ps.opEnd; o++)
                    fprintf(stderr, " %d(t%d,%d c%llx)", prog.ops[(size_t)o].kind, prog.ops[(size_t)o].t[0],
                            prog.ops[(size_t)o].t[1], (unsigned long long)prog.ops[(size_t)o].ctrlIn);
                fprintf(stderr, "\n");
            }
            runTilePass(re, im, L, prog, ps);
        }
        stats().passes++;
        if (ps.opEnd - ps.opBegin > 1) stats().fusedOps += ps.opEnd - ps.opBegin;
    }
}

int fuseQubits() {
    int k = rt().fuseMaxQubits;
    return k > 0 ? std::max(k, 8) : 10;
}

}  // namespace

// ---------------------------------------------------------------------------

void envInit(int, int, int) {}
void envFinalize() {}
void deviceSync() {}

namespace {
std::chrono::steady_clock::time_point g_swapT0;
long long g_swapUs = 0;
bool g_swapOpen = false;
}  // namespace

void swapMark(bool begin) {
    const auto now = std::chrono::steady_clock::now();
    if (begin) {
        g_swapT0 = now;
        g_swapOpen = true;
    } else if (g_swapOpen) {
        g_swapUs += std::chrono::duration_cast<std::chrono::microseconds>(now - g_swapT0).count();
        g_swapOpen = false;
    }
}
long long swapMicros(bool) { return g_swapUs; }
void swapMicrosReset() { g_swapUs = 0; }

bool swapOverlapBegin(QuregImpl&, const int*, int, int) { return false; }
void swapOverlapEnd(QuregImpl&) {}
bool preSwap(QuregImpl&, const int*, int, int) { return false; }
void swapRanges(QuregImpl&, const int*, int) {}
void swapRangeLanded(QuregImpl&, int) {}

u64 queuedTargets(const QuregImpl& q) {
    u64 m = 0xffull;   // the always-resident low positions of every wave tile (cmin <= 8)
    for (const Op& op : q.pending)
        for (int j = 0; j < op.nt; j++) m |= 1ull << op.t[j];
    return m;
}
std::string describe() { return "host C++ (plumbing build, no GPU)"; }
const char* shortName() { return "CPU"; }
bool stateOnHost() { return true; }

namespace {
// QUEST_PLAN_ONLY=1 (planner studies of registers larger than host memory):
// the state is a lazily backed, unreserved mapping; pages no one touches
// cost nothing
bool planOnlyMode() {
    static const bool on = getenv("QUEST_PLAN_ONLY") && atoi(getenv("QUEST_PLAN_ONLY")) != 0;
    return on;
}
}  // namespace

void allocState(QuregImpl& q) {
    const size_t bytes = sizeof(real) * (size_t)q.numAmpsPerChunk;
    if (planOnlyMode()) {
        void* r = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
        void* i = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
        q.re = r == MAP_FAILED ? nullptr : static_cast<real*>(r);
        q.im = i == MAP_FAILED ? nullptr : static_cast<real*>(i);
    } else {
        q.re = (real*)calloc((size_t)q.numAmpsPerChunk, sizeof(real));
        q.im = (real*)calloc((size_t)q.numAmpsPerChunk, sizeof(real));
    }
    if (!q.re || !q.im) {
        fprintf(stderr, "QuEST: could not allocate %lld amplitudes\n", q.numAmpsPerChunk);
        exit(EXIT_FAILURE);
    }
}

void freeState(QuregImpl& q) {
    if (planOnlyMode()) {
        const size_t bytes = sizeof(real) * (size_t)q.numAmpsPerChunk;
        munmap(q.re, bytes);
        munmap(q.im, bytes);
    } else {
        free(q.re);
        free(q.im);
    }
    q.re = q.im = nullptr;
}

void* allocComm(size_t bytes) { return malloc(bytes ? bytes : 1); }
void freeComm(void* p) { free(p); }

// ops queued before a flush: the HIP backend's 1024 (QUEST_QUEUE_OPS), so
// that the emulated wave plans are the GPU's
namespace {
void flushImpl(QuregImpl& q, bool front);
}  // namespace

void enqueue(QuregImpl& q, const Op& op) {
    static const size_t limit = [] {
        const char* e = getenv("QUEST_QUEUE_OPS");
        const long v = e ? atol(e) : 1024;
        return (size_t)std::max(1L, std::min(v, 1024L));
    }();
    q.pending.push_back(op);
    if (q.pending.size() >= limit) {
        flush(q);
        return;
    }
    // front flushes of the wave planner, exactly as the HIP backend's
    // (QUEST_FRONT_FLUSH, default 600 ops): the emulated plans stay the GPU's
    static const size_t front = [] {
        const char* e = getenv("QUEST_FRONT_FLUSH");
        return (size_t)std::max(0L, e ? atol(e) : 600L);
    }();
    if (front && q.pending.size() >= front && ((q.pending.size() - front) & 15) == 0) flushImpl(q, true);
}

void flush(QuregImpl& q) { flushImpl(q, false); }

namespace {
void flushImpl(QuregImpl& q, bool front) {
    if (q.pending.empty()) return;
    const RankSkipScope rankScope(q);
    // the window's first pass now, the strategy search over the rest while it
    // runs (waveSearchSplitFirst); `searched` is then that search's choice for
    // exactly the queue left
    int searched = -1;
    if (!front && waveSearchSplitFirst(q)) {
        flushImpl(q, true);
        if (q.pending.empty()) return;
        if (q.strategySearch.valid()) {
            searched = q.strategySearch.get();
            q.planStrategy = searched;
        }
    }
    TileProgram prog;
    std::vector<Op> raw;
    if (rt().verify) raw = q.pending;
    // QUEST_CPU_PLANNER: 0 op by op (default, fastest on the host), 1 register
    // phases, 2 dense blocks, 3 wave tiles -- 1..3 emulate the GPU tile modes
    // exactly (same plans, same per-thread / per-lane decomposition) for
    // testing them here
    static const int planner = [] {
        const char* e = getenv("QUEST_CPU_PLANNER");
        return e ? atoi(e) : 0;
    }();
    const bool wave = planner == 3 && q.L >= kWaveBits;
    static const int waveCmin = getenv("QUEST_WAVE_CMIN") ? atoi(getenv("QUEST_WAVE_CMIN")) : kWaveVecBits + 5;  // as the HIP backend
    bool channels = false;   // as the HIP backend: density-channel flushes keep one low position fewer
    for (const Op& op : q.pending) channels = channels || op.kind == OpKind::Mat4 || op.kind == OpKind::DensChan2;
    // (QUEST_WAVE_CMIN_CHAN: the always-resident low positions of channel
    // flushes, kWaveVecBits + 3 .. kWaveBits - 2; the density damping trade)
    static const int cminChan = [] {
        const char* e = getenv("QUEST_WAVE_CMIN_CHAN");
        return e ? std::max(kWaveVecBits + 3, std::min(atoi(e), kWaveBits - 2)) : kWaveVecBits + 4;
    }();
    const int cminWave = channels ? cminChan : waveCmin;
    // QUEST_WAVE_CHAN_RELABEL=1: channel flushes relabel too (a channel needs
    // its row and column bits in one tile; relabelling lets the low positions
    // hold different qubits pass by pass)
    static const bool chanRelabel = getenv("QUEST_WAVE_CHAN_RELABEL") && atoi(getenv("QUEST_WAVE_CHAN_RELABEL")) != 0;
    const bool relabel = wave && (!channels || chanRelabel) && rt().fusion && waveRelabel() && !rt().verify;
    // as the HIP backend (streamed wave flushes): relabel only passes the wave
    // engine lowers -- the same plans (QUEST_PLAN_STREAM=0: the fallback below)
    static const bool streamOn = !getenv("QUEST_PLAN_STREAM") || atoi(getenv("QUEST_PLAN_STREAM")) != 0;
    PlanHooks hooks;
    hooks.avoidMask = q.tileAvoid;
    hooks.firstPassAvoid = q.firstPassAvoid;   // (router: a swap's receive ranges; QUEST_SWAP_RANGES_STUDY on this build)
    hooks.firstAvoidPasses = q.firstAvoidLeft;
    hooks.relabelOk = [](const TilePass& ps, const TileOp* ops) { return waveLowers(ps, ops); };
    hooks.lowPerm = [](const TilePass& ps, const TileOp* ops, int c, int* sigma) {
        return waveLowPerm(ps, ops, c, sigma);
    };
    if (q.L >= waveCostMinQubits()) waveCostHooks(hooks);
    std::vector<Op> leftover;
    if (front) {
        // as the HIP backend: plain wave queues of wave-sized registers only
        bool plain = relabel && streamOn && q.L >= kWaveBits + 6;
        for (const Op& op : q.pending) plain = plain && (op.kind == OpKind::Mat2 || op.kind == OpKind::Diag);
        if (!plain) return;
        hooks.maxPasses = 1;
        hooks.leftover = &leftover;
    }
    // counted (and global state touched) only once the flush is certain to run
    stats().flushes++;
    const double tFlush0 = trace::on() ? trace::now() : 0.0;
    const size_t opsIn = q.pending.size();
    fuseBlockQubits() = wave ? 1 : 2;
    std::vector<Op> orig;
    if (relabel && !front) orig = q.pending;
    // as the HIP backend: 6 or 7 always-resident low positions, whichever
    // plans this queue in fewer passes
    int cminUse = (relabel && streamOn && !getenv("QUEST_WAVE_CMIN")) ? chooseWaveCmin(q, cminWave, hooks) : cminWave;
    // Strategy search (searchWaveStrategy): full flushes search their own
    // queue on worker threads while the GPU works through the passes the front
    // flushes launched; front flushes use the strategy a background search
    // picked from the queue left after the window's first front flush (the
    // default until then).  Deterministic: a choice depends on queues only.
    const bool searchable = relabel && streamOn && !getenv("QUEST_WAVE_CMIN");
    int strategy = -1;
    if (searchable) {
        if (q.strategySearch.valid()) q.planStrategy = q.strategySearch.get();
        strategy = front ? (q.planStrategy >= 0 ? q.planStrategy : waveFrontStrategy())
                         : searched >= 0 ? searched : searchWaveStrategy(q.pending, q.L, cminUse, hooks);
    }
    const int cminBase = cminUse;
    WaveStrategyScope strategyScope(strategy, cminBase, hooks, &cminUse);
    planTiles(q.pending, q.L, wave ? kWaveBits : fuseQubits(), wave ? cminUse : 4, rt().fusion, prog,
              relabel ? kWaveVecBits : -1, relabel && streamOn ? &hooks : nullptr);
    consumeFirstAvoid(q, (int)prog.passes.size());
    if (leftover.empty()) {   // the queue drained: choose afresh next time
        q.waveCmin = -1;
        q.planStrategy = -1;
    } else if (front && searchable && waveFrontSearch() && waveSearchOn() && q.planStrategy < 0 &&
               !q.strategySearch.valid() &&
               leftover.size() >= waveSearchMinOps() && q.L >= waveSearchMinQubits()) {
        PlanHooks base;
        base.relabelOk = hooks.relabelOk;
        base.lowPerm = hooks.lowPerm;
        q.strategySearch = std::async(std::launch::async, [ops = leftover, L = q.L, c = cminBase, base,
                                                           fuse = fuseBlockQubits()]() {
            fuseBlockQubits() = fuse;   // (thread-local: this flush's setting)
            return std::max(0, searchWaveStrategy(ops, L, c, base));
        });
    }
    if (!front && relabel && programRelabels(prog) && !relabelsLower(prog)) {
        q.pending.swap(orig);
        planTiles(q.pending, q.L, kWaveBits, cminWave, rt().fusion, prog);
    }
    if (trace::on())
        trace::event("flush", "\"qubits\": %d, \"ops\": %zu, \"ops_fused\": %zu, \"passes\": %zu, \"plan_ms\": %.3f",
                     q.L, opsIn, q.pending.size(), prog.passes.size(), 1e3 * (trace::now() - tFlush0));
    // QUEST_TRACE_PASS_CYCLES=1: each wave pass's modeled cycles (plan studies
    // of the pass-time model, tools/experiments/score_study.py)
    static const bool passCycles = getenv("QUEST_TRACE_PASS_CYCLES") != nullptr;
    if (trace::on() && passCycles && wave)
        for (const TilePass& ps : prog.passes)
            trace::event("pass", "\"qubits\": %d, \"ops\": %d, \"engine\": \"plan\", \"wave_cycles\": %.0f", q.L,
                         ps.opEnd - ps.opBegin, wavePassCycles(ps, prog.ops.data() + ps.opBegin));
    if (planner == 1)
        planPhases(prog, -1, regSlots());
    else if (planner == 2)
        planDenseBlocks(prog, -1, regSlots());
    q.pending.swap(leftover);   // front flush: the ops not planned yet; else empty
    // QUEST_PLAN_ONLY=1 (planner studies): plan, count, do not touch the
    // state -- pass counts of large registers in no time (tools/plan_study.py)
    static const bool planOnly = getenv("QUEST_PLAN_ONLY") && atoi(getenv("QUEST_PLAN_ONLY")) != 0;
    // QUEST_SWAP_STUDY=1: the passes of a pre-swap flush after the last one
    // whose tile holds a victim of the swap (they could run split around it)
    static const bool swapStudy = getenv("QUEST_SWAP_STUDY") != nullptr;
    if (swapStudy && q.nSwapVictims > 0 && rt().rank == 0) {
        int cur[8];
        for (int m = 0; m < q.nSwapVictims; m++) cur[m] = q.l2p[q.swapVictims[m]];
        int last = -1;
        double opsAfter = 0, opsAll = 0;
        for (size_t p = 0; p < prog.passes.size(); p++) {
            const TilePass& ps = prog.passes[p];
            bool in = false;
            for (int m = 0; m < q.nSwapVictims; m++)
                for (int b = 0; b < ps.k; b++)
                    if (ps.pos[b] == cur[m]) {
                        in = true;
                        cur[m] = ps.stPos[b];
                        break;
                    }
            if (in) last = (int)p;
        }
        for (size_t p = 0; p < prog.passes.size(); p++) {
            const double n = prog.passes[p].opEnd - prog.passes[p].opBegin;
            opsAll += n;
            if ((int)p > last) opsAfter += n;
        }
        fprintf(stderr, "swap study: %zu passes before the swap, %zu after the last holding a victim (%.0f of %.0f ops)\n",
                prog.passes.size(), prog.passes.size() - (size_t)(last + 1), opsAfter, opsAll);
    }
    if (planOnly) {
        for (const TilePass& ps : prog.passes) {
            WaveProgram wp;
            if (wave && planWavePass(ps, prog.ops.data() + ps.opBegin, ps.opEnd - ps.opBegin, wp)) {
                stats().wavePasses++;
                dumpWavePass(wp, wp.passes.back());
            }
            stats().passes++;
        }
        applyProgramPerm(q, prog);
        return;
    }
    if (!rt().verify) {
        runProgram(q.re, q.im, q.L, prog, wave);
        applyProgramPerm(q, prog);
        return;
    }
    // debug mode: the same ops one pass each, in order, on a shadow copy
    std::vector<real> sr(q.re, q.re + q.numAmpsPerChunk), si(q.im, q.im + q.numAmpsPerChunk);
    runProgram(q.re, q.im, q.L, prog, wave);
    const Stats keep = stats();
    TileProgram ref;
    planTiles(raw, q.L, fuseQubits(), 4, false, ref);
    runProgram(sr.data(), si.data(), q.L, ref);
    stats() = keep;
    if (rt().verifyInject) {
        rt().verifyInject = false;
        q.re[0] += (real)0.5;
    }
    double diff = 0;
    for (i64 i = 0; i < q.numAmpsPerChunk; i++) {
        const double d = std::hypot((double)q.re[i] - sr[i], (double)q.im[i] - si[i]);
        diff = (d != d) ? INFINITY : std::max(diff, d);
    }
    verifyFlush(q.L, raw.size(), prog.passes.size(), diff);
}
}  // namespace

void fill(QuregImpl& q, real re, real im) {
    flush(q);
    if (planOnlyMode()) return;   // the planner study never reads amplitudes
#pragma omp parallel for if (q.numAmpsPerChunk >= kOmpMin)
    for (i64 i = 0; i < q.numAmpsPerChunk; i++) {
        q.re[i] = re;
        q.im[i] = im;
    }
}

void setAmp(QuregImpl& q, i64 local, real re, real im) {
    flush(q);
    q.re[local] = re;
    q.im[local] = im;
}

void initDebug(QuregImpl& q, i64 globalOffset) {
    flush(q);
#pragma omp parallel for if (q.numAmpsPerChunk >= kOmpMin)
    for (i64 i = 0; i < q.numAmpsPerChunk; i++) {
        i64 g = globalOffset + i;
        q.re[i] = (real)((g * 2.0) / 10.0);
        q.im[i] = (real)((g * 2.0 + 1.0) / 10.0);
    }
}

void fillWhereBit(QuregImpl& q, int bit, int outcome, real val) {
    flush(q);
#pragma omp parallel for if (q.numAmpsPerChunk >= kOmpMin)
    for (i64 i = 0; i < q.numAmpsPerChunk; i++) {
        q.re[i] = (((i >> bit) & 1) == outcome) ? val : 0;
        q.im[i] = 0;
    }
}

void writeAmps(QuregImpl& q, i64 local, const real* re, const real* im, i64 n) {
    flush(q);
    memcpy(q.re + local, re, sizeof(real) * n);
    memcpy(q.im + local, im, sizeof(real) * n);
}

void readAmps(QuregImpl& q, i64 local, real* re, real* im, i64 n) {
    flush(q);
    memcpy(re, q.re + local, sizeof(real) * n);
    memcpy(im, q.im + local, sizeof(real) * n);
}

void copyState(QuregImpl& dst, QuregImpl& src) {
    flush(src);
    flush(dst);
    memcpy(dst.re, src.re, sizeof(real) * dst.numAmpsPerChunk);
    memcpy(dst.im, src.im, sizeof(real) * dst.numAmpsPerChunk);
}

double sumSq(QuregImpl& q, int bit, int bitVal) {
    flush(q);
    double s = 0;
#pragma omp parallel for reduction(+ : s) if (q.numAmpsPerChunk >= kOmpMin)
    for (i64 i = 0; i < q.numAmpsPerChunk; i++) {
        if (bit >= 0 && (int)((i >> bit) & 1) != bitVal) continue;
        s += (double)q.re[i] * q.re[i] + (double)q.im[i] * q.im[i];
    }
    return s;
}

// One pass over blocks of 2^12 amplitudes: bits inside a block per element,
// bits above it from the block total.
void marginals(QuregImpl& q, double* zeroSums, double* total) {
    flush(q);
    const int L = q.L, kb = std::min(L, 12);
    const i64 blk = (i64)1 << kb, nBlk = q.numAmpsPerChunk >> kb;
    // per-thread partials summed in thread order: deterministic
    std::vector<double> parts;
#pragma omp parallel if (q.numAmpsPerChunk >= kOmpMin)
    {
        double mine[65] = {0};
#pragma omp single
        parts.assign(65 * (size_t)omp_get_num_threads(), 0.0);
#pragma omp for schedule(static)
        for (i64 B = 0; B < nBlk; B++) {
            double bs = 0;
            for (i64 i = 0; i < blk; i++) {
                const i64 k = B * blk + i;
                const double x = (double)q.re[k] * q.re[k] + (double)q.im[k] * q.im[k];
                bs += x;
                for (int b = 0; b < kb; b++)
                    if (!((i >> b) & 1)) mine[b] += x;
            }
            for (int b = kb; b < L; b++)
                if (!((B >> (b - kb)) & 1)) mine[b] += bs;
            mine[64] += bs;
        }
        memcpy(&parts[65 * (size_t)omp_get_thread_num()], mine, sizeof mine);
    }
    double acc[65] = {0};
    for (size_t t = 0; t < parts.size(); t += 65)
        for (int b = 0; b < 65; b++) acc[b] += parts[t + b];
    for (int b = 0; b < L; b++) zeroSums[b] = acc[b];
    *total = acc[64];
}

void innerProduct(QuregImpl& bra, QuregImpl& ket, double out[2]) {
    flush(bra);
    flush(ket);
    double r = 0, i = 0;
#pragma omp parallel for reduction(+ : r, i) if (bra.numAmpsPerChunk >= kOmpMin)
    for (i64 k = 0; k < bra.numAmpsPerChunk; k++) {
        r += (double)bra.re[k] * ket.re[k] + (double)bra.im[k] * ket.im[k];
        i += (double)bra.re[k] * ket.im[k] - (double)bra.im[k] * ket.re[k];
    }
    out[0] = r;
    out[1] = i;
}

namespace {
// sigma(i) of the permuted kernels: the bits of i moved to sig[] positions,
// through two 2^h tables
struct BitMap {
    int h;
    std::vector<i64> lo, hi;
    BitMap(int L, const int* sig) : h(L / 2), lo((size_t)1 << (L / 2)), hi((size_t)1 << (L - L / 2)) {
        for (size_t x = 0; x < lo.size(); x++)
            for (int b = 0; b < h; b++)
                if ((x >> b) & 1) lo[x] |= (i64)1 << sig[b];
        for (size_t x = 0; x < hi.size(); x++)
            for (int b = 0; b < L - h; b++)
                if ((x >> b) & 1) hi[x] |= (i64)1 << sig[h + b];
    }
    i64 operator()(i64 i) const { return lo[(size_t)(i & (((i64)1 << h) - 1))] | hi[(size_t)(i >> h)]; }
};
}  // namespace

bool permuteLocal(QuregImpl& q, const int* dest) {
    // the wave engine's relayout passes on its host emulation (QUEST_CPU_PLANNER=3)
    static const bool wave = getenv("QUEST_CPU_PLANNER") && atoi(getenv("QUEST_CPU_PLANNER")) == 3;
    if (!wave || q.L < kWaveBits + 6 || rt().verify) return false;
    TileProgram prog;
    if (!planRelayout(q.L, dest, prog)) return false;
    flush(q);
    runProgram(q.re, q.im, q.L, prog, true);
    return true;
}

void innerProductPerm(QuregImpl& bra, QuregImpl& ket, const int* sig, double out[2]) {
    flush(bra);
    flush(ket);
    const BitMap map(bra.L, sig);
    double r = 0, i = 0;
#pragma omp parallel for reduction(+ : r, i) if (bra.numAmpsPerChunk >= kOmpMin)
    for (i64 k = 0; k < bra.numAmpsPerChunk; k++) {
        const i64 j = map(k);
        r += (double)bra.re[k] * ket.re[j] + (double)bra.im[k] * ket.im[j];
        i += (double)bra.re[k] * ket.im[j] - (double)bra.im[k] * ket.re[j];
    }
    out[0] = r;
    out[1] = i;
}

void axpbyPerm(QuregImpl& a, real alpha, QuregImpl& b, real beta, const int* sig) {
    flush(a);
    flush(b);
    const BitMap map(a.L, sig);
#pragma omp parallel for if (a.numAmpsPerChunk >= kOmpMin)
    for (i64 k = 0; k < a.numAmpsPerChunk; k++) {
        const i64 j = map(k);
        a.re[k] = alpha * a.re[k] + beta * b.re[j];
        a.im[k] = alpha * a.im[k] + beta * b.im[j];
    }
}

double densDiagSum(QuregImpl& q, const u64* offs, int n, int skipBit, i64 chunkStart) {
    flush(q);
    double s = 0;
    const i64 dim = (i64)1 << n;
    for (i64 r = 0; r < dim; r++) {
        if (skipBit >= 0 && ((r >> skipBit) & 1)) continue;
        i64 p = 0;
        for (int j = 0; j < n; j++)
            if ((r >> j) & 1) p |= (i64)offs[j];
        p -= chunkStart;
        if (p >= 0 && p < q.numAmpsPerChunk) s += q.re[p];
    }
    return s;
}

void axpby(QuregImpl& a, real alpha, QuregImpl& b, real beta) {
    flush(a);
    flush(b);
#pragma omp parallel for if (a.numAmpsPerChunk >= kOmpMin)
    for (i64 i = 0; i < a.numAmpsPerChunk; i++) {
        a.re[i] = alpha * a.re[i] + beta * b.re[i];
        a.im[i] = alpha * a.im[i] + beta * b.im[i];
    }
}

void densInitPure(QuregImpl& rho, const real* pr, const real* pi, int n, i64 chunkStart) {
    flush(rho);
    const i64 mask = ((i64)1 << n) - 1;
#pragma omp parallel for if (rho.numAmpsPerChunk >= kOmpMin)
    for (i64 k = 0; k < rho.numAmpsPerChunk; k++) {
        i64 g = chunkStart + k, r = g & mask, c = g >> n;
        // psi_r * conj(psi_c)
        rho.re[k] = pr[r] * pr[c] + pi[r] * pi[c];
        rho.im[k] = pi[r] * pr[c] - pr[r] * pi[c];
    }
}

double densFidelity(QuregImpl& rho, const real* pr, const real* pi, int n, i64 chunkStart) {
    flush(rho);
    const i64 mask = ((i64)1 << n) - 1;
    double s = 0;
    for (i64 k = 0; k < rho.numAmpsPerChunk; k++) {
        i64 g = chunkStart + k, r = g & mask, c = g >> n;
        // Re[ conj(psi_r) rho psi_c ]
        double ar = rho.re[k] * pr[c] - rho.im[k] * pi[c];
        double ai = rho.re[k] * pi[c] + rho.im[k] * pr[c];
        s += pr[r] * ar + pi[r] * ai;
    }
    return s;
}

namespace {
// positions sorted ascending, for bit insertion
int sortedPositions(const int* pos, int k, int* out) {
    for (int i = 0; i < k; i++) out[i] = pos[i];
    std::sort(out, out + k);
    return k;
}
}  // namespace

void swapPartsWithPeer(QuregImpl&, real*, real*, const int*, int, u64, u64, i64, i64) {
    fprintf(stderr, "QuEST: in-place peer swaps need the HIP build's IPC transport\n");
    exit(EXIT_FAILURE);
}

void packBits(QuregImpl& q, const int* pos, int k, u64 setMask, i64 start, i64 count, real* br, real* bi) {
    flush(q);
    int sp[8];
    sortedPositions(pos, k, sp);
#pragma omp parallel for if (count >= kOmpMin)
    for (i64 j = 0; j < count; j++) {
        i64 i = start + j;
        for (int m = 0; m < k; m++) i = insertZero(i, sp[m]);
        i |= (i64)setMask;
        br[j] = q.re[i];
        bi[j] = q.im[i];
    }
}

void unpackBits(QuregImpl& q, const int* pos, int k, u64 setMask, i64 start, i64 count, const real* br,
                const real* bi) {
    flush(q);
    int sp[8];
    sortedPositions(pos, k, sp);
#pragma omp parallel for if (count >= kOmpMin)
    for (i64 j = 0; j < count; j++) {
        i64 i = start + j;
        for (int m = 0; m < k; m++) i = insertZero(i, sp[m]);
        i |= (i64)setMask;
        q.re[i] = br[j];
        q.im[i] = bi[j];
    }
}

void toBuffer(QuregImpl& q, i64 local, i64 n, real* br, real* bi) {
    flush(q);
    memcpy(br, q.re + local, sizeof(real) * n);
    memcpy(bi, q.im + local, sizeof(real) * n);
}

void fromBuffer(QuregImpl& q, i64 local, i64 n, const real* br, const real* bi) {
    flush(q);
    memcpy(q.re + local, br, sizeof(real) * n);
    memcpy(q.im + local, bi, sizeof(real) * n);
}

void bufferToHost(const real* buf, real* host, i64 n) { memcpy(host, buf, sizeof(real) * n); }
void hostToBuffer(const real* host, real* buf, i64 n) { memcpy(buf, host, sizeof(real) * n); }

}  // namespace be
}  // namespace qa

namespace qa {
namespace be {
bool setTuning(const char*, int) { return false; }
bool memoryInfo(size_t*, size_t*) { return false; }
bool getTuning(const char*, int*) { return false; }
}  // namespace be
}  // namespace qa
