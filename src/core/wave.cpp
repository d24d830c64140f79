#include "wave.hpp"

#include <chrono>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>

#include "router.hpp"

namespace qa {

extern thread_local int t_planQuiet;
namespace {

constexpr int kInf = 1 << 30;

// where[b]: < kWaveSlots: register slot; else lane bit (where - kWaveSlots)
inline bool inSlot(int w) { return w < kWaveSlots; }
inline int laneOf(int w) { return w - kWaveSlots; }

// How a Mat2 is executed.  Diagonal matrices need no slot.
enum class M2Class { Diag, Swap, Anti, Real, RealImag, General };

M2Class classify(const real* m) {
    // m: m00 re,im  m01 re,im  m10 re,im  m11 re,im
    const bool offZero = m[2] == 0 && m[3] == 0 && m[4] == 0 && m[5] == 0;
    const bool diagZero = m[0] == 0 && m[1] == 0 && m[6] == 0 && m[7] == 0;
    if (offZero) return M2Class::Diag;
    if (diagZero) {
        if (m[2] == 1 && m[3] == 0 && m[4] == 1 && m[5] == 0) return M2Class::Swap;
        return M2Class::Anti;
    }
    if (m[1] == 0 && m[3] == 0 && m[5] == 0 && m[7] == 0) return M2Class::Real;
    if (m[1] == 0 && m[7] == 0 && m[2] == 0 && m[4] == 0) return M2Class::RealImag;
    return M2Class::General;
}

struct Layout {
    int where[kWaveBits];
    int slotBit[kWaveSlots];
    int laneBit[kWaveLaneBits];

    void put(int b, int w) {
        where[b] = w;
        if (inSlot(w))
            slotBit[w] = b;
        else
            laneBit[laneOf(w)] = b;
    }
};

void masks(const Layout& lay, unsigned ctrlIn, unsigned& cReg, unsigned& cLane) {
    cReg = cLane = 0;
    for (int b = 0; b < kWaveBits; b++) {
        if (!((ctrlIn >> b) & 1)) continue;
        const int w = lay.where[b];
        if (inSlot(w))
            cReg |= 1u << w;
        else
            cLane |= 1u << laneOf(w);
    }
}

WaveOp blank(int kind) {
    WaveOp w;
    memset(&w, 0, sizeof w);
    w.kind = kind;
    return w;
}

// ---- cheaper gate forms (tools/gen_wave_asm.py KINDS2 / PH_KINDS) ----------
// A rotation [[c, -s], [s, c]] (c^2 + s^2 = 1) runs as three shears with
// t = tan(phi/2) = s / (1 + c), sn = sin(phi) = s; for c < 0 it is -R(phi - pi):
// the shears of phi - pi and a factor -1 for the pass (`neg`).
// tolerances for recognising unit-modulus / structured matrices: a few ulps
// of the build's precision (the matrices arrive in qreal)
constexpr double kUnitTol = sizeof(real) >= 8 ? 1e-14 : 1e-6;
constexpr double kNearTol = sizeof(real) >= 8 ? 1e-15 : 1e-7;
inline bool unitCircle(double c, double s) { return std::fabs(c * c + s * s - 1) <= kUnitTol; }

void rotParams(double c, double s, real* m, bool* neg) {
    *neg = c < 0;
    if (*neg) c = -c, s = -s;
    m[0] = (real)(s / (1 + c));
    m[1] = (real)s;
}

inline bool near(double a, double b) { return std::fabs(a - b) <= kNearTol; }

// Kind of a unit-modulus phase p (false: not unit modulus).  DROT / DROTN
// get their shear parameters in m[0], m[1]; identity phases give kind -1.
bool phaseKind(double pr, double pi, int* kind, real* m) {
    if (!unitCircle(pr, pi)) return false;
    if (near(pr, 1) && near(pi, 0)) *kind = -1;
    else if (near(pr, -1) && near(pi, 0)) *kind = (int)WKind::DNEG;
    else if (near(pr, 0) && near(pi, 1)) *kind = (int)WKind::DMULI;
    else if (near(pr, 0) && near(pi, -1)) *kind = (int)WKind::DMULNI;
    else {
        bool neg;
        rotParams(pr, pi, m, &neg);
        *kind = neg ? (int)WKind::DROTN : (int)WKind::DROT;
    }
    return true;
}

struct Scale {  // complex factor the pass still owes its amplitudes
    double re = 1, im = 0;
    void mul(double r, double i) {
        const double x = re * r - im * i;
        im = re * i + im * r;
        re = x;
    }
    bool one() const { return re == 1 && im == 0; }
};

bool isPhaseKind(int k) {
    return k == (int)WKind::DNEG || k == (int)WKind::DMULI || k == (int)WKind::DMULNI || k == (int)WKind::DROT ||
           k == (int)WKind::DROTN;
}

// The unit phase a phase op applies (phaseKind's inverse).
void phaseOf(const WaveOp& w, double* pr, double* pi) {
    switch ((WKind)w.kind) {
        case WKind::DNEG: *pr = -1, *pi = 0; return;
        case WKind::DMULI: *pr = 0, *pi = 1; return;
        case WKind::DMULNI: *pr = 0, *pi = -1; return;
        default: {
            // rotParams: m[0] = tan(phi / 2), m[1] = sin(phi) of the phase with
            // non-negative real part; DROTN negates it
            const double t = w.m[0];
            double c = (1 - t * t) / (1 + t * t), sn = w.m[1];
            if (w.kind == (int)WKind::DROTN) c = -c, sn = -sn;
            *pr = c;
            *pi = sn;
        }
    }
}

// Phase frame (round 5, QUEST_WAVE_ZFRAME=0 to disable; QUEST_WAVE_PFRAME=0:
// signs only): a unit phase on one register location -- a slot, a real lane
// bit or a wave bit: the DNEG / DMULI / DROT ops a pass emits for Z, S, T, Rz
// and for the conditional frame's bookkeeping, about a fifth of the bench
// passes' VALU instructions -- is not executed where it stands but multiplied
// into the location's pending phase and applied once, where an op needs it or
// at the end of the pass (phases on one location between two of its gates
// merge into one op or cancel).  Pending phases commute with diagonal ops and
// controls and move with transpositions; a 2x2 op on the location applies a
// general phase first.  A pending sign (Z) goes further:
//   * diagonal ops and ops controlled by the location commute with it;
//   * a transposition moves it with the bit (TR swaps two locations);
//   * a 2x2 op on the location is conjugated instead, U Z = Z (Z U Z): the
//     off-diagonal entries of its matrix change sign (general, real, Rx-form,
//     anti-diagonal kinds on slots and lanes), a rotation's angle too, Y <-> -Y;
//   * an X / CNOT on it (SWAP, LSWAP) with one plain control c: CX Z_t =
//     Z_t Z_c CX, the op stays and c joins the pending set;
//   * an uncontrolled X (X Z = -Z X: a global sign with nowhere to go here),
//     a multi-controlled X, an unnormalised Hadamard and channels apply the
//     pending Z first.
// Emulated and GPU passes run the transformed list, so the host emulation
// (QUEST_CPU_PLANNER=3) checks it against the oracle like any other plan.
void zFrame(WaveProgram& out, size_t begin) {
    static const bool on = !getenv("QUEST_WAVE_ZFRAME") || atoi(getenv("QUEST_WAVE_ZFRAME")) != 0;
    // QUEST_WAVE_PFRAME=0: carry only signs (Z), not general unit phases
    static const bool phases = !getenv("QUEST_WAVE_PFRAME") || atoi(getenv("QUEST_WAVE_PFRAME")) != 0;
    if (!on || out.ops.size() <= begin) return;
    constexpr int nLoc = kWaveSlots + kWaveLaneBits;   // slots, then lane / wave bits
    double zr[nLoc], zi[nLoc];                         // pending unit phase per location
    for (int l = 0; l < nLoc; l++) zr[l] = 1, zi[l] = 0;
    auto pending = [&](int l) { return !(zr[l] == 1 && zi[l] == 0); };
    auto isZ = [&](int l) { return near(zr[l], -1) && near(zi[l], 0); };
    std::vector<WaveOp> res(out.ops.begin(), out.ops.begin() + (long)begin);
    static long long why[4];   // QUEST_ZFRAME_STATS: HADD / 2x2 op, X, channel, end
    static const bool zst = getenv("QUEST_ZFRAME_STATS") != nullptr;
    static struct P { ~P() { if (zst) fprintf(stderr, "zframe flushes: op %lld X %lld chan %lld end %lld\n", why[0], why[1], why[2], why[3]); } } printer;
    int reason = 3;
    auto flush = [&](int loc) {   // apply the pending phase of loc here
        if (loc < 0 || loc >= nLoc || !pending(loc)) return;
        WaveOp w;
        memset(&w, 0, sizeof w);
        int kind;
        real pm[2] = {0, 0};
        if (phaseKind(zr[loc], zi[loc], &kind, pm) && kind >= 0) {
            w.kind = kind;
            w.m[0] = pm[0];
            w.m[1] = pm[1];
            if (loc < kWaveSlots)
                w.cReg = 1u << loc;
            else
                w.cLane = 1u << (loc - kWaveSlots);
            res.push_back(w);
            if (!t_planQuiet) why[reason]++;
        }
        zr[loc] = 1, zi[loc] = 0;
    };
    auto single = [](const WaveOp& w, int* loc) {   // one plain control location, nothing else
        if (w.ctrlOut || w.ctrlOutZero || w.cLaneZero || (w.cReg & w.fReg) || (w.cLane & w.fLane)) return false;
        const int n = __builtin_popcount(w.cReg) + __builtin_popcount(w.cLane);
        if (n != 1) return false;
        *loc = w.cReg ? __builtin_ctz(w.cReg) : kWaveSlots + __builtin_ctz(w.cLane);
        return true;
    };
    for (size_t o = begin; o < out.ops.size(); o++) {
        WaveOp w = out.ops[o];
        const WKind k = (WKind)w.kind;
        int loc = -1;
        if ((phases ? isPhaseKind(w.kind) : k == WKind::DNEG) && single(w, &loc)) {
            double pr, pi;
            phaseOf(w, &pr, &pi);
            const double r = zr[loc] * pr - zi[loc] * pi;
            zi[loc] = zr[loc] * pi + zi[loc] * pr;
            zr[loc] = r;
            if (near(zr[loc], 1) && near(zi[loc], 0)) zr[loc] = 1, zi[loc] = 0;   // (cancelled)
            continue;
        }
        if (k == WKind::TR) {
            std::swap(zr[w.a], zr[kWaveSlots + w.b]);
            std::swap(zi[w.a], zi[kWaveSlots + w.b]);
            res.push_back(w);
            continue;
        }
        const bool slotTarget = k == WKind::M2 || k == WKind::M2R || k == WKind::M2RI || k == WKind::ANTI ||
                                k == WKind::SWAP || k == WKind::ROTY || k == WKind::ROTX || k == WKind::HADD ||
                                k == WKind::YSW || k == WKind::YSWC;
        const bool laneTarget = k == WKind::LM2R || k == WKind::LM2RI || k == WKind::LANTI || k == WKind::LSWAP;
        if (k == WKind::CH1 || k == WKind::CHD) {
            reason = 2;
            flush(w.a);
            flush(w.b);
            res.push_back(w);
            continue;
        }
        if (!slotTarget && !laneTarget) {   // diagonal kinds: commute
            res.push_back(w);
            continue;
        }
        const int t = slotTarget ? w.a : kWaveSlots + w.a;
        if (!pending(t)) {
            res.push_back(w);
            continue;
        }
        if (!isZ(t)) {   // a general phase: applied before the op
            reason = 0;
            flush(t);
            res.push_back(w);
            continue;
        }
        switch (k) {
            case WKind::M2:   // (re, im) pairs: u00, u01, u10, u11
                for (int i = 2; i < 6; i++) w.m[i] = -w.m[i];
                break;
            case WKind::M2R: case WKind::M2RI: case WKind::LM2R: case WKind::LM2RI:
                w.m[1] = -w.m[1];
                w.m[2] = -w.m[2];
                break;
            case WKind::ANTI: case WKind::LANTI:
                for (int i = 0; i < 4; i++) w.m[i] = -w.m[i];
                break;
            case WKind::ROTY: case WKind::ROTX:
                w.m[0] = -w.m[0];
                w.m[1] = -w.m[1];
                break;
            case WKind::YSW: w.kind = (int)WKind::YSWC; break;
            case WKind::YSWC: w.kind = (int)WKind::YSW; break;
            case WKind::SWAP: case WKind::LSWAP: {
                int c = -1;
                if (single(w, &c)) {   // CX Z_t = Z_t Z_c CX
                    const double r = -zr[c];
                    zi[c] = -zi[c];
                    zr[c] = r;
                    if (near(zr[c], 1) && near(zi[c], 0)) zr[c] = 1, zi[c] = 0;
                } else {
                    reason = 1;
                    flush(t);
                }
                break;
            }
            default:   // HADD
                reason = 0;
                flush(t);
                break;
        }
        res.push_back(w);
    }
    reason = 3;
    for (int loc = 0; loc < nLoc; loc++) flush(loc);
    out.ops.swap(res);
}

// Merge the phase ops of every run of consecutive diagonal ops in
// out.ops[begin..) that act on the same amplitudes (same register / lane /
// wave / out-of-tile predicates): the product goes to the first of them,
// identities disappear.
void mergePhases(WaveProgram& out, size_t begin) {
    std::vector<WaveOp>& ops = out.ops;
    auto diag = [](int k) { return isPhaseKind(k) || k == (int)WKind::DIAG || k == (int)WKind::DSC; };
    auto same = [](const WaveOp& x, const WaveOp& y) {
        return x.a == y.a && x.b == y.b && x.cReg == y.cReg && x.cLane == y.cLane && x.cLaneZero == y.cLaneZero &&
               x.fReg == y.fReg && x.fLane == y.fLane && x.ctrlOut == y.ctrlOut && x.ctrlOutZero == y.ctrlOutZero;
    };
    std::vector<char> gone(ops.size(), 0);
    bool any = false;
    size_t run = begin;
    for (size_t k = begin; k <= ops.size(); k++) {
        if (k < ops.size() && diag(ops[k].kind)) continue;
        for (size_t x = run; x < k; x++) {
            if (gone[x] || !isPhaseKind(ops[x].kind)) continue;
            double pr, pi;
            phaseOf(ops[x], &pr, &pi);
            std::vector<size_t> ys;
            for (size_t y = x + 1; y < k; y++) {
                if (gone[y] || !isPhaseKind(ops[y].kind) || !same(ops[x], ops[y])) continue;
                double qr, qi;
                phaseOf(ops[y], &qr, &qi);
                const double r = pr * qr - pi * qi, i = pr * qi + pi * qr;
                pr = r, pi = i;
                ys.push_back(y);
            }
            int kind;
            real pm[2] = {0, 0};
            if (ys.empty() || !phaseKind(pr, pi, &kind, pm)) continue;   // (products of unit phases stay unit)
            for (size_t y : ys) gone[y] = 1;
            any = true;
            if (kind < 0) {
                gone[x] = 1;
                continue;
            }
            ops[x].kind = kind;
            ops[x].m[0] = pm[0];
            ops[x].m[1] = pm[1];
        }
        run = k + 1;
    }
    if (!any) return;
    size_t w = begin;
    for (size_t k = begin; k < ops.size(); k++)
        if (!gone[k]) ops[w++] = ops[k];
    ops.resize(w);
}

}  // namespace

// Absorb the factor (sr, si) a pass owes its amplitudes: scale the matrix of
// one uncontrolled op that takes it at no cost (complex: M2, ANTI, D2S, D2L,
// LANTI; real: also M2R, M2RI, LM2R, LM2RI); else turn an unnormalised
// Hadamard or a rotation back into a scaled M2R / M2RI; else append a phase op.
void settleScale(WaveProgram& out, int begin, double sr, double si) {
    auto free = [](const WaveOp& w) {
        return w.cReg == 0 && w.cLane == 0 && w.cLaneZero == 0 && w.ctrlOut == 0 && w.ctrlOutZero == 0;
    };
    const bool realF = si == 0;
    auto cm = [&](real* p) {  // p[0] + i p[1] *= (sr + i si)
        const double x = p[0] * sr - p[1] * si, y = p[0] * si + p[1] * sr;
        p[0] = (real)x;
        p[1] = (real)y;
    };
    for (size_t k = (size_t)begin; k < out.ops.size(); k++) {
        WaveOp& w = out.ops[k];
        if (!free(w)) continue;
        switch ((WKind)w.kind) {
            case WKind::M2:
                for (int e = 0; e < 4; e++) cm(w.m + 2 * e);
                return;
            case WKind::ANTI:
            case WKind::LANTI:
            case WKind::D2S:
            case WKind::D2L:
                cm(w.m);
                cm(w.m + 2);
                return;
            case WKind::M2R:
            case WKind::M2RI:
            case WKind::LM2R:
            case WKind::LM2RI:
                if (!realF) break;
                for (int e = 0; e < 4; e++) w.m[e] = (real)(w.m[e] * sr);
                return;
            default: break;
        }
    }
    if (realF)
        for (size_t k = (size_t)begin; k < out.ops.size(); k++) {
            WaveOp& w = out.ops[k];
            if (!free(w)) continue;
            if (w.kind == (int)WKind::HADD) {  // computed [[1, 1], [1, -1]]
                w.kind = (int)WKind::M2R;
                w.m[0] = w.m[1] = w.m[2] = (real)sr;
                w.m[3] = (real)-sr;
                return;
            }
            if (w.kind == (int)WKind::ROTY || w.kind == (int)WKind::ROTX) {
                // the emitted rotation: cos = 1 - t sin, sin
                const double c = 1 - (double)w.m[0] * w.m[1], s = w.m[1];
                if (w.kind == (int)WKind::ROTY) {
                    w.m[0] = (real)(c * sr);
                    w.m[1] = (real)(-s * sr);
                    w.m[2] = (real)(s * sr);
                    w.m[3] = (real)(c * sr);
                    w.kind = (int)WKind::M2R;
                } else {  // [[c, -is], [-is, c]] as M2RI (m00, Im m01, Im m10, m11)
                    w.m[0] = (real)(c * sr);
                    w.m[1] = (real)(-s * sr);
                    w.m[2] = (real)(-s * sr);
                    w.m[3] = (real)(c * sr);
                    w.kind = (int)WKind::M2RI;
                }
                return;
            }
        }
    WaveOp w = blank((int)WKind::DIAG);   // every amplitude
    w.m[0] = (real)sr;
    w.m[1] = (real)si;
    out.ops.push_back(w);
}

bool& waveRelabel() {
    static bool on = !getenv("QUEST_WAVE_RELABEL") || atoi(getenv("QUEST_WAVE_RELABEL")) != 0;
    return on;
}

bool waveStoresInPlace(const WavePass& wp) {
    if (wp.stFlipLane >> kWaveLanes) return false;   // wave w stores where wave w ^ f loaded
    for (int l = kWaveLanes; l < kWaveLaneBits; l++)
        if (wp.stCondLane[l]) return false;          // ... or where a wave-conditioned flip sends it
    for (int l = kWaveLanes; l < kWaveLaneBits; l++)
        if (wp.pos[wp.ldLane[l]] != wp.stPos[wp.stLane[l]]) return false;
    return true;
}

bool waveLowPerm(const TilePass& ps, const TileOp* ops, int cmin, int* sigma) {
    // on by default for the fp32 tile (5 slots x 3 wave bits); off for the fp64
    // tile of 5 slots x 2 wave bits, whose plans it made worse on one of five
    // circuit seeds (15 -> 20 passes; same passes and 0.7 % faster without it,
    // profiles/r3/wave_shape_variants.txt)
    static const bool on = getenv("QUEST_WAVE_LOW_PERM") ? atoi(getenv("QUEST_WAVE_LOW_PERM")) != 0
                                                          : !(kWaveSlots == 5 && kWaveWBits == 2);
    for (int p = 0; p < 64; p++) sigma[p] = p;
    if (!on || ps.k != kWaveBits) return false;
    WaveProgram tmp;
    int endLanes[3];
    bool ok;
    {
        QuietPlan quiet;
        ok = planWavePass(ps, ops, ps.opEnd - ps.opBegin, tmp, endLanes);
    }
    if (!ok) return false;
    constexpr int VB = kWaveVecBits;
    // tile bits stored to the always-resident positions [VB, cmin)
    int bitAt[64];
    for (int p = 0; p < 64; p++) bitAt[p] = -1;
    for (int b = 0; b < ps.k; b++)
        if (ps.stPos[b] >= VB && ps.stPos[b] < cmin) bitAt[ps.stPos[b]] = b;
    for (int p = VB; p < cmin; p++)
        if (bitAt[p] < 0) return false;   // (a wave tile holds every position below cmin)
    int newPos[64];
    for (int b = 0; b < 64; b++) newPos[b] = -1;
    bool used[64] = {false};
    for (int l = 0; l < 3 && VB + l < cmin; l++) {
        const int b = endLanes[l];
        if (b >= 0 && ps.stPos[b] >= VB && ps.stPos[b] < cmin && newPos[b] < 0) {
            newPos[b] = VB + l;
            used[VB + l] = true;
        }
    }
    int next = VB;
    for (int p = VB; p < cmin; p++) {
        const int b = bitAt[p];
        if (newPos[b] >= 0) continue;
        while (used[next]) next++;
        newPos[b] = next;
        used[next] = true;
    }
    bool moved = false;
    for (int p = VB; p < cmin; p++) {
        sigma[p] = newPos[bitAt[p]];
        moved = moved || sigma[p] != p;
    }
    if (!moved) return false;
    // the adjusted layout must still lower (it only spares transpositions)
    TilePass cand = ps;
    for (int i = 0; i < cand.k; i++) cand.stPos[i] = sigma[cand.stPos[i]];
    if (!waveLowers(cand, ops)) {
        for (int p = 0; p < 64; p++) sigma[p] = p;
        return false;
    }
    return true;
}

int& waveLaneOrder() {
    static int order = getenv("QUEST_WAVE_LANE_ORDER") ? atoi(getenv("QUEST_WAVE_LANE_ORDER")) : 1;
    return order;
}

bool relabelsLower(const TileProgram& prog) {
    QuietPlan quiet;
    bool ok = true;
    for (const TilePass& ps : prog.passes) {
        bool perm = false;
        for (int i = 0; i < ps.k; i++) perm |= ps.stPos[i] != ps.pos[i];
        if (!perm) continue;
        WaveProgram tmp;
        if (!planWavePass(ps, prog.ops.data() + ps.opBegin, ps.opEnd - ps.opBegin, tmp)) {
            ok = false;
            break;
        }
    }
    return ok;
}

long long g_waveStoreTrCost = 0;

// QUEST_CNOT_STATS=1 (planner study): why deferred CNOTs were executed, by
// reason and by the domains of control / target -- printed at exit
namespace {
const char* kCnotReason[] = {"ctrl-of-deferred-has-conds", "target-conditions-others", "channel", "op-control-has-conds",
                             "phase-mask-has-conds", "gate-on-control", "gate-on-target", "diag-run", "end-of-pass"};
long long g_cnotStats[9][3][3];
bool cnotStatsOn() {
    static const bool on = getenv("QUEST_CNOT_STATS") != nullptr;
    return on;
}
struct CnotStatsPrinter {
    ~CnotStatsPrinter() {
        if (!cnotStatsOn()) return;
        const char* dn[] = {"slot", "lane", "wave"};
        long long tot = 0;
        for (auto& a : g_cnotStats)
            for (auto& b : a)
                for (long long v : b) tot += v;
        fprintf(stderr, "executed deferred CNOTs: %lld\n", tot);
        for (int r = 0; r < 9; r++)
            for (int c = 0; c < 3; c++)
                for (int t = 0; t < 3; t++)
                    if (g_cnotStats[r][c][t])
                        fprintf(stderr, "  %-28s control %-4s target %-4s %6lld (%.1f %%)\n", kCnotReason[r], dn[c], dn[t],
                                g_cnotStats[r][c][t], 100.0 * g_cnotStats[r][c][t] / tot);
    }
} g_cnotStatsPrinter;
// QUEST_CTRL_STATS=1 (kernel study): ops of the executed wave passes by kind
// and slot-control count (0, 1, 2+) / lane controls, with modeled cycles
long long g_ctrlOps[32][3][2];
double g_ctrlCyc[32][3][2];
double g_trByBit[16][2];   // TR ops by lane / wave bit: count, modeled cycles
bool ctrlStatsOn() {
    static const bool on = getenv("QUEST_CTRL_STATS") != nullptr;
    return on;
}
struct CtrlStatsPrinter {
    ~CtrlStatsPrinter() {
        if (!ctrlStatsOn()) return;
        double tot = 0;
        for (auto& a : g_ctrlCyc)
            for (auto& b : a)
                for (double v : b) tot += v;
        fprintf(stderr, "wave ops by kind / slot controls / lane controls (modeled cycles %.3g):\n", tot);
        for (int k = 0; k < 32; k++)
            for (int c = 0; c < 3; c++)
                for (int l = 0; l < 2; l++)
                    if (g_ctrlOps[k][c][l])
                        fprintf(stderr, "  kind %2d cReg %d%s lanes %d %8lld ops %5.1f %% cycles\n", k, c, c == 2 ? "+" : " ", l,
                                g_ctrlOps[k][c][l], 100.0 * g_ctrlCyc[k][c][l] / tot);
        for (int b = 0; b < 16; b++)
            if (g_trByBit[b][0] > 0)
                fprintf(stderr, "  TR with bit %2d: %6.0f ops %5.1f %% cycles\n", b, g_trByBit[b][0], 100.0 * g_trByBit[b][1] / tot);
    }
} g_ctrlStatsPrinter;
}  // namespace
thread_local int t_planQuiet = 0;
thread_local int t_waveCframe = -1;

bool waveLowers(const TilePass& ps, const TileOp* ops) {
    QuietPlan quiet;
    WaveProgram tmp;
    return planWavePass(ps, ops, ps.opEnd - ps.opBegin, tmp);
}

// Issue cycles per wave of one op (uncontrolled), from the measured cost of
// the generated handlers (tools/wave_cost.py over the bench plans, issue
// costs of profiles/r2/isa_micro_gfx950.txt); slot-controlled ops branch over
// the registers that fail their controls.
double waveOpCycles(const WaveOp& w) {
    // round-4 calibration (tools/cost_fit.py: the per-pass compute of the
    // --nomem kernel over 64 passes of three circuits against the handler
    // mix): matrix handlers 1.5x, phases 1.25x, Ry / Rx 1.28x, register
    // swaps 0.67x, lane swaps 0.75x, lane-0/1 transpositions 0.74x -- rms
    // error per pass 0.27 -> 0.21 ms, same total (QUEST_WAVE_COST_MODEL=0:
    // the round-3 table)
    static const bool cal = !getenv("QUEST_WAVE_COST_MODEL") || atoi(getenv("QUEST_WAVE_COST_MODEL")) != 0;
    double c;
    switch ((WKind)w.kind) {
        case WKind::M2: c = 600; break;
        case WKind::M2R: case WKind::M2RI: case WKind::D2S: c = 300; break;
        case WKind::ANTI: c = 450; break;
        case WKind::SWAP: c = 211; break;
        case WKind::DIAG: c = 256; break;
        case WKind::D2L: c = 300; break;
        case WKind::TR: {
            static const double lane[kWaveLanes] = {517, 563, 341, 339, 264, 259};
            c = w.b < kWaveLanes ? lane[w.b] : 300;   // wave bits: LDS round trip
            break;
        }
        case WKind::LM2R: c = 724; break;
        case WKind::LM2RI: c = 578; break;
        case WKind::LANTI: c = 600; break;
        case WKind::LSWAP: c = 425; break;
        case WKind::ROTY: case WKind::ROTX: c = 207; break;
        case WKind::HADD: c = 140; break;
        case WKind::YSW: case WKind::YSWC: c = 250; break;
        case WKind::DROT: c = 190; break;
        case WKind::DNEG: c = 61; break;
        case WKind::DMULI: case WKind::DMULNI: c = 236; break;
        case WKind::DROTN: c = 259; break;
        case WKind::DSC: c = 128; break;
        default: c = 300; break;   // channels
    }
    if (cal) {
        switch ((WKind)w.kind) {
            case WKind::M2: case WKind::M2R: case WKind::M2RI: case WKind::ANTI: case WKind::D2S: case WKind::D2L:
            case WKind::YSW: case WKind::YSWC: c *= 1.5; break;
            case WKind::SWAP: c *= 0.67; break;
            case WKind::LSWAP: c *= 0.75; break;
            case WKind::TR: if (w.b < 2) c *= 0.74; else if (w.b >= kWaveLanes) c *= 0.88; break;
            case WKind::ROTY: case WKind::ROTX: c *= 1.28; break;
            case WKind::HADD: c *= 0.79; break;
            case WKind::DNEG: c *= 1.31; break;
            case WKind::DIAG: case WKind::DROT: case WKind::DMULI: case WKind::DMULNI: case WKind::DROTN:
            case WKind::DSC: c *= 1.25; break;
            default: break;
        }
    }
    const bool slotKind = w.kind != (int)WKind::TR && w.kind != (int)WKind::D2L &&
                          (w.kind < (int)WKind::LM2R || w.kind > (int)WKind::LSWAP);
    if (slotKind && w.cReg) c *= std::ldexp(1.0, -__builtin_popcount(w.cReg));
    return c;
}

double wavePassCycles(const TilePass& ps, const TileOp* ops) {
    QuietPlan quiet;
    WaveProgram tmp;
    double c = -1;
    if (planWavePass(ps, ops, ps.opEnd - ps.opBegin, tmp)) {
        c = 0;
        for (const WaveOp& w : tmp.ops) c += waveOpCycles(w);
    }
    return c;
}

void waveCostHooks(PlanHooks& hooks) {
    // One pass's HBM stream in the units of wavePassCycles: a 30-qubit pass
    // streams in about 5.6 ms, the time the kernel issues about 12800 modeled
    // cycles per wave and tile (profiles/r3/overlap_study_one_tile_per_wg.txt
    // against the plan's modeled cycles); both scale with the tile count.
    // (fp32: the handler table is fp64's and the 2^14 tile's balance differs;
    // trimming measured 1.7-2.6 % slower there, profiles/r4/f32_mem_ab.txt: off)
    static const double mem = getenv("QUEST_PLAN_MEM_CYCLES") ? atof(getenv("QUEST_PLAN_MEM_CYCLES"))
                                                              : (sizeof(real) == 4 ? 0.0 : 12800.0);
    static const double margin = getenv("QUEST_PLAN_COST_MARGIN") ? atof(getenv("QUEST_PLAN_COST_MARGIN")) : 0.1;
    if (mem <= 0) return;
    hooks.passCost = [](const TilePass& ps, const TileOp* ops) { return wavePassCycles(ps, ops); };
    hooks.memCost = mem;
    hooks.costMargin = margin;
}

namespace {
struct WaveStrategy {
    int dc;        // always-resident low positions - cdefault
    int cost;      // compute-aware passes: 1 as waveCostHooks, 0 off, 2 without margin
    int seeds;     // seed candidates per pass (0: default)
    double look;   // one-pass lookahead weight (< 0: default)
    int cframe;    // conditional exchange frame: 1 as configured, 0 off
    int commute;   // class-aware commutation in the scheduler (t_planCommute): -1 as configured, 0 off, 1 on
    double mem = 0;  // trimming bound in modeled cycles (0: waveCostHooks')
    int roll = 0;    // rollout scoring of candidate passes (PlanHooks::rollout)
};
// 0 is the configured default (cost = -1, cframe = -1: waveCostHooks and the
// environment as they are); the 8th is the round-3 planner (no compute-aware
// passes, no conditional frame); then class-aware commutation variants
const WaveStrategy kStrategies[] = {{0, -1, 0, -1, -1, -1}, {1, 1, 0, -1, 1, -1}, {0, 0, 0, -1, 1, -1},
                                    {1, 0, 0, -1, 1, -1},   {0, 2, 0, -1, 1, -1},  {0, 1, 96, -1, 1, -1},
                                    {0, 1, 0, 0.5, 1, -1},  {0, 0, 0, -1, 0, -1},  {0, -1, 0, -1, -1, 1},
                                    {1, 1, 0, -1, 1, 1},    {0, 0, 0, -1, 1, 1},   {1, 0, 0, -1, 1, 1},
                                    {-1, 1, 0, -1, 1, -1},  {-1, 0, 0, -1, 1, -1},  {0, 1, 0, -1, 1, -1, 15000},
                                    {0, 1, 0, -1, 1, -1, 17500},
                                    // round 6: candidate lookahead off / strong (the default is 0.3)
                                    {0, -1, 0, 0.0, -1, -1}, {0, 1, 0, 0.0, 1, -1}, {1, 1, 0, 0.0, 1, -1},
                                    {0, 1, 0, 1.0, 1, -1},
                                    // round 6: rollout-scored candidates
                                    {0, 1, 0, -1, 1, -1, 0, 1}, {1, 1, 0, -1, 1, -1, 0, 2}, {0, 0, 0, -1, 1, -1, 0, 1},
                                    {0, 1, 0, -1, 1, -1, 0, 2}};
constexpr int kNumStrategies = (int)(sizeof kStrategies / sizeof kStrategies[0]);
// strategies the search tries (QUEST_PLAN_STRATEGIES, default all 16: with
// the commutation and one-fewer-resident-position variants the five bench
// seeds plan 80 passes instead of 82, 0.1306 vs 0.1317 ms / gate over three
// interleaved rounds on one box, profiles/r5/search_strategies_ab.txt; 11
// circuit seeds 177 instead of 183 passes in the host model; the last two,
// trimming against a larger memory budget, leave the bench seeds' plans as
// they are and take fresh seeds 14-20 from 96 to 94 passes, 0.1247 -> 0.1233
// ms / gate, profiles/r5/trim_budget_strategies_ab.txt)
int searchStrategies(int L) {
    // from 30 local qubits (passes of 6 ms and more hide the longer search)
    // the four lookahead variants join: host study, seeds 11-20 152 -> 150
    // passes, the other seed sets -0.1 .. -2 % predicted (plan_seeds.txt)
    if (!getenv("QUEST_PLAN_STRATEGIES")) return L >= 30 ? 20 : 16;
    static const int n = [] {
        const char* e = getenv("QUEST_PLAN_STRATEGIES");
        // (round 6: strategies 16-19, lookahead variants, and the four rollout
        // ones after them are opt-in -- QUEST_PLAN_STRATEGIES=20: bench seeds
        // 512 -> 502 predicted ms, fresh seeds 21-80 / 141-200 unchanged;
        // =24: rollouts, fresh seeds 21-30 166 -> 163 passes at ten times the
        // host time per strategy, profiles/r6/rollout_strategies.txt)
        const int v = e ? atoi(e) : 16;
        return v < 1 ? 1 : v > kNumStrategies ? kNumStrategies : v;
    }();
    return n;
}

void strategyHooks(const WaveStrategy& st, PlanHooks& h) {
    PlanHooks costed;
    waveCostHooks(costed);
    const double M = costed.memCost > 0 ? costed.memCost : 12800.0;
    h.seeds = st.seeds;
    h.lookahead = st.look;
    h.rollout = st.roll;
    if (st.cost < 0) {   // as configured
        h.passCost = nullptr;
        h.memCost = 0;
        waveCostHooks(h);
        return;
    }
    h.passCost = nullptr;
    h.memCost = 0;
    if (st.cost) {
        h.passCost = [](const TilePass& ps, const TileOp* o) { return wavePassCycles(ps, o); };
        h.memCost = st.mem > 0 ? st.mem : M;
        h.costMargin = st.cost == 2 ? 0.0 : costed.costMargin;
    }
    h.seeds = st.seeds;
    h.lookahead = st.look;
}
}  // namespace

size_t waveSearchMinOps() {
    static const size_t v = getenv("QUEST_PLAN_SEARCH_OPS") ? (size_t)atol(getenv("QUEST_PLAN_SEARCH_OPS")) : 256;
    return v;
}

int waveCostMinQubits() {
    // compute-aware trimming costs a wave lowering per candidate pass: at 20
    // local qubits (passes of ~10 us) that host time outweighs what it saves
    // (profiles/r4/search_small_registers.txt: 2.11 -> 1.79 us / gate without).
    // Round 6 (fused_sweep windows, profiles/r6/cost_qubits_ab.txt): below 30
    // local qubits the passes it shortens are not memory-bound enough to pay
    // for the passes it adds -- 22-26 qubits 1-30 % faster without it, 27 / 29
    // neutral, 28 -2.8 % (22 before)
    static const int v = getenv("QUEST_PLAN_COST_QUBITS") ? atoi(getenv("QUEST_PLAN_COST_QUBITS")) : 30;
    return v;
}

int waveSearchMinQubits() {
    // below it a pass streams in well under a millisecond and the search's
    // host time (several ms a window) costs more than the passes it saves:
    // 20-24 local qubits ran 2-3x slower with it, 26 13 % slower, 28 7 %
    // faster (profiles/r4/search_small_registers.txt)
    static const int v = getenv("QUEST_PLAN_SEARCH_QUBITS") ? atoi(getenv("QUEST_PLAN_SEARCH_QUBITS")) : 27;
    return v;
}

bool waveSearchSplitFirst(const QuregImpl& q) {
    // (28 qubits, 10-layer windows of ~400 ops: the search held the window's
    // first pass back by 1.2-2.2 ms, profiles/r6/search_split_ab.txt)
    static const bool on = !getenv("QUEST_PLAN_SEARCH_SPLIT") || atoi(getenv("QUEST_PLAN_SEARCH_SPLIT")) != 0;
    return on && waveSearchOn() && waveFrontSearch() && q.planStrategy < 0 && !q.strategySearch.valid() &&
           q.L >= waveSearchMinQubits() && q.pending.size() > waveSearchMinOps() && !getenv("QUEST_WAVE_CMIN");
}

bool waveFrontSearch() {
    static const bool v = !getenv("QUEST_PLAN_SEARCH_FRONT") || atoi(getenv("QUEST_PLAN_SEARCH_FRONT")) != 0;
    return v;
}

int waveFrontStrategy() {
    static const int v = getenv("QUEST_PLAN_FRONT_STRATEGY") ? atoi(getenv("QUEST_PLAN_FRONT_STRATEGY")) : -1;
    return v;
}

bool waveSearchOn() {
    static const bool on = !getenv("QUEST_PLAN_SEARCH") || atoi(getenv("QUEST_PLAN_SEARCH")) != 0;
    return on;
}

int searchWaveStrategy(const std::vector<Op>& ops, int L, int cdefault, const PlanHooks& base) {
    if (!waveSearchOn() || ops.size() < waveSearchMinOps() || L < kWaveBits + 6 || L < waveSearchMinQubits()) return -1;
    PlanHooks costed;
    waveCostHooks(costed);
    const double M = costed.memCost > 0 ? costed.memCost : 12800.0;
    const int fuse = fuseBlockQubits();
    double score[kNumStrategies], took[kNumStrategies] = {0};
    auto run = [&](int i) {
        const auto tRun0 = std::chrono::steady_clock::now();
        QuietPlan quiet;
        fuseBlockQubits() = fuse;              // (thread-local)
        t_waveCframe = kStrategies[i].cframe;  // (thread-local)
        t_planCommute = kStrategies[i].commute;
        const int c = cdefault + kStrategies[i].dc;
        score[i] = 1e300;
        if (c < kWaveBits - 1) {
            PlanHooks h;
            h.relabelOk = base.relabelOk;
            h.lowPerm = base.lowPerm;
            strategyHooks(kStrategies[i], h);
            std::vector<Op> mine = ops;
            TileProgram prog;
            planTiles(mine, L, kWaveBits, c, true, prog, kWaveVecBits, &h);
            // score: sum over passes of max(C, M) + alpha min(C, M) -- a one-tile
            // workgroup overlaps compute and memory worst when they are close
            // (round 5: T = 1.2 sum max with C near M); QUEST_PLAN_SCORE_OVERLAP = alpha
            static const double alpha = getenv("QUEST_PLAN_SCORE_OVERLAP") ? atof(getenv("QUEST_PLAN_SCORE_OVERLAP")) : 0.0;
            // a pass costs M + slope * max(0, C - knee): the hinge fitted to
            // measured pass times (profiles/r6/pass_time_model.txt: 5.81 ms +
            // 0.345 us per modeled cycle above 11500, i.e. 0.76 of M / 12800 per
            // cycle); QUEST_PLAN_SCORE_KNEE=0: round 5's max(C, M)
            // (fp64's fit; fp32 keeps max(C, M): five seeds 73 vs 77 passes with
            // round 5's planner knobs in the host study)
            static const double knee = getenv("QUEST_PLAN_SCORE_KNEE") ? atof(getenv("QUEST_PLAN_SCORE_KNEE"))
                                                                       : (sizeof(real) == 8 ? 11500.0 : 0.0);
            static const double slope = getenv("QUEST_PLAN_SCORE_SLOPE") ? atof(getenv("QUEST_PLAN_SCORE_SLOPE")) : 0.76;
            double t = 0;
            for (const TilePass& ps : prog.passes) {
                const double cyc = wavePassCycles(ps, prog.ops.data() + ps.opBegin);
                const double c = cyc < 0 ? M : cyc;
                t += knee > 0 ? M + slope * std::max(0.0, c - knee) : std::max(c, M) + alpha * std::min(c, M);
            }
            score[i] = t;
        }
        t_waveCframe = -1;
        t_planCommute = -1;
        took[i] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tRun0).count();
    };
    std::vector<std::thread> pool;
    const int nStrat = searchStrategies(L);
    const auto tSearch0 = std::chrono::steady_clock::now();
    for (int i = 1; i < nStrat; i++) pool.emplace_back(run, i);
    run(0);
    for (std::thread& th : pool) th.join();
    int best = 0;
    for (int i = 1; i < nStrat; i++)
        if (score[i] < score[best] * (1 - 1e-9)) best = i;
    static const bool dbg = getenv("QUEST_PLAN_SEARCH_DEBUG") != nullptr;
    if (dbg) {
        fprintf(stderr, "search over %zu ops (%.1f ms):", ops.size(),
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tSearch0).count());
        for (int i = 0; i < nStrat; i++) fprintf(stderr, " %.0f (%.1f ms)", score[i], took[i]);
        fprintf(stderr, " -> %d\n", best);
    }
    return best;
}

WaveStrategyScope::WaveStrategyScope(int idx, int cdefault, PlanHooks& hooks, int* cmin) {
    *cmin = cdefault;
    if (idx <= 0 || idx >= kNumStrategies) return;   // 0 / -1: as configured
    *cmin = cdefault + kStrategies[idx].dc;
    strategyHooks(kStrategies[idx], hooks);
    t_waveCframe = kStrategies[idx].cframe;
    t_planCommute = kStrategies[idx].commute;
    active = true;
}

WaveStrategyScope::~WaveStrategyScope() {
    if (active) {
        t_waveCframe = -1;
        t_planCommute = -1;
    }
}

int chooseWaveCmin(QuregImpl& q, int cdefault, const PlanHooks& hooks) {
    // off by default: the two trial plans (about 2 ms on the host, before the
    // window's first pass starts) cost more than the passes saved on four of
    // five bench seeds (profiles/r3/cmin_search_ab.txt: +0.7..+1.0 %, one seed
    // -7.5 %); QUEST_WAVE_CMIN_SEARCH=1 turns it on
    static const bool on = getenv("QUEST_WAVE_CMIN_SEARCH") && atoi(getenv("QUEST_WAVE_CMIN_SEARCH")) != 0;
    if (!on || q.pending.size() < 64) return cdefault;
    if (q.waveCmin >= 0) return q.waveCmin;
    // plan the queue with cdefault and cdefault + 1 always-resident low
    // positions (plans only: the relabel / low-permutation hooks, nothing
    // launched) and keep the one with fewer passes; the choice holds until
    // the queue drains.  Which one wins varies with the circuit: 15-21 vs
    // 16-20 passes on five bench seeds (profiles/r3/prof_end_r3.txt)
    PlanHooks trialHooks;
    trialHooks.relabelOk = hooks.relabelOk;
    trialHooks.lowPerm = hooks.lowPerm;
    QuietPlan quiet;
    size_t best = (size_t)-1;
    int choice = cdefault;
    for (int c = cdefault; c <= cdefault + 1 && c < kWaveBits - 1; c++) {
        std::vector<Op> ops = q.pending;
        TileProgram prog;
        planTiles(ops, q.L, kWaveBits, c, true, prog, kWaveVecBits, &trialHooks);
        if (prog.passes.size() < best) {
            best = prog.passes.size();
            choice = c;
        }
    }
    q.waveCmin = choice;
    return choice;
}

void applyProgramPerm(QuregImpl& q, const TileProgram& prog) {
    if ((int)prog.perm.size() != q.L) return;
    bool id = true;
    for (int x = 0; x < q.L; x++) id = id && prog.perm[x] == x;
    if (id) return;
    for (int lg = 0; lg < q.nSV; lg++)
        if (q.l2p[lg] < q.L) q.l2p[lg] = prog.perm[q.l2p[lg]];
    for (int lg = 0; lg < q.nSV; lg++) q.p2l[q.l2p[lg]] = lg;
}

bool planRelayout(int L, const int* destIn, TileProgram& prog) {
    constexpr int VB = kWaveVecBits, K = kWaveBits, fixedLow = kWaveVecBits + 3;
    prog.passes.clear();
    prog.ops.clear();
    prog.phases.clear();
    prog.perm.resize((size_t)L);
    for (int x = 0; x < L; x++) prog.perm[(size_t)x] = x;
    if (L < K) return false;
    int dest[64];
    for (int p = 0; p < L; p++) dest[p] = destIn[p];
    for (int v = 0; v < VB; v++)
        if (dest[v] != v) return false;   // the vector bits never move in a wave pass
    for (int guard = 0; guard < 4 * L; guard++) {
        bool done = true;
        for (int p = 0; p < L && done; p++) done = dest[p] == p;
        if (done) return true;
        // the tile: positions 0 .. fixedLow-1 (every wave tile holds them),
        // then whole cycles of dest that fit (those through the fixed low
        // positions first), then a run of the next cycle
        std::vector<char> inT((size_t)L, 0);
        int count = 0;
        for (int p = 0; p < fixedLow; p++) inT[(size_t)p] = 1, count++;
        std::vector<std::vector<int>> cycles;
        std::vector<char> seen((size_t)L, 0);
        for (int p = 0; p < L; p++) {
            if (seen[(size_t)p] || dest[p] == p) continue;
            std::vector<int> c;
            for (int x = p; !seen[(size_t)x]; x = dest[x]) {
                seen[(size_t)x] = 1;
                c.push_back(x);
            }
            cycles.push_back(c);
        }
        auto touchesLow = [&](const std::vector<int>& c) {
            for (int x : c)
                if (x < fixedLow) return true;
            return false;
        };
        std::stable_sort(cycles.begin(), cycles.end(), [&](const std::vector<int>& a, const std::vector<int>& b) {
            const bool la = touchesLow(a), lb = touchesLow(b);
            if (la != lb) return la;
            return a.size() < b.size();
        });
        for (const std::vector<int>& c : cycles) {
            int missing = 0;
            for (int x : c) missing += !inT[(size_t)x];
            if (count + missing <= K) {
                for (int x : c)
                    if (!inT[(size_t)x]) inT[(size_t)x] = 1, count++;
                continue;
            }
            if (count >= K) break;
            // a run c_a, c_a+1, ... from a member already in the tile (else c_0)
            const int m = (int)c.size();
            int a = 0;
            for (int i = 0; i < m; i++)
                if (inT[(size_t)c[(size_t)i]]) {
                    a = i;
                    break;
                }
            for (int i = 0; i < m && count < K; i++) {
                const int x = c[(size_t)((a + i) % m)];
                if (!inT[(size_t)x]) inT[(size_t)x] = 1, count++;
            }
        }
        for (int p = 0; p < L && count < K; p++)
            if (!inT[(size_t)p]) inT[(size_t)p] = 1, count++;
        // within the tile: every qubit whose destination is in the tile goes
        // there; the others take the positions nobody in the tile moves to
        int pi[64];
        std::vector<char> taken((size_t)L, 0);
        std::vector<int> waiting;
        for (int p = 0; p < L; p++) {
            if (!inT[(size_t)p]) continue;
            if (inT[(size_t)dest[p]]) {
                pi[p] = dest[p];
                taken[(size_t)dest[p]] = 1;
            } else {
                waiting.push_back(p);
            }
        }
        size_t w = 0;
        for (int p = 0; p < L; p++)
            if (inT[(size_t)p] && !taken[(size_t)p]) pi[waiting[w++]] = p;
        TilePass ps;
        ps.k = K;
        int n = 0;
        for (int p = 0; p < L; p++)
            if (inT[(size_t)p]) {
                ps.pos[n] = p;
                ps.stPos[n++] = pi[p];
                ps.qmask |= 1ull << p;
            }
        ps.opBegin = ps.opEnd = (int)prog.ops.size();
        if (!waveLowers(ps, prog.ops.data())) return false;
        prog.passes.push_back(ps);
        int nd[64];
        for (int p = 0; p < L; p++) nd[p] = dest[p];
        for (int p = 0; p < L; p++)
            if (inT[(size_t)p]) nd[pi[p]] = dest[p];
        for (int p = 0; p < L; p++) dest[p] = nd[p];
        for (int x = 0; x < L; x++) prog.perm[(size_t)x] = inT[(size_t)prog.perm[(size_t)x]] ? pi[prog.perm[(size_t)x]] : prog.perm[(size_t)x];
    }
    return false;
}

int waveTransposeCost(int laneBit) { return laneBit >= kWaveLanes ? 3 : laneBit >= 4 ? 1 : laneBit >= 2 ? 2 : 4; }

bool waveChannel(const real* m) {
    for (int e = 0; e < 16; e++) {
        if (m[2 * e + 1] != 0) return false;
        const int r = e >> 2, c = e & 3;
        const bool allowed = (r == c) || (r == 0 && c == 3) || (r == 3 && c == 0);
        if (!allowed && m[2 * e] != 0) return false;
    }
    return m[2 * 5] == m[2 * 10];
}

bool planWavePass(const TilePass& ps, const TileOp* ops, int nOps, WaveProgram& out, int* endLanes) {
    if (ps.k != kWaveBits) return false;
    for (int i = 0; i < kWaveVecBits + 3; i++)
        if (ps.pos[i] != i) return false;
    std::vector<M2Class> cls(nOps, M2Class::Diag);
    std::vector<char> chan(nOps, 0);   // one-qubit density channel (CH1 / CHD) on t[0], t[1]
    for (int i = 0; i < nOps; i++) {
        const OpKind k = (OpKind)ops[i].kind;
        if (k == OpKind::Mat2)
            cls[i] = classify(ops[i].m);
        else if (k == OpKind::Mat4 && waveChannel(ops[i].m) && ops[i].ctrlIn == 0 && ops[i].ctrlOut == 0)
            chan[i] = 1;
        else if (k != OpKind::Diag)
            return false;
    }
    // Conditional exchange frame (QUEST_WAVE_CFRAME=0 disables; needs the
    // exchange frame below): a CNOT with one control inside the tile and no
    // control outside is not executed either -- its target is marked flipped
    // where its control is 1 (see Cnd below), so it needs no register slot
    static const bool xframeEnv = !getenv("QUEST_WAVE_XFRAME") || atoi(getenv("QUEST_WAVE_XFRAME")) != 0;
    static const bool cframeEnv = xframeEnv && (!getenv("QUEST_WAVE_CFRAME") || atoi(getenv("QUEST_WAVE_CFRAME")) != 0);
    // a planner strategy may switch it off for the flush it plans (t_waveCframe)
    const bool cframeOn = t_waveCframe >= 0 ? (xframeEnv && t_waveCframe != 0) : cframeEnv;
    auto deferCnot = [&](int i) {
        const TileOp& op = ops[i];
        return cframeOn && (OpKind)op.kind == OpKind::Mat2 && cls[i] == M2Class::Swap && op.ctrlOut == 0 &&
               __builtin_popcount(op.ctrlIn) == 1 && op.t[0] >= kWaveVecBits;
    };
    // ops that need their target(s) in a register slot
    auto needsSlot = [&](int i) { return (OpKind)ops[i].kind == OpKind::Mat2 && cls[i] != M2Class::Diag; };
    auto slotTargets = [&](int i, int* t) {
        if (chan[i]) {
            t[0] = ops[i].t[0];
            t[1] = ops[i].t[1];
            return 2;
        }
        t[0] = ops[i].t[0];
        return needsSlot(i) && !deferCnot(i) ? 1 : 0;
    };
    // next[i][b]: first op >= i needing tile bit b in a slot
    std::vector<int> nextNeed((size_t)(nOps + 1) * kWaveBits, kInf);
    for (int i = nOps - 1; i >= 0; i--) {
        for (int b = 0; b < kWaveBits; b++) nextNeed[(size_t)i * kWaveBits + b] = nextNeed[(size_t)(i + 1) * kWaveBits + b];
        int t[2];
        for (int k = 0, n = slotTargets(i, t); k < n; k++) nextNeed[(size_t)i * kWaveBits + t[k]] = i;
    }
    auto nextUse = [&](int i, int b) { return nextNeed[(size_t)i * kWaveBits + b]; };
    // remaining[i][b]: ops >= i needing tile bit b in a slot
    std::vector<int> remaining((size_t)(nOps + 1) * kWaveBits, 0);
    for (int i = nOps - 1; i >= 0; i--) {
        for (int b = 0; b < kWaveBits; b++)
            remaining[(size_t)i * kWaveBits + b] = remaining[(size_t)(i + 1) * kWaveBits + b];
        int t[2];
        for (int k = 0, n = slotTargets(i, t); k < n; k++) remaining[(size_t)i * kWaveBits + t[k]]++;
    }
    // a gate on lane bit 0-2 runs there directly (DPP partner fetch: about one
    // transposition of work, twice a slot gate) unless the bit has enough slot
    // uses left in the pass to pay for a transposition in -- and, for tile
    // bits 1-3, the one back before the store; QUEST_WAVE_LANE_OPS=0 disables
    static const bool laneOps = !getenv("QUEST_WAVE_LANE_OPS") || atoi(getenv("QUEST_WAVE_LANE_OPS")) != 0;
    auto laneOpsMax = [&](int b) { return !laneOps ? 0 : (b >= 1 && b <= 3) ? 4 : 2; };

    WavePass wp;
    for (int i = 0; i < kWaveBits; i++) {
        wp.pos[i] = ps.pos[i];
        wp.stPos[i] = ps.stPos[i];
    }
    // the vector bits never move (no slot-0 transpositions)
    for (int v = 0; v < kWaveVecBits; v++)
        if (ps.stPos[v] != v) return false;
    // load layout: the vector bits (fp64: tile bit 0, fp32: bits 0-1) in
    // slots 0.., the next three on lanes 0-2 (8 lanes x 16 bytes = one 128-byte
    // line); of the higher tile bits those needed in a slot earliest take the
    // other slots, the rest lanes 3-5 and the wave bits
    constexpr int VB = kWaveVecBits;
    Layout lay;
    for (int v = 0; v < VB; v++) lay.put(v, v);
    for (int l = 0; l < 3; l++) lay.put(VB + l, kWaveSlots + l);
    std::vector<int> high;
    for (int b = VB + 3; b < kWaveBits; b++) high.push_back(b);
    // bits above kWaveLanePosMax may not sit on real lanes (32-bit per-lane
    // offsets); wave bits take any position (per-wave uniform offsets)
    auto farPos = [&](int b) { return ps.pos[b] > kWaveLanePosMax; };
    int nFar = 0;
    for (int b : high) nFar += farPos(b);
    if (nFar > (kWaveSlots - VB) + kWaveWBits) return false;
    // slots: the bits needed in a slot earliest; then real lanes 3-5 for the
    // next near bits, wave bits for the rest (LDS transpositions are dearest)
    std::stable_sort(high.begin(), high.end(), [&](int x, int y) { return nextUse(0, x) < nextUse(0, y); });
    std::vector<int> slots(high.begin(), high.begin() + (kWaveSlots - VB));
    std::vector<int> rest(high.begin() + (kWaveSlots - VB), high.end());
    // real lanes 3-5: three near bits, from the rest first (in need order);
    // if the rest has fewer, near bits leave the slots for them and far bits
    // of the rest take their slot places
    std::vector<int> lanes, waves;
    // lanes 3-5 take the lowest positions of the rest: a 16-byte load / store
    // of 64 lanes then spans the fewest DRAM pages and translations
    // (lane order 0: in need order instead; 2: the wave bits -- LDS
    // transpositions -- take the latest-needed of the rest first, lanes 3-5
    // the others by position)
    const int laneOrder = waveLaneOrder();
    if (laneOrder == 2) {
        std::vector<int> byNeed(rest);  // need order already; latest last
        std::vector<int> wv;
        for (int x = (int)byNeed.size() - 1; x >= 0 && (int)wv.size() < kWaveWBits; x--) wv.push_back(byNeed[x]);
        std::vector<int> ln;
        for (int b : rest)
            if (std::find(wv.begin(), wv.end(), b) == wv.end()) ln.push_back(b);
        std::sort(ln.begin(), ln.end());
        rest = ln;
        rest.insert(rest.end(), wv.begin(), wv.end());
        // far bits among the lane candidates still go to waves below
    } else if (laneOrder == 1) {
        std::sort(rest.begin(), rest.end());
    }
    for (int b : rest)
        if (!farPos(b) && (int)lanes.size() < kWaveLanes - 3) lanes.push_back(b);
        else waves.push_back(b);
    for (int k = (int)slots.size() - 1; k >= 0 && (int)lanes.size() < kWaveLanes - 3; k--) {
        if (farPos(slots[k])) continue;
        int far = -1;
        for (int x = 0; x < (int)waves.size() && far < 0; x++)
            if (farPos(waves[x])) far = x;
        if (far < 0) return false;
        lanes.push_back(slots[k]);
        slots[k] = waves[far];
        waves.erase(waves.begin() + far);
    }
    if ((int)lanes.size() != kWaveLanes - 3 || (int)waves.size() != kWaveWBits) return false;
    for (int s = VB; s < kWaveSlots; s++) lay.put(slots[s - VB], s);
    for (int l = 3; l < kWaveLanes; l++) lay.put(lanes[l - 3], kWaveSlots + l);
    for (int l = kWaveLanes; l < kWaveLaneBits; l++) lay.put(waves[l - kWaveLanes], kWaveSlots + l);
    for (int s = 0; s < kWaveSlots; s++) wp.ldSlot[s] = lay.slotBit[s];
    for (int l = 0; l < kWaveLaneBits; l++) wp.ldLane[l] = lay.laneBit[l];

    wp.opBegin = (int)out.ops.size();
    // Exchange frame: an uncontrolled X on a tile bit (not a vector bit) is
    // not executed; the bit is marked flipped (F) -- its amplitude pairs sit
    // in each other's places, wherever the bit moves (slots, lanes, waves).
    // Later gates on a flipped bit take X M X (same handler, conjugated
    // matrix); controls on flipped bits test for 0 (register masks computed by
    // the host, lane masks through the record's aux word, wave bits swapped
    // between cLane and cLaneZero); phases on a flipped register bit split in
    // two (p on the mask without it, 1/p on the whole mask); channels and
    // unnormalised Hadamards get the exchange first.  What is left at the end
    // of the pass is folded into the store addresses (WavePass::stFlip*).
    // QUEST_WAVE_XFRAME=0 executes every X.
    static const bool frameOn = !getenv("QUEST_WAVE_XFRAME") || atoi(getenv("QUEST_WAVE_XFRAME")) != 0;
    unsigned F = 0;
    Scale sig;
    auto slotFlips = [&]() {
        unsigned m = 0;
        for (int s = 0; s < kWaveSlots; s++) m |= ((F >> lay.slotBit[s]) & 1u) << s;
        return m;
    };
    auto laneFlips = [&]() {   // real lanes and wave bits, as cLane bits
        unsigned m = 0;
        for (int l = 0; l < kWaveLaneBits; l++) m |= ((F >> lay.laneBit[l]) & 1u) << l;
        return m;
    };
    // conditional flips (deferred CNOTs, see below); declared here because a
    // physical X on a condition bit toggles its dependents' flips
    unsigned Cnd[kWaveBits] = {0};
    auto materialize = [&](unsigned slots) {
        for (unsigned m = slots & slotFlips(); m; m &= m - 1) {
            WaveOp x = blank((int)WKind::SWAP);
            x.a = __builtin_ctz(m);
            out.ops.push_back(x);
            const int b = lay.slotBit[x.a];
            F &= ~(1u << b);
            // x_t = p_t ^ F_t ^ p_b for t conditioned on b: p_b just flipped
            for (int t = 0; t < kWaveBits; t++)
                if ((Cnd[t] >> b) & 1u) F ^= 1u << t;
        }
    };
    // the unit phase p of a phase op (DIAG: its complex factor)
    auto phaseOf = [](const WaveOp& w, double& pr, double& pi) {
        const double t = w.m[0], sn = w.m[1], c = 1 - t * sn;
        switch ((WKind)w.kind) {
            case WKind::DROT: pr = c, pi = sn; break;
            case WKind::DROTN: pr = -c, pi = -sn; break;
            case WKind::DNEG: pr = -1, pi = 0; break;
            case WKind::DMULI: pr = 0, pi = 1; break;
            case WKind::DMULNI: pr = 0, pi = -1; break;
            default: pr = w.m[0], pi = w.m[1]; break;   // DIAG
        }
    };
    auto invertPhase = [](WaveOp& w) {   // p -> 1/p
        switch ((WKind)w.kind) {
            case WKind::DROT:
            case WKind::DROTN:
                w.m[0] = -w.m[0];
                w.m[1] = -w.m[1];
                break;
            case WKind::DMULI: w.kind = (int)WKind::DMULNI; break;
            case WKind::DMULNI: w.kind = (int)WKind::DMULI; break;
            case WKind::DNEG: break;
            default: {   // DIAG
                const double r = w.m[0], i = w.m[1], n = r * r + i * i;
                w.m[0] = (real)(r / n);
                w.m[1] = (real)(-i / n);
            }
        }
    };
    std::function<void(WaveOp)> emit = [&](WaveOp w) {
        const bool free = w.cReg == 0 && w.cLane == 0 && w.cLaneZero == 0 && w.ctrlOut == 0 && w.ctrlOutZero == 0;
        if (frameOn && free && w.kind == (int)WKind::SWAP && w.a >= VB) {
            F ^= 1u << lay.slotBit[w.a];
            return;
        }
        if (frameOn && free && w.kind == (int)WKind::LSWAP) {
            F ^= 1u << lay.laneBit[w.a];
            return;
        }
        // Y = i X Z (-Y = -i X Z): a sign flip on the bit's 1 half, the X into
        // the frame, the i to the pass's owed factor
        const bool laneY = w.kind == (int)WKind::LANTI && w.m[0] == 0 && w.m[2] == 0 && std::fabs(w.m[1]) == 1 &&
                           w.m[3] == -w.m[1];
        if (frameOn && free && (((w.kind == (int)WKind::YSW || w.kind == (int)WKind::YSWC) && w.a >= VB) || laneY)) {
            // YSW is Y, YSWC -Y; a lane Y has m01 = -i (m[1] = -1)
            const bool minus = laneY ? w.m[1] > 0 : w.kind == (int)WKind::YSWC;
            WaveOp z = blank((int)WKind::DNEG);
            if (laneY)
                z.cLane = 1u << w.a;
            else
                z.cReg = 1u << w.a;
            emit(z);
            WaveOp x = blank(laneY ? (int)WKind::LSWAP : (int)WKind::SWAP);
            x.a = w.a;
            emit(x);
            sig.mul(0, minus ? -1 : 1);
            return;
        }
        if (!F) {
            out.ops.push_back(w);
            return;
        }
        const unsigned fs = slotFlips(), fl = laneFlips();
        const bool isPhase = w.kind == (int)WKind::DIAG || (w.kind >= (int)WKind::DROT && w.kind <= (int)WKind::DROTN);
        if (isPhase) {
            const unsigned T = w.cReg & fs;
            if (T && (__builtin_popcount(T) > 1 || (w.kind == (int)WKind::DIAG && w.m[0] == 0 && w.m[1] == 0)))
                materialize(T);
            else if (T) {
                WaveOp rest = w;
                rest.cReg &= ~T;
                if (rest.cReg == 0 && rest.cLane == 0 && rest.cLaneZero == 0 && rest.ctrlOut == 0 &&
                    rest.ctrlOutZero == 0) {
                    double pr, pi;
                    phaseOf(rest, pr, pi);
                    sig.mul(pr, pi);   // a global factor: absorbed by the pass
                } else {
                    rest.fLane = fl & 63u;
                    const unsigned wv = (fl >> kWaveLanes) << kWaveLanes;
                    const unsigned one = rest.cLane & wv, zero = rest.cLaneZero & wv;
                    rest.cLane = (rest.cLane & ~wv) | zero;
                    rest.cLaneZero = (rest.cLaneZero & ~wv) | one;
                    out.ops.push_back(rest);
                }
                invertPhase(w);   // 1/p on the whole mask (physical bits, no flips)
            }
        }
        const bool slotFlipped = inSlot(w.a) && ((fs >> w.a) & 1);
        auto swapPairs = [&](int x, int y, int n) {
            for (int k = 0; k < n; k++) std::swap(w.m[x + k], w.m[y + k]);
        };
        switch ((WKind)w.kind) {
            case WKind::TR: break;   // the flip travels with the tile bit
            case WKind::CH1:
            case WKind::CHD: materialize((1u << w.a) | (1u << w.b)); break;
            case WKind::HADD:
                // on a flipped slot: H gives (a0 + a1, -(a0 - a1)) in (low, high), the
                // logical order with the high half negated: clear the flip, then Z
                if (slotFlipped) {
                    F &= ~(1u << lay.slotBit[w.a]);
                    out.ops.push_back(w);
                    WaveOp z = blank((int)WKind::DNEG);   // the slot is unflipped now: no frame work
                    z.cReg = 1u << w.a;
                    out.ops.push_back(z);
                    return;
                }
                break;
            case WKind::M2:   // X M X: m00 <-> m11, m01 <-> m10 (complex)
                if (slotFlipped) {
                    swapPairs(0, 6, 2);
                    swapPairs(2, 4, 2);
                }
                break;
            case WKind::M2R:
            case WKind::M2RI:   // (m00, m01, m10, m11) -> (m11, m10, m01, m00)
                if (slotFlipped) {
                    std::swap(w.m[0], w.m[3]);
                    std::swap(w.m[1], w.m[2]);
                }
                break;
            case WKind::LM2R:
            case WKind::LM2RI:
                if ((fl >> w.a) & 1) {
                    std::swap(w.m[0], w.m[3]);
                    std::swap(w.m[1], w.m[2]);
                }
                break;
            case WKind::ANTI:   // m01 <-> m10
            case WKind::D2S:    // d0 <-> d1
                if (slotFlipped) swapPairs(0, 2, 2);
                break;
            case WKind::LANTI:
            case WKind::D2L:
                if ((fl >> w.a) & 1) swapPairs(0, 2, 2);
                break;
            case WKind::ROTY:   // X Ry(phi) X = Ry(-phi)
                if (slotFlipped) {
                    w.m[0] = -w.m[0];
                    w.m[1] = -w.m[1];
                }
                break;
            case WKind::YSW:
            case WKind::YSWC:   // X Y X = -Y
                if (slotFlipped) w.kind = w.kind == (int)WKind::YSW ? (int)WKind::YSWC : (int)WKind::YSW;
                break;
            default: break;   // ROTX, SWAP, LSWAP commute with X; phases handled above
        }
        // controls on flipped bits
        if (!isPhase) w.fReg = slotFlips() & w.cReg;
        w.fLane = laneFlips() & w.cLane & 63u;
        const unsigned wv = ((laneFlips() >> kWaveLanes) << kWaveLanes);
        const unsigned one = w.cLane & wv, zero = w.cLaneZero & wv;
        w.cLane = (w.cLane & ~wv) | zero;
        w.cLaneZero = (w.cLaneZero & ~wv) | one;
        out.ops.push_back(w);
    };
    auto transpose = [&](int s, int l) {
        WaveOp w = blank((int)WKind::TR);
        w.a = s;
        w.b = l;
        emit(w);
        const int bs = lay.slotBit[s], bl = lay.laneBit[l];
        lay.put(bs, kWaveSlots + l);
        lay.put(bl, s);
    };

    // Factors the pass owes its amplitudes (unnormalised Hadamards, rotations
    // run as -R, global phases split off diagonal gates) are absorbed at the
    // end by one uncontrolled op whose matrix can take them at no cost (or a
    // final phase op).  QUEST_WAVE_CHEAP=0 keeps the round-1 kinds only.
    static const bool cheap = !getenv("QUEST_WAVE_CHEAP") || atoi(getenv("QUEST_WAVE_CHEAP")) != 0;
    auto uncontrolled = [&](const TileOp& op) { return op.ctrlIn == 0 && op.ctrlOut == 0; };
    // an uncontrolled general 2x2 absorbs any factor: then every uncontrolled
    // diagonal gate can drop its global phase; otherwise the first one stays
    // a D2S / D2L (complex absorber) and the later ones are split
    bool haveComplexAbsorber = false;
    for (int i = 0; i < nOps && cheap; i++)
        if (needsSlot(i) && cls[i] == M2Class::General && uncontrolled(ops[i])) haveComplexAbsorber = true;
    // phase p on the amplitudes whose tile bits in `mask` are all 1
    auto emitPhase = [&](unsigned mask, const TileOp& op, double pr, double pi) -> bool {
        int kind;
        real pm[2] = {0, 0};
        if (!cheap || !phaseKind(pr, pi, &kind, pm)) return false;
        if (kind < 0) return true;   // identity
        WaveOp w = blank(kind);
        masks(lay, mask, w.cReg, w.cLane);
        w.ctrlOut = op.ctrlOut;
        w.m[0] = pm[0];
        w.m[1] = pm[1];
        emit(w);
        return true;
    };
    // bring tile bit b into a register slot (not the slot `keep`), evicting
    // the slot whose next use lies furthest (slot 0 keeps tile bit 0)
    auto toSlot = [&](int i, int b, int keep) {
        if (inSlot(lay.where[b])) return;
        const int l = laneOf(lay.where[b]);
        int victim = -1, far = -1;
        for (int s = VB; s < kWaveSlots; s++) {
            if (s == keep) continue;
            const int nu = nextUse(i, lay.slotBit[s]);
            if (nu > far) {
                far = nu;
                victim = s;
            }
        }
        transpose(victim, l);
    };
    // Conditional flips: tile bit t additionally flipped where the tile bits
    // in Cnd[t] have odd parity.  With p the physical coordinates of an
    // amplitude (the bits where each tile bit currently lives), its logical
    // tile index x has x_t = p_t ^ F_t ^ parity(p & Cnd[t]).  Invariant: a
    // condition bit has no conditions itself, so the pairs of a gate on a
    // target t are still the pairs along p_t (t is never a condition) and the
    // gate only has to be oriented: X M X where the parity is odd.  Deferred
    // CNOTs are executed (SWAP with the condition as its control) only when an
    // op needs it; at the end of the pass the flips whose target and
    // conditions are in one domain (slots, real lanes, wave bits) are folded
    // into the store maps (WavePass::stCondSlot / stCondLane).
    auto deps = [&](int c) {
        unsigned m = 0;
        for (int u = 0; u < kWaveBits; u++) m |= ((Cnd[u] >> c) & 1u) << u;
        return m;
    };
    // ops in physical terms (no frame adjustment): a CNOT c -> t, a Z, a CZ
    int cnotReason = 0;
    auto rawCnot = [&](int i, int c, int t) {
        WaveOp x;
        const int wt = lay.where[t];
        if (cnotStatsOn() && !t_planQuiet) {
            auto dom = [&](int w) { return inSlot(w) ? 0 : laneOf(w) < kWaveLanes ? 1 : 2; };
            g_cnotStats[cnotReason][dom(lay.where[c])][dom(wt)]++;
        }
        if (!inSlot(wt) && laneOf(wt) < kWaveLaneOps) {
            x = blank((int)WKind::LSWAP);
            x.a = laneOf(wt);
        } else {
            if (!inSlot(wt)) toSlot(i, t, inSlot(lay.where[c]) ? lay.where[c] : -1);
            x = blank((int)WKind::SWAP);
            x.a = lay.where[t];
        }
        masks(lay, 1u << c, x.cReg, x.cLane);
        out.ops.push_back(x);
        Cnd[t] &= ~(1u << c);
    };
    auto rawZ = [&](unsigned tileMask) {
        WaveOp z = blank((int)WKind::DNEG);
        masks(lay, tileMask, z.cReg, z.cLane);
        out.ops.push_back(z);
    };
    auto execConds = [&](int i, int t) {   // execute t's deferred CNOTs
        for (unsigned m = Cnd[t]; m; m &= m - 1) rawCnot(i, __builtin_ctz(m), t);
    };
    auto clean = [&](int i, int c) {          // execute the deferred CNOTs controlled by c
        for (unsigned m = deps(c); m; m &= m - 1) rawCnot(i, c, __builtin_ctz(m));
    };
    auto laneOpPath = [&](int i, int t) {
        return !inSlot(lay.where[t]) && laneOf(lay.where[t]) < kWaveLaneOps && cls[i] != M2Class::General &&
               remaining[(size_t)i * kWaveBits + t] <= laneOpsMax(t);
    };
    // Resolve the conditional frame before op i: 1 = the op was applied here
    // (a deferred CNOT, a Z or Y on a conditioned bit); postT / postCZ / postClear:
    // CZs to emit after the op (orientation by Z M Z, or the Z an H leaves)
    int postT = -1;
    unsigned postCZ = 0;
    bool postClear = false;
    auto frameBefore = [&](int i) -> int {
        const TileOp& op = ops[i];
        postT = -1;
        postCZ = 0;
        postClear = false;
        if (deferCnot(i)) {
            const int t = op.t[0], k = __builtin_ctz(op.ctrlIn);
            cnotReason = 0;
            if (Cnd[k]) execConds(i, k);   // the control must be a plain physical bit
            cnotReason = 1;
            if (deps(t)) clean(i, t);       // the target must not condition other bits
            Cnd[t] ^= 1u << k;
            F ^= ((F >> k) & 1u) << t;     // x_t ^= x_k = p_k ^ F_k
            return 1;
        }
        if (chan[i]) {
            cnotReason = 2;
            for (int b : {op.t[0], op.t[1]}) {
                execConds(i, b);
                clean(i, b);
            }
            return 0;
        }
        cnotReason = 3;
        for (unsigned m = op.ctrlIn; m; m &= m - 1)
            if (Cnd[__builtin_ctz(m)]) execConds(i, __builtin_ctz(m));
        const real* m = op.m;
        const bool isMat2 = (OpKind)op.kind == OpKind::Mat2;
        if (!isMat2 || cls[i] == M2Class::Diag) {
            const unsigned mask = op.ctrlIn | (isMat2 ? 1u << op.t[0] : 0u);
            // Z on one bit: (-1)^x_t = (-1)^p_t (-1)^F_t prod_c (-1)^p_c
            int zt = -1;
            if (op.ctrlOut == 0 && !isMat2 && __builtin_popcount(mask) == 1 && m[0] == -1 && m[1] == 0)
                zt = __builtin_ctz(mask);
            if (op.ctrlOut == 0 && isMat2 && op.ctrlIn == 0 && m[0] == 1 && m[1] == 0 && m[6] == -1 && m[7] == 0)
                zt = op.t[0];
            if (zt >= 0 && Cnd[zt]) {
                rawZ(1u << zt);
                for (unsigned c = Cnd[zt]; c; c &= c - 1) rawZ(1u << __builtin_ctz(c));
                if ((F >> zt) & 1u) sig.mul(-1, 0);
                return 1;
            }
            cnotReason = 4;
            for (unsigned b = mask; b; b &= b - 1)
                if (Cnd[__builtin_ctz(b)]) execConds(i, __builtin_ctz(b));
            return 0;
        }
        const int t = op.t[0];
        const bool unc = op.ctrlIn == 0 && op.ctrlOut == 0;
        const bool isY = cls[i] == M2Class::Anti && m[2] == 0 && m[4] == 0 && std::fabs(m[3]) == 1 && m[5] == -m[3];
        // an uncontrolled X / Y on a condition only toggles F_t (and a Z on p_t)
        cnotReason = 5;
        if (deps(t) && !(unc && t >= VB && (cls[i] == M2Class::Swap || isY))) clean(i, t);
        if (!Cnd[t] || cls[i] == M2Class::Swap) return 0;   // X commutes with the orientation
        const bool commX = near(m[0], m[6]) && near(m[1], m[7]) && near(m[2], m[4]) && near(m[3], m[5]);
        const bool zmz = near(m[0], m[6]) && near(m[1], m[7]) && near(m[2], -m[4]) && near(m[3], -m[5]);
        const bool isH = cheap && unc && cls[i] == M2Class::Real && near(m[0], m[2]) && near(m[0], m[4]) &&
                         near(m[0], -m[6]);
        if (commX) return 0;
        if (unc && isY) {   // Y = i X Z (-Y = -i X Z): Z on x_t, then X into the frame
            rawZ(1u << t);
            for (unsigned c = Cnd[t]; c; c &= c - 1) rawZ(1u << __builtin_ctz(c));
            if ((F >> t) & 1u) sig.mul(-1, 0);
            F ^= 1u << t;
            sig.mul(0, m[3] < 0 ? 1 : -1);
            return 1;
        }
        if (zmz) {   // X M X = Z M Z: CZ(c, t) for every condition before and after
            for (unsigned c = Cnd[t]; c; c &= c - 1) rawZ((1u << __builtin_ctz(c)) | (1u << t));
            postT = t;
            postCZ = Cnd[t];
            return 0;
        }
        if (isH && !laneOpPath(i, t)) {   // H X^s = Z^s H: the CZs after clear the conditions
            postT = t;
            postCZ = Cnd[t];
            postClear = true;
            return 0;
        }
        cnotReason = 6;
        execConds(i, t);
        return 0;
    };
    auto frameAfter = [&]() {
        if (postT < 0) return;
        for (unsigned c = postCZ; c; c &= c - 1) rawZ((1u << __builtin_ctz(c)) | (1u << postT));
        if (postClear) Cnd[postT] = 0;
        postT = -1;
    };
    static const bool foldOn = !getenv("QUEST_WAVE_FOLD_DIAG") || atoi(getenv("QUEST_WAVE_FOLD_DIAG")) != 0;
    // a real diagonal factor that is not a unit phase (those have cheap kinds)
    auto foldable = [&](int x) {
        const real* m = ops[x].m;
        return foldOn && m[1] == 0 && m[0] != 0 && std::fabs((double)m[0]) != 1 && !(ops[x].ctrlOut & kRankTagMask);
    };
    for (int i = 0; i < nOps; i++) {
        if (cframeOn) {
            frameAfter();
            // a run of foldable diagonal ops resolves the frame itself (below)
            const bool run = (OpKind)ops[i].kind == OpKind::Diag && foldable(i) && i + 1 < nOps &&
                             (OpKind)ops[i + 1].kind == OpKind::Diag && foldable(i + 1);
            if (!run && frameBefore(i)) continue;
        }
        const TileOp& op = ops[i];
        if (chan[i]) {
            const int r = op.t[0], c = op.t[1];
            toSlot(i, r, inSlot(lay.where[c]) ? lay.where[c] : -1);
            toSlot(i, c, lay.where[r]);
            const real* m = op.m;
            const bool dephaseOnly = m[0] == 1 && m[2 * 3] == 0 && m[2 * 12] == 0 && m[2 * 15] == 1;
            WaveOp w = blank(dephaseOnly ? (int)WKind::CHD : (int)WKind::CH1);
            w.a = lay.where[r];
            w.b = lay.where[c];
            w.m[0] = m[0];
            w.m[1] = m[2 * 3];
            w.m[2] = m[2 * 12];
            w.m[3] = m[2 * 15];
            w.m[4] = m[2 * 5];
            emit(w);
            continue;
        }
        if ((OpKind)op.kind == OpKind::Diag && foldable(i)) {
            // A run of real diagonal factors (density dephasing lowered to
            // diagonal ops: 15 per two-qubit channel, most of their masks
            // partly or wholly outside the tile): group the run's ops by their
            // in-tile mask; per group the out-of-tile bits U of its ops take
            // 2^|U| values, so ONE op per value carries the product of the
            // group's factors for it (ctrlOut = the 1 bits, ctrlOutZero = the
            // 0 bits) -- each tile executes at most one op per group instead of
            // every op whose outside bits it matches.  QUEST_WAVE_FOLD_DIAG=0 off.
            int j = i;
            while (j < nOps && (OpKind)ops[j].kind == OpKind::Diag && foldable(j)) j++;
            if (j - i >= 2) {
                for (int x = i; x < j; x++)
                    for (unsigned b = ops[x].ctrlIn; b; b &= b - 1)
                        if (cframeOn && Cnd[__builtin_ctz(b)]) {
                            cnotReason = 7;
                            execConds(x, __builtin_ctz(b));
                        }
                std::vector<unsigned> masksIn;
                for (int x = i; x < j; x++)
                    if (std::find(masksIn.begin(), masksIn.end(), ops[x].ctrlIn) == masksIn.end())
                        masksIn.push_back(ops[x].ctrlIn);
                for (unsigned mi : masksIn) {
                    u64 U = 0;
                    for (int x = i; x < j; x++)
                        if (ops[x].ctrlIn == mi) U |= ops[x].ctrlOut;
                    const int nu = __builtin_popcountll(U);
                    if (nu > 3) {   // too many combinations: the ops as they are
                        for (int x = i; x < j; x++) {
                            if (ops[x].ctrlIn != mi) continue;
                            WaveOp w = blank((int)WKind::DIAG);
                            masks(lay, mi, w.cReg, w.cLane);
                            w.ctrlOut = ops[x].ctrlOut;
                            w.m[0] = ops[x].m[0];
                            emit(w);
                        }
                        continue;
                    }
                    int ub[3], k = 0;
                    for (u64 u = U; u; u &= u - 1) ub[k++] = __builtin_ctzll(u);
                    for (int v = 0; v < (1 << nu); v++) {
                        u64 one = 0;
                        for (int q = 0; q < nu; q++)
                            if ((v >> q) & 1) one |= 1ull << ub[q];
                        double f = 1;
                        for (int x = i; x < j; x++)
                            if (ops[x].ctrlIn == mi && (ops[x].ctrlOut & ~one) == 0) f *= ops[x].m[0];
                        if (f == 1) continue;
                        WaveOp w = blank((int)WKind::DIAG);
                        masks(lay, mi, w.cReg, w.cLane);
                        w.ctrlOut = one;
                        w.ctrlOutZero = U & ~one;
                        w.m[0] = (real)f;
                        emit(w);
                    }
                }
                i = j - 1;
                continue;
            }
        }
        if ((OpKind)op.kind == OpKind::Diag) {
            if (emitPhase(op.ctrlIn, op, op.m[0], op.m[1])) continue;
            WaveOp w = blank((int)WKind::DIAG);
            masks(lay, op.ctrlIn, w.cReg, w.cLane);
            w.ctrlOut = op.ctrlOut;
            w.m[0] = op.m[0];
            w.m[1] = op.m[1];
            emit(w);
            continue;
        }
        const int t = op.t[0];
        const real* m = op.m;
        if (cls[i] == M2Class::Diag) {
            WaveOp w;
            if (m[0] == 1 && m[1] == 0) {  // phase on |1>: diagonal op on ctrl + target
                if (emitPhase(op.ctrlIn | (1u << t), op, m[6], m[7])) continue;
                w = blank((int)WKind::DIAG);
                masks(lay, op.ctrlIn | (1u << t), w.cReg, w.cLane);
                w.m[0] = m[6];
                w.m[1] = m[7];
            } else if (cheap && uncontrolled(op) && haveComplexAbsorber && unitCircle(m[0], m[1]) &&
                       unitCircle(m[6], m[7])) {
                // diag(d0, d1) = d0 diag(1, d1 / d0): the pass owes d0
                sig.mul(m[0], m[1]);
                const double qr = m[6] * m[0] + m[7] * m[1], qi = m[7] * m[0] - m[6] * m[1];
                if (emitPhase(1u << t, op, qr, qi)) continue;
                sig.mul(m[0], -m[1]);  // (not reached: the quotient is unit modulus)
                w = blank((int)WKind::D2S);
            } else if (!inSlot(lay.where[t]) && laneOf(lay.where[t]) >= kWaveLanes) {
                // target on a wave bit: d1 on the waves with the bit set, d0
                // on the others (two wave-uniform phase ops)
                const unsigned wb = 1u << laneOf(lay.where[t]);
                for (int v = 0; v < 2; v++) {
                    WaveOp d = blank((int)WKind::DIAG);
                    masks(lay, op.ctrlIn, d.cReg, d.cLane);
                    if (v) d.cLane |= wb; else d.cLaneZero |= wb;
                    d.m[0] = m[v ? 6 : 0];
                    d.m[1] = m[v ? 7 : 1];
                    d.ctrlOut = op.ctrlOut;
                    emit(d);
                }
                continue;
            } else {
                const int wt = lay.where[t];
                w = blank(inSlot(wt) ? (int)WKind::D2S : (int)WKind::D2L);
                w.a = inSlot(wt) ? wt : laneOf(wt);
                masks(lay, op.ctrlIn, w.cReg, w.cLane);
                w.m[0] = m[0];
                w.m[1] = m[1];
                w.m[2] = m[6];
                w.m[3] = m[7];
                if (uncontrolled(op)) haveComplexAbsorber = true;  // later diagonals may split
            }
            w.ctrlOut = op.ctrlOut;
            emit(w);
            continue;
        }
        if (!inSlot(lay.where[t]) && laneOf(lay.where[t]) < kWaveLaneOps && cls[i] != M2Class::General &&
            remaining[(size_t)i * kWaveBits + t] <= laneOpsMax(t)) {
            WaveOp w;
            switch (cls[i]) {
                case M2Class::Swap: w = blank((int)WKind::LSWAP); break;
                case M2Class::Anti:
                    w = blank((int)WKind::LANTI);
                    w.m[0] = m[2];
                    w.m[1] = m[3];
                    w.m[2] = m[4];
                    w.m[3] = m[5];
                    break;
                case M2Class::Real:
                    w = blank((int)WKind::LM2R);
                    w.m[0] = m[0];
                    w.m[1] = m[2];
                    w.m[2] = m[4];
                    w.m[3] = m[6];
                    break;
                default:
                    w = blank((int)WKind::LM2RI);
                    w.m[0] = m[0];
                    w.m[1] = m[3];
                    w.m[2] = m[5];
                    w.m[3] = m[6];
                    break;
            }
            w.a = laneOf(lay.where[t]);
            masks(lay, op.ctrlIn, w.cReg, w.cLane);
            w.ctrlOut = op.ctrlOut;
            emit(w);
            continue;
        }
        // target into a slot (slot 0 keeps tile bit 0 for the whole pass)
        if (!inSlot(lay.where[t])) {
            const int l = laneOf(lay.where[t]);
            int victim = 1, far = -1;
            for (int s = VB; s < kWaveSlots; s++) {
                const int nu = nextUse(i, lay.slotBit[s]);
                if (nu > far) {
                    far = nu;
                    victim = s;
                }
            }
            transpose(victim, l);
        }
        WaveOp w;
        bool neg = false;
        switch (cls[i]) {
            case M2Class::Swap: w = blank((int)WKind::SWAP); break;
            case M2Class::Anti:
                if (cheap && m[2] == 0 && m[4] == 0 && std::fabs(m[3]) == 1 && m[5] == -m[3]) {
                    w = blank(m[3] < 0 ? (int)WKind::YSW : (int)WKind::YSWC);   // Y = [[0, -i], [i, 0]]
                    break;
                }
                w = blank((int)WKind::ANTI);
                w.m[0] = m[2];
                w.m[1] = m[3];
                w.m[2] = m[4];
                w.m[3] = m[5];
                break;
            case M2Class::Real:
                if (cheap && uncontrolled(op) && near(m[0], m[2]) && near(m[0], m[4]) && near(m[0], -m[6])) {
                    w = blank((int)WKind::HADD);   // m00 [[1, 1], [1, -1]]
                    sig.mul(m[0], 0);
                    break;
                }
                if (cheap && near(m[0], m[6]) && near(m[2], -m[4]) && unitCircle(m[0], m[4])) {
                    rotParams(m[0], m[4], w.m, &neg);
                    if (!neg || uncontrolled(op)) {
                        const real t0 = w.m[0], t1 = w.m[1];
                        w = blank((int)WKind::ROTY);
                        w.m[0] = t0;
                        w.m[1] = t1;
                        if (neg) sig.mul(-1, 0);
                        break;
                    }
                }
                w = blank((int)WKind::M2R);
                w.m[0] = m[0];
                w.m[1] = m[2];
                w.m[2] = m[4];
                w.m[3] = m[6];
                break;
            case M2Class::RealImag:
                // [[c, -is], [-is, c]]: m00 = m11 = c, Im m01 = Im m10 = -s
                if (cheap && near(m[0], m[6]) && near(m[3], m[5]) && unitCircle(m[0], m[5])) {
                    rotParams(m[0], -m[5], w.m, &neg);
                    if (!neg || uncontrolled(op)) {
                        const real t0 = w.m[0], t1 = w.m[1];
                        w = blank((int)WKind::ROTX);
                        w.m[0] = t0;
                        w.m[1] = t1;
                        if (neg) sig.mul(-1, 0);
                        break;
                    }
                }
                w = blank((int)WKind::M2RI);
                w.m[0] = m[0];
                w.m[1] = m[3];
                w.m[2] = m[5];
                w.m[3] = m[6];
                break;
            default:
                w = blank((int)WKind::M2);
                for (int x = 0; x < 8; x++) w.m[x] = m[x];
                break;
        }
        w.a = lay.where[t];
        masks(lay, op.ctrlIn, w.cReg, w.cLane);
        w.ctrlOut = op.ctrlOut;
        emit(w);
    }
    if (cframeOn) frameAfter();
    if (!sig.one()) settleScale(out, wp.opBegin, sig.re, sig.im);
    // real diagonal factors (density dephasing) as DSC: two multiplies per
    // amplitude instead of a complex product (QUEST_WAVE_DSC=0: keep DIAG)
    static const bool dscOn = !getenv("QUEST_WAVE_DSC") || atoi(getenv("QUEST_WAVE_DSC")) != 0;
    for (size_t o = (size_t)wp.opBegin; o < out.ops.size() && dscOn; o++)
        if (out.ops[o].kind == (int)WKind::DIAG && out.ops[o].m[1] == 0) out.ops[o].kind = (int)WKind::DSC;
    // phase ops on the same amplitudes inside a run of diagonal ops (they
    // all commute) multiply into one, or vanish (Z Z, the CZ pairs the
    // conditional frame puts around consecutive Ry / Rx on a conditioned
    // target, T T -> S, ...): QUEST_WAVE_MERGE_PHASES=0 to keep them
    static const bool mergeOn = !getenv("QUEST_WAVE_MERGE_PHASES") || atoi(getenv("QUEST_WAVE_MERGE_PHASES")) != 0;
    if (mergeOn) mergePhases(out, (size_t)wp.opBegin);
    if (endLanes)
        for (int l = 0; l < 3; l++) endLanes[l] = lay.laneBit[l];
    // store layout: the tile bits STORED to positions VB..VB+2 on lane bits
    // 0-2 (one 128-byte line per 8 lanes; the vector bits never left their
    // slots); with a relabelling pass these are other bits than at the load
    const size_t trBeforeStore = out.ops.size();
    int stBit[kWaveBits];
    for (int b = 0; b < kWaveBits; b++) stBit[b] = -1;
    for (int b = 0; b < kWaveBits; b++)
        if (ps.stPos[b] < kWaveBits) stBit[ps.stPos[b]] = b;
    // (these transpositions are about 40 % of a pass's weighted transposition
    // cost on the bench circuit, but stores that skip them are not 128-byte
    // coalesced: 0.284 instead of 0.199 ms/gate, same-box A/B)
    // the store layout's transpositions on `L2` (real: emitted, L2 is lay;
    // else only L2 is updated -- a dry run)
    auto farSt = [&](int b) { return ps.stPos[b] > kWaveLanePosMax; };
    auto storeLayout = [&](Layout& L2, bool real) -> bool {
        auto tr = [&](int s, int l) {
            if (real) {
                transpose(s, l);
                return;
            }
            const int bs = L2.slotBit[s], bl = L2.laneBit[l];
            L2.put(bs, kWaveSlots + l);
            L2.put(bl, s);
        };
        for (int l = 0; l < 3; l++) {
            const int b = stBit[VB + l];
            if (b < 0) return false;
            const int w = L2.where[b];
            if (w == kWaveSlots + l) continue;
            if (inSlot(w)) {
                tr(w, l);
            } else {
                // b sits on another lane bit (>= 3): through the first free slot
                tr(VB, laneOf(w));
                tr(VB, l);
            }
        }
        // real lane bits 3.. may not carry positions above kWaveLanePosMax at store
        for (int l = 3; l < kWaveLanes; l++) {
            if (!farSt(L2.laneBit[l])) continue;
            int s = -1;
            for (int x = VB; x < kWaveSlots && s < 0; x++)
                if (!farSt(L2.slotBit[x])) s = x;
            if (s < 0) return false;  // cannot happen: at most kWaveSlots - 1 far bits
            tr(s, l);
        }
        return true;
    };
    // conditional flips left at the end: those whose target and conditions
    // sit in one domain of the store layout (slots >= VB, real lanes, wave
    // bits) become store maps; the others are executed now
    auto domain = [](int w) { return inSlot(w) ? (w >= VB ? 0 : -1) : (laneOf(w) < kWaveLanes ? 1 : 2); };
    for (int guard = 0; cframeOn && guard < 4 * kWaveBits; guard++) {
        Layout fin = lay;
        if (!storeLayout(fin, false)) return false;
        int bad = -1;
        for (int t = 0; t < kWaveBits && bad < 0; t++) {
            if (!Cnd[t]) continue;
            const int d = domain(fin.where[t]);
            bool ok = d >= 0;
            for (unsigned c = Cnd[t]; c && ok; c &= c - 1) ok = domain(fin.where[__builtin_ctz(c)]) == d;
            if (!ok) bad = t;
        }
        if (bad < 0) break;
        cnotReason = 8;
        execConds(nOps, bad);
    }
    if (!storeLayout(lay, true)) return false;
    for (int t = 0; t < kWaveBits; t++) {
        if (!Cnd[t]) continue;
        const int w = lay.where[t];
        for (unsigned c = Cnd[t]; c; c &= c - 1) {
            const int wc = lay.where[__builtin_ctz(c)];
            if (inSlot(w))
                wp.stCondSlot[w] |= 1u << wc;
            else
                wp.stCondLane[laneOf(w)] |= 1u << laneOf(wc);
        }
    }
    if (!t_planQuiet)
        for (size_t o = trBeforeStore; o < out.ops.size(); o++)
            if (out.ops[o].kind == (int)WKind::TR) g_waveStoreTrCost += waveTransposeCost(out.ops[o].b);
    // flips still pending: folded into the store offsets
    wp.stFlip = slotFlips();
    wp.stFlipLane = laneFlips();
    for (int s = 0; s < kWaveSlots; s++) wp.stSlot[s] = lay.slotBit[s];
    for (int l = 0; l < kWaveLaneBits; l++) wp.stLane[l] = lay.laneBit[l];
    zFrame(out, (size_t)wp.opBegin);
    if (ctrlStatsOn() && !t_planQuiet)
        for (size_t o = (size_t)wp.opBegin; o < out.ops.size(); o++) {
            const WaveOp& w = out.ops[o];
            const int pc = __builtin_popcount(w.cReg), c = pc > 2 ? 2 : pc, l = (w.cLane & 63u) ? 1 : 0;
            g_ctrlOps[w.kind & 31][c][l]++;
            if (w.kind == (int)WKind::TR) g_trByBit[w.b & 15][0]++, g_trByBit[w.b & 15][1] += waveOpCycles(w);
            g_ctrlCyc[w.kind & 31][c][l] += waveOpCycles(w);
        }
    wp.opEnd = (int)out.ops.size();
    for (int o = wp.opBegin; o < wp.opEnd; o++)
        wp.waveExchange = wp.waveExchange || (out.ops[(size_t)o].kind == (int)WKind::TR && out.ops[(size_t)o].b >= kWaveLanes);
    // QUEST_WAVE_NO_STORE_BARRIER=1 (test hook): plan as before round 3, to
    // show that the emulation's wave-by-wave schedule catches the race
    static const bool noBarrier = getenv("QUEST_WAVE_NO_STORE_BARRIER") && atoi(getenv("QUEST_WAVE_NO_STORE_BARRIER"));
    wp.storeBarrier = !wp.waveExchange && !waveStoresInPlace(wp) && !noBarrier;
    out.passes.push_back(wp);
    if (t_planQuiet) return true;   // a trial plan: the statistics are the launched passes'
    stats().waveOps += wp.opEnd - wp.opBegin;
    for (int o = wp.opBegin; o < wp.opEnd; o++) stats().waveTransposes += out.ops[o].kind == (int)WKind::TR;
    return true;
}

}  // namespace qa
