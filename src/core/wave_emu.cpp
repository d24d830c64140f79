// Host emulation of wave-tile passes (src/core/wave.hpp): 64 lanes x the
// waves of a tile x 2^kWaveSlots registers, moved and combined exactly as the
// gfx950 kernel of tools/gen_wave_asm.py does.  The CPU backend runs wave
// plans through it (QUEST_CPU_PLANNER=3); the HIP backend uses it as the
// per-pass oracle of its shadow check (tuning "wave_shadow").
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <utility>
#include <vector>

#include "wave.hpp"

namespace qa {

namespace {
constexpr int kWaveRegs = 1 << kWaveSlots;
constexpr int kVLanes = 1 << kWaveLaneBits;  // 64 lanes x the waves sharing a tile

void applyWaveOp(const WaveOp& w, real (*vr)[kWaveRegs], real (*vi)[kWaveRegs]) {
    const WKind kind = (WKind)w.kind;
    if (kind == WKind::TR) {
        const int s = w.a, l = w.b;
        for (int j = 0; j < kWaveRegs; j++) {
            if ((j >> s) & 1) continue;
            const int f = j | (1 << s);
            for (int L0 = 0; L0 < kVLanes; L0++) {
                if ((L0 >> l) & 1) continue;
                const int L1 = L0 | (1 << l);
                std::swap(vr[L1][j], vr[L0][f]);
                std::swap(vi[L1][j], vi[L0][f]);
            }
        }
        return;
    }
    const real* m = w.m;
    // the shear rotation of tools/gen_wave_asm.py rot(): same operation order
    auto rot = [&](real& x, real& y, bool neg) {
        const real t = neg ? -m[0] : m[0], sn = neg ? -m[1] : m[1];
        x = std::fma(-t, y, x);
        y = std::fma(sn, x, y);
        x = std::fma(-t, y, x);
    };
    if (kind >= WKind::LM2R && kind <= WKind::LSWAP) {
        // target on lane bit a: lane pairs (L0, L1 = L0 | 2^a), per register
        const int a = w.a;
        for (int L0 = 0; L0 < kVLanes; L0++) {
            if ((L0 >> a) & 1) continue;
            if ((((unsigned)L0 ^ w.fLane) & w.cLane) != w.cLane || ((unsigned)L0 & w.cLaneZero)) continue;
            const int L1 = L0 | (1 << a);
            for (int j = 0; j < kWaveRegs; j++) {
                if ((((unsigned)j ^ w.fReg) & w.cReg) != w.cReg) continue;
                const real r0 = vr[L0][j], i0 = vi[L0][j], r1 = vr[L1][j], i1 = vi[L1][j];
                real *R0 = &vr[L0][j], *I0 = &vi[L0][j], *R1 = &vr[L1][j], *I1 = &vi[L1][j];
                switch (kind) {
                    case WKind::LM2R:
                        *R0 = m[0] * r0 + m[1] * r1;
                        *I0 = m[0] * i0 + m[1] * i1;
                        *R1 = m[2] * r0 + m[3] * r1;
                        *I1 = m[2] * i0 + m[3] * i1;
                        break;
                    case WKind::LM2RI:
                        *R0 = m[0] * r0 - m[1] * i1;
                        *I0 = m[0] * i0 + m[1] * r1;
                        *R1 = m[3] * r1 - m[2] * i0;
                        *I1 = m[3] * i1 + m[2] * r0;
                        break;
                    case WKind::LANTI:
                        *R0 = m[0] * r1 - m[1] * i1;
                        *I0 = m[0] * i1 + m[1] * r1;
                        *R1 = m[2] * r0 - m[3] * i0;
                        *I1 = m[2] * i0 + m[3] * r0;
                        break;
                    default:  // LSWAP
                        *R0 = r1;
                        *I0 = i1;
                        *R1 = r0;
                        *I1 = i0;
                        break;
                }
            }
        }
        return;
    }
    for (int lane = 0; lane < kVLanes; lane++) {
        if ((((unsigned)lane ^ w.fLane) & w.cLane) != w.cLane) continue;
        if ((unsigned)lane & w.cLaneZero) continue;
        real* r = vr[lane];
        real* i = vi[lane];
        if (kind == WKind::CH1 || kind == WKind::CHD) {
            const int a = w.a, b = w.b;
            for (int j = 0; j < kWaveRegs; j++) {
                if (((j >> a) & 1) || ((j >> b) & 1)) continue;
                const int x1 = j | (1 << a), x2 = j | (1 << b), x3 = x1 | (1 << b);
                for (real* v : {r, i}) {
                    v[x1] *= m[4];
                    v[x2] *= m[4];
                    if (kind == WKind::CH1) {
                        const real t = m[2] * v[j];
                        v[j] = std::fma(m[1], v[x3], m[0] * v[j]);
                        v[x3] = std::fma(m[3], v[x3], t);
                    }
                }
            }
            continue;
        }
        if (kind == WKind::DSC) {
            for (int j = 0; j < kWaveRegs; j++) {
                if ((((unsigned)j ^ w.fReg) & w.cReg) != w.cReg) continue;
                r[j] *= m[0];
                i[j] *= m[0];
            }
            continue;
        }
        if (kind >= WKind::DROT && kind <= WKind::DROTN) {
            for (int j = 0; j < kWaveRegs; j++) {
                if ((((unsigned)j ^ w.fReg) & w.cReg) != w.cReg) continue;
                real &x = r[j], &y = i[j];
                if (kind == WKind::DNEG || kind == WKind::DROTN) x = -x, y = -y;
                if (kind == WKind::DROT || kind == WKind::DROTN) rot(x, y, false);
                if (kind == WKind::DMULI) {
                    const real t = x;
                    x = -y;
                    y = t;
                } else if (kind == WKind::DMULNI) {
                    const real t = x;
                    x = y;
                    y = -t;
                }
            }
            continue;
        }
        if (kind == WKind::DIAG || kind == WKind::D2S || kind == WKind::D2L) {
            for (int j = 0; j < kWaveRegs; j++) {
                if ((((unsigned)j ^ w.fReg) & w.cReg) != w.cReg) continue;
                real tr = m[0], ti = m[1];
                if (kind == WKind::D2S && ((j >> w.a) & 1)) tr = m[2], ti = m[3];
                if (kind == WKind::D2L && ((lane >> w.a) & 1)) tr = m[2], ti = m[3];
                const real x = r[j], y = i[j];
                r[j] = tr * x - ti * y;
                i[j] = tr * y + ti * x;
            }
            continue;
        }
        const int a = w.a;
        for (int j = 0; j < kWaveRegs; j++) {
            if ((j >> a) & 1) continue;
            if ((((unsigned)j ^ w.fReg) & w.cReg) != w.cReg) continue;
            const int f = j | (1 << a);
            const real r0 = r[j], i0 = i[j], r1 = r[f], i1 = i[f];
            switch (kind) {
                case WKind::M2:
                    r[j] = m[0] * r0 - m[1] * i0 + m[2] * r1 - m[3] * i1;
                    i[j] = m[0] * i0 + m[1] * r0 + m[2] * i1 + m[3] * r1;
                    r[f] = m[4] * r0 - m[5] * i0 + m[6] * r1 - m[7] * i1;
                    i[f] = m[4] * i0 + m[5] * r0 + m[6] * i1 + m[7] * r1;
                    break;
                case WKind::M2R:
                    r[j] = m[0] * r0 + m[1] * r1;
                    i[j] = m[0] * i0 + m[1] * i1;
                    r[f] = m[2] * r0 + m[3] * r1;
                    i[f] = m[2] * i0 + m[3] * i1;
                    break;
                case WKind::M2RI:
                    r[j] = m[0] * r0 - m[1] * i1;
                    i[j] = m[0] * i0 + m[1] * r1;
                    r[f] = m[3] * r1 - m[2] * i0;
                    i[f] = m[3] * i1 + m[2] * r0;
                    break;
                case WKind::ANTI:
                    r[j] = m[0] * r1 - m[1] * i1;
                    i[j] = m[0] * i1 + m[1] * r1;
                    r[f] = m[2] * r0 - m[3] * i0;
                    i[f] = m[2] * i0 + m[3] * r0;
                    break;
                case WKind::SWAP:
                    r[j] = r1;
                    i[j] = i1;
                    r[f] = r0;
                    i[f] = i0;
                    break;
                case WKind::ROTY:
                    rot(r[j], r[f], false);
                    rot(i[j], i[f], false);
                    break;
                case WKind::ROTX:
                    rot(i[j], r[f], false);
                    rot(r[j], i[f], true);
                    break;
                case WKind::HADD:
                    r[f] = r0 - r1;
                    r[j] = std::fma((real)2, r0, -r[f]);
                    i[f] = i0 - i1;
                    i[j] = std::fma((real)2, i0, -i[f]);
                    break;
                case WKind::YSW:  // a -> -i b, b -> i a
                    r[j] = i1;
                    i[j] = -r1;
                    r[f] = -i0;
                    i[f] = r0;
                    break;
                case WKind::YSWC:
                    r[j] = -i1;
                    i[j] = r1;
                    r[f] = i0;
                    i[f] = -r0;
                    break;
                default: break;
            }
        }
    }
}

}  // namespace

long long g_trCost = 0;  // QUEST_WAVE_DUMP: weighted transposition cost (planner study)

// QUEST_WAVE_DUMP (planner study): the op mix of every wave pass on stderr
void dumpWavePass(const WaveProgram& wp, const WavePass& ps) {
    static const bool dump = getenv("QUEST_WAVE_DUMP") != nullptr;
    if (!dump) return;
    // QUEST_WAVE_DUMP=2: the GPU handler of every op (names of
    // tools/gen_wave_asm.py, for tools/wave_cost.py)
    static const bool perOp = atoi(getenv("QUEST_WAVE_DUMP")) >= 2;
    // QUEST_WAVE_DUMP=3: also every op's fields (planner studies)
    static const bool fields = atoi(getenv("QUEST_WAVE_DUMP")) == 3;
    for (int i = ps.opBegin; i < ps.opEnd && fields; i++) {
        const WaveOp& w = wp.ops[(size_t)i];
        fprintf(stderr, "O %d %d %d %x %x %x %llx\n", w.kind, w.a, w.b, w.cReg, w.cLane, w.cLaneZero,
                (unsigned long long)w.ctrlOut);
    }
    static const char* kName[] = {"M2", "M2R", "M2RI", "ANTI", "SWAP", "DIAG", "D2S", "D2L", "TR", "LM2R", "LM2RI",
                                  "LANTI", "LSWAP", "ROTY", "ROTX", "HADD", "YSW", "YSWC", "DROT", "DNEG", "DMULI",
                                  "DMULNI", "DROTN", "CH1", "CHD", "DSC"};
    for (int i = ps.opBegin; i < ps.opEnd && perOp; i++) {
        const WaveOp& w = wp.ops[(size_t)i];
        const unsigned lanes = w.cLane & 63u;
        const int ctrl = (w.cReg | lanes) == 0 ? 0 : (w.cReg == 0 ? 2 : 1);
        const char* k = kName[w.kind];
        switch ((WKind)w.kind) {
            case WKind::TR:
                if (w.b < kWaveLanes) fprintf(stderr, "H wh_TR_s%d_l%d\n", w.a, w.b);
                else fprintf(stderr, "H wh_TRW_s%d_b%d\n", w.a, w.b - kWaveLanes);
                break;
            case WKind::DIAG: case WKind::DROT: case WKind::DNEG: case WKind::DMULI: case WKind::DMULNI:
            case WKind::DROTN: case WKind::DSC:
                fprintf(stderr, "H wh_%s_m%u_l%d\n", k, w.cReg, lanes ? 1 : 0);
                break;
            case WKind::D2L: fprintf(stderr, "H wh_D2L_c%d\n", ctrl ? 1 : 0); break;
            case WKind::LM2R: case WKind::LM2RI: case WKind::LANTI: case WKind::LSWAP:
                fprintf(stderr, "H wh_%s_l%d_c%d\n", k, w.a, ctrl ? 1 : 0);
                break;
            case WKind::CH1: case WKind::CHD: fprintf(stderr, "H wh_%s_a%d_b%d\n", k, w.a, w.b); break;
            default: fprintf(stderr, "H wh_%s_s%d_c%d\n", k, w.a, ctrl); break;
        }
    }
    int cnt[32] = {0}, trw = 0, ctl = 0;
    double cyc = 0;
    for (int i = ps.opBegin; i < ps.opEnd; i++) {
        const WaveOp& w = wp.ops[(size_t)i];
        cyc += waveOpCycles(w);
        cnt[w.kind]++;
        if (w.kind == (int)WKind::TR && w.b >= kWaveLanes) trw++;
        if (w.kind == (int)WKind::TR) g_trCost += waveTransposeCost(w.b);
        if (w.kind != (int)WKind::DIAG && (w.cReg || w.cLane)) ctl++;
    }
    fprintf(stderr, "wave pass: %d ops  M2 %d M2R %d M2RI %d ANTI %d SWAP %d DIAG %d D2S %d D2L %d TR %d (TRW %d) lane %d "
            "ctl %d | ROTY %d ROTX %d HADD %d Y %d phase %d chan %d | cycles %.0f\n",
            ps.opEnd - ps.opBegin, cnt[0], cnt[1], cnt[2], cnt[3], cnt[4], cnt[5], cnt[6], cnt[7], cnt[8], trw,
            cnt[9] + cnt[10] + cnt[11] + cnt[12], ctl, cnt[13], cnt[14], cnt[15], cnt[16] + cnt[17],
            cnt[18] + cnt[19] + cnt[20] + cnt[21] + cnt[22], cnt[23] + cnt[24], cyc);
    // memory pattern: physical positions of the lane bits (one load / store
    // instruction spans the vector bit and the real lane bits) and the slots
    fprintf(stderr, "wave: ld lanes");
    for (int l = 0; l < kWaveLaneBits; l++) fprintf(stderr, " %d", ps.pos[ps.ldLane[l]]);
    fprintf(stderr, " slots");
    for (int r = 0; r < kWaveSlots; r++) fprintf(stderr, " %d", ps.pos[ps.ldSlot[r]]);
    fprintf(stderr, " | st lanes");
    for (int l = 0; l < kWaveLaneBits; l++) fprintf(stderr, " %d", ps.stPos[ps.stLane[l]]);
    fprintf(stderr, " slots");
    for (int r = 0; r < kWaveSlots; r++) fprintf(stderr, " %d", ps.stPos[ps.stSlot[r]]);
    fprintf(stderr, "\n");
    int trb[16] = {0};
    for (int i = ps.opBegin; i < ps.opEnd; i++)
        if (wp.ops[(size_t)i].kind == (int)WKind::TR) trb[wp.ops[(size_t)i].b & 15]++;
    fprintf(stderr, "wave: TR per bit:");
    for (int b = 0; b < 9; b++) fprintf(stderr, " %d", trb[b]);
    fprintf(stderr, "\nwave: cumulative weighted transposition cost %lld (store layout %lld)\n", g_trCost,
            g_waveStoreTrCost);
}

void emulateWavePass(real* re, real* im, int L, const WaveProgram& wp, const WavePass& ps) {
    // shared by the threads of the parallel region below (a thread_local
    // table here was filled by the calling thread only)
    std::vector<i64> ldv((size_t)kVLanes * kWaveRegs), stv(ldv.size());
    auto ld = reinterpret_cast<i64(*)[kWaveRegs]>(ldv.data());
    auto st = reinterpret_cast<i64(*)[kWaveRegs]>(stv.data());
    auto offsetOf = [&](const int* pos, const int* slotBit, const int* laneBit, int lane, int j) {
        i64 off = 0;
        for (int s = 0; s < kWaveSlots; s++)
            if ((j >> s) & 1) off |= (i64)1 << pos[slotBit[s]];
        for (int l = 0; l < kWaveLaneBits; l++)
            if ((lane >> l) & 1) off |= (i64)1 << pos[laneBit[l]];
        return off;
    };
    for (int lane = 0; lane < kVLanes; lane++)
        for (int j = 0; j < kWaveRegs; j++) {
            ld[lane][j] = offsetOf(ps.pos, ps.ldSlot, ps.ldLane, lane, j);
            // relabelling passes store permuted; pending exchanges (stFlip,
            // conditional flips) store register j where its partner belongs
            st[lane][j] = offsetOf(ps.stPos, ps.stSlot, ps.stLane, waveStLane(ps, lane), waveStReg(ps, j));
        }
    dumpWavePass(wp, ps);
    TilePass tp;
    tp.k = kWaveBits;
    for (int b = 0; b < kWaveBits; b++) tp.pos[b] = ps.pos[b];
    const i64 tiles = (i64)1 << (L - kWaveBits);
    // The kernel's waves are unordered between their loads and stores unless
    // a barrier lies between (a wave-bit transposition, or the store barrier
    // the planner requests when waves store onto each other's load
    // addresses).  Without one, emulate the worst legal order -- each wave
    // loads, computes and stores before the next wave loads -- so that a plan
    // that needs a barrier and lacks it gives a wrong result here as well
    // (the kernel's race, made deterministic).  Passes whose waves store in
    // place give the same result either way and take the fast path.
    const bool waveByWave = kWaveWBits > 0 && !ps.storeBarrier && !ps.waveExchange && !waveStoresInPlace(ps);
    auto work = [&](i64 t0, i64 t1) {
        std::vector<real> bufR(kVLanes * kWaveRegs), bufI(kVLanes * kWaveRegs);
        real(*vr)[kWaveRegs] = reinterpret_cast<real(*)[kWaveRegs]>(bufR.data());
        real(*vi)[kWaveRegs] = reinterpret_cast<real(*)[kWaveRegs]>(bufI.data());
        const int groups = waveByWave ? 1 << kWaveWBits : 1, per = kVLanes / groups;
        for (i64 T = t0; T < t1; T++) {
            const i64 base = tileBase(tp, T, L);
            for (int g = 0; g < groups; g++) {
                for (int lane = g * per; lane < (g + 1) * per; lane++)
                    for (int j = 0; j < kWaveRegs; j++) {
                        vr[lane][j] = re[base + ld[lane][j]];
                        vi[lane][j] = im[base + ld[lane][j]];
                    }
                for (int o = ps.opBegin; o < ps.opEnd; o++) {
                    const WaveOp& w = wp.ops[o];
                    if (((u64)base & w.ctrlOut) != w.ctrlOut || ((u64)base & w.ctrlOutZero)) continue;
                    applyWaveOp(w, vr, vi);
                }
                for (int lane = g * per; lane < (g + 1) * per; lane++)
                    for (int j = 0; j < kWaveRegs; j++) {
                        re[base + st[lane][j]] = vr[lane][j];
                        im[base + st[lane][j]] = vi[lane][j];
                    }
            }
        }
    };
    // below ~4M amplitudes thread start-up costs more than it saves
    const int nt = ((i64)1 << L) >= ((i64)1 << 22)
                       ? (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()))
                       : 1;
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; t++) pool.emplace_back(work, tiles * t / nt, tiles * (t + 1) / nt);
    work(0, tiles / nt);
    for (std::thread& th : pool) th.join();
}


}  // namespace qa
