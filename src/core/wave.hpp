// Wave-tile programs: the register-resident pass engine of the HIP backend
// (fp64 and fp32), planned on the host.
//
// A pass of the ordinary tile planner (tiles.hpp) with exactly kWaveBits tile
// bits is executed by ONE wave per tile: each of the 64 lanes holds 16
// amplitudes in registers, so the wave holds the whole 2^10-amplitude tile
// and no LDS and no barrier is involved.  A tile bit lives either in a
// register *slot* (bit s of the register index j, s < 5) or in a *lane bit*
// (bit l of the lane id, l < 6):
//
//   * gates whose target is in a slot run in registers (pairs j, j | 2^s);
//   * diagonal gates and every control work wherever their bits are
//     (per-register uniform predicates / per-lane predicates);
//   * a target held by a lane bit is first exchanged with a slot by a
//     cross-lane transposition (TR): DPP row shifts / quad permutes for lane
//     bits 0-3, v_permlane16/32_swap for lane bits 4-5 -- VALU work only.
//
// Loads and stores need tile bit 0 in slot 0 (the two halves of a 16-byte
// vector) and tile bits 1-3 in lane bits 0-2 (eight lanes cover one 128-byte
// line); the other 7 tile bits can sit in any of slots 1-4 / lane bits 3-5,
// chosen per pass for loads and whatever the ops left for stores.
//
// Gates are lowered to structure-specific kinds (real, real-diagonal /
// imaginary-off-diagonal, anti-diagonal, Pauli-X swap, diagonal), so e.g. a
// Hadamard costs 4 fp64 operations per amplitude instead of 8 and an X or a
// CNOT none -- the fused LDS kernel was bound by fp64 FMA issue and LDS.
#pragma once

#include <vector>

#include "tiles.hpp"

namespace qa {

// Register slots: 2^5 amplitudes per lane for fp64 (128 VGPRs of tile, four
// waves per tile) and fp32 (64 VGPRs, eight waves); QA_WAVE_SLOTS_F64 / _F32
// and QA_WAVE_WBITS_F64 / _F32 override (make WAVE_SLOTS=... WAVE_WBITS=...)
#ifndef QA_WAVE_SLOTS_F64
#define QA_WAVE_SLOTS_F64 5
#endif
#ifndef QA_WAVE_SLOTS_F32
#define QA_WAVE_SLOTS_F32 5
#endif
#if QuEST_PREC == 1
constexpr int kWaveSlots = QA_WAVE_SLOTS_F32;
#else
constexpr int kWaveSlots = QA_WAVE_SLOTS_F64;
#endif
// the kernel's register-control masks hold one bit per register in 32 bits
static_assert(kWaveSlots <= 5, "at most 2^5 registers per lane (32-bit register masks)");
// tile bits inside one 16-byte vector (they stay in slots 0.. for the whole
// pass): fp64 tile bit 0, fp32 tile bits 0-1
constexpr int kWaveVecBits = sizeof(real) == 8 ? 1 : 2;
constexpr int kWaveLanes = 6;   // 64 lanes
// A tile is shared by 2^kWaveWBits waves of a workgroup: "wave bits" are
// virtual lane bits 6.. of the tile (transpositions with a slot go through
// LDS, controls on them are wave-uniform predicates).  fp64: 5 slots x 2 wave
// bits (profiles/r3/wave_shape_variants.txt; round 2-3 before: 4 x 3)
#ifndef QA_WAVE_WBITS_F64
#define QA_WAVE_WBITS_F64 2
#endif
#ifndef QA_WAVE_WBITS_F32
#define QA_WAVE_WBITS_F32 3
#endif
#if QuEST_PREC == 1
constexpr int kWaveWBits = QA_WAVE_WBITS_F32;
#else
constexpr int kWaveWBits = QA_WAVE_WBITS_F64;
#endif
constexpr int kWaveLaneBits = kWaveLanes + kWaveWBits;  // real + wave lane bits
constexpr int kWaveBits = kWaveSlots + kWaveLaneBits;
// real lane bits carry positions up to this (32-bit per-lane byte offsets)
constexpr int kWaveLanePosMax = sizeof(real) == 8 ? 27 : 28;

enum class WKind : int {
    M2 = 0,    // general 2x2 on slot a
    M2R = 1,   // real 2x2 on slot a (m[0..3] = m00 m01 m10 m11)
    M2RI = 2,  // real diagonal / imaginary off-diagonal on slot a (m = m00 Im(m01) Im(m10) m11)
    ANTI = 3,  // anti-diagonal on slot a (m = m01 re,im, m10 re,im)
    SWAP = 4,  // Pauli X on slot a (controls make it CNOT / Toffoli)
    DIAG = 5,  // multiply every element whose (cReg, cLane) bits are 1 by m[0] + i m[1]
    D2S = 6,   // diagonal 2x2 on the bit of slot a (m = d0 re,im, d1 re,im)
    D2L = 7,   // diagonal 2x2 on lane bit a
    TR = 8,    // transpose slot a with lane bit b (b >= 6: wave bit, through LDS; never masked)
    // the same gates with their target on real lane bit a < kWaveLaneOps (lane
    // pairs combined through DPP, per-lane coefficients; m as for the slot kinds)
    LM2R = 9,
    LM2RI = 10,
    LANTI = 11,
    LSWAP = 12,
    // cheaper forms of common gates on slot a (tools/gen_wave_asm.py KINDS2):
    ROTY = 13,   // real rotation [[c, -s], [s, c]] by three shears (m = tan(phi/2), sin(phi))
    ROTX = 14,   // [[c, -is], [-is, c]] (Rx): (a_im, b_re) by +phi, (a_re, b_im) by -phi
    HADD = 15,   // unnormalised Hadamard (a + b, a - b); never controlled (the pass absorbs 1/sqrt2)
    YSW = 16,    // Pauli Y as register swaps + sign flips
    YSWC = 17,   // -Y
    // unit-modulus phases on the (cReg, cLane) registers (PH_KINDS):
    DROT = 18,   // multiply by e^{i phi}, |phi| <= pi/2: (re, im) rotated by shears (m as ROTY)
    DNEG = 19,   // multiply by -1
    DMULI = 20,  // multiply by i
    DMULNI = 21, // multiply by -i
    DROTN = 22,  // multiply by -e^{i phi} (negation + DROT)
    // one-qubit density channels on the 4-group of slots (a = row bit, b =
    // column bit; g = bit a + 2 bit b): x0, x3 mixed by the real 2x2 m[0..3],
    // x1, x2 scaled by m[4] (CHD: the scaling only)
    CH1 = 23,
    CHD = 24,
    // real factor m[0] on the (cReg, cLane) registers (PH_KINDS "DSC"): the
    // real diagonal factors of density dephasing, half a complex product
    DSC = 25,
};

// Whether a Mat4 (4x4, row-major, interleaved re/im as in TileOp::m) is a
// one-qubit channel superoperator the wave engine runs (CH1 / CHD): real,
// nonzero only at (0,0) (0,3) (3,0) (3,3) and (1,1) = (2,2).
bool waveChannel(const real* m);
constexpr int kWaveLaneOps = 3;  // lane bits with direct gate handlers

// One op, uploaded as-is (uniform: read through the scalar cache).
struct WaveOp {
    int kind;
    int a, b;
    unsigned cReg;    // register slots that must be 1
    unsigned cLane;   // lane bits that must be 1 (bits >= 6: wave bits)
    unsigned cLaneZero;  // lane bits that must be 0 (wave bits only)
    // controls on tile bits the pass has flipped (deferred X, see
    // planWavePass): register j passes when ((j ^ fReg) & cReg) == cReg,
    // lane L when ((L ^ fLane) & cLane) == cLane (real lane bits)
    unsigned fReg, fLane;
    u64 ctrlOut;      // physical bits outside the tile that must be 1
    u64 ctrlOutZero;  // ... that must be 0 (DIAG only: folded diagonal runs, planWavePass)
    real m[8];
};

struct WavePass {
    int pos[kWaveBits];        // tile bit -> physical position (pos[i] = i for i < 4)
    int stPos[kWaveBits];      // tile bit -> physical position it is stored to (TilePass::stPos)
    int opBegin = 0, opEnd = 0;
    int ldSlot[kWaveSlots];    // tile bit held by slot s at load
    int ldLane[kWaveLaneBits]; // tile bit held by lane bit l at load (l >= 6: wave bits)
    int stSlot[kWaveSlots];    // ... at store
    // tile bits flipped at the end of the pass (X the planner did not
    // execute, planWavePass): register j of lane L is stored where register
    // j ^ stFlip of lane L ^ stFlipLane belongs (stFlipLane: real lane bits
    // 0-5 and the wave bits above them)
    unsigned stFlip = 0, stFlipLane = 0;
    // conditional flips (deferred CNOTs, planWavePass): the bit of slot s is
    // further flipped in the registers where the parity of the slots in
    // stCondSlot[s] is odd; the bit of lane bit l in the lanes where the parity
    // of the lane bits in stCondLane[l] is odd (real lanes condition real
    // lanes, wave bits wave bits; vector slots never take part)
    unsigned stCondSlot[kWaveSlots] = {0};
    unsigned stCondLane[kWaveLaneBits] = {0};
    int stLane[kWaveLaneBits];
    // The waves of a workgroup run unsynchronised between their loads and
    // stores unless a wave-bit transposition (LDS, two barriers) lies between.
    // A pass whose store moves a tile bit held by a wave bit to another
    // position (relabelling, or a deferred X on a wave bit) has each wave
    // store onto addresses other waves load: the kernel then waits at a
    // barrier before the stores (launch record, tileMap bit 30).
    bool storeBarrier = false;
    bool waveExchange = false;  // the pass has a wave-bit transposition (its barriers order loads before stores)
};

// Store maps of a pass: register j of lane L (L: real lane bits, then the
// wave bits) is stored where register waveStReg(wp, j) of lane
// waveStLane(wp, L) belongs in the store layout (stSlot / stLane / stPos).
inline int waveStReg(const WavePass& wp, int j) {
    int r = j ^ (int)wp.stFlip;
    for (int s = 0; s < kWaveSlots; s++)
        if (__builtin_popcount((unsigned)j & wp.stCondSlot[s]) & 1) r ^= 1 << s;
    return r;
}
inline int waveStLane(const WavePass& wp, int L) {
    int r = L ^ (int)wp.stFlipLane;
    for (int l = 0; l < kWaveLaneBits; l++)
        if (__builtin_popcount((unsigned)L & wp.stCondLane[l]) & 1) r ^= 1 << l;
    return r;
}

// Whether every wave of a tile stores to exactly the addresses it loaded
// (false: the pass needs storeBarrier or a wave-bit transposition).
bool waveStoresInPlace(const WavePass& wp);

struct WaveProgram {
    std::vector<WavePass> passes;
    std::vector<WaveOp> ops;
};

// Lower one tile pass (its ops in tile-local coordinates) to a wave pass.
// False if the pass cannot run on the wave engine (tile size other than
// kWaveBits, non-contiguous low bits, Mat4 / DensChan2 ops, too many tile
// bits above kWaveLanePosMax).
// endLanes (optional): the tile bits on real lane bits 0-2 after the ops,
// before the store layout is restored.
bool planWavePass(const TilePass& ps, const TileOp* ops, int nOps, WaveProgram& out, int* endLanes = nullptr);

// PlanHooks::lowPerm of wave plans: reorder the tile bits stored to the
// always-resident positions [kWaveVecBits, cmin) so that those already on
// lanes 0-2 at the end of the pass are stored to positions 1-3 (fp64) from
// there -- the store layout then needs no transposition for them.
bool waveLowPerm(const TilePass& ps, const TileOp* ops, int cmin, int* sigma);

// In-place relabelling passes (planTiles relabelFrom): on by default for
// wave programs (QUEST_WAVE_RELABEL=0 / tuning "wave_relabel" turn it off).
bool& waveRelabel();
// Every relabelling pass of the program lowers to the wave engine (the LDS
// and direct kernels store in place); false -> plan again without relabelling.
bool relabelsLower(const TileProgram& prog);

// The wave engine can lower this pass (planWavePass on a scratch program; the
// statistics are left alone): the planner's relabelOk hook.
bool waveLowers(const TilePass& ps, const TileOp* ops);
// Estimated issue cycles per wave of one wave op / of a whole tile pass as
// the wave engine would run it (-1: the pass does not lower) -- the planner's
// pass-balancing cost (PlanHooks::passCost).
double waveOpCycles(const WaveOp& w);
double wavePassCycles(const TilePass& ps, const TileOp* ops);
// The compute-aware planner hooks of wave plans (PlanHooks::passCost /
// memCost / costMargin): QUEST_PLAN_MEM_CYCLES (0: off) and
// QUEST_PLAN_COST_MARGIN.
void waveCostHooks(PlanHooks& hooks);
// Planner strategy search (QUEST_PLAN_SEARCH, default on).  The greedy
// planner's pass count swings by several passes from circuit to circuit with
// any single knob; searchWaveStrategy plans a queue of at least
// QUEST_PLAN_SEARCH_OPS (256) plain wave ops with every strategy at once on
// worker threads (always-resident positions cdefault / cdefault + 1,
// compute-aware passes on / off / without margin, more seed candidates,
// one-pass lookahead, and the round-3 planner without the conditional frame;
// statistics untouched), scores each plan by sum over passes of max(modeled
// compute, memory stream) and returns the best one's index (-1: no search).
// Thread-safe: the backends run it synchronously (worker threads) on full
// flushes and in the background after a window's first front flush.
int searchWaveStrategy(const std::vector<Op>& ops, int L, int cdefault, const PlanHooks& base);
size_t waveSearchMinOps();
// local qubits from which the strategy search runs (QUEST_PLAN_SEARCH_QUBITS, 27)
int waveSearchMinQubits();
// local qubits from which passes are planned compute-aware (QUEST_PLAN_COST_QUBITS, 22)
int waveCostMinQubits();
// QUEST_PLAN_SEARCH_FRONT=0: no background search after front flushes;
// QUEST_PLAN_FRONT_STRATEGY: the strategy of front flushes until a search
// has chosen one (default 0)
bool waveFrontSearch();
bool waveSearchOn();   // QUEST_PLAN_SEARCH (default 1)
// A full flush of a queue the search would plan, with no front flush of the
// window before it (the GPU is idle): launch the first pass at once (planned
// as a front flush, the whole queue its lookahead) and search the rest while
// it runs, instead of searching first (QUEST_PLAN_SEARCH_SPLIT, default 1).
bool waveSearchSplitFirst(const QuregImpl& q);
int waveFrontStrategy();
// Plan (and lower) a flush with strategy idx (< 0: the default): sets the
// hooks' knobs and *cmin, and the thread's conditional-frame switch until
// the scope ends -- the lowering of the streamed passes must see the planner's.
struct WaveStrategyScope {
    WaveStrategyScope(int idx, int cdefault, PlanHooks& hooks, int* cmin);
    ~WaveStrategyScope();
    WaveStrategyScope(const WaveStrategyScope&) = delete;
    WaveStrategyScope& operator=(const WaveStrategyScope&) = delete;
    bool active = false;
};
extern thread_local int t_waveCframe;   // conditional frame of this thread's plans: -1 env, 0 off, 1 on
// Always-resident low positions for a relabelling wave plan of q.pending:
// cdefault or cdefault + 1, whichever plans fewer passes (QUEST_WAVE_CMIN_SEARCH
// =1; default: cdefault); sticky in q.waveCmin until the queue drains.
int chooseWaveCmin(QuregImpl& q, int cdefault, const PlanHooks& hooks);
// After a program ran: the register's qubits moved by prog.perm.
void applyProgramPerm(QuregImpl& q, const TileProgram& prog);
// A local qubit permutation as op-free relabelling wave passes (load a tile,
// store it with its positions permuted: no arithmetic, one HBM round trip per
// pass, at most 12 moved positions each): dest[p] = the position the qubit on
// local position p must move to.  False if the wave engine cannot (a moved
// vector bit, or a pass it does not lower); prog.passes then is unusable.
bool planRelayout(int L, const int* dest, TileProgram& prog);

// Cost in VALU instructions per lane of one transposition with lane bit l
// (for the planner's statistics and tests).
int waveTransposeCost(int laneBit);
extern long long g_waveStoreTrCost;   // planner study: weighted transpositions for the store layout
// Plans made while a QuietPlan lives on this thread (lowering checks, cost
// estimates, trial plans -- possibly on planner worker threads) leave the
// global statistics alone.
extern thread_local int t_planQuiet;
struct QuietPlan {
    QuietPlan() { t_planQuiet++; }
    ~QuietPlan() { t_planQuiet--; }
    QuietPlan(const QuietPlan&) = delete;
    QuietPlan& operator=(const QuietPlan&) = delete;
};

// Load layout of the bits beyond the slots (QUEST_WAVE_LANE_ORDER / tuning
// "wave_lane_order"): 1 (default) lanes 3-5 take the lowest positions, 0 need
// order, 2 the wave bits take the latest-needed bits.
int& waveLaneOrder();

// Host emulation of one wave pass on a host copy of the state
// (src/core/wave_emu.cpp): the CPU backend's wave planner mode and the HIP
// backend's per-pass shadow oracle.
void emulateWavePass(real* re, real* im, int L, const WaveProgram& wp, const WavePass& ps);
// QUEST_WAVE_DUMP: the pass's op mix (and with =2 its handlers) on stderr
void dumpWavePass(const WaveProgram& wp, const WavePass& ps);

}  // namespace qa
