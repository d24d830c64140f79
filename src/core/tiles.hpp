// Gate-fusion planner and tile-program compiler (host code shared by both
// backends, so the CPU build executes the exact tile decomposition the GPU
// kernel does and can be tested without a GPU).
//
// A *pass* streams the chunk once: it is cut into 2^(L-k) independent tiles of
// 2^k amplitudes that share every physical bit outside the tile's qubit set Q
// (|Q| = k).  Q always contains the lowest `cmin` bits, so every tile is made
// of contiguous runs of >= 2^cmin amplitudes (whole 128-B lines in HBM), plus
// every TARGET of the pass's ops.  Inside a tile the ops run back to back on
// the LDS copy; controls / diagonal bits outside Q are per-tile predicates.
// Ops are never reordered, so fused and unfused execution are identical up to
// floating-point rounding of the same operations in the same order.
//
// The reference has no equivalent: every gate is one kernel launch streaming
// the full state (QuEST/src/GPU/QuEST_gpu.cu, e.g. :586-592).
#pragma once

#include <functional>
#include <vector>

#include "core.hpp"

namespace qa {

// One op in tile-local coordinates.  Plain data: uploaded as-is to the GPU.
struct TileOp {
    int kind;            // OpKind
    int t[4];            // tile-local target bits
    int rt[4];           // register slots of the targets inside a register phase
    unsigned ctrlIn;     // tile-local mask of bits that must be 1
    int nsw;             // element-bit swaps applied to the work-item index (below)
    unsigned char swA[4], swB[4];
    unsigned du[16];     // element of work item 256 u (u < 16), after insertion + swaps
    unsigned sdu[16];    // ldsSwizzle(du[u])
    u64 ctrlOut;         // physical bits outside the tile that must be 1
    real m[32];          // matrix, interleaved re/im, row-major
};

// GPU op-by-op LDS access: work item j of an op (a pair / quad / element) is
// expanded to tile element p by inserting zeros at the target bits; the
// first 5 bits of j then come from the lowest free bits.  When targets sit
// low, those give 32 lanes colliding LDS slots under ldsSwizzle.  The host
// records up to 4 element-bit swaps (swA[i] <-> swB[i], applied to p in
// order) that re-map lane bits 0-4 to free bits with independent slot
// vectors (reads: 32-lane groups, slot = 8-byte word mod 32; writes: 16-lane
// groups, mod 16), making every access of the op conflict-free.
// Also fills du / sdu, the wave-uniform parts of the work-item addresses.
void laneSwaps(TileOp& op, int k);

// Threads per workgroup of the GPU tile kernel for a tile of k bits: 256 up
// to 2^11 fp64 / 2^12 fp32 amplitudes (32 KiB), 512 for the double tile, so
// that every thread keeps 8 (fp64) / 16 (fp32) amplitudes.
constexpr unsigned tileThreads(int k) { return k > (sizeof(real) == 8 ? 11 : 12) ? 512u : 256u; }

// A phase of a pass: a run of ops executed with each thread holding 2^R
// amplitudes in registers, namely the tile elements spanned by the R tile
// bits reg[0..R-1] (reg slot r <-> tile bit reg[r]).  Ops whose targets are
// register bits run without touching LDS; only phase boundaries re-shuffle
// the tile through LDS.  `lds` = 1 marks a fallback phase whose ops are
// applied directly on the LDS tile (ops that do not fit the register scheme).
struct TilePhase {
    int opBegin = 0, opEnd = 0;
    int lds = 0;
    int mat = -1;        // >= 0: dense block phase, matrix index in TileProgram::mats
    int reg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // tile bit carried by bit i of the thread index (the non-register bits,
    // ordered so that the 32 lanes of a half-wave hit 32 distinct LDS slots
    // under the GPU's XOR swizzle, see ldsSwizzle below)
    int lane[16] = {0};
};

// XOR swizzle of the GPU tile layout in LDS: element p of a tile lives at
// p ^ h(p >> 5).  With it, for (almost) any choice of register bits there is
// an assignment of lanes to the remaining bits that makes every 8-byte LDS
// access of a half-wave conflict-free (32 distinct 8-byte slots mod 256 B).
inline unsigned ldsSwizzleHash(unsigned hi) {
    unsigned h = hi & 31u;
    if ((hi >> 5) & 1u) h ^= 31u;
    if ((hi >> 6) & 1u) h ^= 21u;
    return h;
}
inline unsigned ldsSwizzle(unsigned p) { return p ^ ldsSwizzleHash(p >> 5); }

struct TilePass {
    int k = 0;           // tile qubits
    int pos[32];         // tile bit i -> physical bit position (ascending)
    // tile bit -> physical position it is STORED to: a permutation of pos
    // when the pass relabels qubits in place (planTiles relabelFrom >= 0);
    // later passes and the register's qubit map follow the new layout
    int stPos[32];
    u64 qmask = 0;       // physical mask of Q
    int opBegin = 0;     // range in the program's op array
    int opEnd = 0;
    int phaseBegin = 0;  // range in the program's phase array (0,0: no phases)
    int phaseEnd = 0;
};

struct TileProgram {
    std::vector<TilePass> passes;
    // physical position at the start of the program -> position at its end
    // (identity unless passes relabel); size L
    std::vector<int> perm;
    std::vector<TileOp> ops;
    std::vector<TilePhase> phases;
    // dense block matrices: 2^R x 2^R complex, row-major, interleaved re/im
    std::vector<real> mats;
};

// Fuse the ops of every pass with exactly `k` tile bits into dense blocks of
// at most R qubits (the product of the block's gates, computed on the host):
// each block is one register phase with one 2^R x 2^R matrix-vector product
// per thread, i.e. ONE LDS round trip however many gates it absorbed.  Ops
// with controls outside the tile, or more than R qubits, become LDS phases.
void planDenseBlocks(TileProgram& prog, int k, int R);

// Split every pass with exactly `k` tile bits (k < 0: every pass with more
// than R tile bits) into register phases of R slots (fills TileOp::rt and
// TileProgram::phases).
void planPhases(TileProgram& prog, int k, int R);

// Multiply runs of gates acting on at most two qubits into one 2x2 / 4x4
// matrix each (a run may interleave with gates on other qubits; ops keep
// their relative order where they do not commute).  Diagonal-only runs and
// single gates are left as they are.
void fuseGates(std::vector<Op>& ops);
// Gate-block fusion in planTiles (env QUEST_FUSE_BLOCKS=0 / setQuESTTuning
// "fuse_blocks" turn it off).
bool& fuseBlocks();
// Largest block fuseGates forms: 2 (4x4 blocks, default) or 1 (runs of
// one-qubit gates only; the wave engine keeps CNOTs and controls apart)
int& fuseBlockQubits();
// Most ops one fused pass takes (0: no limit; env QUEST_PLAN_MAX_OPS,
// setQuESTTuning "plan_max_ops").  A pass whose ops cost more VALU time than
// its HBM stream is compute-bound while the passes after it wait on memory;
// a cap moves the surplus into them.
int& planMaxOps();

// Split `ops` (physical local positions, L local qubits) into passes of at
// most kmax tile qubits (kmax >= cmin + 4).  With fuse=true ops are reordered
// where they commute to fill each pass (`ops` is left in execution order);
// with fuse=false every op gets its own pass, in order.
//
// relabelFrom >= 0 (wave engine): a pass of two or more ops may store its
// tile with the qubits permuted among the tile's positions >= relabelFrom,
// so that the qubits the rest of the queue needs soonest land on the low
// positions below cmin, which every later tile contains.  The remaining ops
// are remapped to the new layout and out.perm records the composition.
// Optional callbacks of planTiles.  relabelOk: a relabelling store layout
// for the pass just emitted is kept only if it accepts the pass with that
// layout (e.g. the wave engine can lower it).  passReady: called once per pass
// as soon as it is final (its store layout decided), in program order, with
// the scheduled ops so far (the pass's ops are order[opBegin, opEnd)) -- the
// backend launches it while the planner works on the next pass.
struct PlanHooks {
    std::function<bool(const TilePass&, const TileOp*)> relabelOk;
    std::function<void(const TileProgram&, int pass, const std::vector<Op>& order)> passReady;
    // lowPerm (relabelling plans): a permutation sigma of the always-resident
    // positions [relabelFrom, cmin) to compose with the pass's store layout
    // (every later tile holds all of them, so their order does not change the
    // plan) -- the wave engine picks the one that spares it transpositions at
    // the store.  Returns false to keep the layout.
    std::function<bool(const TilePass&, const TileOp*, int cmin, int* sigma)> lowPerm;
    // maxPasses > 0: stop after that many passes (a front flush: the pass is
    // planned with the whole queue as lookahead, the rest waits for more ops).
    // The ops not planned go to *leftover, in queue order, already in the
    // layout the planned passes leave (out.perm applied); `ops` then holds only
    // the planned ones.
    int maxPasses = 0;
    std::vector<Op>* leftover = nullptr;
    // Compute-aware passes (passCost set, memCost > 0): passCost predicts the
    // compute of a pass (e.g. wave issue cycles per tile, -1: unknown) and
    // memCost is the same measure of one pass's memory stream.  A pass whose
    // predicted compute exceeds memCost * (1 + costMargin) leaves some of its
    // ops that any later pass can take (phases, targets on always-resident
    // positions, nothing after them in the pass depending on them) to the
    // passes after it, which are memory-bound more often than not.
    std::function<double(const TilePass&, const TileOp*)> passCost;
    double memCost = 0;
    double costMargin = 0.1;
    // candidate passes seeded per pass (0: QUEST_PLAN_SEEDS, default 24) and
    // the one-pass lookahead weight (< 0: QUEST_PLAN_LOOKAHEAD, default 0):
    // knobs of the wave planner's strategy search (searchWavePlan)
    int seeds = 0;
    double lookahead = -1;
    // local positions no tile may take as padding (the victims of a qubit
    // swap about to run, router planSwap): passes whose ops do not target
    // them then leave them out, so the swap can overlap those passes
    u64 avoidMask = 0;
    // rollout scoring of candidate passes (-1: QUEST_PLAN_ROLLOUT, default 0;
    // 1: the greedy plan of the rest of the queue with first-use relabelling
    // counts the passes a candidate leaves) -- a strategy of the search
    int rollout = -1;
    // positions the first `firstAvoidPasses` passes of this plan keep out of
    // their tiles even as targets (ops targeting them wait for a later pass)
    u64 firstPassAvoid = 0;
    int firstAvoidPasses = 1;
};

void planTiles(std::vector<Op>& ops, int L, int kmax, int cmin, bool fuse, TileProgram& out, int relabelFrom = -1,
               const PlanHooks* hooks = nullptr);
// class-aware commutation in the pass scheduler for this thread's plans
// (-1: QUEST_PLAN_COMMUTE, default off; 0 off; 1 on) -- a strategy of the
// wave planner's search (searchWaveStrategy)
extern thread_local int t_planCommute;
// Whether any pass of the program stores with a permuted layout.
bool programRelabels(const TileProgram& prog);

// Physical chunk index of element p of tile T in a pass.
inline i64 tileBase(const TilePass& ps, i64 T, int L) {
    // insert the k tile bits as zeros into T (positions ascending)
    i64 base = T;
    for (int i = 0; i < ps.k; i++) {
        i64 low = base & (((i64)1 << ps.pos[i]) - 1);
        base = ((base >> ps.pos[i]) << (ps.pos[i] + 1)) | low;
    }
    (void)L;
    return base;
}

inline i64 tileOffset(const TilePass& ps, unsigned p) {
    i64 off = 0;
    for (int i = 0; i < ps.k; i++)
        if ((p >> i) & 1) off |= (i64)1 << ps.pos[i];
    return off;
}

}  // namespace qa
