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

#include <vector>

#include "core.hpp"

namespace qa {

// One op in tile-local coordinates.  Plain data: uploaded as-is to the GPU.
struct TileOp {
    int kind;            // OpKind
    int t[4];            // tile-local target bits
    unsigned ctrlIn;     // tile-local mask of bits that must be 1
    unsigned pad;
    u64 ctrlOut;         // physical bits outside the tile that must be 1
    real m[32];          // matrix, interleaved re/im, row-major
};

struct TilePass {
    int k = 0;           // tile qubits
    int pos[32];         // tile bit i -> physical bit position (ascending)
    u64 qmask = 0;       // physical mask of Q
    int opBegin = 0;     // range in the program's op array
    int opEnd = 0;
};

struct TileProgram {
    std::vector<TilePass> passes;
    std::vector<TileOp> ops;
};

// Split `ops` (physical local positions, L local qubits) into passes of at
// most kmax tile qubits (kmax >= cmin + 4).  With fuse=false every op gets its
// own pass.
void planTiles(const std::vector<Op>& ops, int L, int kmax, int cmin, bool fuse, TileProgram& out);

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
