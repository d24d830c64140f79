#include "tiles.hpp"

#include <algorithm>
#include <cstring>

namespace qa {

namespace {

u64 targetMask(const Op& op) {
    u64 m = 0;
    for (int i = 0; i < op.nt; i++) m |= 1ull << op.t[i];
    return m;
}

int popcount64(u64 x) { return __builtin_popcountll(x); }

void emitPass(const std::vector<Op>& ops, int b, int e, u64 tmask, int L, int k, int cmin, TileProgram& out) {
    TilePass ps;
    ps.k = k;
    // Q = low cmin bits + targets, padded with the lowest remaining bits
    u64 q = tmask | ((cmin >= 64) ? ~0ull : ((1ull << cmin) - 1));
    for (int bit = 0; popcount64(q) < k && bit < L; bit++) q |= 1ull << bit;
    ps.qmask = q;
    int n = 0;
    int tileOf[64];
    for (int bit = 0; bit < L; bit++) {
        tileOf[bit] = -1;
        if ((q >> bit) & 1) {
            tileOf[bit] = n;
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
        int nm = op.kind == OpKind::Mat2 ? 4 : op.kind == OpKind::Mat4 ? 16 : op.kind == OpKind::Diag ? 1 : 3;
        for (int j = 0; j < nm; j++) {
            t.m[2 * j] = op.m[j].re;
            t.m[2 * j + 1] = op.m[j].im;
        }
        out.ops.push_back(t);
    }
    ps.opEnd = (int)out.ops.size();
    out.passes.push_back(ps);
}

}  // namespace

void planTiles(const std::vector<Op>& ops, int L, int kmax, int cmin, bool fuse, TileProgram& out) {
    out.passes.clear();
    out.ops.clear();
    if (ops.empty()) return;
    const int k = std::min(kmax, L);
    const int c = std::min(cmin, k);
    const u64 low = (c >= 64) ? ~0ull : ((1ull << c) - 1);
    // high targets allowed per pass besides the always-present low bits
    const int highSlots = k - c;

    int begin = 0;
    u64 cur = 0;
    for (int i = 0; i < (int)ops.size(); i++) {
        u64 tm = targetMask(ops[i]);
        u64 merged = cur | tm;
        bool fits = popcount64(merged & ~low) <= highSlots;
        if (i > begin && (!fuse || !fits)) {
            emitPass(ops, begin, i, cur, L, k, c, out);
            begin = i;
            cur = tm;
        } else {
            cur = merged;
        }
    }
    emitPass(ops, begin, (int)ops.size(), cur, L, k, c, out);
}

}  // namespace qa
