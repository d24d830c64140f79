// Gate kernels for CDNA4 (gfx950): the LDS-tiled fused pass.
//
// One launch = one pass over the chunk (src/core/tiles.hpp).  Each 256-thread
// workgroup (4 waves of 64) walks tiles of 2^K amplitudes with a grid-stride
// loop.  Per tile:
//   1. load  : 16-byte vector loads (double2 / float4) of the re and im
//              arrays; the tile's lowest c >= 4 (fp64) bits are contiguous, so
//              every wave instruction reads whole 128-B lines.  The loads of
//              tile i+1 are issued into registers before tile i is processed;
//   2. ops   : the pass's gates run in *register phases*: each thread holds
//              2^R amplitudes (R = K - 8) spanning the phase's register bits,
//              and every gate whose target is a register bit is applied in
//              registers; only a phase change re-shuffles the tile through
//              LDS.  Controls and phase bits are per-element predicates inside
//              the tile and per-tile (wave-uniform) predicates outside it;
//   3. store : 16-byte vector stores back to HBM.
// The tile lives in LDS under an XOR swizzle (ldsSwizzle, tiles.hpp) and the
// host assigns lanes to tile bits so that every 8-byte LDS access of a
// half-wave hits 32 distinct slots.
//
// A pass of G fused gates costs one HBM read + write of the chunk instead of
// G (the reference launches one kernel per gate, QuEST_gpu.cu:586-592, whose
// pair loop reads 8-byte scalars from 128-thread blocks).
#include "qa_hip.h"

namespace qa {
namespace hipk {

namespace {

__device__ __forceinline__ unsigned ins0(unsigned x, int b) {
    unsigned low = x & ((1u << b) - 1u);
    return ((x >> b) << (b + 1)) | low;
}

__device__ __forceinline__ unsigned swz(unsigned p) {
    unsigned hi = p >> 5;
    unsigned h = hi & 31u;
    h ^= ((hi >> 5) & 1u) ? 31u : 0u;
    h ^= ((hi >> 6) & 1u) ? 21u : 0u;
    return p ^ h;
}

template <bool SW>
__device__ __forceinline__ unsigned li(unsigned p) {
    if constexpr (SW)
        return swz(p);
    else
        return p;
}

// ---------------------------------------------------------------------------
// ops applied directly on the LDS tile (generic kernel, and fallback phases)
// ---------------------------------------------------------------------------

// host-chosen element-bit swaps that make the op's lane -> element map free
// of LDS bank conflicts under the swizzle (tiles.hpp: laneSwaps)
template <bool SW>
__device__ __forceinline__ unsigned laneMap(unsigned p, const TileOp& op) {
    if constexpr (SW) {
        for (int s = 0; s < op.nsw; s++) {
            const unsigned a = op.swA[s], b = op.swB[s];
            const unsigned x = ((p >> a) ^ (p >> b)) & 1u;
            p ^= (x << a) | (x << b);
        }
    }
    return p;
}

template <typename T, bool SW>
__device__ __forceinline__ void applyMat2(T* __restrict__ sre, T* __restrict__ sim, unsigned n, const TileOp& op) {
    const int t = op.t[0];
    const unsigned cin = op.ctrlIn;
    const T m0r = (T)op.m[0], m0i = (T)op.m[1], m1r = (T)op.m[2], m1i = (T)op.m[3];
    const T m2r = (T)op.m[4], m2i = (T)op.m[5], m3r = (T)op.m[6], m3i = (T)op.m[7];
    for (unsigned j = threadIdx.x; j < (n >> 1); j += blockDim.x) {
        const unsigned p0 = laneMap<SW>(ins0(j, t), op);
        if ((p0 & cin) != cin) continue;
        const unsigned a0 = li<SW>(p0), a1 = li<SW>(p0 | (1u << t));
        const T r0 = sre[a0], i0 = sim[a0], r1 = sre[a1], i1 = sim[a1];
        sre[a0] = m0r * r0 - m0i * i0 + m1r * r1 - m1i * i1;
        sim[a0] = m0r * i0 + m0i * r0 + m1r * i1 + m1i * r1;
        sre[a1] = m2r * r0 - m2i * i0 + m3r * r1 - m3i * i1;
        sim[a1] = m2r * i0 + m2i * r0 + m3r * i1 + m3i * r1;
    }
}

template <typename T, bool SW>
__device__ __forceinline__ void applyDiag(T* __restrict__ sre, T* __restrict__ sim, unsigned n, const TileOp& op) {
    const unsigned cin = op.ctrlIn;
    const T tr = (T)op.m[0], ti = (T)op.m[1];
    for (unsigned p = threadIdx.x; p < n; p += blockDim.x) {
        if ((p & cin) != cin) continue;
        const unsigned a = li<SW>(p);
        const T r = sre[a], i = sim[a];
        sre[a] = tr * r - ti * i;
        sim[a] = tr * i + ti * r;
    }
}

template <typename T, bool SW>
__device__ __forceinline__ void applyMat4(T* __restrict__ sre, T* __restrict__ sim, unsigned n, const TileOp& op) {
    const int a = op.t[0], b = op.t[1];
    const int lo = a < b ? a : b, hi = a < b ? b : a;
    const unsigned cin = op.ctrlIn;
    for (unsigned j = threadIdx.x; j < (n >> 2); j += blockDim.x) {
        const unsigned p = laneMap<SW>(ins0(ins0(j, lo), hi), op);
        if ((p & cin) != cin) continue;
        unsigned idx[4];
        T vr[4], vi[4];
#pragma unroll
        for (int g = 0; g < 4; g++) {
            idx[g] = li<SW>(p | ((unsigned)(g & 1) << a) | ((unsigned)(g >> 1) << b));
            vr[g] = sre[idx[g]];
            vi[g] = sim[idx[g]];
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            T sr = 0, si = 0;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const T mr = (T)op.m[2 * (4 * r + c)], mi = (T)op.m[2 * (4 * r + c) + 1];
                sr += mr * vr[c] - mi * vi[c];
                si += mr * vi[c] + mi * vr[c];
            }
            sre[idx[r]] = sr;
            sim[idx[r]] = si;
        }
    }
}

template <typename T, bool SW>
__device__ __forceinline__ void applyDensChan2(T* __restrict__ sre, T* __restrict__ sim, unsigned n,
                                               const TileOp& op) {
    const int s0 = op.t[0], s1 = op.t[1], s2 = op.t[2], s3 = op.t[3];
    int s[4] = {s0, s1, s2, s3};
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 3 - i; j++)
            if (s[j] > s[j + 1]) {
                int tmp = s[j];
                s[j] = s[j + 1];
                s[j + 1] = tmp;
            }
    const T off = (T)op.m[0], keep = (T)op.m[2], mix = (T)op.m[4] * (T)0.25;
    for (unsigned j = threadIdx.x; j < (n >> 4); j += blockDim.x) {
        const unsigned p = ins0(ins0(ins0(ins0(j, s[0]), s[1]), s[2]), s[3]);
        T sr = 0, si = 0;
#pragma unroll
        for (int a = 0; a < 4; a++) {
            const unsigned d = li<SW>(p | ((unsigned)(a & 1) << s0) | ((unsigned)(a >> 1) << s1) |
                                      ((unsigned)(a & 1) << s2) | ((unsigned)(a >> 1) << s3));
            sr += sre[d];
            si += sim[d];
        }
#pragma unroll
        for (int e = 0; e < 16; e++) {
            const int a = e & 3, b = e >> 2;
            const unsigned i = li<SW>(p | ((unsigned)(e & 1) << s0) | ((unsigned)((e >> 1) & 1) << s1) |
                                      ((unsigned)((e >> 2) & 1) << s2) | ((unsigned)((e >> 3) & 1) << s3));
            if (a != b) {
                sre[i] *= off;
                sim[i] *= off;
            } else {
                sre[i] = keep * sre[i] + mix * sr;
                sim[i] = keep * sim[i] + mix * si;
            }
        }
    }
}

template <typename T, bool SW>
__device__ __forceinline__ void applyLdsOp(T* sre, T* sim, unsigned n, const TileOp& op) {
    switch ((OpKind)op.kind) {
        case OpKind::Mat2: applyMat2<T, SW>(sre, sim, n, op); break;
        case OpKind::Diag: applyDiag<T, SW>(sre, sim, n, op); break;
        case OpKind::Mat4: applyMat4<T, SW>(sre, sim, n, op); break;
        case OpKind::DensChan2: applyDensChan2<T, SW>(sre, sim, n, op); break;
    }
}

// ---------------------------------------------------------------------------
// ops on the swizzled tile of the compile-time kernel (N elements, 256
// threads).  Work item j = tid + 256 u of an op maps to element
// laneMap(ins0(.., targets)) and then to LDS word swz(.): every step is a
// bit permutation or XOR-linear, so the word of item u, member g is
//     swz(map(tid)) ^ swz(map(256 u) | g-bits)
// -- one per-thread base plus a wave-uniform (scalar) term: a single v_xor
// per access instead of recomputing the insertion and the swizzle.
// ---------------------------------------------------------------------------

template <typename T, unsigned N, unsigned TH>
__device__ __forceinline__ void mat2Tile(T* __restrict__ sre, T* __restrict__ sim, const TileOp& op) {
    constexpr int P = N / 2 / TH;
    static_assert(P <= 16, "TileOp::du holds 16 work-item groups");
    const int t = op.t[0];
    const unsigned cin = op.ctrlIn;
    const T m0r = (T)op.m[0], m0i = (T)op.m[1], m1r = (T)op.m[2], m1i = (T)op.m[3];
    const T m2r = (T)op.m[4], m2i = (T)op.m[5], m3r = (T)op.m[6], m3i = (T)op.m[7];
    const unsigned p0 = laneMap<true>(ins0(threadIdx.x, t), op);
    const unsigned a0 = swz(p0);
    const unsigned tb = swz(1u << t);
#pragma unroll
    for (int u = 0; u < P; u++) {
        const unsigned du = op.du[u];  // uniform, precomputed on the host
        if (((p0 ^ du) & cin) != cin) continue;
        const unsigned i0 = a0 ^ op.sdu[u], i1 = i0 ^ tb;
        const T r0 = sre[i0], im0 = sim[i0], r1 = sre[i1], im1 = sim[i1];
        sre[i0] = m0r * r0 - m0i * im0 + m1r * r1 - m1i * im1;
        sim[i0] = m0r * im0 + m0i * r0 + m1r * im1 + m1i * r1;
        sre[i1] = m2r * r0 - m2i * im0 + m3r * r1 - m3i * im1;
        sim[i1] = m2r * im0 + m2i * r0 + m3r * im1 + m3i * r1;
    }
}

template <typename T, unsigned N, unsigned TH>
__device__ __forceinline__ void mat4Tile(T* __restrict__ sre, T* __restrict__ sim, const TileOp& op) {
    constexpr int P = N / 4 / TH;
    static_assert(P <= 16, "TileOp::du holds 16 work-item groups");
    const int a = op.t[0], b = op.t[1];
    const int lo = a < b ? a : b, hi = a < b ? b : a;
    const unsigned cin = op.ctrlIn;
    const unsigned p0 = laneMap<true>(ins0(ins0(threadIdx.x, lo), hi), op);
    const unsigned a0 = swz(p0);
    const unsigned ga = swz(1u << a), gb = swz(1u << b);
#pragma unroll
    for (int u = 0; u < P; u++) {
        const unsigned du = op.du[u];  // uniform, precomputed on the host
        if (((p0 ^ du) & cin) != cin) continue;
        const unsigned b0 = a0 ^ op.sdu[u];
        const unsigned idx[4] = {b0, b0 ^ ga, b0 ^ gb, b0 ^ ga ^ gb};
        T vr[4], vi[4];
#pragma unroll
        for (int g = 0; g < 4; g++) {
            vr[g] = sre[idx[g]];
            vi[g] = sim[idx[g]];
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            T sr = 0, si = 0;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const T mr = (T)op.m[2 * (4 * r + c)], mi = (T)op.m[2 * (4 * r + c) + 1];
                sr += mr * vr[c] - mi * vi[c];
                si += mr * vi[c] + mi * vr[c];
            }
            sre[idx[r]] = sr;
            sim[idx[r]] = si;
        }
    }
}

template <typename T, unsigned N, unsigned TH>
__device__ __forceinline__ void diagTile(T* __restrict__ sre, T* __restrict__ sim, const TileOp& op) {
    constexpr int P = N / TH;
    const unsigned cin = op.ctrlIn;
    const T tr = (T)op.m[0], ti = (T)op.m[1];
    const unsigned a0 = swz(threadIdx.x);
#pragma unroll
    for (int u = 0; u < P; u++) {
        const unsigned p = threadIdx.x + TH * u;
        if ((p & cin) != cin) continue;
        const unsigned i = a0 ^ swz(TH * u);  // compile-time constant
        const T r = sre[i], im = sim[i];
        sre[i] = tr * r - ti * im;
        sim[i] = tr * im + ti * r;
    }
}

template <typename T, unsigned N, unsigned TH>
__device__ __forceinline__ void applyTileOp(T* sre, T* sim, const TileOp& op) {
    switch ((OpKind)op.kind) {
        case OpKind::Mat2: mat2Tile<T, N, TH>(sre, sim, op); break;
        case OpKind::Diag: diagTile<T, N, TH>(sre, sim, op); break;
        case OpKind::Mat4: mat4Tile<T, N, TH>(sre, sim, op); break;
        case OpKind::DensChan2: applyDensChan2<T, true>(sre, sim, N, op); break;
    }
}

// ---------------------------------------------------------------------------
// generic tile kernel: any tile size (small chunks), no swizzle, op by op
// ---------------------------------------------------------------------------

template <typename T, bool VEC>
__global__ __launch_bounds__(256) void tilePassKernel(T* __restrict__ re, T* __restrict__ im, TileArgs a,
                                                      const TileOp* __restrict__ ops) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int k = a.k, c = a.c;
    const unsigned n = 1u << k;
    T* sre = reinterpret_cast<T*>(smem);
    T* sim = sre + n;
    long long* hiOff = reinterpret_cast<long long*>(sim + n);
    const int nh = 1 << (k - c);
    for (int h = threadIdx.x; h < nh; h += blockDim.x) {
        long long off = 0;
        for (int i = c; i < k; i++)
            if ((h >> (i - c)) & 1) off |= 1ll << a.pos[i];
        hiOff[h] = off;
    }
    __syncthreads();

    using V = typename Vec16<T>::type;
    constexpr int VN = VEC ? Vec16<T>::n : 1;
    const unsigned lowMask = (1u << c) - 1u;

    for (long long tile = blockIdx.x; tile < a.numTiles; tile += gridDim.x) {
        long long base = tile;
        for (int i = 0; i < k; i++) {
            const int p = a.pos[i];
            const long long low = base & ((1ll << p) - 1);
            base = ((base >> p) << (p + 1)) | low;
        }
        for (unsigned u = threadIdx.x; u < n / VN; u += blockDim.x) {
            const unsigned p = u * VN;
            const long long g = base + (p & lowMask) + hiOff[p >> c];
            if constexpr (VEC) {
                *reinterpret_cast<V*>(sre + p) = *reinterpret_cast<const V*>(re + g);
                *reinterpret_cast<V*>(sim + p) = *reinterpret_cast<const V*>(im + g);
            } else {
                sre[p] = re[g];
                sim[p] = im[g];
            }
        }
        __syncthreads();
        for (int o = 0; o < a.nOps; o++) {
            const TileOp& op = ops[o];
            if (((unsigned long long)base & op.ctrlOut) != op.ctrlOut) continue;  // uniform per tile
            applyLdsOp<T, false>(sre, sim, n, op);
            __syncthreads();
        }
        for (unsigned u = threadIdx.x; u < n / VN; u += blockDim.x) {
            const unsigned p = u * VN;
            const long long g = base + (p & lowMask) + hiOff[p >> c];
            if constexpr (VEC) {
                *reinterpret_cast<V*>(re + g) = *reinterpret_cast<const V*>(sre + p);
                *reinterpret_cast<V*>(im + g) = *reinterpret_cast<const V*>(sim + p);
            } else {
                re[g] = sre[p];
                im[g] = sim[p];
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// register phases
// ---------------------------------------------------------------------------

template <typename T, int R, int A>
__device__ __forceinline__ void regMat2(T (&vr)[1 << R], T (&vi)[1 << R], const unsigned (&idx)[1 << R],
                                        const TileOp& op) {
    const unsigned cin = op.ctrlIn;
    const T m0r = (T)op.m[0], m0i = (T)op.m[1], m1r = (T)op.m[2], m1i = (T)op.m[3];
    const T m2r = (T)op.m[4], m2i = (T)op.m[5], m3r = (T)op.m[6], m3i = (T)op.m[7];
#pragma unroll
    for (int j = 0; j < (1 << R); j++) {
        if ((j >> A) & 1) continue;
        const int f = j | (1 << A);
        if ((idx[j] & cin) != cin) continue;
        const T r0 = vr[j], i0 = vi[j], r1 = vr[f], i1 = vi[f];
        vr[j] = m0r * r0 - m0i * i0 + m1r * r1 - m1i * i1;
        vi[j] = m0r * i0 + m0i * r0 + m1r * i1 + m1i * r1;
        vr[f] = m2r * r0 - m2i * i0 + m3r * r1 - m3i * i1;
        vi[f] = m2r * i0 + m2i * r0 + m3r * i1 + m3i * r1;
    }
}

// Mat4 targets are pinned to register slots 0 (low) and 1 by the planner
template <typename T, int R>
__device__ __forceinline__ void regMat4(T (&vr)[1 << R], T (&vi)[1 << R], const unsigned (&idx)[1 << R],
                                        const TileOp& op) {
    const unsigned cin = op.ctrlIn;
#pragma unroll
    for (int j = 0; j < (1 << R); j += 4) {
        if ((idx[j] & cin) != cin) continue;
        T xr[4], xi[4];
#pragma unroll
        for (int g = 0; g < 4; g++) {
            xr[g] = vr[j + g];
            xi[g] = vi[j + g];
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            T sr = 0, si = 0;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const T mr = (T)op.m[2 * (4 * r + c)], mi = (T)op.m[2 * (4 * r + c) + 1];
                sr += mr * xr[c] - mi * xi[c];
                si += mr * xi[c] + mi * xr[c];
            }
            vr[j + r] = sr;
            vi[j + r] = si;
        }
    }
}

// DensChan2 targets pinned to slots 0..3: element e of each 16-group is j + e
template <typename T, int R>
__device__ __forceinline__ void regChan2(T (&vr)[1 << R], T (&vi)[1 << R], const TileOp& op) {
    const T off = (T)op.m[0], keep = (T)op.m[2], mix = (T)op.m[4] * (T)0.25;
#pragma unroll
    for (int j = 0; j < (1 << R); j += 16) {
        const T sr = vr[j] + vr[j + 5] + vr[j + 10] + vr[j + 15];
        const T si = vi[j] + vi[j + 5] + vi[j + 10] + vi[j + 15];
#pragma unroll
        for (int e = 0; e < 16; e++) {
            if ((e & 3) != (e >> 2)) {
                vr[j + e] *= off;
                vi[j + e] *= off;
            } else {
                vr[j + e] = keep * vr[j + e] + mix * sr;
                vi[j + e] = keep * vi[j + e] + mix * si;
            }
        }
    }
}

template <typename T, int K, int R>
__device__ __forceinline__ void runRegPhase(T* __restrict__ sre, T* __restrict__ sim, const TilePhase& ph,
                                            const TileOp* __restrict__ ops, unsigned long long base) {
    constexpr int M = 1 << R;
    unsigned ro[R];
#pragma unroll
    for (int r = 0; r < R; r++) ro[r] = 1u << ph.reg[r];
    unsigned tb = 0;
#pragma unroll
    for (int i = 0; i < K - R; i++) tb |= ((threadIdx.x >> i) & 1u) << ph.lane[i];
    unsigned idx[M];
    T vr[M], vi[M];
#pragma unroll
    for (int j = 0; j < M; j++) {
        unsigned o = 0;
#pragma unroll
        for (int r = 0; r < R; r++)
            if ((j >> r) & 1) o |= ro[r];
        idx[j] = tb | o;
        const unsigned a = swz(idx[j]);
        vr[j] = sre[a];
        vi[j] = sim[a];
    }
    for (int o = ph.opBegin; o < ph.opEnd; o++) {
        const TileOp& op = ops[o];
        if ((base & op.ctrlOut) != op.ctrlOut) continue;
        switch ((OpKind)op.kind) {
            case OpKind::Mat2: {
                // an if-chain of explicit instantiations keeps vr/vi in
                // registers (a recursive dispatch pushed them to scratch)
                const int a = op.rt[0];
                if (a == 0)
                    regMat2<T, R, 0>(vr, vi, idx, op);
                else if (a == 1)
                    regMat2<T, R, 1>(vr, vi, idx, op);
                else if (a == 2)
                    regMat2<T, R, 2>(vr, vi, idx, op);
                else if constexpr (R > 3)
                    regMat2<T, R, (R > 3 ? 3 : 0)>(vr, vi, idx, op);
                break;
            }
            case OpKind::Diag: {
                const unsigned cin = op.ctrlIn;
                const T tr = (T)op.m[0], ti = (T)op.m[1];
#pragma unroll
                for (int j = 0; j < M; j++) {
                    if ((idx[j] & cin) != cin) continue;
                    const T x = vr[j], y = vi[j];
                    vr[j] = tr * x - ti * y;
                    vi[j] = tr * y + ti * x;
                }
                break;
            }
            case OpKind::Mat4: regMat4<T, R>(vr, vi, idx, op); break;
            case OpKind::DensChan2:
                if constexpr (R >= 4) regChan2<T, R>(vr, vi, op);
                break;
        }
    }
#pragma unroll
    for (int j = 0; j < M; j++) {
        const unsigned a = swz(idx[j]);
        sre[a] = vr[j];
        sim[a] = vi[j];
    }
}

// Dense block phase: y = U x on the thread's 2^R amplitudes, U composed on
// the host from every gate of the block (uniform -> scalar loads).
template <typename T, int K, int R>
__device__ __forceinline__ void runDensePhase(T* __restrict__ sre, T* __restrict__ sim, const TilePhase& ph,
                                              const real* __restrict__ mats) {
    constexpr int M = 1 << R;
    unsigned ro[R];
#pragma unroll
    for (int r = 0; r < R; r++) ro[r] = 1u << ph.reg[r];
    unsigned tb = 0;
#pragma unroll
    for (int i = 0; i < K - R; i++) tb |= ((threadIdx.x >> i) & 1u) << ph.lane[i];
    unsigned addr[M];
    T xr[M], xi[M];
#pragma unroll
    for (int j = 0; j < M; j++) {
        unsigned o = 0;
#pragma unroll
        for (int r = 0; r < R; r++)
            if ((j >> r) & 1) o |= ro[r];
        addr[j] = swz(tb | o);
        xr[j] = sre[addr[j]];
        xi[j] = sim[addr[j]];
    }
    const real* U = mats + (size_t)ph.mat * 2 * M * M;
#pragma unroll
    for (int r = 0; r < M; r++) {
        T sr = 0, si = 0;
#pragma unroll
        for (int c = 0; c < M; c++) {
            const T ur = (T)U[2 * (r * M + c)], ui = (T)U[2 * (r * M + c) + 1];
            sr += ur * xr[c] - ui * xi[c];
            si += ur * xi[c] + ui * xr[c];
        }
        sre[addr[r]] = sr;
        sim[addr[r]] = si;
    }
}

// 16-byte vector of tile elements p..p+VN-1 (p aligned) to / from the
// swizzled LDS tile: the group stays one aligned vector, its element order
// permuted by x = swz(p) mod VN
// element permutation e -> e ^ x with selects only (a runtime index into a
// vector would be lowered to scratch memory)
__device__ __forceinline__ double2 xorPerm(double2 v, unsigned x) {
    double2 w;
    w.x = (x & 1u) ? v.y : v.x;
    w.y = (x & 1u) ? v.x : v.y;
    return w;
}

__device__ __forceinline__ float4 xorPerm(float4 v, unsigned x) {
    float4 a;  // swap neighbours if bit 0
    a.x = (x & 1u) ? v.y : v.x;
    a.y = (x & 1u) ? v.x : v.y;
    a.z = (x & 1u) ? v.w : v.z;
    a.w = (x & 1u) ? v.z : v.w;
    float4 b;  // swap pairs if bit 1
    b.x = (x & 2u) ? a.z : a.x;
    b.y = (x & 2u) ? a.w : a.y;
    b.z = (x & 2u) ? a.x : a.z;
    b.w = (x & 2u) ? a.y : a.w;
    return b;
}

template <typename T>
__device__ __forceinline__ void ldsPutVec(T* s, unsigned p, typename Vec16<T>::type v) {
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::n;
    const unsigned q = swz(p);
    *reinterpret_cast<V*>(s + (q & ~(unsigned)(VN - 1))) = xorPerm(v, q & (VN - 1));
}

template <typename T>
__device__ __forceinline__ typename Vec16<T>::type ldsGetVec(const T* s, unsigned p) {
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::n;
    const unsigned q = swz(p);
    return xorPerm(*reinterpret_cast<const V*>(s + (q & ~(unsigned)(VN - 1))), q & (VN - 1));
}

// Tile kernel with the tile size fixed at compile time (every chunk of at
// least 2^(K+7) amplitudes).  Each thread owns U = 2^K/VN/256 16-byte
// vectors per array for the HBM <-> LDS moves.
// MODE 0: ops one by one on LDS; 1: register phases; 2: dense blocks
template <typename T, int K, int MODE>
__global__ __launch_bounds__(tileThreads(K), (MODE == 1 || K > kTileQubits) ? 2 : 4) void tilePassKernelK(T* __restrict__ re, T* __restrict__ im, TileArgs a,
                                                       const TileOp* __restrict__ ops,
                                                       const TilePhase* __restrict__ phases,
                                                       const real* __restrict__ mats) {
    constexpr unsigned TH = tileThreads(K);
    constexpr int R = K - 8;  // 256 threads x 2^R = 2^K (register phases: TH = 256)
    constexpr bool PHASES = MODE != 0;
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::n;
    constexpr unsigned N = 1u << K;
    constexpr int U = N / VN / TH;
    static_assert(U >= 1, "tile too small for the vector layout");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* sre = reinterpret_cast<T*>(smem);
    T* sim = sre + N;
    long long* hiOff = reinterpret_cast<long long*>(sim + N);
    const int c = a.c;
    const int nh = 1 << (K - c);
    for (int h = threadIdx.x; h < nh; h += TH) {
        long long off = 0;
        for (int i = c; i < K; i++)
            if ((h >> (i - c)) & 1) off |= 1ll << a.pos[i];
        hiOff[h] = off;
    }
    __syncthreads();
    const unsigned lowMask = (1u << c) - 1u;

    long long off[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const unsigned p = (threadIdx.x + TH * u) * VN;
        off[u] = (long long)(p & lowMask) + hiOff[p >> c];
    }

    auto tileBaseOf = [&](long long tile) {
        long long base = tile;
        for (int i = 0; i < K; i++) {
            const int p = a.pos[i];
            const long long low = base & ((1ll << p) - 1);
            base = ((base >> p) << (p + 1)) | low;
        }
        return base;
    };

    // Software pipeline, one tile ahead: the loads of tile i+1 are issued
    // before the ops of tile i and are only consumed (register -> LDS) after
    // the stores of tile i, in the same iteration, so the wait on them leaves
    // those stores in flight.  The prefetch is branch-free (the last
    // iteration re-reads its own tile) to keep the vmcnt accounting exact.
    V rr[U], ri[U];
    long long tile = blockIdx.x;
    if (tile >= a.numTiles) return;
    long long base = tileBaseOf(tile);
#pragma unroll
    for (int u = 0; u < U; u++) {
        rr[u] = streamLoad(reinterpret_cast<const V*>(re + base + off[u]));
        ri[u] = streamLoad(reinterpret_cast<const V*>(im + base + off[u]));
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const unsigned p = (threadIdx.x + TH * u) * VN;
        ldsPutVec<T>(sre, p, rr[u]);
        ldsPutVec<T>(sim, p, ri[u]);
    }
    __syncthreads();
    for (; tile < a.numTiles; tile += gridDim.x) {
        const long long next = tile + gridDim.x;
        const long long nbase = next < a.numTiles ? tileBaseOf(next) : base;
#pragma unroll
        for (int u = 0; u < U; u++) {
            rr[u] = streamLoad(reinterpret_cast<const V*>(re + nbase + off[u]));
            ri[u] = streamLoad(reinterpret_cast<const V*>(im + nbase + off[u]));
        }
        if constexpr (PHASES) {
            for (int h = 0; h < a.nPhases; h++) {
                const TilePhase& ph = phases[h];
                if (ph.lds) {
                    for (int o = ph.opBegin; o < ph.opEnd; o++) {
                        const TileOp& op = ops[o];
                        if (((unsigned long long)base & op.ctrlOut) != op.ctrlOut) continue;
                        applyTileOp<T, N, TH>(sre, sim, op);
                        __syncthreads();
                    }
                } else if constexpr (MODE == 2) {
                    runDensePhase<T, K, R>(sre, sim, ph, mats);
                    __syncthreads();
                } else {
                    runRegPhase<T, K, R>(sre, sim, ph, ops, (unsigned long long)base);
                    __syncthreads();
                }
            }
        } else {
            for (int o = 0; o < a.nOps; o++) {
                const TileOp& op = ops[o];
                if (((unsigned long long)base & op.ctrlOut) != op.ctrlOut) continue;
                applyTileOp<T, N, TH>(sre, sim, op);
                __syncthreads();
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const unsigned p = (threadIdx.x + TH * u) * VN;
            streamStore(reinterpret_cast<V*>(re + base + off[u]), ldsGetVec<T>(sre, p));
            streamStore(reinterpret_cast<V*>(im + base + off[u]), ldsGetVec<T>(sim, p));
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < U; u++) {
            const unsigned p = (threadIdx.x + TH * u) * VN;
            ldsPutVec<T>(sre, p, rr[u]);
            ldsPutVec<T>(sim, p, ri[u]);
        }
        __syncthreads();
        base = nbase;
    }
}

}  // namespace

void launchTilePass(real* re, real* im, const TileArgs& a, const TileOp* dOps, const TilePhase* dPhases,
                    const real* dMats, int mode) {
    const unsigned n = 1u << a.k;
    const size_t lds = 2 * n * sizeof(real) + sizeof(long long) * (1u << (a.k - a.c));
    const long long maxGrid = (long long)numCUs() * 8;
    const int grid = (int)(a.numTiles < maxGrid ? a.numTiles : maxGrid);
    const int vecBits = sizeof(real) == 8 ? 1 : 2;
    if (a.k == kTileQubits && a.c >= vecBits) {
        // register phases: ~170 VGPRs -> 2 resident workgroups per CU; op by
        // op / dense blocks: <= 128 VGPRs -> LDS-limited at 4 per CU
        if (a.nPhases == 0) mode = 0;
        long long perCU = mode == 1 ? tuning().tileWgPerCU : 4;
        if (perCU <= 0) perCU = 2;
        const long long g2 = a.numTiles < (long long)numCUs() * perCU ? a.numTiles : (long long)numCUs() * perCU;
        if (mode == 2)
            hipLaunchKernelGGL((tilePassKernelK<real, kTileQubits, 2>), dim3((int)g2), dim3(256), lds, stream(), re,
                               im, a, dOps, dPhases, dMats);
        else if (mode == 1)
            hipLaunchKernelGGL((tilePassKernelK<real, kTileQubits, 1>), dim3((int)g2), dim3(256), lds, stream(), re,
                               im, a, dOps, dPhases, dMats);
        else
            hipLaunchKernelGGL((tilePassKernelK<real, kTileQubits, 0>), dim3((int)g2), dim3(256), lds, stream(), re,
                               im, a, dOps, dPhases, dMats);
    } else if (a.k == kTileQubits + 1 && a.c >= vecBits && a.nPhases == 0) {
        // double tile (64 KiB of LDS): op by op, 2 resident workgroups per CU
        const long long g2 = a.numTiles < (long long)numCUs() * 2 ? a.numTiles : (long long)numCUs() * 2;
        hipLaunchKernelGGL((tilePassKernelK<real, kTileQubits + 1, 0>), dim3((int)g2),
                           dim3(tileThreads(kTileQubits + 1)), lds, stream(), re,
                           im, a, dOps, dPhases, dMats);
    } else if (a.c >= vecBits) {
        hipLaunchKernelGGL((tilePassKernel<real, true>), dim3(grid), dim3(256), lds, stream(), re, im, a, dOps);
    } else {
        hipLaunchKernelGGL((tilePassKernel<real, false>), dim3(grid), dim3(256), lds, stream(), re, im, a, dOps);
    }
    QA_HIP_CHECK(hipGetLastError());
}

}  // namespace hipk
}  // namespace qa
