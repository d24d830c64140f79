// Gate kernels for CDNA4 (gfx950): the LDS-tiled fused pass.
//
// One launch = one pass over the chunk (src/core/tiles.hpp).  Each 256-thread
// workgroup (4 waves of 64) walks tiles of 2^k amplitudes with a grid-stride
// loop.  Per tile:
//   1. load  : 16-byte vector loads (double2 / float4) of the re and im
//              arrays; the tile's lowest c >= 4 (fp64) bits are contiguous, so
//              every wave instruction reads whole 128-B lines;
//   2. ops   : every queued gate of the pass is applied to the LDS copy in
//              program order, one __syncthreads() between ops; controls and
//              phase bits outside the tile are a per-tile (wave-uniform)
//              predicate, so a tile failing a control skips the op entirely;
//   3. store : 16-byte vector stores back to HBM.
// So a pass of G fused gates costs one HBM read + write of the chunk instead
// of G (the reference launches one kernel per gate, QuEST_gpu.cu:586-592, and
// its pair loop reads 8-byte scalars with a 128-thread block).
#include "qa_hip.h"

namespace qa {
namespace hipk {

namespace {

__device__ __forceinline__ unsigned ins0(unsigned x, int b) {
    unsigned low = x & ((1u << b) - 1u);
    return ((x >> b) << (b + 1)) | low;
}

template <typename T>
__device__ __forceinline__ void applyMat2(T* __restrict__ sre, T* __restrict__ sim, unsigned n, const TileOp& op) {
    const int t = op.t[0];
    const unsigned cin = op.ctrlIn;
    const T m0r = (T)op.m[0], m0i = (T)op.m[1], m1r = (T)op.m[2], m1i = (T)op.m[3];
    const T m2r = (T)op.m[4], m2i = (T)op.m[5], m3r = (T)op.m[6], m3i = (T)op.m[7];
    for (unsigned j = threadIdx.x; j < (n >> 1); j += blockDim.x) {
        const unsigned p0 = ins0(j, t);
        if ((p0 & cin) != cin) continue;
        const unsigned p1 = p0 | (1u << t);
        const T r0 = sre[p0], i0 = sim[p0], r1 = sre[p1], i1 = sim[p1];
        sre[p0] = m0r * r0 - m0i * i0 + m1r * r1 - m1i * i1;
        sim[p0] = m0r * i0 + m0i * r0 + m1r * i1 + m1i * r1;
        sre[p1] = m2r * r0 - m2i * i0 + m3r * r1 - m3i * i1;
        sim[p1] = m2r * i0 + m2i * r0 + m3r * i1 + m3i * r1;
    }
}

template <typename T>
__device__ __forceinline__ void applyDiag(T* __restrict__ sre, T* __restrict__ sim, unsigned n, const TileOp& op) {
    const unsigned cin = op.ctrlIn;
    const T tr = (T)op.m[0], ti = (T)op.m[1];
    for (unsigned p = threadIdx.x; p < n; p += blockDim.x) {
        if ((p & cin) != cin) continue;
        const T r = sre[p], i = sim[p];
        sre[p] = tr * r - ti * i;
        sim[p] = tr * i + ti * r;
    }
}

template <typename T>
__device__ __forceinline__ void applyMat4(T* __restrict__ sre, T* __restrict__ sim, unsigned n, const TileOp& op) {
    const int a = op.t[0], b = op.t[1];
    const int lo = a < b ? a : b, hi = a < b ? b : a;
    const unsigned cin = op.ctrlIn;
    for (unsigned j = threadIdx.x; j < (n >> 2); j += blockDim.x) {
        const unsigned p = ins0(ins0(j, lo), hi);
        if ((p & cin) != cin) continue;
        unsigned idx[4];
        T vr[4], vi[4];
#pragma unroll
        for (int g = 0; g < 4; g++) {
            idx[g] = p | ((unsigned)(g & 1) << a) | ((unsigned)(g >> 1) << b);
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

template <typename T>
__device__ __forceinline__ void applyDensChan2(T* __restrict__ sre, T* __restrict__ sim, unsigned n,
                                               const TileOp& op) {
    int s0 = op.t[0], s1 = op.t[1], s2 = op.t[2], s3 = op.t[3];
    // sort the four positions (uniform, tiny)
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
        // diagonal-type elements (row bits == col bits): e = a + 4a
        unsigned d[4];
        T sr = 0, si = 0;
#pragma unroll
        for (int a = 0; a < 4; a++) {
            d[a] = p | ((unsigned)(a & 1) << s0) | ((unsigned)(a >> 1) << s1) | ((unsigned)(a & 1) << s2) |
                   ((unsigned)(a >> 1) << s3);
            sr += sre[d[a]];
            si += sim[d[a]];
        }
#pragma unroll
        for (int e = 0; e < 16; e++) {
            const int a = e & 3, b = e >> 2;
            const unsigned i = p | ((unsigned)(e & 1) << s0) | ((unsigned)((e >> 1) & 1) << s1) |
                               ((unsigned)((e >> 2) & 1) << s2) | ((unsigned)((e >> 3) & 1) << s3);
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
        // ---- load tile ----
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
        // ---- apply the pass's ops ----
        for (int o = 0; o < a.nOps; o++) {
            const TileOp& op = ops[o];
            if (((unsigned long long)base & op.ctrlOut) != op.ctrlOut) continue;  // uniform per tile
            switch ((OpKind)op.kind) {
                case OpKind::Mat2: applyMat2<T>(sre, sim, n, op); break;
                case OpKind::Diag: applyDiag<T>(sre, sim, n, op); break;
                case OpKind::Mat4: applyMat4<T>(sre, sim, n, op); break;
                case OpKind::DensChan2: applyDensChan2<T>(sre, sim, n, op); break;
            }
            __syncthreads();
        }
        // ---- store tile ----
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

}  // namespace

void launchTilePass(real* re, real* im, const TileArgs& a, const TileOp* dOps) {
    const unsigned n = 1u << a.k;
    const size_t lds = 2 * n * sizeof(real) + sizeof(long long) * (1u << (a.k - a.c));
    const long long maxGrid = (long long)numCUs() * 8;
    const int grid = (int)(a.numTiles < maxGrid ? a.numTiles : maxGrid);
    const int vecBits = sizeof(real) == 8 ? 1 : 2;
    if (a.c >= vecBits)
        hipLaunchKernelGGL((tilePassKernel<real, true>), dim3(grid), dim3(256), lds, stream(), re, im, a, dOps);
    else
        hipLaunchKernelGGL((tilePassKernel<real, false>), dim3(grid), dim3(256), lds, stream(), re, im, a, dOps);
    QA_HIP_CHECK(hipGetLastError());
}

}  // namespace hipk
}  // namespace qa
