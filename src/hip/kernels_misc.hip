// State preparation, distributed pack/unpack and elementwise kernels.
// All grid-stride, 256 threads, 16-byte vector accesses where the layout
// allows; launched on the backend stream.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include <type_traits>

#include "qa_hip.h"

namespace qa {
namespace hipk {

namespace {

constexpr int kThreads = 256;

int gridFor(long long work) {
    long long g = (work + kThreads - 1) / kThreads;
    long long mx = (long long)numCUs() * 16;
    if (g > mx) g = mx;
    if (g < 1) g = 1;
    return (int)g;
}

__device__ __forceinline__ long long ins0(long long x, int b) {
    long long low = x & ((1ll << b) - 1);
    return ((x >> b) << (b + 1)) | low;
}

template <typename T>
__global__ __launch_bounds__(kThreads) void fillKernel(T* __restrict__ re, T* __restrict__ im, long long n, T vr,
                                                       T vi) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        re[i] = vr;
        im[i] = vi;
    }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void debugKernel(T* __restrict__ re, T* __restrict__ im, long long n,
                                                        long long offset) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const long long g = offset + i;
        re[i] = (T)((g * 2.0) / 10.0);
        im[i] = (T)((g * 2.0 + 1.0) / 10.0);
    }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void fillBitKernel(T* __restrict__ re, T* __restrict__ im, long long n,
                                                          int bit, int outcome, T val) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        re[i] = (((i >> bit) & 1) == outcome) ? val : (T)0;
        im[i] = 0;
    }
}

// Bit positions inserted into a packed index (ascending) and the values
// they take.
struct PackBits {
    int k;
    int pos[8];
    long long setMask;
};

// gather (UNPACK=false) / scatter (UNPACK=true) of the amplitudes whose bits
// pos[] equal those of setMask; VN consecutive items per thread when the
// lowest inserted bit is above the vector width
template <typename T, bool UNPACK, bool VEC>
__global__ __launch_bounds__(kThreads) void packKernel(T* __restrict__ re, T* __restrict__ im, PackBits pb,
                                                       long long start, long long count, T* __restrict__ br,
                                                       T* __restrict__ bi) {
    using V = typename Vec16<T>::type;
    constexpr int VN = VEC ? Vec16<T>::n : 1;
    const long long units = count / VN;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long u = (long long)blockIdx.x * blockDim.x + threadIdx.x; u < units; u += stride) {
        const long long j = u * VN;
        long long i = start + j;
        for (int m = 0; m < pb.k; m++) i = ins0(i, pb.pos[m]);
        i |= pb.setMask;
        if constexpr (VEC) {
            if constexpr (UNPACK) {
                *reinterpret_cast<V*>(re + i) = *reinterpret_cast<const V*>(br + j);
                *reinterpret_cast<V*>(im + i) = *reinterpret_cast<const V*>(bi + j);
            } else {
                *reinterpret_cast<V*>(br + j) = *reinterpret_cast<const V*>(re + i);
                *reinterpret_cast<V*>(bi + j) = *reinterpret_cast<const V*>(im + i);
            }
        } else {
            if constexpr (UNPACK) {
                re[i] = br[j];
                im[i] = bi[j];
            } else {
                br[j] = re[i];
                bi[j] = im[i];
            }
        }
    }
}

// The same gather / scatter for the 16-byte-vector case, streamed the way
// the direct gate kernels stream: each workgroup owns one run of 256 x 4
// vector units, every thread issues its four re and four im loads before the
// first store (0.5-1 TB/s with one vector per thread
// and a grid-stride loop; tools/swap_trace.sh).  `units` is a multiple of
// 256 x 4 (the launcher falls back to packKernel otherwise).
template <typename T, bool UNPACK>
__global__ __launch_bounds__(kThreads) void packRunKernel(T* __restrict__ re, T* __restrict__ im, PackBits pb,
                                                          long long start, T* __restrict__ br,
                                                          T* __restrict__ bi) {
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::n, UNR = 4;
    const long long u0 = (long long)blockIdx.x * (kThreads * UNR) + threadIdx.x;
    long long si[UNR], bj[UNR];
    for (int k = 0; k < UNR; k++) {
        const long long j = (u0 + k * kThreads) * VN;
        long long i = start + j;
        for (int m = 0; m < pb.k; m++) i = ins0(i, pb.pos[m]);
        si[k] = i | pb.setMask;
        bj[k] = j;
    }
    V vr[UNR], vi[UNR];
    if constexpr (UNPACK) {
        for (int k = 0; k < UNR; k++) {
            vr[k] = *(reinterpret_cast<const V*>(br + bj[k]));
            vi[k] = *(reinterpret_cast<const V*>(bi + bj[k]));
        }
        for (int k = 0; k < UNR; k++) {
            *(reinterpret_cast<V*>(re + si[k])) = vr[k];
            *(reinterpret_cast<V*>(im + si[k])) = vi[k];
        }
    } else {
        for (int k = 0; k < UNR; k++) {
            vr[k] = *(reinterpret_cast<const V*>(re + si[k]));
            vi[k] = *(reinterpret_cast<const V*>(im + si[k]));
        }
        for (int k = 0; k < UNR; k++) {
            *(reinterpret_cast<V*>(br + bj[k])) = vr[k];
            *(reinterpret_cast<V*>(bi + bj[k])) = vi[k];
        }
    }
}

// In-place exchange of two parts through a peer's mapped memory (the IPC
// transport's swaps): a's amplitude at packed index j (bits pos[] = pb.setMask)
// trades places with b's at the same j (bits pos[] = bMask).  Each amplitude
// is read once and written once; the buffered pipeline (pack, pull, unpack)
// moves it three times.  VEC: 16-byte units when the lowest inserted bit is
// above the vector width.
template <typename T, bool VEC>
__global__ __launch_bounds__(kThreads) void swapPartsKernel(T* __restrict__ ar, T* __restrict__ ai,
                                                            T* __restrict__ br, T* __restrict__ bi, PackBits pb,
                                                            long long bMask, long long start, long long count) {
    using V = typename std::conditional<VEC, typename Vec16<T>::type, T>::type;
    constexpr int VN = VEC ? Vec16<T>::n : 1;
    const long long units = count / VN;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long u = (long long)blockIdx.x * blockDim.x + threadIdx.x; u < units; u += stride) {
        long long i = start + u * VN;
        for (int m = 0; m < pb.k; m++) i = ins0(i, pb.pos[m]);
        const long long ia = i | pb.setMask, ib = i | bMask;
        V* pa = reinterpret_cast<V*>(ar + ia);
        V* qa = reinterpret_cast<V*>(ai + ia);
        V* pbv = reinterpret_cast<V*>(br + ib);
        V* qb = reinterpret_cast<V*>(bi + ib);
        const V x = *pa, y = *qa, z = *pbv, w = *qb;
        *pa = z;
        *qa = w;
        *pbv = x;
        *qb = y;
    }
}

// Device-to-device copy of n 16-byte vectors (runs of 256 x 4 per workgroup,
// plus a tail loop): the IPC transport's pull from a peer's mapped buffer on
// the same GPU, instead of the runtime's blit (~1 TB/s under contention).
__global__ __launch_bounds__(kThreads) void copyVecKernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                          long long n) {
    constexpr int UNR = 4;
    const long long u0 = (long long)blockIdx.x * (kThreads * UNR) + threadIdx.x;
    if (u0 + (UNR - 1) * kThreads < n) {
        uint4 v[UNR];
        for (int k = 0; k < UNR; k++) v[k] = *(src + u0 + k * kThreads);
        for (int k = 0; k < UNR; k++) *(dst + u0 + k * kThreads) = v[k];
        return;
    }
    for (int k = 0; k < UNR; k++) {
        const long long u = u0 + k * kThreads;
        if (u < n) dst[u] = src[u];
    }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void axpbyKernel(T* __restrict__ ar, T* __restrict__ ai, T alpha,
                                                        const T* __restrict__ br, const T* __restrict__ bi, T beta,
                                                        long long n) {
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::n;
    const long long stride = (long long)gridDim.x * blockDim.x;
    const long long nv = n / VN;
    for (long long u = (long long)blockIdx.x * blockDim.x + threadIdx.x; u < nv; u += stride) {
        V a = reinterpret_cast<V*>(ar)[u], b = reinterpret_cast<V*>(ai)[u];
        const V c = reinterpret_cast<const V*>(br)[u], d = reinterpret_cast<const V*>(bi)[u];
        T* pa = reinterpret_cast<T*>(&a);
        T* pb = reinterpret_cast<T*>(&b);
        const T* pc = reinterpret_cast<const T*>(&c);
        const T* pd = reinterpret_cast<const T*>(&d);
#pragma unroll
        for (int e = 0; e < VN; e++) {
            pa[e] = alpha * pa[e] + beta * pc[e];
            pb[e] = alpha * pb[e] + beta * pd[e];
        }
        reinterpret_cast<V*>(ar)[u] = a;
        reinterpret_cast<V*>(ai)[u] = b;
    }
    for (long long i = nv * VN + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        ar[i] = alpha * ar[i] + beta * br[i];
        ai[i] = alpha * ai[i] + beta * bi[i];
    }
}

// rho(r, c) = psi_r conj(psi_c); consecutive threads walk consecutive rows of
// one column, so rho writes and psi_r reads are coalesced and psi_c is a
// broadcast (the reference gives each thread a whole row: column-strided
// writes, QuEST_gpu.cu:67-84)
template <typename T>
__global__ __launch_bounds__(kThreads) void densPureKernel(T* __restrict__ re, T* __restrict__ im, long long n,
                                                           const T* __restrict__ pr, const T* __restrict__ pi, int nq,
                                                           long long chunkStart) {
    const long long mask = (1ll << nq) - 1;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
        const long long g = chunkStart + k, r = g & mask, c = g >> nq;
        const T ar = pr[r], ai = pi[r], cr = pr[c], ci = pi[c];
        re[k] = ar * cr + ai * ci;
        im[k] = ai * cr - ar * ci;
    }
}

}  // namespace

void launchFill(real* re, real* im, i64 n, real vr, real vi) {
    if (vr == 0 && vi == 0) {
        QA_HIP_CHECK(hipMemsetAsync(re, 0, sizeof(real) * n, stream()));
        QA_HIP_CHECK(hipMemsetAsync(im, 0, sizeof(real) * n, stream()));
        return;
    }
    hipLaunchKernelGGL(fillKernel<real>, dim3(gridFor(n)), dim3(kThreads), 0, stream(), re, im, n, vr, vi);
    QA_HIP_CHECK(hipGetLastError());
}

void launchInitDebug(real* re, real* im, i64 n, i64 offset) {
    hipLaunchKernelGGL(debugKernel<real>, dim3(gridFor(n)), dim3(kThreads), 0, stream(), re, im, n, offset);
    QA_HIP_CHECK(hipGetLastError());
}

void launchFillWhereBit(real* re, real* im, i64 n, int bit, int outcome, real val) {
    hipLaunchKernelGGL(fillBitKernel<real>, dim3(gridFor(n)), dim3(kThreads), 0, stream(), re, im, n, bit, outcome,
                       val);
    QA_HIP_CHECK(hipGetLastError());
}

void launchPackBits(const real* re, const real* im, const int* pos, int k, u64 setMask, i64 start, i64 count,
                    real* br, real* bi, bool unpack) {
    constexpr int VN = Vec16<real>::n;
    PackBits pb;
    pb.k = k;
    for (int m = 0; m < 8; m++) pb.pos[m] = m < k ? pos[m] : 0;
    std::sort(pb.pos, pb.pos + k);
    pb.setMask = (long long)setMask;
    const bool vec = (k == 0 || (1ll << pb.pos[0]) >= VN) && (start % VN == 0) && (count % VN == 0);
    real* r = const_cast<real*>(re);
    real* m = const_cast<real*>(im);
    constexpr long long kRun = (long long)kThreads * 4;
    if (vec && (count / VN) % kRun == 0) {
        const dim3 grid((unsigned)((count / VN) / kRun));
        if (unpack)
            hipLaunchKernelGGL((packRunKernel<real, true>), grid, dim3(kThreads), 0, stream(), r, m, pb, start, br, bi);
        else
            hipLaunchKernelGGL((packRunKernel<real, false>), grid, dim3(kThreads), 0, stream(), r, m, pb, start, br, bi);
        QA_HIP_CHECK(hipGetLastError());
        return;
    }
    const int g = gridFor(vec ? count / VN : count);
    if (unpack) {
        if (vec)
            hipLaunchKernelGGL((packKernel<real, true, true>), dim3(g), dim3(kThreads), 0, stream(), r, m, pb, start,
                               count, br, bi);
        else
            hipLaunchKernelGGL((packKernel<real, true, false>), dim3(g), dim3(kThreads), 0, stream(), r, m, pb, start,
                               count, br, bi);
    } else {
        if (vec)
            hipLaunchKernelGGL((packKernel<real, false, true>), dim3(g), dim3(kThreads), 0, stream(), r, m, pb,
                               start, count, br, bi);
        else
            hipLaunchKernelGGL((packKernel<real, false, false>), dim3(g), dim3(kThreads), 0, stream(), r, m, pb,
                               start, count, br, bi);
    }
    QA_HIP_CHECK(hipGetLastError());
}

void launchCopyVec(void* dst, const void* src, size_t bytes, hipStream_t st) {
    if (bytes % 16 != 0 || ((uintptr_t)dst | (uintptr_t)src) % 16 != 0) {
        QA_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st));
        return;
    }
    const long long n = (long long)(bytes / 16);
    const long long per = (long long)kThreads * 4;
    const long long g = (n + per - 1) / per;
    if (g <= 0) return;
    hipLaunchKernelGGL(copyVecKernel, dim3((unsigned)g), dim3(kThreads), 0, st, static_cast<const uint4*>(src),
                       static_cast<uint4*>(dst), n);
    QA_HIP_CHECK(hipGetLastError());
}

// a = alpha a + beta b, b in another qubit layout (PermArgs): per tile, b's
// runs into LDS in a's element order (as innerPermKernel), then a streamed in
// place, two elements per access
template <typename T, int NP>
__global__ __launch_bounds__(kThreads) void axpbyPermKernel(T* __restrict__ ar, T* __restrict__ ai, T alpha,
                                                            const T* __restrict__ br, const T* __restrict__ bi,
                                                            T beta, PermArgs pa) {
    using V2 = typename std::conditional<sizeof(T) == 8, double2, float2>::type;
    extern __shared__ unsigned char smem[];
    T* sr = reinterpret_cast<T*>(smem);
    T* si = sr + (1 << pa.K);
    const PermLanes<NP> pl(pa);
    const long long tiles = 1ll << pa.nOut;
    // b's runs of the next tile load while this one is updated (as innerPermKernel)
    V2 ub[NP], vb[NP];
    auto loadB = [&](long long tt) {
        const unsigned long long baseB = scatterBits((unsigned long long)tt, pa.oB, pa.nOut);
#pragma unroll
        for (int q = 0; q < NP; q++) {
            if (!pl.live[q]) continue;
            ub[q] = streamLoad(reinterpret_cast<const V2*>(br + (baseB | pl.offB[q])));
            vb[q] = streamLoad(reinterpret_cast<const V2*>(bi + (baseB | pl.offB[q])));
        }
    };
    if ((long long)blockIdx.x < tiles) loadB(blockIdx.x);
    for (long long t = blockIdx.x; t < tiles; t += gridDim.x) {
        const unsigned long long baseA = scatterBits((unsigned long long)t, pa.oA, pa.nOut);
#pragma unroll
        for (int q = 0; q < NP; q++) {
            if (!pl.live[q]) continue;
            sr[pl.slotB0[q]] = ub[q].x;
            sr[pl.slotB1[q]] = ub[q].y;
            si[pl.slotB0[q]] = vb[q].x;
            si[pl.slotB1[q]] = vb[q].y;
        }
        V2 xa[NP], ya[NP];
#pragma unroll
        for (int q = 0; q < NP; q++) {
            if (!pl.live[q]) continue;
            xa[q] = streamLoad(reinterpret_cast<const V2*>(ar + (baseA | pl.offA[q])));
            ya[q] = streamLoad(reinterpret_cast<const V2*>(ai + (baseA | pl.offA[q])));
        }
        if (t + gridDim.x < tiles) loadB(t + gridDim.x);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < NP; q++) {
            if (!pl.live[q]) continue;
            V2* xr = reinterpret_cast<V2*>(ar + (baseA | pl.offA[q]));
            V2* xi = reinterpret_cast<V2*>(ai + (baseA | pl.offA[q]));
            const int s0 = pl.slotA[q], s1 = s0 ^ 1;
            V2 x = xa[q], y = ya[q];
            x.x = alpha * x.x + beta * sr[s0];
            x.y = alpha * x.y + beta * sr[s1];
            y.x = alpha * y.x + beta * si[s0];
            y.y = alpha * y.y + beta * si[s1];
            streamStore(xr, x);
            streamStore(xi, y);
        }
        __syncthreads();
    }
}


void launchSwapParts(real* ar, real* ai, real* br, real* bi, const int* pos, int k, u64 aMask, u64 bMask, i64 start,
                     i64 count) {
    constexpr int VN = Vec16<real>::n;
    PackBits pb;
    pb.k = k;
    for (int m = 0; m < 8; m++) pb.pos[m] = m < k ? pos[m] : 0;
    std::sort(pb.pos, pb.pos + k);
    pb.setMask = (long long)aMask;
    const bool vec = (k == 0 || (1ll << pb.pos[0]) >= VN) && start % VN == 0 && count % VN == 0;
    if (vec)
        hipLaunchKernelGGL((swapPartsKernel<real, true>), dim3(gridFor(count / VN)), dim3(kThreads), 0, stream(), ar,
                           ai, br, bi, pb, (long long)bMask, start, count);
    else
        hipLaunchKernelGGL((swapPartsKernel<real, false>), dim3(gridFor(count)), dim3(kThreads), 0, stream(), ar, ai,
                           br, bi, pb, (long long)bMask, start, count);
    QA_HIP_CHECK(hipGetLastError());
}

void launchAxpby(real* ar, real* ai, real alpha, const real* br, const real* bi, real beta, i64 n) {
    hipLaunchKernelGGL(axpbyKernel<real>, dim3(gridFor(n / Vec16<real>::n)), dim3(kThreads), 0, stream(), ar, ai,
                       alpha, br, bi, beta, n);
    QA_HIP_CHECK(hipGetLastError());
}

PermArgs makePermArgs(int L, const int* sig) {
    PermArgs pa;
    std::memset(&pa, 0, sizeof pa);
    // tile: a's positions 0-3 and those b holds on 0-3 (16-element runs on
    // both sides), then alternately a's and b's next lowest positions, so that
    // both streams read runs as long as the tile allows
    bool inTile[64] = {false};
    int inv[64];
    for (int p = 0; p < L; p++) inv[sig[p]] = p;
    const int c = std::min(L, 4);
    for (int p = 0; p < c; p++) inTile[p] = inTile[inv[p]] = true;
    // tile bits: more pairs per thread keep more loads in flight, fewer
    // workgroups fit the LDS (QUEST_PERM_TILE_BITS, 8..12, default 11)
    static const int bits = [] {
        const char* e = std::getenv("QUEST_PERM_TILE_BITS");
        return e ? std::max(8, std::min(kPermMaxBits, std::atoi(e))) : 11;
    }();
    const int K = std::min(L, bits);
    int k = 0;
    for (int p = 0; p < L; p++) k += inTile[p];
    for (int p = c; p < L && k < K; p++) {
        if (!inTile[p]) inTile[p] = true, k++;
        if (k < K && !inTile[inv[p]]) inTile[inv[p]] = true, k++;
    }
    pa.K = k;
    int n = 0, m = 0;
    for (int p = 0; p < L; p++) {
        if (inTile[p]) {
            pa.tA[n] = (signed char)p;
            pa.tB[n++] = (signed char)sig[p];
        } else {
            pa.oA[m] = (signed char)p;
            pa.oB[m++] = (signed char)sig[p];
        }
    }
    pa.nOut = m;
    // b order: tile bits by ascending b-position
    int ord[16];
    for (int x = 0; x < n; x++) ord[x] = x;
    std::sort(ord, ord + n, [&](int a, int b) { return pa.tB[a] < pa.tB[b]; });
    for (int x = 0; x < n; x++) pa.bOrd[x] = (signed char)ord[x];
    return pa;
}

void launchAxpbyPerm(real* ar, real* ai, real alpha, const real* br, const real* bi, real beta, const PermArgs& pa) {
    const long long tiles = 1ll << pa.nOut;
    const int grid = (int)std::min<long long>(tiles, 8ll * numCUs());
    const size_t lds = 2 * sizeof(real) << pa.K;
    switch (permPairsFor(pa.K)) {
#define QA_AXPBY_PERM(NP)                                                                                            \
    case NP:                                                                                                         \
        hipLaunchKernelGGL((axpbyPermKernel<real, NP>), dim3(grid), dim3(kThreads), lds, stream(), ar, ai, alpha, br, \
                           bi, beta, pa);                                                                            \
        break;
        QA_AXPBY_PERM(1)
        QA_AXPBY_PERM(2)
        QA_AXPBY_PERM(4)
        QA_AXPBY_PERM(8)
#undef QA_AXPBY_PERM
    default:
        fatal("launchAxpbyPerm", "tile bits out of range", __FILE__, __LINE__);
    }
    QA_HIP_CHECK(hipGetLastError());
}

void launchDensInitPure(real* re, real* im, i64 n, const real* pr, const real* pi, int nq, i64 chunkStart) {
    hipLaunchKernelGGL(densPureKernel<real>, dim3(gridFor(n)), dim3(kThreads), 0, stream(), re, im, n, pr, pi, nq,
                       chunkStart);
    QA_HIP_CHECK(hipGetLastError());
}

}  // namespace hipk
}  // namespace qa
