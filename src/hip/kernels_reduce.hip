// Reductions for CDNA4: probabilities, norms, inner products, density-matrix
// traces and fidelities.
//
// Two launches per reduction, both deterministic (no float atomics, fixed
// summation tree):  a grid-stride first level where each thread accumulates
// in fp64 over 16-byte vector loads, a 64-lane wave reduction with
// __shfl_xor, and one partial per workgroup; then a single-workgroup finish.
// The reference instead runs one kernel per 512-element level with a
// cudaDeviceSynchronize between levels and a divergent __syncthreads
// (QuEST_gpu.cu:1335-1352, :1515-1551), and sums calcTotalProb on the host
// after copying the whole state back (:1121, :1143-1163).
#include "qa_hip.h"

#include <algorithm>
#include <type_traits>

namespace qa {
namespace hipk {

namespace {

constexpr int kThreads = 256;
constexpr int kMaxBlocks = 2048;

double* g_partials = nullptr;  // 2 * kMaxBlocks doubles
double* g_out = nullptr;       // 2 doubles (device)
double* g_outHost = nullptr;   // 2 doubles (pinned)

void ensureScratch() {
    if (g_partials) return;
    QA_HIP_CHECK(hipMalloc(&g_partials, sizeof(double) * 2 * kMaxBlocks));
    QA_HIP_CHECK(hipMalloc(&g_out, sizeof(double) * 2));
    QA_HIP_CHECK(hipHostMalloc(&g_outHost, sizeof(double) * 2, hipHostMallocDefault));
}

__device__ __forceinline__ double waveSum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// sum over the block; result valid in thread 0
__device__ __forceinline__ double blockSum(double v) {
    __shared__ double sh[kThreads / 64];
    v = waveSum(v);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) sh[w] = v;
    __syncthreads();
    double r = 0;
    if (threadIdx.x < 64) {
        r = (threadIdx.x < kThreads / 64) ? sh[threadIdx.x] : 0.0;
        r = waveSum(r);
    }
    return r;
}

__device__ __forceinline__ long long ins0(long long x, int b) {
    long long low = x & ((1ll << b) - 1);
    return ((x >> b) << (b + 1)) | low;
}

template <typename T>
__global__ __launch_bounds__(kThreads) void sumSqAllKernel(const T* __restrict__ re, const T* __restrict__ im,
                                                           long long n, double* __restrict__ part) {
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::n;
    double acc = 0;
    const long long nv = n / VN;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long u = (long long)blockIdx.x * blockDim.x + threadIdx.x; u < nv; u += stride) {
        const V a = reinterpret_cast<const V*>(re)[u];
        const V b = reinterpret_cast<const V*>(im)[u];
        const T* pa = reinterpret_cast<const T*>(&a);
        const T* pb = reinterpret_cast<const T*>(&b);
#pragma unroll
        for (int e = 0; e < VN; e++) acc += (double)pa[e] * pa[e] + (double)pb[e] * pb[e];
    }
    for (long long i = nv * VN + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        acc += (double)re[i] * re[i] + (double)im[i] * im[i];
    const double s = blockSum(acc);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// amplitudes whose bit `bit` == bitVal; VN consecutive per unit when 2^bit >= VN
template <typename T, bool VEC>
__global__ __launch_bounds__(kThreads) void sumSqBitKernel(const T* __restrict__ re, const T* __restrict__ im,
                                                           long long n, int bit, int bitVal,
                                                           double* __restrict__ part) {
    using V = typename Vec16<T>::type;
    constexpr int VN = VEC ? Vec16<T>::n : 1;
    double acc = 0;
    const long long units = (n >> 1) / VN;
    const long long stride = (long long)gridDim.x * blockDim.x;
    const long long set = (long long)bitVal << bit;
    for (long long u = (long long)blockIdx.x * blockDim.x + threadIdx.x; u < units; u += stride) {
        const long long i = ins0(u * VN, bit) | set;
        if constexpr (VEC) {
            const V a = *reinterpret_cast<const V*>(re + i);
            const V b = *reinterpret_cast<const V*>(im + i);
            const T* pa = reinterpret_cast<const T*>(&a);
            const T* pb = reinterpret_cast<const T*>(&b);
#pragma unroll
            for (int e = 0; e < VN; e++) acc += (double)pa[e] * pa[e] + (double)pb[e] * pb[e];
        } else {
            acc += (double)re[i] * re[i] + (double)im[i] * im[i];
        }
    }
    const double s = blockSum(acc);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// All one-qubit marginals in ONE pass: out[b] = sum of |a_i|^2 over i with
// bit b == 0, for every local bit b, plus the total.  The fork's program asks
// for P(q = 1) of all 30 qubits back to back (tutorial_example.c:521-525);
// one sumSqBitKernel per qubit re-streams half the state each time
// (QuEST_gpu.cu:1515-1551 streams it per call too).
//
// A tile of 2^m amplitudes is 256 threads x kMargUnits 16-byte units x VN
// elements: element bits [0, vb), thread bits [vb, vb + 8), unit bits
// [vb + 8, vb + 11), tile bits above.  Workgroup w of G = 2^g takes tiles
// w, w + G, ...: tile bits [m, m + g) are blockIdx's (applied by the finish
// kernel to the workgroup total), the rest vary per iteration.  Partial slots
// per workgroup: 0 total, 1 .. vb element bits, then 8 thread bits, 3 unit
// bits, then the varying tile bits.
constexpr int kMargUnits = 8;
constexpr int kMargSlots = 64;
double* g_margPartials = nullptr;  // kMargSlots * kMaxBlocks

template <typename T>
__global__ __launch_bounds__(kThreads) void marginalsKernel(const T* __restrict__ re, const T* __restrict__ im,
                                                            long long numTiles, int g, int nVary,
                                                            double* __restrict__ part) {
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::n;
    constexpr int VB = VN == 2 ? 1 : 2;
    constexpr int kMaxVary = 32;
    const int G = gridDim.x;
    double tot = 0, ez[VB], uz[3], hz[kMaxVary];
#pragma unroll
    for (int e = 0; e < VB; e++) ez[e] = 0;
#pragma unroll
    for (int e = 0; e < 3; e++) uz[e] = 0;
#pragma unroll
    for (int e = 0; e < kMaxVary; e++) hz[e] = 0;
    for (long long t = blockIdx.x; t < numTiles; t += G) {
        const long long base = t * (kThreads * kMargUnits);   // in units
        double s[kMargUnits];
#pragma unroll
        for (int k = 0; k < kMargUnits; k++) {
            const V a = reinterpret_cast<const V*>(re)[base + k * kThreads + threadIdx.x];
            const V b = reinterpret_cast<const V*>(im)[base + k * kThreads + threadIdx.x];
            const T* pa = reinterpret_cast<const T*>(&a);
            const T* pb = reinterpret_cast<const T*>(&b);
            double x[VN];
#pragma unroll
            for (int e = 0; e < VN; e++) x[e] = (double)pa[e] * pa[e] + (double)pb[e] * pb[e];
            double sk = 0;
#pragma unroll
            for (int e = 0; e < VN; e++) {
                sk += x[e];
#pragma unroll
                for (int eb = 0; eb < VB; eb++)
                    if (!((e >> eb) & 1)) ez[eb] += x[e];
            }
            s[k] = sk;
        }
        double st = 0;
#pragma unroll
        for (int k = 0; k < kMargUnits; k++) {
            st += s[k];
#pragma unroll
            for (int kb = 0; kb < 3; kb++)
                if (!((k >> kb) & 1)) uz[kb] += s[k];
        }
        tot += st;
        const long long hi = t >> g;   // tile bits that vary across this workgroup's tiles
#pragma unroll
        for (int h = 0; h < kMaxVary; h++)
            if (h < nVary && !((hi >> h) & 1)) hz[h] += st;
    }
    // block sums of every slot (thread bits: the thread's total where its bit is 0)
    __shared__ double red[kMargSlots][kThreads / 64];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    auto put = [&](int slot, double v) {
        v = waveSum(v);
        if (l == 0) red[slot][w] = v;
    };
    int slot = 0;
    put(slot++, tot);
#pragma unroll
    for (int e = 0; e < VB; e++) put(slot++, ez[e]);
#pragma unroll
    for (int b = 0; b < 8; b++) put(slot++, ((threadIdx.x >> b) & 1) ? 0.0 : tot);
#pragma unroll
    for (int e = 0; e < 3; e++) put(slot++, uz[e]);
#pragma unroll
    for (int h = 0; h < kMaxVary; h++)
        if (h < nVary) put(slot++, hz[h]);
    __syncthreads();
    if (threadIdx.x < slot) {
        double v = 0;
#pragma unroll
        for (int k = 0; k < kThreads / 64; k++) v += red[threadIdx.x][k];
        part[(long long)threadIdx.x * kMaxBlocks + blockIdx.x] = v;
    }
}

// out[b] for b < L (zero-bit sums), out[L] = total, from the per-workgroup slots
__global__ __launch_bounds__(kThreads) void marginalsFinishKernel(const double* __restrict__ part, int G, int g,
                                                                  int vb, int L, double* __restrict__ out) {
    const int m = vb + 11;
    for (int b = 0; b <= L; b++) {
        double acc = 0;
        if (b == L) {
            for (int i = threadIdx.x; i < G; i += blockDim.x) acc += part[i];
        } else if (b >= m && b < m + g) {   // workgroup-index bits: totals of the workgroups with the bit clear
            for (int i = threadIdx.x; i < G; i += blockDim.x)
                if (!((i >> (b - m)) & 1)) acc += part[i];
        } else {
            const int slot = b < m ? 1 + b : 1 + m + (b - m - g);
            for (int i = threadIdx.x; i < G; i += blockDim.x) acc += part[(long long)slot * kMaxBlocks + i];
        }
        const double s = blockSum(acc);
        if (threadIdx.x == 0) out[b] = s;
        __syncthreads();
    }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void innerKernel(const T* __restrict__ ar, const T* __restrict__ ai,
                                                        const T* __restrict__ br, const T* __restrict__ bi,
                                                        long long n, double* __restrict__ part) {
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::n;
    double sr = 0, si = 0;
    const long long nv = n / VN;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long u = (long long)blockIdx.x * blockDim.x + threadIdx.x; u < nv; u += stride) {
        const V a = reinterpret_cast<const V*>(ar)[u], b = reinterpret_cast<const V*>(ai)[u];
        const V c = reinterpret_cast<const V*>(br)[u], d = reinterpret_cast<const V*>(bi)[u];
        const T *pa = reinterpret_cast<const T*>(&a), *pb = reinterpret_cast<const T*>(&b);
        const T *pc = reinterpret_cast<const T*>(&c), *pd = reinterpret_cast<const T*>(&d);
#pragma unroll
        for (int e = 0; e < VN; e++) {
            sr += (double)pa[e] * pc[e] + (double)pb[e] * pd[e];
            si += (double)pa[e] * pd[e] - (double)pb[e] * pc[e];
        }
    }
    for (long long i = nv * VN + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        sr += (double)ar[i] * br[i] + (double)ai[i] * bi[i];
        si += (double)ar[i] * bi[i] - (double)ai[i] * br[i];
    }
    const double s0 = blockSum(sr);
    const double s1 = blockSum(si);
    if (threadIdx.x == 0) {
        part[blockIdx.x] = s0;
        part[kMaxBlocks + blockIdx.x] = s1;
    }
}


// sum conj(a_i) b_sigma(i) with b in another qubit layout (PermArgs): per
// tile, b's 16-element runs into LDS in a's element order (2-element vector
// loads, swizzled slots), then a streamed the same way
template <typename T, int NP>
__global__ __launch_bounds__(kThreads) void innerPermKernel(const T* __restrict__ ar, const T* __restrict__ ai,
                                                            const T* __restrict__ br, const T* __restrict__ bi,
                                                            PermArgs pa, double* __restrict__ part) {
    using V2 = typename std::conditional<sizeof(T) == 8, double2, float2>::type;
    extern __shared__ unsigned char smem[];
    T* sr = reinterpret_cast<T*>(smem);
    T* si = sr + (1 << pa.K);
    const PermLanes<NP> pl(pa);
    const long long tiles = 1ll << pa.nOut;
    double accR = 0, accI = 0;
    // b's runs of the next tile are loaded while this one is reduced
    // (software pipeline: one tile of b in registers ahead)
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
            const V2 x = xa[q], y = ya[q];
            const int s0 = pl.slotA[q], s1 = s0 ^ 1;  // element f + 1: bit 0 is never swizzled
            const double u0 = sr[s0], v0 = si[s0], u1 = sr[s1], v1 = si[s1];
            accR += (double)x.x * u0 + (double)y.x * v0 + (double)x.y * u1 + (double)y.y * v1;
            accI += (double)x.x * v0 - (double)y.x * u0 + (double)x.y * v1 - (double)y.y * u1;
        }
        __syncthreads();
    }
    const double s0 = blockSum(accR);
    const double s1 = blockSum(accI);
    if (threadIdx.x == 0) {
        part[blockIdx.x] = s0;
        part[kMaxBlocks + blockIdx.x] = s1;
    }
}

struct Offs {
    unsigned long long o[32];
};

template <typename T>
__global__ __launch_bounds__(kThreads) void densDiagKernel(const T* __restrict__ re, long long chunkAmps, Offs offs,
                                                           int nq, int skipBit, long long chunkStart,
                                                           double* __restrict__ part) {
    double acc = 0;
    const long long dim = skipBit >= 0 ? (1ll << (nq - 1)) : (1ll << nq);
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x; j < dim; j += stride) {
        const long long r = skipBit >= 0 ? ins0(j, skipBit) : j;
        long long p = 0;
        for (int b = 0; b < nq; b++)
            if ((r >> b) & 1) p |= (long long)offs.o[b];
        p -= chunkStart;
        if (p >= 0 && p < chunkAmps) acc += (double)re[p];
    }
    const double s = blockSum(acc);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

template <typename T>
__global__ __launch_bounds__(kThreads) void densFidelityKernel(const T* __restrict__ re, const T* __restrict__ im,
                                                               long long n, const T* __restrict__ pr,
                                                               const T* __restrict__ pi, int nq,
                                                               long long chunkStart, double* __restrict__ part) {
    double acc = 0;
    const long long mask = (1ll << nq) - 1;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
        const long long g = chunkStart + k, r = g & mask, c = g >> nq;
        const double ar = (double)re[k] * pr[c] - (double)im[k] * pi[c];
        const double ai = (double)re[k] * pi[c] + (double)im[k] * pr[c];
        acc += (double)pr[r] * ar + (double)pi[r] * ai;
    }
    const double s = blockSum(acc);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// max over the block of a non-negative value; result valid in thread 0
__device__ __forceinline__ double blockMax(double v) {
    __shared__ double sh[kThreads / 64];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) sh[w] = v;
    __syncthreads();
    double r = 0;
    if (threadIdx.x < 64) {
        r = (threadIdx.x < kThreads / 64) ? sh[threadIdx.x] : 0.0;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) r = fmax(r, __shfl_xor(r, off, 64));
    }
    return r;
}

// max_i |a_i - b_i| over complex amplitudes (QUEST_VERIFY)
template <typename T>
__global__ __launch_bounds__(kThreads) void maxDiffKernel(const T* __restrict__ ar, const T* __restrict__ ai,
                                                          const T* __restrict__ br, const T* __restrict__ bi,
                                                          long long n, double* __restrict__ part) {
    double m = 0;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const double dr = (double)ar[i] - br[i], di = (double)ai[i] - bi[i];
        // NaN anywhere must fail the check: fmax would drop it
        const double d = sqrt(dr * dr + di * di);
        m = (d != d) ? INFINITY : fmax(m, d);
    }
    const double s = blockMax(m);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(kThreads) void finishMaxKernel(const double* __restrict__ part, int nb,
                                                            double* __restrict__ out) {
    double m = 0;
    for (int i = threadIdx.x; i < nb; i += blockDim.x) m = fmax(m, part[i]);
    const double s = blockMax(m);
    if (threadIdx.x == 0) out[0] = s;
}

__global__ __launch_bounds__(kThreads) void finishKernel(const double* __restrict__ part, int nb, int nvals,
                                                         double* __restrict__ out) {
    for (int v = 0; v < nvals; v++) {
        double acc = 0;
        for (int i = threadIdx.x; i < nb; i += blockDim.x) acc += part[v * kMaxBlocks + i];
        const double s = blockSum(acc);
        if (threadIdx.x == 0) out[v] = s;
        __syncthreads();
    }
}

int blocksFor(long long work) {
    long long b = (work + kThreads * 4 - 1) / (kThreads * 4);
    if (b < 1) b = 1;
    if (b > kMaxBlocks) b = kMaxBlocks;
    return (int)b;
}

void finish(int nb, int nvals, double* result) {
    hipLaunchKernelGGL(finishKernel, dim3(1), dim3(kThreads), 0, stream(), g_partials, nb, nvals, g_out);
    QA_HIP_CHECK(hipGetLastError());
    QA_HIP_CHECK(hipMemcpyAsync(g_outHost, g_out, sizeof(double) * nvals, hipMemcpyDeviceToHost, stream()));
    syncStream();
    for (int v = 0; v < nvals; v++) result[v] = g_outHost[v];
}

}  // namespace

double reduceSumSq(const real* re, const real* im, i64 n, int bit, int bitVal) {
    ensureScratch();
    constexpr int VN = Vec16<real>::n;
    int nb;
    if (bit < 0) {
        nb = blocksFor(n / VN);
        hipLaunchKernelGGL(sumSqAllKernel<real>, dim3(nb), dim3(kThreads), 0, stream(), re, im, n, g_partials);
    } else if ((1ll << bit) >= VN) {
        nb = blocksFor(n / 2 / VN);
        hipLaunchKernelGGL((sumSqBitKernel<real, true>), dim3(nb), dim3(kThreads), 0, stream(), re, im, n, bit,
                           bitVal, g_partials);
    } else {
        nb = blocksFor(n / 2);
        hipLaunchKernelGGL((sumSqBitKernel<real, false>), dim3(nb), dim3(kThreads), 0, stream(), re, im, n, bit,
                           bitVal, g_partials);
    }
    QA_HIP_CHECK(hipGetLastError());
    double r;
    finish(nb, 1, &r);
    return r;
}

void reduceMarginals(const real* re, const real* im, int L, double* zeroSums, double* total) {
    ensureScratch();
    constexpr int VN = Vec16<real>::n;
    constexpr int vb = VN == 2 ? 1 : 2;
    const int m = vb + 11;
    if (L < m) {   // small chunk: one bit at a time (tiny launches)
        for (int b = 0; b < L; b++) zeroSums[b] = reduceSumSq(re, im, 1ll << L, b, 0);
        *total = reduceSumSq(re, im, 1ll << L, -1, 0);
        return;
    }
    static double* dOut = nullptr;
    static double* hOut = nullptr;
    if (!g_margPartials) {
        QA_HIP_CHECK(hipMalloc(&g_margPartials, sizeof(double) * kMargSlots * kMaxBlocks));
        QA_HIP_CHECK(hipMalloc(&dOut, sizeof(double) * 64));
        QA_HIP_CHECK(hipHostMalloc(&hOut, sizeof(double) * 64, hipHostMallocDefault));
    }
    const int tileBits = L - m;
    int g = 0;
    while (g < tileBits && (2 << g) <= kMaxBlocks) g++;
    const int nVary = tileBits - g;
    if (nVary > 32 || 1 + vb + 11 + nVary > kMargSlots) {
        fprintf(stderr, "QuEST: marginals of %d local qubits exceed the kernel's slots\n", L);
        exit(EXIT_FAILURE);
    }
    const long long numTiles = 1ll << tileBits;
    hipLaunchKernelGGL(marginalsKernel<real>, dim3(1 << g), dim3(kThreads), 0, stream(), re, im, numTiles, g, nVary,
                       g_margPartials);
    QA_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(marginalsFinishKernel, dim3(1), dim3(kThreads), 0, stream(), g_margPartials, 1 << g, g, vb, L,
                       dOut);
    QA_HIP_CHECK(hipGetLastError());
    QA_HIP_CHECK(hipMemcpyAsync(hOut, dOut, sizeof(double) * (L + 1), hipMemcpyDeviceToHost, stream()));
    syncStream();
    for (int b = 0; b < L; b++) zeroSums[b] = hOut[b];
    *total = hOut[L];
}

void reduceInner(const real* ar, const real* ai, const real* br, const real* bi, i64 n, double out[2]) {
    ensureScratch();
    const int nb = blocksFor(n / Vec16<real>::n);
    hipLaunchKernelGGL(innerKernel<real>, dim3(nb), dim3(kThreads), 0, stream(), ar, ai, br, bi, n, g_partials);
    QA_HIP_CHECK(hipGetLastError());
    finish(nb, 2, out);
}

void reduceInnerPerm(const real* ar, const real* ai, const real* br, const real* bi, const PermArgs& pa,
                     double out[2]) {
    ensureScratch();
    const long long tiles = 1ll << pa.nOut;
    const int nb = (int)std::min<long long>(tiles, kMaxBlocks);
    const size_t lds = 2 * sizeof(real) << pa.K;
    switch (permPairsFor(pa.K)) {
#define QA_INNER_PERM(NP)                                                                                            \
    case NP:                                                                                                         \
        hipLaunchKernelGGL((innerPermKernel<real, NP>), dim3(nb), dim3(kThreads), lds, stream(), ar, ai, br, bi, pa,  \
                           g_partials);                                                                              \
        break;
        QA_INNER_PERM(1)
        QA_INNER_PERM(2)
        QA_INNER_PERM(4)
        QA_INNER_PERM(8)
#undef QA_INNER_PERM
    default:
        fatal("reduceInnerPerm", "tile bits out of range", __FILE__, __LINE__);
    }
    QA_HIP_CHECK(hipGetLastError());
    finish(nb, 2, out);
}

double reduceMaxDiff(const real* ar, const real* ai, const real* br, const real* bi, i64 n) {
    ensureScratch();
    const int nb = blocksFor(n);
    hipLaunchKernelGGL(maxDiffKernel<real>, dim3(nb), dim3(kThreads), 0, stream(), ar, ai, br, bi, n, g_partials);
    QA_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(finishMaxKernel, dim3(1), dim3(kThreads), 0, stream(), g_partials, nb, g_out);
    QA_HIP_CHECK(hipGetLastError());
    QA_HIP_CHECK(hipMemcpyAsync(g_outHost, g_out, sizeof(double), hipMemcpyDeviceToHost, stream()));
    syncStream();
    return g_outHost[0];
}

double reduceDensDiag(const real* re, i64 chunkAmps, const u64* offs, int nq, int skipBit, i64 chunkStart) {
    ensureScratch();
    Offs o;
    for (int i = 0; i < 32; i++) o.o[i] = i < nq ? offs[i] : 0;
    const long long dim = 1ll << nq;
    const int nb = blocksFor(dim);
    hipLaunchKernelGGL(densDiagKernel<real>, dim3(nb), dim3(kThreads), 0, stream(), re, chunkAmps, o, nq, skipBit,
                       chunkStart, g_partials);
    QA_HIP_CHECK(hipGetLastError());
    double r;
    finish(nb, 1, &r);
    return r;
}

double reduceDensFidelity(const real* re, const real* im, i64 n, const real* pr, const real* pi, int nq,
                          i64 chunkStart) {
    ensureScratch();
    const int nb = blocksFor(n);
    hipLaunchKernelGGL(densFidelityKernel<real>, dim3(nb), dim3(kThreads), 0, stream(), re, im, n, pr, pi, nq,
                       chunkStart, g_partials);
    QA_HIP_CHECK(hipGetLastError());
    double r;
    finish(nb, 1, &r);
    return r;
}

}  // namespace hipk
}  // namespace qa
