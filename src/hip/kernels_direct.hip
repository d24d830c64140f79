// Direct (LDS-free) streaming kernels for a pass that holds ONE op - the
// eager path, and the common case for a gate that cannot be fused with its
// neighbours.
//
// Index space: the bits of the op that would halve the work (target, and
// control / phase bits at or above the 128-byte line, LINE = 4 for fp64 and
// 5 for fp32) are *inserted* into a compressed counter, so the kernel only
// visits amplitudes it changes.  Control / phase bits BELOW the line are not
// inserted - skipping them would still fetch the whole line - but evaluated
// per element as a predicate.  Every thread moves UNR x 16-byte vectors per
// array, all loads issued before the first use.
#include "qa_hip.h"

namespace qa {
namespace hipk {

namespace {

__device__ __forceinline__ long long ins0ll(long long x, int b) {
    const long long low = x & ((1ll << b) - 1);
    return ((x >> b) << (b + 1)) | low;
}

struct InsertBits {
    int n;              // inserted bit positions, ascending
    int pos[8];
    long long setMask;  // inserted bits forced to 1 (high controls / phase bits)
    unsigned predMask;  // low bits (< LINE) that must be 1, checked per element
    unsigned pad;
};

__device__ __forceinline__ long long insertAll(long long j, const InsertBits& ib) {
    for (int i = 0; i < ib.n; i++) j = ins0ll(j, ib.pos[i]);
    return j | ib.setMask;
}

template <typename T>
struct Cm2 {
    T r[4], i[4];
};

template <typename T>
__device__ __forceinline__ void mat2apply(const Cm2<T>& m, T& r0, T& i0, T& r1, T& i1) {
    const T a = r0, b = i0, c = r1, d = i1;
    r0 = m.r[0] * a - m.i[0] * b + m.r[1] * c - m.i[1] * d;
    i0 = m.r[0] * b + m.i[0] * a + m.r[1] * d + m.i[1] * c;
    r1 = m.r[2] * a - m.i[2] * b + m.r[3] * c - m.i[3] * d;
    i1 = m.r[2] * b + m.i[2] * a + m.r[3] * d + m.i[3] * c;
}

// This thread's groups of UNR units: u0 + k * step, k < UNR.  BLK = false:
// grid-stride (consecutive groups of one thread lie a whole grid apart);
// BLK = true: each workgroup owns a contiguous run of 256 * UNR units, so
// the UNR loads of a wave are 4 KiB apart instead of a grid's worth.
template <bool BLK, int UNR, typename F>
__device__ __forceinline__ void forUnits(long long units, F&& f) {
    if constexpr (BLK) {
        const long long per = (long long)blockDim.x * UNR;
        for (long long c = blockIdx.x; c * per < units; c += gridDim.x) f(c * per + threadIdx.x, (long long)blockDim.x);
    } else {
        const long long stride = (long long)gridDim.x * blockDim.x;
        for (long long u0 = (long long)blockIdx.x * blockDim.x + threadIdx.x; u0 < units; u0 += stride * UNR)
            f(u0, stride);
    }
}

// target >= log2(VN): a vector at `up` (target bit 0) pairs with the vector
// at up + 2^t.
template <typename T, bool BLK>
__global__ __launch_bounds__(256) void mat2DirectKernel(T* __restrict__ re, T* __restrict__ im, long long units,
                                                        InsertBits ib, long long tbit, Cm2<T> m) {
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::n;
    constexpr int UNR = 2;
    forUnits<BLK, UNR>(units, [&](long long u0, long long step) {
        long long up[UNR];
        V ar[UNR], ai[UNR], br[UNR], bi[UNR];
#pragma unroll
        for (int k = 0; k < UNR; k++) {
            const long long u = u0 + k * step;
            up[k] = u < units ? insertAll(u * VN, ib) : -1;
            if (up[k] >= 0) {
                ar[k] = streamLoad(reinterpret_cast<const V*>(re + up[k]));
                ai[k] = streamLoad(reinterpret_cast<const V*>(im + up[k]));
                br[k] = streamLoad(reinterpret_cast<const V*>(re + up[k] + tbit));
                bi[k] = streamLoad(reinterpret_cast<const V*>(im + up[k] + tbit));
            }
        }
#pragma unroll
        for (int k = 0; k < UNR; k++) {
            if (up[k] < 0) continue;
            T* pr = reinterpret_cast<T*>(&ar[k]);
            T* pi = reinterpret_cast<T*>(&ai[k]);
            T* qr = reinterpret_cast<T*>(&br[k]);
            T* qi = reinterpret_cast<T*>(&bi[k]);
#pragma unroll
            for (int e = 0; e < VN; e++) {
                if ((((unsigned)up[k] + e) & ib.predMask) != ib.predMask) continue;
                mat2apply(m, pr[e], pi[e], qr[e], qi[e]);
            }
            streamStore(reinterpret_cast<V*>(re + up[k]), ar[k]);
            streamStore(reinterpret_cast<V*>(im + up[k]), ai[k]);
            streamStore(reinterpret_cast<V*>(re + up[k] + tbit), br[k]);
            streamStore(reinterpret_cast<V*>(im + up[k] + tbit), bi[k]);
        }
    });
}

// target inside one vector (bit 0 for fp64, bits 0-1 for fp32)
template <typename T, bool BLK>
__global__ __launch_bounds__(256) void mat2LowKernel(T* __restrict__ re, T* __restrict__ im, long long units,
                                                     InsertBits ib, int t, Cm2<T> m) {
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::n;
    constexpr int UNR = 4;
    forUnits<BLK, UNR>(units, [&](long long u0, long long step) {
        long long at[UNR];
        V vr[UNR], vi[UNR];
#pragma unroll
        for (int k = 0; k < UNR; k++) {
            const long long u = u0 + k * step;
            at[k] = u < units ? insertAll(u * VN, ib) : -1;
            if (at[k] >= 0) {
                vr[k] = streamLoad(reinterpret_cast<const V*>(re + at[k]));
                vi[k] = streamLoad(reinterpret_cast<const V*>(im + at[k]));
            }
        }
#pragma unroll
        for (int k = 0; k < UNR; k++) {
            if (at[k] < 0) continue;
            T* pr = reinterpret_cast<T*>(&vr[k]);
            T* pi = reinterpret_cast<T*>(&vi[k]);
#pragma unroll
            for (int e = 0; e < VN; e++) {
                if (e & (1 << t)) continue;
                if ((((unsigned)at[k] + e) & ib.predMask) != ib.predMask) continue;
                const int f = e | (1 << t);
                mat2apply(m, pr[e], pi[e], pr[f], pi[f]);
            }
            streamStore(reinterpret_cast<V*>(re + at[k]), vr[k]);
            streamStore(reinterpret_cast<V*>(im + at[k]), vi[k]);
        }
    });
}

// multiply the amplitudes whose mask bits are all 1
template <typename T, bool BLK>
__global__ __launch_bounds__(256) void diagDirectKernel(T* __restrict__ re, T* __restrict__ im, long long units,
                                                        InsertBits ib, T tr, T ti) {
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::n;
    constexpr int UNR = 4;
    forUnits<BLK, UNR>(units, [&](long long u0, long long step) {
        long long at[UNR];
        V vr[UNR], vi[UNR];
#pragma unroll
        for (int k = 0; k < UNR; k++) {
            const long long u = u0 + k * step;
            at[k] = u < units ? insertAll(u * VN, ib) : -1;
            if (at[k] >= 0) {
                vr[k] = streamLoad(reinterpret_cast<const V*>(re + at[k]));
                vi[k] = streamLoad(reinterpret_cast<const V*>(im + at[k]));
            }
        }
#pragma unroll
        for (int k = 0; k < UNR; k++) {
            if (at[k] < 0) continue;
            T* pr = reinterpret_cast<T*>(&vr[k]);
            T* pi = reinterpret_cast<T*>(&vi[k]);
#pragma unroll
            for (int e = 0; e < VN; e++) {
                if ((((unsigned)at[k] + e) & ib.predMask) != ib.predMask) continue;
                const T a = pr[e], b = pi[e];
                pr[e] = tr * a - ti * b;
                pi[e] = tr * b + ti * a;
            }
            streamStore(reinterpret_cast<V*>(re + at[k]), vr[k]);
            streamStore(reinterpret_cast<V*>(im + at[k]), vi[k]);
        }
    });
}

int directGrid(long long units) {
    long long g = (units + 255) / 256;
    const long long mx = (long long)numCUs() * 16;
    if (g > mx) g = mx;
    return (int)(g < 1 ? 1 : g);
}

}  // namespace

bool launchDirectOp(real* re, real* im, int L, const Op& op) {
    constexpr int VN = Vec16<real>::n;
    constexpr int vbits = VN == 2 ? 1 : 2;
    constexpr int LINE = sizeof(real) == 8 ? 4 : 5;  // log2(amps per 128-byte line)
    const long long N = 1ll << L;
    if (N < (long long)VN * 2048) return false;  // small states: one tile pass is as good
    if (op.kind != OpKind::Mat2 && op.kind != OpKind::Diag) return false;
    const bool blk = tuning().directLayout == 1;
    // Targets / masks inside a 128-byte line: the LDS tile pass streams
    // faster than the in-register pair kernels (measured 6.7 vs 7.3-8.9 ms
    // per H on 30 qubits, tools/layout_probe.py), so leave those to it.
    if (tuning().directLowToTile) {
        if (op.kind == OpKind::Mat2 && op.t[0] < LINE) return false;
        if ((op.ctrl & ((1ull << LINE) - 1)) != 0) return false;
    }

    InsertBits ib;
    ib.n = 0;
    ib.setMask = 0;
    ib.predMask = 0;
    ib.pad = 0;
    int ins[64];
    int ni = 0;
    for (int b = 0; b < L; b++) {
        if (!((op.ctrl >> b) & 1)) continue;
        if (b < LINE)
            ib.predMask |= 1u << b;
        else
            ins[ni++] = b;
    }
    for (int i = 0; i < ni; i++) ib.setMask |= 1ll << ins[i];

    if (op.kind == OpKind::Diag) {
        if (ni > 8) return false;
        for (int i = 0; i < ni; i++) ib.pos[ib.n++] = ins[i];
        const long long units = (N >> ni) / VN;
        if (blk)
            hipLaunchKernelGGL((diagDirectKernel<real, true>), dim3(directGrid(units)), dim3(256), 0, stream(), re, im,
                               units, ib, op.m[0].re, op.m[0].im);
        else
            hipLaunchKernelGGL((diagDirectKernel<real, false>), dim3(directGrid(units)), dim3(256), 0, stream(), re, im,
                               units, ib, op.m[0].re, op.m[0].im);
        QA_HIP_CHECK(hipGetLastError());
        return true;
    }

    const int t = op.t[0];
    Cm2<real> m;
    for (int i = 0; i < 4; i++) {
        m.r[i] = op.m[i].re;
        m.i[i] = op.m[i].im;
    }
    if (t >= vbits) {
        if (ni > 7) return false;
        // insert the target among the (ascending) high controls
        int all[9], na = 0;
        bool placed = false;
        for (int i = 0; i < ni; i++) {
            if (!placed && t < ins[i]) {
                all[na++] = t;
                placed = true;
            }
            all[na++] = ins[i];
        }
        if (!placed) all[na++] = t;
        for (int i = 0; i < na; i++) ib.pos[ib.n++] = all[i];
        const long long units = (N >> na) / VN;
        if (blk)
            hipLaunchKernelGGL((mat2DirectKernel<real, true>), dim3(directGrid(units)), dim3(256), 0, stream(), re, im,
                               units, ib, 1ll << t, m);
        else
            hipLaunchKernelGGL((mat2DirectKernel<real, false>), dim3(directGrid(units)), dim3(256), 0, stream(), re, im,
                               units, ib, 1ll << t, m);
    } else {
        if (ni > 8) return false;
        for (int i = 0; i < ni; i++) ib.pos[ib.n++] = ins[i];
        const long long units = (N >> ni) / VN;
        if (blk)
            hipLaunchKernelGGL((mat2LowKernel<real, true>), dim3(directGrid(units)), dim3(256), 0, stream(), re, im,
                               units, ib, t, m);
        else
            hipLaunchKernelGGL((mat2LowKernel<real, false>), dim3(directGrid(units)), dim3(256), 0, stream(), re, im,
                               units, ib, t, m);
    }
    QA_HIP_CHECK(hipGetLastError());
    return true;
}

}  // namespace hipk
}  // namespace qa
