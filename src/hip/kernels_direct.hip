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

#include <type_traits>

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

// This thread's groups of UNR units: u0 + k * step, k < UNR.  MODE 0:
// grid-stride (consecutive groups of one thread lie a whole grid apart);
// MODE 1: each workgroup owns contiguous runs of 256 * UNR units, so the UNR
// loads of a wave are 4 KiB apart instead of a grid's worth; MODE 2: as 1
// with exactly one run per workgroup and units a multiple of the run (no
// bounds checks: every load is unconditional and issued back to back).
template <int MODE, int UNR, typename F>
__device__ __forceinline__ void forUnits(long long units, F&& f) {
    if constexpr (MODE == 2) {
        f((long long)blockIdx.x * blockDim.x * UNR + threadIdx.x, (long long)blockDim.x);
    } else if constexpr (MODE == 1) {
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
template <typename T, int MODE, bool NT>
__global__ __launch_bounds__(256) void mat2DirectKernel(T* __restrict__ re, T* __restrict__ im, long long units,
                                                        InsertBits ib, long long tbit, Cm2<T> m) {
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::n;
    constexpr int UNR = 4;  // tools/stream_variants.hip: 4 pairs per thread 1-4 % faster than 2
    forUnits<MODE, UNR>(units, [&](long long u0, long long step) {
        long long up[UNR];
        V ar[UNR], ai[UNR], br[UNR], bi[UNR];
#pragma unroll
        for (int k = 0; k < UNR; k++) {
            const long long u = u0 + k * step;
            up[k] = (MODE == 2 || u < units) ? insertAll(u * VN, ib) : -1;
            if (MODE == 2 || up[k] >= 0) {
                ar[k] = streamLoad<V, NT>(reinterpret_cast<const V*>(re + up[k]));
                ai[k] = streamLoad<V, NT>(reinterpret_cast<const V*>(im + up[k]));
                br[k] = streamLoad<V, NT>(reinterpret_cast<const V*>(re + up[k] + tbit));
                bi[k] = streamLoad<V, NT>(reinterpret_cast<const V*>(im + up[k] + tbit));
            }
        }
#pragma unroll
        for (int k = 0; k < UNR; k++) {
            if (MODE != 2 && up[k] < 0) continue;
            T* pr = reinterpret_cast<T*>(&ar[k]);
            T* pi = reinterpret_cast<T*>(&ai[k]);
            T* qr = reinterpret_cast<T*>(&br[k]);
            T* qi = reinterpret_cast<T*>(&bi[k]);
#pragma unroll
            for (int e = 0; e < VN; e++) {
                if ((((unsigned)up[k] + e) & ib.predMask) != ib.predMask) continue;
                mat2apply(m, pr[e], pi[e], qr[e], qi[e]);
            }
            streamStore<V, NT>(reinterpret_cast<V*>(re + up[k]), ar[k]);
            streamStore<V, NT>(reinterpret_cast<V*>(im + up[k]), ai[k]);
            streamStore<V, NT>(reinterpret_cast<V*>(re + up[k] + tbit), br[k]);
            streamStore<V, NT>(reinterpret_cast<V*>(im + up[k] + tbit), bi[k]);
        }
    });
}

// target inside one vector (bit 0 for fp64, bits 0-1 for fp32)
template <typename T, int MODE, bool NT>
__global__ __launch_bounds__(256) void mat2LowKernel(T* __restrict__ re, T* __restrict__ im, long long units,
                                                     InsertBits ib, int t, Cm2<T> m) {
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::n;
    constexpr int UNR = 4;
    forUnits<MODE, UNR>(units, [&](long long u0, long long step) {
        long long at[UNR];
        V vr[UNR], vi[UNR];
#pragma unroll
        for (int k = 0; k < UNR; k++) {
            const long long u = u0 + k * step;
            at[k] = (MODE == 2 || u < units) ? insertAll(u * VN, ib) : -1;
            if (MODE == 2 || at[k] >= 0) {
                vr[k] = streamLoad<V, NT>(reinterpret_cast<const V*>(re + at[k]));
                vi[k] = streamLoad<V, NT>(reinterpret_cast<const V*>(im + at[k]));
            }
        }
#pragma unroll
        for (int k = 0; k < UNR; k++) {
            if (MODE != 2 && at[k] < 0) continue;
            T* pr = reinterpret_cast<T*>(&vr[k]);
            T* pi = reinterpret_cast<T*>(&vi[k]);
            // element indices must be compile-time (a runtime-indexed
            // register array goes to scratch: 7.7 instead of 5.9 ms per H)
            auto pairs = [&](auto tc) {
                constexpr int TT = decltype(tc)::value;
#pragma unroll
                for (int e = 0; e < VN; e++) {
                    if (e & (1 << TT)) continue;
                    if ((((unsigned)at[k] + e) & ib.predMask) != ib.predMask) continue;
                    mat2apply(m, pr[e], pi[e], pr[e | (1 << TT)], pi[e | (1 << TT)]);
                }
            };
            if (VN == 2 || t == 0)
                pairs(std::integral_constant<int, 0>{});
            else
                pairs(std::integral_constant<int, 1>{});
            streamStore<V, NT>(reinterpret_cast<V*>(re + at[k]), vr[k]);
            streamStore<V, NT>(reinterpret_cast<V*>(im + at[k]), vi[k]);
        }
    });
}

// target inside the 128-byte line but above one vector (fp64 bits 1-3,
// fp32 bits 2-4): every lane loads ONE contiguous vector per array (the
// access pattern of the in-vector kernel: 1 KiB per wave instruction), gets
// its partner's vector -- lane ^ 2^(t - vbits), the same line -- by a lane
// shuffle and computes its own half of the pair.  The pair kernel above
// would load two half-used 2 KiB spans per instruction instead (10.5 ms per
// H at 30 qubits against 7.3 in-vector, tools/direct_ab.py).  Controls
// below the line are per-element predicates; both halves of a pair agree on
// them, so a lane that fails keeps its amplitudes.
template <typename T, int MODE, bool NT>
__global__ __launch_bounds__(256) void mat2ShflKernel(T* __restrict__ re, T* __restrict__ im, long long units,
                                                      InsertBits ib, int t, int lx, Cm2<T> m) {
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::n;
    constexpr int UNR = 4;
    forUnits<MODE, UNR>(units, [&](long long u0, long long step) {
        long long at[UNR];
        V vr[UNR], vi[UNR];
#pragma unroll
        for (int k = 0; k < UNR; k++) {
            const long long u = u0 + k * step;
            // out-of-range lanes still take part in the shuffles (whole
            // 8-lane partner groups are in or out together)
            at[k] = (MODE == 2 || u < units) ? insertAll(u * VN, ib) : -1;
            if (MODE == 2 || at[k] >= 0) {
                vr[k] = streamLoad<V, NT>(reinterpret_cast<const V*>(re + at[k]));
                vi[k] = streamLoad<V, NT>(reinterpret_cast<const V*>(im + at[k]));
            } else {
                vr[k] = V{};
                vi[k] = V{};
            }
        }
#pragma unroll
        for (int k = 0; k < UNR; k++) {
            T* pr = reinterpret_cast<T*>(&vr[k]);
            T* pi = reinterpret_cast<T*>(&vi[k]);
            T qr[VN], qi[VN];
#pragma unroll
            for (int e = 0; e < VN; e++) {
                qr[e] = __shfl_xor(pr[e], lx);
                qi[e] = __shfl_xor(pi[e], lx);
            }
            if (MODE != 2 && at[k] < 0) continue;
            const bool hi = ((at[k] >> t) & 1) != 0;
            // own amplitude a (row `hi` of the matrix), partner b
            const T ar = hi ? m.r[3] : m.r[0], ai = hi ? m.i[3] : m.i[0];
            const T br = hi ? m.r[2] : m.r[1], bi = hi ? m.i[2] : m.i[1];
#pragma unroll
            for (int e = 0; e < VN; e++) {
                if ((((unsigned)at[k] + e) & ib.predMask) != ib.predMask) continue;
                const T x = pr[e], y = pi[e];
                pr[e] = ar * x - ai * y + br * qr[e] - bi * qi[e];
                pi[e] = ar * y + ai * x + br * qi[e] + bi * qr[e];
            }
            streamStore<V, NT>(reinterpret_cast<V*>(re + at[k]), vr[k]);
            streamStore<V, NT>(reinterpret_cast<V*>(im + at[k]), vi[k]);
        }
    });
}

// multiply the amplitudes whose mask bits are all 1
template <typename T, int MODE, bool NT>
__global__ __launch_bounds__(256) void diagDirectKernel(T* __restrict__ re, T* __restrict__ im, long long units,
                                                        InsertBits ib, T tr, T ti) {
    using V = typename Vec16<T>::type;
    constexpr int VN = Vec16<T>::n;
    constexpr int UNR = 4;
    forUnits<MODE, UNR>(units, [&](long long u0, long long step) {
        long long at[UNR];
        V vr[UNR], vi[UNR];
#pragma unroll
        for (int k = 0; k < UNR; k++) {
            const long long u = u0 + k * step;
            at[k] = (MODE == 2 || u < units) ? insertAll(u * VN, ib) : -1;
            if (MODE == 2 || at[k] >= 0) {
                vr[k] = streamLoad<V, NT>(reinterpret_cast<const V*>(re + at[k]));
                vi[k] = streamLoad<V, NT>(reinterpret_cast<const V*>(im + at[k]));
            }
        }
#pragma unroll
        for (int k = 0; k < UNR; k++) {
            if (MODE != 2 && at[k] < 0) continue;
            T* pr = reinterpret_cast<T*>(&vr[k]);
            T* pi = reinterpret_cast<T*>(&vi[k]);
#pragma unroll
            for (int e = 0; e < VN; e++) {
                if ((((unsigned)at[k] + e) & ib.predMask) != ib.predMask) continue;
                const T a = pr[e], b = pi[e];
                pr[e] = tr * a - ti * b;
                pi[e] = tr * b + ti * a;
            }
            streamStore<V, NT>(reinterpret_cast<V*>(re + at[k]), vr[k]);
            streamStore<V, NT>(reinterpret_cast<V*>(im + at[k]), vi[k]);
        }
    });
}

// directLayout 2 (default): one run of 256 * UNR units per workgroup and
// as many workgroups as runs -- no loop, the dispatcher keeps every CU fed
// (tools/stream_variants.hip: 5.28 ms per H at 30 qubits, 6.5 TB/s, against
// 5.40 ms with 16 looping workgroups per CU on the same box; in the library
// 6.15-6.38 vs 6.65-7.12 ms on a slower box, tools/direct_ab.py).  1: at
// most 16 workgroups per CU, each looping over runs; 0: grid-stride units.
int directMode(long long units, int unr) {
    const int lay = tuning().directLayout;
    if (lay >= 2) return units % (256ll * unr) == 0 ? 2 : 1;
    return lay;
}

int directGrid(long long units, int unr) {
    const long long per = 256ll * (tuning().directLayout >= 2 ? unr : 1);
    long long g = (units + per - 1) / per;
    if (tuning().directLayout < 2) {
        const long long mx = (long long)numCUs() * 16;
        if (g > mx) g = mx;
    }
    if (g > 0x7fffffffll) g = 0x7fffffffll;
    return (int)(g < 1 ? 1 : g);
}

}  // namespace

// States of at most QUEST_CACHED_STATE_MB (default 128 MiB, re + im) stay in
// the 256 MB Infinity Cache from one gate to the next: their kernels use plain
// loads and stores, larger ones non-temporal accesses (one HBM pass each).
static bool stateCached(long long amps) {
    static const long long limit = [] {
        const char* e = getenv("QUEST_CACHED_STATE_MB");
        return (e ? atoll(e) : 128ll) << 20;
    }();
    return 2ll * (long long)sizeof(real) * amps <= limit;
}

#define QA_DIRECT_LAUNCH_NT(KER, NT, ...)                                                                          \
    do {                                                                                                        \
        switch (directMode(units, 4)) {                                                                          \
            case 2: hipLaunchKernelGGL((KER<real, 2, NT>), grid_, dim3(256), 0, stream(), __VA_ARGS__); break;   \
            case 1: hipLaunchKernelGGL((KER<real, 1, NT>), grid_, dim3(256), 0, stream(), __VA_ARGS__); break;   \
            default: hipLaunchKernelGGL((KER<real, 0, NT>), grid_, dim3(256), 0, stream(), __VA_ARGS__); break;  \
        }                                                                                                        \
    } while (0)

#define QA_DIRECT_LAUNCH(KER, UNR, ...)                                 \
    do {                                                             \
        static_assert(UNR == 4, "the direct kernels move 4 units");  \
        const dim3 grid_(directGrid(units, UNR));                     \
        if (stateCached(N))                                           \
            QA_DIRECT_LAUNCH_NT(KER, false, __VA_ARGS__);             \
        else                                                          \
            QA_DIRECT_LAUNCH_NT(KER, true, __VA_ARGS__);              \
        QA_HIP_CHECK(hipGetLastError());                              \
    } while (0)

bool launchDirectOp(real* re, real* im, int L, const Op& op, bool launch) {
    constexpr int VN = Vec16<real>::n;
    constexpr int vbits = VN == 2 ? 1 : 2;
    constexpr int LINE = sizeof(real) == 8 ? 4 : 5;  // log2(amps per 128-byte line)
    const long long N = 1ll << L;
    if (N < (long long)VN * 2048) return false;  // small states: one tile pass is as good
    if (op.kind != OpKind::Mat2 && op.kind != OpKind::Diag) return false;
    // a rank predicate still tagged after resolution: the op does not apply on
    // this rank (core.hpp kRankTagMask) -- nothing to launch
    if (op.ctrl & kRankTagMask) return true;
    // directLowToTile = 1: targets / controls inside a 128-byte line go to
    // the LDS tile pass instead of the in-vector and lane-shuffle kernels.
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
        if (!launch) return true;
        QA_DIRECT_LAUNCH(diagDirectKernel, 4, re, im, units, ib, op.m[0].re, op.m[0].im);
        return true;
    }

    const int t = op.t[0];
    Cm2<real> m;
    for (int i = 0; i < 4; i++) {
        m.r[i] = op.m[i].re;
        m.i[i] = op.m[i].im;
    }
    if (t >= LINE) {
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
        if (!launch) return true;
        QA_DIRECT_LAUNCH(mat2DirectKernel, 4, re, im, units, ib, 1ll << t, m);
    } else if (t >= vbits) {
        if (ni > 8) return false;
        for (int i = 0; i < ni; i++) ib.pos[ib.n++] = ins[i];
        const long long units = (N >> ni) / VN;
        if (!launch) return true;
        QA_DIRECT_LAUNCH(mat2ShflKernel, 4, re, im, units, ib, t, 1 << (t - vbits), m);
    } else {
        if (ni > 8) return false;
        for (int i = 0; i < ni; i++) ib.pos[ib.n++] = ins[i];
        const long long units = (N >> ni) / VN;
        if (!launch) return true;
        QA_DIRECT_LAUNCH(mat2LowKernel, 4, re, im, units, ib, t, m);
    }
    return true;
}

}  // namespace hipk
}  // namespace qa
