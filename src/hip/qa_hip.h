// Shared declarations of the HIP (gfx950) backend translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../core/core.hpp"
#include "../core/tiles.hpp"
#include "../core/wave.hpp"

#define QA_HIP_CHECK(expr)                                                                        \
    do {                                                                                          \
        hipError_t _e = (expr);                                                                   \
        if (_e != hipSuccess) qa::hipk::fatal(#expr, hipGetErrorString(_e), __FILE__, __LINE__); \
    } while (0)

namespace qa {
namespace hipk {

[[noreturn]] void fatal(const char* expr, const char* err, const char* file, int line);

hipStream_t stream();   // the backend's compute stream (RCCL ops are ordered on it too)
// Order the compute stream after an overlapped swap still in flight
// (be::swapOverlapBegin) and run its deferred pass parts; the transport calls
// it before any other collective or exchange.
void settleSwaps();
int numCUs();

// Wait until `ev` (nullptr: everything queued on the stream) has completed.
// With a watchdog -- installed by the RCCL transport, or QUEST_SYNC_TIMEOUT
// seconds -- the wait polls instead of blocking, so a dead peer rank or a
// kernel that never finishes ends the process with a report instead of a
// silent hang.
void syncStream(hipEvent_t ev = nullptr);
// poll(elapsedSeconds) is called about every 10 ms while a wait is pending
void setSyncWatchdog(void (*poll)(double elapsedSeconds));

// runtime knobs (env QUEST_* at start-up, setQuESTTuning() afterwards)
struct Tuning {
    int directKernels = 1;  // LDS-free kernels for single-op passes
    int tileMode = 0;       // fused tiles: 0 op by op, 1 register phases, 2 dense blocks, 3 wave tiles (fp64 default)
    int tileWgPerCU = 2;    // grid of the register-phase tile kernel, per CU
    int waveWgPerCU = 0;    // grid of the wave-tile kernel: 0 one workgroup per tile, else workgroups per CU (looping)
    int directLayout = 2;   // direct kernels: 0 grid-stride units, 1 looping contiguous chunks, 2 one chunk per workgroup
    int directLowToTile = 0;  // 1: ops on bits inside a 128-byte line go to the tile pass (0: in-vector / lane-shuffle kernels)
    int tileQubits = 0;     // tile bits of fused passes (0: kTileQubits; kTileQubits + 1 = 64 KiB tiles)
    int waveTileMap = 0;    // wave kernel: XCD / CU-aware tile order (QUEST_WAVE_TILE_MAP)
    int waveDynamic = 1;    // looping wave grids claim tiles through an atomic counter (QUEST_WAVE_DYNAMIC)
};
Tuning& tuning();

// vector type moving 16 bytes of amplitudes (2 doubles or 4 floats)
template <typename T>
struct Vec16;
template <>
struct Vec16<double> {
    using type = double2;
    static constexpr int n = 2;
};
template <>
struct Vec16<float> {
    using type = float4;
    static constexpr int n = 4;
};

#ifdef __HIPCC__
// HBM streaming of the state: every amplitude is read and written once per
// pass, so the accesses are marked non-temporal (QA_NONTEMPORAL=0 at build
// time: plain accesses)
#ifndef QA_NONTEMPORAL
#define QA_NONTEMPORAL 1
#endif
typedef double qa_nd2 __attribute__((ext_vector_type(2)));
typedef float qa_nf4 __attribute__((ext_vector_type(4)));
template <typename V>
struct NativeVec;
template <>
struct NativeVec<double2> {
    using type = qa_nd2;
};
template <>
struct NativeVec<float4> {
    using type = qa_nf4;
};
typedef float qa_nf2 __attribute__((ext_vector_type(2)));
template <>
struct NativeVec<float2> {
    using type = qa_nf2;
};

// NT = false: plain accesses (the direct kernels on states that stay in the
// 256 MB Infinity Cache between gates, hipk::stateCached)
template <typename V, bool NT = (QA_NONTEMPORAL != 0)>
__device__ __forceinline__ V streamLoad(const V* p) {
    if constexpr (NT) {
        using N = typename NativeVec<V>::type;
        const N n = __builtin_nontemporal_load(reinterpret_cast<const N*>(p));
        V v;
        __builtin_memcpy(&v, &n, sizeof v);
        return v;
    } else {
        return *p;
    }
}
template <typename V, bool NT = (QA_NONTEMPORAL != 0)>
__device__ __forceinline__ void streamStore(V* p, V v) {
    if constexpr (NT) {
        using N = typename NativeVec<V>::type;
        N n;
        __builtin_memcpy(&n, &v, sizeof n);
        __builtin_nontemporal_store(n, reinterpret_cast<N*>(p));
    } else {
        *p = v;
    }
}

// LDS slot of tile element e in the permuted kernels: b's elements are written
// in its own order, scattered over a's; the XOR fold spreads a wave's writes
// over the banks (a's reads of consecutive elements stay conflict-free)
__device__ __forceinline__ int permSlot(int e) { return e ^ ((e >> 5) & 31) ^ ((e >> 10) & 31); }

// PermArgs helpers: the bits of x scattered to positions pos[0..n)
__device__ __forceinline__ unsigned long long scatterBits(unsigned long long x, const signed char* pos, int n) {
    unsigned long long r = 0;
    for (int m = 0; m < n; m++)
        if ((x >> m) & 1) r |= 1ull << pos[m];
    return r;
}

#endif  // __HIPCC__

// Tile size of the compile-time tile kernel (2^K amplitudes, 256 threads x
// 2^(K-8) registers): 32 KiB of LDS for fp64 and fp32 alike.
constexpr int kTileQubits = sizeof(real) == 8 ? 11 : 12;
constexpr int kRegSlots = kTileQubits - 8;

// Kernel launch parameters of one tile pass.
struct TileArgs {
    int L;               // local qubits of the chunk
    int k;               // tile qubits
    int c;               // contiguous low tile bits (pos[i] == i for i < c)
    int nOps;
    int nPhases;         // register phases (0: op-by-op on LDS)
    int pad;
    long long numTiles;  // 2^(L-k)
    int pos[32];         // tile bit -> physical bit
};

// Two registers of one rank whose local qubits sit on different positions:
// amplitude i of `a` pairs with amplitude sigma(i) of `b`, sigma a permutation
// of the index bits (a's position p -> b's position sig[p]).  The permuted
// kernels (innerPermKernel, axpbyPermKernel) take tiles of 2^K amplitudes
// whose a-positions include 0-3 and every position b holds on 0-3, so both
// sides load 16-element runs; b goes through LDS into a's order.
// most tile bits of the permuted kernels (4096 elements: 8 pairs a thread)
constexpr int kPermMaxBits = 12;
struct PermArgs {
    int K;                    // tile bits
    int nOut;                 // the other bits (L - K)
    signed char tA[16], tB[16];  // tile bit k: position in a / in b
    signed char bOrd[16];     // b-order bit m (b-positions ascending) -> tile bit k
    signed char oA[48], oB[48];  // other bit m: position in a / in b
};
PermArgs makePermArgs(int L, const int* sig);

#ifdef __HIPCC__
// Per-thread element pairs of a permuted tile (E = 2^K elements, 256
// threads, NP = max(1, E / 512) pairs a thread, compile-time so that the
// per-pair state stays in registers): pair g = threadIdx.x + 256 q.  b side, in
// b's order: its elements 2g, 2g+1 (b-position 0 inside the pair: one
// 2-element load) and their a-order LDS slots; a side: a's elements 2g, 2g+1
// (a-position 0).  live: g < E / 2 (only tiles under 512 elements leave
// threads idle).
template <int NP>
struct PermLanes {
    unsigned long long offB[NP], offA[NP];
    int slotB0[NP], slotB1[NP], slotA[NP];
    bool live[NP];

    __device__ __forceinline__ explicit PermLanes(const PermArgs& pa) {
        const int pairs = 1 << (pa.K - 1);
#pragma unroll
        for (int q = 0; q < NP; q++) {
            const int g = threadIdx.x + 256 * q;
            live[q] = g < pairs;
            const int f = 2 * g;
            unsigned long long ob = 0;
            int e = 0;
            for (int m = 1; m < pa.K; m++)
                if ((f >> m) & 1) {
                    ob |= 1ull << pa.tB[pa.bOrd[m]];
                    e |= 1 << pa.bOrd[m];
                }
            offB[q] = ob;
            slotB0[q] = permSlot(e);
            slotB1[q] = permSlot(e | (1 << pa.bOrd[0]));
            offA[q] = scatterBits((unsigned long long)f, pa.tA, pa.K);
            slotA[q] = permSlot(f);
        }
    }
};
// pairs per thread of a tile of K bits
constexpr int permPairsFor(int K) { return K <= 9 ? 1 : 1 << (K - 9); }
#endif  // __HIPCC__

// ---- launchers (defined in kernels_*.hip) ----------------------------------
void launchTilePass(real* re, real* im, const TileArgs& a, const TileOp* dOps, const TilePhase* dPhases,
                    const real* dMats, int mode);
// one-op pass as a streaming kernel without LDS; false if not applicable
// Run a single-op pass with an LDS-free streaming kernel if one applies
// (launch = false: only report whether one does).
bool launchDirectOp(real* re, real* im, int L, const Op& op, bool launch = true);
void launchFill(real* re, real* im, i64 n, real vr, real vi);
void launchInitDebug(real* re, real* im, i64 n, i64 offset);
void launchFillWhereBit(real* re, real* im, i64 n, int bit, int outcome, real val);
// Device-to-device copy on stream st by a streaming kernel (hipMemcpyAsync
// for unaligned sizes): the IPC transport's pulls.
void launchCopyVec(void* dst, const void* src, size_t bytes, hipStream_t st);
void launchPackBits(const real* re, const real* im, const int* pos, int k, u64 setMask, i64 start, i64 count,
                    real* br, real* bi, bool unpack);
// swap a's amplitudes with bits pos[0..k) = aMask and b's with bits = bMask,
// at equal packed index in [start, start + count) (b may be a peer's mapped
// memory)
void launchSwapParts(real* ar, real* ai, real* br, real* bi, const int* pos, int k, u64 aMask, u64 bMask, i64 start,
                     i64 count);
void launchAxpby(real* ar, real* ai, real alpha, const real* br, const real* bi, real beta, i64 n);
// a = alpha a + beta b with b's amplitude sigma(i) for a's i (PermArgs)
void launchAxpbyPerm(real* ar, real* ai, real alpha, const real* br, const real* bi, real beta, const PermArgs& pa);
void launchDensInitPure(real* re, real* im, i64 n, const real* pr, const real* pi, int nq, i64 chunkStart);

// reductions: results are written to `out` (device, doubles) and copied back
double reduceSumSq(const real* re, const real* im, i64 n, int bit, int bitVal);
// zeroSums[b] = sum |a_i|^2 over i with bit b clear (b < L), *total = sum |a_i|^2, one pass
void reduceMarginals(const real* re, const real* im, int L, double* zeroSums, double* total);
void reduceInner(const real* ar, const real* ai, const real* br, const real* bi, i64 n, double out[2]);
// sum conj(a_i) b_sigma(i) (PermArgs: one streaming pass over both, no relayout)
void reduceInnerPerm(const real* ar, const real* ai, const real* br, const real* bi, const PermArgs& pa,
                     double out[2]);
double reduceMaxDiff(const real* ar, const real* ai, const real* br, const real* bi, i64 n);
double reduceDensDiag(const real* re, i64 chunkAmps, const u64* offs, int nq, int skipBit, i64 chunkStart);
double reduceDensFidelity(const real* re, const real* im, i64 n, const real* pr, const real* pi, int nq,
                          i64 chunkStart);

}  // namespace hipk
}  // namespace qa
