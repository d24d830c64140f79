// Streaming-kernel probe for the unfused (one gate = one pass) path: in-place
// Hadamard over a fp64 state held as two arrays (re, im) of 2^n doubles, as a
// register stores it, in several launch / unroll / cache-policy shapes, next
// to a device-to-device copy of the same bytes.  All variants run in one
// process on the same allocation, so the table is a same-box A/B.
//
//   hipcc -O3 --offload-arch=gfx950 tools/stream_variants.hip -o build/stream_variants
//   ./build/stream_variants [n=30] [reps=7]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ d2 ld(const d2* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT>
__device__ __forceinline__ void st(d2* p, d2 v) {
    if constexpr (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

constexpr double kS = 0.70710678118654752440;

// H on bit 0: both amplitudes of a pair are in one 16-byte vector.
// GRID = 0: one chunk of 256*UNR vectors per workgroup, no loop (grid = units / (256*UNR));
// GRID > 0: GRID workgroups per CU, each looping over chunks.
template <int UNR, bool NT, bool STRIDE>
__global__ __launch_bounds__(256) void hLow(d2* __restrict__ re, d2* __restrict__ im, long long units, int loopChunks) {
    const long long per = 256ll * UNR;
    for (long long c = blockIdx.x; c * per < units; c += gridDim.x) {
        d2 a[UNR], b[UNR];
        long long at[UNR];
#pragma unroll
        for (int k = 0; k < UNR; k++) {
            at[k] = STRIDE ? c * per + k * 256 + threadIdx.x : c * per + threadIdx.x * UNR + k;
            a[k] = ld<NT>(re + at[k]);
            b[k] = ld<NT>(im + at[k]);
        }
#pragma unroll
        for (int k = 0; k < UNR; k++) {
            d2 x = a[k], y = b[k];
            a[k] = d2{(x.x + x.y) * kS, (x.x - x.y) * kS};
            b[k] = d2{(y.x + y.y) * kS, (y.x - y.y) * kS};
            st<NT>(re + at[k], a[k]);
            st<NT>(im + at[k], b[k]);
        }
        if (!loopChunks) break;
    }
}

// H on bit t >= 1 (vector index bit tv = t - 1): vector u pairs with u + 2^tv.
template <int UNR, bool NT>
__global__ __launch_bounds__(256) void hHigh(d2* __restrict__ re, d2* __restrict__ im, long long units, int tv,
                                             int loopChunks) {
    const long long per = 256ll * UNR;
    const long long half = units / 2;
    const long long off = 1ll << tv;
    for (long long c = blockIdx.x; c * per < half; c += gridDim.x) {
        d2 a0[UNR], b0[UNR], a1[UNR], b1[UNR];
        long long at[UNR];
#pragma unroll
        for (int k = 0; k < UNR; k++) {
            const long long u = c * per + k * 256 + threadIdx.x;
            at[k] = ((u >> tv) << (tv + 1)) | (u & (off - 1));
            a0[k] = ld<NT>(re + at[k]);
            b0[k] = ld<NT>(im + at[k]);
            a1[k] = ld<NT>(re + at[k] + off);
            b1[k] = ld<NT>(im + at[k] + off);
        }
#pragma unroll
        for (int k = 0; k < UNR; k++) {
            st<NT>(re + at[k], (a0[k] + a1[k]) * kS);
            st<NT>(im + at[k], (b0[k] + b1[k]) * kS);
            st<NT>(re + at[k] + off, (a0[k] - a1[k]) * kS);
            st<NT>(im + at[k] + off, (b0[k] - b1[k]) * kS);
        }
        if (!loopChunks) break;
    }
}

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 30;
    const int reps = argc > 2 ? atoi(argv[2]) : 7;
    const long long N = 1ll << n, units = N / 2;
    const double traffic = 2.0 * 16.0 * (double)N;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    d2 *re, *im, *cp;
    CK(hipMalloc(&re, N * 8));
    CK(hipMalloc(&im, N * 8));
    CK(hipMalloc(&cp, N * 8));
    CK(hipMemset(re, 0, N * 8));
    CK(hipMemset(im, 0, N * 8));
    CK(hipMemset(cp, 0, N * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto&& launch) {
        launch();
        CK(hipDeviceSynchronize());
        std::vector<double> ts;
        for (int r = 0; r < reps; r++) {
            CK(hipEventRecord(e0, 0));
            launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        const double m = median(ts);
        printf("%-44s %8.3f ms  %5.2f TB/s\n", name, m, traffic / (m * 1e-3) / 1e12);
        fflush(stdout);
    };
    printf("n=%d, %d CUs, state 2 x %.1f GiB, traffic %.1f GB per pass\n", n, cus, N * 8.0 / (1 << 30), traffic / 1e9);
    // same bytes as one pass: read 16 GiB + write 16 GiB
    timeit("hipMemcpy D2D re->cp, im->re (same bytes)", [&] {
        CK(hipMemcpyAsync(cp, re, N * 8, hipMemcpyDeviceToDevice, 0));
        CK(hipMemcpyAsync(re, im, N * 8, hipMemcpyDeviceToDevice, 0));
    });
#define LOW(U, NT, S, G)                                                                                   \
    timeit("low  UNR=" #U " NT=" #NT " stride=" #S " grid=" #G, [&] {                                     \
        const long long chunks = (units + 256ll * U - 1) / (256ll * U);                                   \
        const long long g = G ? std::min<long long>(chunks, (long long)cus * G) : chunks;                 \
        hipLaunchKernelGGL((hLow<U, NT, S>), dim3(g), dim3(256), 0, 0, re, im, units, G ? 1 : 0);         \
    })
    LOW(1, true, true, 0);
    LOW(2, true, true, 0);
    LOW(4, true, true, 0);
    LOW(4, false, true, 0);
    LOW(8, true, true, 0);
    LOW(4, true, false, 0);
    LOW(2, true, true, 16);
    LOW(4, true, true, 16);
    LOW(4, true, true, 32);
    LOW(4, true, true, 64);
    LOW(8, true, true, 32);
#define HIGH(U, NT, T, G)                                                                                   \
    if (T < n) timeit("high UNR=" #U " NT=" #NT " t=" #T " grid=" #G, [&] {                                           \
        const long long chunks = (units / 2 + 256ll * U - 1) / (256ll * U);                                \
        const long long g = G ? std::min<long long>(chunks, (long long)cus * G) : chunks;                  \
        hipLaunchKernelGGL((hHigh<U, NT>), dim3(g), dim3(256), 0, 0, re, im, units, T - 1, G ? 1 : 0);     \
    })
    HIGH(1, true, 15, 0);
    HIGH(2, true, 15, 0);
    HIGH(4, true, 15, 0);
    HIGH(2, false, 15, 0);
    HIGH(2, true, 15, 16);
    HIGH(2, true, 15, 32);
    HIGH(4, true, 15, 32);
    HIGH(2, true, 1, 0);
    HIGH(2, true, 4, 0);
    HIGH(2, true, 8, 0);
    HIGH(2, true, 12, 0);
    HIGH(2, true, 20, 0);
    HIGH(2, true, 29, 0);
    HIGH(1, true, 29, 0);
    CK(hipFree(re));
    CK(hipFree(im));
    CK(hipFree(cp));
    return 0;
}
