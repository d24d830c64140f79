// Latency floor of one launch + host synchronisation on this GPU, next to the
// same through the QuEST C API (no Python): what the small-n end of the
// metric ("single-qubit-gate time vs #qubits", one gate + sync) can reach.
//
//   hipcc --offload-arch=gfx950 -O2 -Iinclude tools/launch_floor.hip -Lquest_amd/lib -lQuEST_hip_f64 \
//         -Wl,-rpath,$PWD/quest_amd/lib -o /tmp/launch_floor && /tmp/launch_floor
//
// Rows (median of 200):
//   empty kernel + hipStreamSynchronize      the runtime's round trip
//   empty kernel + spin on hipStreamQuery    the same, polled
//   H kernel (2^n amplitudes) + sync         a bare in-place Hadamard kernel
//   QuEST hadamard + syncQuESTEnv            the library's path (validation, queue, launch)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#include "QuEST.h"
#include "quest_amd.h"

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            return 1;                                                              \
        }                                                                          \
    } while (0)

__global__ void emptyKernel() {}

// in-place H on qubit t of separate re / im arrays, one pair per thread
__global__ void hKernel(double* re, double* im, long long half, int t) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= half) return;
    const long long lo = ((i >> t) << (t + 1)) | (i & ((1ll << t) - 1));
    const long long hi = lo | (1ll << t);
    const double s = 0.70710678118654752440;
    const double a = re[lo], b = re[hi], c = im[lo], d = im[hi];
    re[lo] = s * (a + b);
    re[hi] = s * (a - b);
    im[lo] = s * (c + d);
    im[hi] = s * (c - d);
}

template <typename F>
double medianUs(F f, int reps = 200) {
    std::vector<double> t;
    for (int r = 0; r < 20; r++) f();
    for (int r = 0; r < reps; r++) {
        const auto t0 = std::chrono::steady_clock::now();
        f();
        t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    printf("empty kernel + hipStreamSynchronize   %6.1f us\n", medianUs([&] {
               hipLaunchKernelGGL(emptyKernel, dim3(1), dim3(64), 0, s);
               (void)hipStreamSynchronize(s);
           }));
    printf("empty kernel + spin on hipStreamQuery %6.1f us\n", medianUs([&] {
               hipLaunchKernelGGL(emptyKernel, dim3(1), dim3(64), 0, s);
               while (hipStreamQuery(s) == hipErrorNotReady) {
               }
           }));
    for (int n : {14, 20, 22}) {
        double *re, *im;
        CHECK(hipMalloc(&re, sizeof(double) << n));
        CHECK(hipMalloc(&im, sizeof(double) << n));
        CHECK(hipMemset(re, 0, sizeof(double) << n));
        CHECK(hipMemset(im, 0, sizeof(double) << n));
        const long long half = 1ll << (n - 1);
        const int bs = 256;
        const unsigned grid = (unsigned)((half + bs - 1) / bs);
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        CHECK(hipEventRecord(e0, s));
        for (int r = 0; r < 100; r++) hipLaunchKernelGGL(hKernel, dim3(grid), dim3(bs), 0, s, re, im, half, n / 2);
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("n=%2d bare H kernel + sync             %6.1f us   (kernel alone, back to back: %.1f us)\n", n,
               medianUs([&] {
                   hipLaunchKernelGGL(hKernel, dim3(grid), dim3(bs), 0, s, re, im, half, n / 2);
                   (void)hipStreamSynchronize(s);
               }),
               1e3 * ms / 100);
        CHECK(hipFree(re));
        CHECK(hipFree(im));
    }
    QuESTEnv env = createQuESTEnv();
    for (int n : {14, 20, 22}) {
        setGateFusion(0);
        Qureg q = createQureg(n, env);
        initPlusState(q);
        printf("n=%2d QuEST hadamard + syncQuESTEnv    %6.1f us\n", n, medianUs([&] {
                   hadamard(q, n / 2);
                   syncQuESTEnv(env);
               }));
        destroyQureg(q, env);
    }
    destroyQuESTEnv(env);
    return 0;
}
