// Re / im placement probe (gfx950): a read-modify-write stream over two arrays
// of S bytes, im starting D bytes after re inside one allocation, for several
// D; then the same for further allocations made after the first (the bench
// creates one register per circuit seed).  Prints TB/s per (allocation, D).
//   placement_probe <S GiB> <regions> <D GiB>...
// Build: hipcc --offload-arch=gfx950 -O3 -o placement_probe placement_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

// each thread: 4 vectors of 16 bytes per array, 256 threads per workgroup
__global__ __launch_bounds__(256) void rmw(double2* re, double2* im, size_t nVec) {
    const size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x;
    double2 a[4], b[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const size_t i = base + 256 * k;
        if (i < nVec) {
            a[k] = re[i];
            b[k] = im[i];
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const size_t i = base + 256 * k;
        if (i < nVec) {
            re[i] = make_double2(a[k].x + 1e-300 * b[k].y, a[k].y);
            im[i] = make_double2(b[k].x, b[k].y - 1e-300 * a[k].x);
        }
    }
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s S_GiB regions D_GiB...\n", argv[0]);
        return 2;
    }
    const size_t GiB = (size_t)1 << 30;
    const size_t S = (size_t)atof(argv[1]) * GiB;
    const int regions = atoi(argv[2]);
    std::vector<double> Ds;
    for (int i = 3; i < argc; i++) Ds.push_back(atof(argv[i]));
    double dmax = 0;
    for (double d : Ds) dmax = d > dmax ? d : dmax;
    const size_t region = (size_t)(dmax * GiB) + S;
    const size_t nVec = S / 16;
    const unsigned grid = (unsigned)((nVec + 1023) / 1024);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<char*> keep;
    for (int r = 0; r < regions; r++) {
        char* p = nullptr;
        size_t f = 0, t = 0;
        CHECK(hipMemGetInfo(&f, &t));
        if (f < region + GiB) {
            printf("region %d: %.1f GiB free, stop\n", r, f / (double)GiB);
            break;
        }
        CHECK(hipMalloc(&p, region));
        CHECK(hipMemset(p, 0, region));
        keep.push_back(p);
        printf("region %d (va %p, %.1f GiB):", r, (void*)p, region / (double)GiB);
        for (double d : Ds) {
            double2* re = reinterpret_cast<double2*>(p);
            double2* im = reinterpret_cast<double2*>(p + (size_t)(d * GiB));
            hipLaunchKernelGGL(rmw, dim3(grid), dim3(256), 0, 0, re, im, nVec);
            float best = 1e30f;
            for (int rep = 0; rep < 3; rep++) {
                CHECK(hipEventRecord(e0));
                hipLaunchKernelGGL(rmw, dim3(grid), dim3(256), 0, 0, re, im, nVec);
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
            }
            printf("  D=%g %.2f", d, 4.0 * S / (best * 1e-3) / 1e12);
        }
        printf("  TB/s\n");
        fflush(stdout);
    }
    for (char* p : keep) CHECK(hipFree(p));
    return 0;
}
