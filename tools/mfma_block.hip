// MFMA experiment (VERDICT r2 "next round" item 2): what a dense 4-qubit
// block costs on the fp64 matrix cores against the VALU gate handlers the wave
// engine uses today, with the state held in registers exactly as a wave of
// qa_wave_tile holds it (64 lanes x 16 amplitudes = 1024 amplitudes).
//
// Layout.  v_mfma_f64_16x16x4_f64 takes one f64 of A (16x4) and of B (4x16)
// per lane: lane l holds A[m = l & 15][k = l >> 4] and B[k = l >> 4][n = l & 15];
// its 16x16 result sits in 4 f64 per lane at row (l >> 4) + 4 i, column l & 15.
// A wave's amplitude (lane l, register j) is viewed, per column block
// cb = j >> 2, as X_cb[k][n] with k = (l >> 4) + 4 (j & 3) (target qubits:
// lane bits 4-5 and slot bits 0-1) and n = l & 15 (lane bits 0-3).  Then
// Y_cb = U X_cb is four k-steps of 4 MFMAs (re / im products); the result
// lands in the same layout (row m = (l >> 4) + 4 i in register i of block cb),
// so a 16x16 complex U is applied in place to two lane bits and two slot bits
// without any cross-lane transposition: 64 MFMAs per wave per block.
//
// Kernels (compute only: the state never leaves the registers):
//   mfma_block   ITER dense 16x16 complex blocks per wave
//   valu_gates   ITER x 4 general complex 2x2 gates on slot bits 0-3 (the
//                engine's M2 handler: 16 fp64 FMA/mul per amplitude pair)
//   valu_rot     ITER x 4 real rotations (ROTY: 3 shears on re and im)
//   split        half of the waves run mfma_block, half valu_gates (matrix
//                and vector pipes shared by waves of one SIMD)
// and a correctness check of the MFMA layout against a host product.
//
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_block.hip -o build/mfma_block && build/mfma_block
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int ITER = 256;

// U (16x16 complex, row-major re / im) as the A operands of the four k-steps:
// lane l, step kb: U[m = l & 15][k = (l >> 4) + 4 kb]
struct UOps {
    double re[4], im[4], nim[4];
};

__device__ inline UOps loadU(const double* ur, const double* ui) {
    const int l = threadIdx.x & 63, m = l & 15, kk = l >> 4;
    UOps u;
    for (int kb = 0; kb < 4; kb++) {
        u.re[kb] = ur[m * 16 + kk + 4 * kb];
        u.im[kb] = ui[m * 16 + kk + 4 * kb];
        u.nim[kb] = -u.im[kb];
    }
    return u;
}

// one dense block on the wave's 16 amplitudes per lane (xr / xi[j])
__device__ inline void mfmaBlock(const UOps& u, double* xr, double* xi) {
#pragma unroll
    for (int cb = 0; cb < 4; cb++) {
        d4 ar = {0, 0, 0, 0}, ai = {0, 0, 0, 0};
#pragma unroll
        for (int kb = 0; kb < 4; kb++) {
            const double br = xr[4 * cb + kb], bi = xi[4 * cb + kb];
            ar = __builtin_amdgcn_mfma_f64_16x16x4f64(u.re[kb], br, ar, 0, 0, 0);
            ar = __builtin_amdgcn_mfma_f64_16x16x4f64(u.nim[kb], bi, ar, 0, 0, 0);
            ai = __builtin_amdgcn_mfma_f64_16x16x4f64(u.re[kb], bi, ai, 0, 0, 0);
            ai = __builtin_amdgcn_mfma_f64_16x16x4f64(u.im[kb], br, ai, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
            xr[4 * cb + i] = ar[i];
            xi[4 * cb + i] = ai[i];
        }
    }
}

// general complex 2x2 on slot bit s (pairs j, j | 2^s): m = 8 reals
__device__ inline void m2(const double* m, int s, double* xr, double* xi) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
        if ((j >> s) & 1) continue;
        const int f = j | (1 << s);
        const double ar = xr[j], ai = xi[j], br = xr[f], bi = xi[f];
        xr[j] = m[0] * ar - m[1] * ai + m[2] * br - m[3] * bi;
        xi[j] = m[0] * ai + m[1] * ar + m[2] * bi + m[3] * br;
        xr[f] = m[4] * ar - m[5] * ai + m[6] * br - m[7] * bi;
        xi[f] = m[4] * ai + m[5] * ar + m[6] * bi + m[7] * br;
    }
}

// real rotation by three shears (the engine's ROTY): t = tan(phi/2), sn = sin(phi)
__device__ inline void roty(double t, double sn, int s, double* xr, double* xi) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
        if ((j >> s) & 1) continue;
        const int f = j | (1 << s);
        xr[j] -= t * xr[f];
        xr[f] += sn * xr[j];
        xr[j] -= t * xr[f];
        xi[j] -= t * xi[f];
        xi[f] += sn * xi[j];
        xi[j] -= t * xi[f];
    }
}

__device__ inline void initState(double* xr, double* xi) {
    const int l = threadIdx.x & 63;
    for (int j = 0; j < 16; j++) {
        xr[j] = 1.0 / 32 + 1e-3 * (l ^ j);
        xi[j] = 1e-3 * (l + j);
    }
}

__device__ inline void sink(const double* xr, const double* xi, double* out) {
    double s = 0;
    for (int j = 0; j < 16; j++) s += xr[j] + xi[j];
    if (s == 12345.678) out[0] = s;   // keeps the work alive
}

__global__ void __launch_bounds__(512) mfma_block(const double* ur, const double* ui, double* out) {
    const UOps u = loadU(ur, ui);
    double xr[16], xi[16];
    initState(xr, xi);
    for (int it = 0; it < ITER; it++) mfmaBlock(u, xr, xi);
    sink(xr, xi, out);
}

__global__ void __launch_bounds__(512) valu_gates(const double* mm, double* out) {
    double m[8];
    for (int i = 0; i < 8; i++) m[i] = mm[i];
    double xr[16], xi[16];
    initState(xr, xi);
    for (int it = 0; it < ITER; it++)
#pragma unroll
        for (int s = 0; s < 4; s++) m2(m, s, xr, xi);
    sink(xr, xi, out);
}

__global__ void __launch_bounds__(512) valu_rot(double t, double sn, double* out) {
    double xr[16], xi[16];
    initState(xr, xi);
    for (int it = 0; it < ITER; it++)
#pragma unroll
        for (int s = 0; s < 4; s++) roty(t, sn, s, xr, xi);
    sink(xr, xi, out);
}

// waves of even index: MFMA blocks, odd: VALU gates (one SIMD hosts both kinds)
__global__ void __launch_bounds__(512) split(const double* ur, const double* ui, const double* mm, double* out) {
    double xr[16], xi[16];
    initState(xr, xi);
    if (((threadIdx.x >> 6) & 1) == 0) {
        const UOps u = loadU(ur, ui);
        for (int it = 0; it < ITER; it++) mfmaBlock(u, xr, xi);
    } else {
        double m[8];
        for (int i = 0; i < 8; i++) m[i] = mm[i];
        for (int it = 0; it < ITER; it++)
#pragma unroll
            for (int s = 0; s < 4; s++) m2(m, s, xr, xi);
    }
    sink(xr, xi, out);
}

// correctness: one wave applies U once to amplitudes read from `in`
// (index lane + 64 j), writes them back the same way
__global__ void mfma_check(const double* ur, const double* ui, const double* inr, const double* ini, double* outr,
                           double* outi) {
    const int l = threadIdx.x;
    const UOps u = loadU(ur, ui);
    double xr[16], xi[16];
    for (int j = 0; j < 16; j++) {
        xr[j] = inr[l + 64 * j];
        xi[j] = ini[l + 64 * j];
    }
    mfmaBlock(u, xr, xi);
    for (int j = 0; j < 16; j++) {
        outr[l + 64 * j] = xr[j];
        outi[l + 64 * j] = xi[j];
    }
}

template <typename F>
double timeKernel(F launch, int reps = 5) {
    launch();
    CHECK(hipDeviceSynchronize());
    double best = 1e30;
    for (int r = 0; r < reps; r++) {
        const auto t0 = std::chrono::steady_clock::now();
        launch();
        CHECK(hipDeviceSynchronize());
        best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    return best;
}

int main() {
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    std::mt19937_64 rng(5);
    std::normal_distribution<double> nd;
    // random unitary: Gram-Schmidt on a complex gaussian 16x16
    std::vector<double> ur(256), ui(256);
    for (int i = 0; i < 256; i++) {
        ur[i] = nd(rng);
        ui[i] = nd(rng);
    }
    for (int r = 0; r < 16; r++) {
        for (int p = 0; p < r; p++) {
            double dr = 0, di = 0;   // <row p, row r>
            for (int c = 0; c < 16; c++) {
                dr += ur[p * 16 + c] * ur[r * 16 + c] + ui[p * 16 + c] * ui[r * 16 + c];
                di += ur[p * 16 + c] * ui[r * 16 + c] - ui[p * 16 + c] * ur[r * 16 + c];
            }
            for (int c = 0; c < 16; c++) {
                ur[r * 16 + c] -= dr * ur[p * 16 + c] - di * ui[p * 16 + c];
                ui[r * 16 + c] -= dr * ui[p * 16 + c] + di * ur[p * 16 + c];
            }
        }
        double nrm = 0;
        for (int c = 0; c < 16; c++) nrm += ur[r * 16 + c] * ur[r * 16 + c] + ui[r * 16 + c] * ui[r * 16 + c];
        nrm = std::sqrt(nrm);
        for (int c = 0; c < 16; c++) {
            ur[r * 16 + c] /= nrm;
            ui[r * 16 + c] /= nrm;
        }
    }
    std::vector<double> xr(1024), xi(1024), yr(1024), yi(1024);
    for (int i = 0; i < 1024; i++) {
        xr[i] = nd(rng);
        xi[i] = nd(rng);
    }
    double *dur, *dui, *dxr, *dxi, *dyr, *dyi, *dm, *dout;
    CHECK(hipMalloc(&dur, 256 * 8));
    CHECK(hipMalloc(&dui, 256 * 8));
    CHECK(hipMalloc(&dxr, 1024 * 8));
    CHECK(hipMalloc(&dxi, 1024 * 8));
    CHECK(hipMalloc(&dyr, 1024 * 8));
    CHECK(hipMalloc(&dyi, 1024 * 8));
    CHECK(hipMalloc(&dm, 8 * 8));
    CHECK(hipMalloc(&dout, 8));
    CHECK(hipMemcpy(dur, ur.data(), 256 * 8, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dui, ui.data(), 256 * 8, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dxr, xr.data(), 1024 * 8, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dxi, xi.data(), 1024 * 8, hipMemcpyHostToDevice));
    const double hm[8] = {0.6, 0.0, 0.0, -0.8, 0.0, -0.8, 0.6, 0.0};   // a unitary 2x2
    CHECK(hipMemcpy(dm, hm, sizeof hm, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(mfma_check, dim3(1), dim3(64), 0, 0, dur, dui, dxr, dxi, dyr, dyi);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(yr.data(), dyr, 1024 * 8, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(yi.data(), dyi, 1024 * 8, hipMemcpyDeviceToHost));
    double err = 0;
    for (int cb = 0; cb < 4; cb++)
        for (int m = 0; m < 16; m++)
            for (int n = 0; n < 16; n++) {
                double sr = 0, si = 0;
                for (int k = 0; k < 16; k++) {
                    const int ix = (n | (k & 3) << 4) + 64 * ((k >> 2) | cb << 2);
                    sr += ur[m * 16 + k] * xr[ix] - ui[m * 16 + k] * xi[ix];
                    si += ur[m * 16 + k] * xi[ix] + ui[m * 16 + k] * xr[ix];
                }
                const int iy = (n | (m & 3) << 4) + 64 * ((m >> 2) | cb << 2);
                err = std::max(err, std::max(std::fabs(sr - yr[iy]), std::fabs(si - yi[iy])));
            }
    printf("mfma layout check: max |MFMA - host| = %.3e over 1024 amplitudes (%s)\n", err, err < 1e-13 ? "ok" : "WRONG");

    // timing: 8-wave workgroups, `per` workgroups per CU
    const int per = 4;
    const dim3 grid(cus * per), block(512);
    const double waveBlocks = (double)cus * per * 8 * ITER;           // wave x iteration
    const double passBlocks = (double)(1u << 30) / 1024;              // wave-blocks of one 2^30 pass
    auto report = [&](const char* name, double s, const char* what) {
        const double ms = 1e3 * s * passBlocks / waveBlocks;
        // 4 SIMDs per CU at the chip's clock: wave-cycles per block of one SIMD
        const double cyc = s * 2.4e9 * 4 * cus / waveBlocks;
        printf("%-12s %8.3f ms  = %6.3f ms per 2^30-amplitude pass, ~%6.0f SIMD-cycles per wave-block at 2.4 GHz  (%s)\n",
               name, 1e3 * s, ms, cyc, what);
    };
    const double tm = timeKernel([&] { hipLaunchKernelGGL(mfma_block, grid, block, 0, 0, dur, dui, dout); });
    report("mfma_block", tm, "dense 16x16 complex on lane bits 4-5 + slot bits 0-1: 64 v_mfma_f64_16x16x4_f64");
    const double tg = timeKernel([&] { hipLaunchKernelGGL(valu_gates, grid, block, 0, 0, dm, dout); });
    report("valu_gates", tg, "4 general complex 2x2 gates on slot bits 0-3 (M2 handler math)");
    const double tr = timeKernel([&] { hipLaunchKernelGGL(valu_rot, grid, block, 0, 0, 0.3, 0.55, dout); });
    report("valu_rot", tr, "4 real rotations on slot bits 0-3 (ROTY handler math)");
    const double ts = timeKernel([&] { hipLaunchKernelGGL(split, grid, block, 0, 0, dur, dui, dm, dout); });
    printf("%-12s %8.3f ms  (half the waves mfma_block, half valu_gates; sum of the halves alone %.3f ms)\n", "split",
           1e3 * ts, 0.5 * 1e3 * (tm + tg));
    return 0;
}
