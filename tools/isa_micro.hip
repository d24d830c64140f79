// Issue cost of single gfx950 VALU / LDS instructions (relative to v_mov_b32):
// every thread runs ITER x 16 independent copies of one instruction, enough
// waves to fill every SIMD; the time of each kernel is printed with the
// implied wave-cycles per instruction at the measured clock-free ratio.
//
//   hipcc --offload-arch=gfx950 -O2 tools/isa_micro.hip -o build/isa_micro && build/isa_micro
//
// Used to choose instruction forms in tools/gen_wave_asm.py (e.g. register
// exchanges as 64-bit moves instead of v_swap_b32).
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                \
            return 1;                                                                              \
        }                                                                                          \
    } while (0)

constexpr int ITER = 2048;

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

// 32-bit operand pairs a[i], b[i]
#define KERNEL32(name, ins)                                                                        \
    __global__ void name(unsigned* out) {                                                          \
        unsigned a[16], b[16];                                                                     \
        for (int i = 0; i < 16; i++) {                                                             \
            a[i] = threadIdx.x + i;                                                                \
            b[i] = threadIdx.x * 3 + i;                                                            \
        }                                                                                          \
        for (int it = 0; it < ITER; it++) {                                                        \
            _Pragma("unroll") for (int i = 0; i < 16; i++) asm volatile(ins : "+v"(a[i]), "+v"(b[i])); \
        }                                                                                          \
        unsigned s = 0;                                                                            \
        for (int i = 0; i < 16; i++) s += a[i] ^ b[i];                                             \
        if (s == 0x12345678u) out[0] = s;                                                          \
    }

// 64-bit operand pairs
#define KERNEL64(name, ins)                                                                        \
    __global__ void name(unsigned* out) {                                                          \
        double a[16], b[16];                                                                       \
        for (int i = 0; i < 16; i++) {                                                             \
            a[i] = threadIdx.x + i;                                                                \
            b[i] = threadIdx.x * 0.5 + i;                                                          \
        }                                                                                          \
        for (int it = 0; it < ITER; it++) {                                                        \
            _Pragma("unroll") for (int i = 0; i < 16; i++) asm volatile(ins : "+v"(a[i]), "+v"(b[i])); \
        }                                                                                          \
        double s = 0;                                                                              \
        for (int i = 0; i < 16; i++) s += a[i] + b[i];                                             \
        if (s == 1234.5) out[0] = 1;                                                               \
    }

KERNEL32(k_mov_b32, "v_mov_b32 %0, %1")
KERNEL32(k_xor_b32, "v_xor_b32 %0, %1, %0")
KERNEL32(k_swap_b32, "v_swap_b32 %0, %1")
KERNEL32(k_dpp_quad, "v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
KERNEL32(k_dpp_rowshl4, "v_mov_b32_dpp %0, %1 row_shl:4 row_mask:0xf bank_mask:0x5")
KERNEL32(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
KERNEL32(k_cndmask_s, "v_cndmask_b32_e64 %0, %0, %1, s[8:9]")
KERNEL32(k_bfi, "v_bfi_b32 %0, %1, %0, %1")
// a realistic select: vcc written once per 16 selects by a compare
__global__ void k_cndmask_cmp(unsigned* out) {
    unsigned a[16], b[16];
    for (int i = 0; i < 16; i++) {
        a[i] = threadIdx.x + i;
        b[i] = threadIdx.x * 3 + i;
    }
    unsigned lane = threadIdx.x & 63;
    for (int it = 0; it < ITER; it++) {
        asm volatile("v_and_b32 %0, 1, %0\n v_cmp_ne_u32 vcc, 0, %0" : "+v"(lane) : : "vcc");
#pragma unroll
        for (int i = 0; i < 16; i++) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]), "+v"(b[i]) : : "vcc");
    }
    unsigned s = 0;
    for (int i = 0; i < 16; i++) s += a[i] ^ b[i];
    if (s == 0x12345678u) out[0] = s;
}
KERNEL32(k_permlane32_swap, "v_permlane32_swap_b32 %0, %1")
KERNEL32(k_permlane16_swap, "v_permlane16_swap_b32 %0, %1")
KERNEL32(k_fma_f32, "v_fma_f32 %0, %1, %0, %1")
KERNEL64(k_mov_b64, "v_mov_b64 %0, %1")
KERNEL64(k_pk_mov_b32, "v_pk_mov_b32 %0, %1, %1 op_sel:[1,0]")
KERNEL64(k_fma_f64, "v_fma_f64 %0, %1, %0, %1")
KERNEL64(k_mul_f64, "v_mul_f64 %0, %1, %0")
KERNEL64(k_add_f64, "v_add_f64 %0, %1, %0")
KERNEL64(k_pk_fma_f32, "v_pk_fma_f32 %0, %1, %0, %1")

struct K {
    const char* name;
    void (*fn)(unsigned*);
};

int main() {
    K ks[] = {{"v_mov_b32", k_mov_b32},
              {"v_xor_b32", k_xor_b32},
              {"v_swap_b32", k_swap_b32},
              {"v_mov_b32_dpp quad_perm", k_dpp_quad},
              {"v_mov_b32_dpp row_shl:4", k_dpp_rowshl4},
              {"v_cndmask_b32 (vcc)", k_cndmask},
              {"v_cndmask_b32_e64 (sgpr)", k_cndmask_s},
              {"v_cndmask_b32 after v_cmp", k_cndmask_cmp},
              {"v_bfi_b32", k_bfi},
              {"v_permlane32_swap_b32", k_permlane32_swap},
              {"v_permlane16_swap_b32", k_permlane16_swap},
              {"v_fma_f32", k_fma_f32},
              {"v_mov_b64", k_mov_b64},
              {"v_pk_mov_b32 (dword swap)", k_pk_mov_b32},
              {"v_fma_f64", k_fma_f64},
              {"v_mul_f64", k_mul_f64},
              {"v_add_f64", k_add_f64},
              {"v_pk_fma_f32", k_pk_fma_f32}};
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    unsigned* out;
    CHECK(hipMalloc(&out, 64));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int threads = 256, blocks = cus * 8;   // 8 x 4 waves per CU
    const double waveInsts = (double)blocks * (threads / 64) * ITER * 16;
    float base = 0;
    printf("%d CUs, clock %d MHz; %d blocks x %d threads, %d x 16 instructions per thread\n", cus,
           prop.clockRate / 1000, blocks, threads, ITER);
    for (const K& k : ks) {
        hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(threads), 0, 0, out);   // warm
        CHECK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 5; r++) {
            CHECK(hipEventRecord(e0));
            hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(threads), 0, 0, out);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        if (base == 0) base = best;
        // wave-cycles per instruction per SIMD at the nominal clock
        const double cyc = best * 1e-3 * (prop.clockRate * 1e3) * cus * 4 / waveInsts;
        printf("%-28s %8.3f ms  %5.2fx v_mov_b32  %5.2f cycles/wave-instruction/SIMD\n", k.name, best, best / base,
               cyc);
    }
    return 0;
}
