// VALU issue cost of the instructions the wave kernel's register exchanges use
// (gfx950): one workgroup of 4 waves per SIMD slot, 3 waves per SIMD (the
// wave kernel's occupancy), a loop of 64 instructions of one kind on
// independent registers.  Prints ns per wave-instruction per SIMD, relative to
// v_fma_f64.  Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/valu_rate valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

#define KERNEL(name, body)                                                                     \
    __global__ __launch_bounds__(256) void name(int iters, float* out) {                      \
        float acc = threadIdx.x;                                                               \
        asm volatile(                                                                          \
            "v_mov_b32 v40, %1\n v_mov_b32 v41, %1\n v_mov_b32 v42, %1\n v_mov_b32 v43, %1\n"  \
            "v_mov_b32 v44, %1\n v_mov_b32 v45, %1\n v_mov_b32 v46, %1\n v_mov_b32 v47, %1\n"  \
            "s_mov_b32 s40, %2\n s_mov_b32 s50, 0x55555555\n s_mov_b32 s51, 0x55555555\n"       \
            "1:\n" body                                                                        \
            "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n"              \
            "v_add_f32 %0, v40, v44\n"                                                         \
            : "=v"(acc)                                                                        \
            : "v"(acc), "s"(iters)                                                             \
            : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "s40", "s50", "s51", "vcc", "scc"); \
        if (acc == 12345.f) out[threadIdx.x] = acc;                                            \
    }

// 64 instructions per loop iteration in every variant
KERNEL(k_fma64, REP64("v_fma_f64 v[40:41], v[42:43], v[44:45], v[40:41]\n"))
KERNEL(k_mov64, REP64("v_mov_b64 v[40:41], v[42:43]\n"))
KERNEL(k_pkmov, REP64("v_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\n"))
KERNEL(k_swap32, REP64("v_swap_b32 v40, v41\n"))
KERNEL(k_mov32, REP64("v_mov_b32 v40, v41\n"))
KERNEL(k_xor32, REP64("v_xor_b32 v40, 0x80000000, v41\n"))
KERNEL(k_dpp, REP64("v_mov_b32_dpp v40, v41 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"))
KERNEL(k_dpprow, REP64("v_mov_b32_dpp v40, v41 row_shr:4 row_mask:0xf bank_mask:0xa\n"))
KERNEL(k_cnd, REP64("v_cndmask_b32 v40, v41, v42, vcc\n"))
KERNEL(k_perm32, REP64("v_permlane32_swap_b32 v40, v41\n"))
KERNEL(k_perm16, REP64("v_permlane16_swap_b32 v40, v41\n"))
KERNEL(k_pkfma, REP64("v_pk_fma_f32 v[40:41], v[42:43], v[44:45], v[40:41]\n"))
KERNEL(k_add64, REP64("v_add_f64 v[40:41], v[42:43], v[44:45]\n"))
// distinct destinations, SGPR-pair mask (the TR lane-0/1 handler's form)
#define CND8 "v_cndmask_b32_e64 v40, v40, v44, s[50:51]\n v_cndmask_b32_e64 v41, v45, v41, s[50:51]\n" \
             "v_cndmask_b32_e64 v42, v42, v46, s[50:51]\n v_cndmask_b32_e64 v43, v47, v43, s[50:51]\n"
KERNEL(k_cnd_e64, REP8(CND8 CND8))
#define DPP8 "v_mov_b32_dpp v44, v40 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n" \
             "v_mov_b32_dpp v45, v41 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n" \
             "v_mov_b32_dpp v46, v42 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n" \
             "v_mov_b32_dpp v47, v43 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
KERNEL(k_dpp_distinct, REP8(DPP8 DPP8))
KERNEL(k_dpp_cnd, REP8(DPP8 CND8))
// lane ^ 4 through the LDS crossbar (no VALU), what a lane-bit-2 exchange could use
KERNEL(k_swz, "s_mov_b32 m0, -1\n" REP64("ds_swizzle_b32 v40, v41 offset:0x101f\n") "s_waitcnt lgkmcnt(0)\n")
// exec-masked DPP exchange of lane bit 0 (3 instructions per dword instead of 2 DPP + 2 cndmask)
#define EXM "v_mov_b32 v44, v40\n s_mov_b64 exec, s[50:51]\n v_mov_b32_dpp v40, v41 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n" \
            "s_not_b64 exec, exec\n v_mov_b32_dpp v41, v44 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n s_mov_b64 exec, -1\n"
KERNEL(k_exm, REP8(EXM EXM EXM EXM EXM EXM EXM EXM) "s_nop 0\n")

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    float* out;
    hipMalloc(&out, 4096);
    const int iters = 4000;
    struct V { const char* n; void (*k)(int, float*); } vs[] = {
        {"v_fma_f64", k_fma64}, {"v_add_f64", k_add64}, {"v_mov_b64", k_mov64}, {"v_pk_mov_b32", k_pkmov},
        {"v_swap_b32", k_swap32}, {"v_mov_b32", k_mov32}, {"v_xor_b32", k_xor32},
        {"v_mov_b32_dpp quad", k_dpp}, {"v_mov_b32_dpp row_shr bank", k_dpprow}, {"v_cndmask_b32", k_cnd},
        {"v_permlane32_swap", k_perm32}, {"v_permlane16_swap", k_perm16}, {"v_pk_fma_f32", k_pkfma},
        {"v_cndmask_b32_e64 s-mask, 4 dst", k_cnd_e64}, {"v_mov_b32_dpp quad, 4 dst", k_dpp_distinct},
        {"dpp x4 + cndmask x4 (TR l0)", k_dpp_cnd}, {"ds_swizzle xor 4 (LDS pipe)", k_swz},
        {"exec-masked dpp pair (3 VALU per 64)", k_exm}};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    double base = 0;
    for (auto& v : vs) {
        // 3 waves per SIMD: 12 waves (3 workgroups of 256) per CU
        hipLaunchKernelGGL(v.k, dim3(cus * 3), dim3(256), 0, 0, 10, out);
        hipEventRecord(a);
        hipLaunchKernelGGL(v.k, dim3(cus * 3), dim3(256), 0, 0, iters, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        // wave-instructions per SIMD: 3 waves x iters x 64
        const double perSimd = 3.0 * iters * 64;
        const double ns = ms * 1e6 / perSimd;
        if (!base) base = ns;
        printf("%-28s %.3f ns / wave-instr / SIMD  (%.2fx v_fma_f64)\n", v.n, ns, ns / base);
    }
    return 0;
}
