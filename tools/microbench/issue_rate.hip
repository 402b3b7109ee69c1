// Issue-rate microbenchmark (gfx950): chip-wide wave-instructions per ns for single
// opcodes, forced with inline asm on 8 independent accumulators per lane, 8 waves/SIMD.
// Used to calibrate the VALU budget of the FAST pre-filter.
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 2048
#define BODY8(INSN)                                                                   \
    asm volatile(INSN " %0, %0, %8\n\t" INSN " %1, %1, %8\n\t" INSN " %2, %2, %8\n\t" \
                 INSN " %3, %3, %8\n\t" INSN " %4, %4, %8\n\t" INSN " %5, %5, %8\n\t" \
                 INSN " %6, %6, %8\n\t" INSN " %7, %7, %8"                            \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                 : "v"(b))
#define BODY8_3(INSN)                                                                         \
    asm volatile(INSN " %0, %0, %8, %8\n\t" INSN " %1, %1, %8, %8\n\t" INSN " %2, %2, %8, %8\n\t" \
                 INSN " %3, %3, %8, %8\n\t" INSN " %4, %4, %8, %8\n\t" INSN " %5, %5, %8, %8\n\t" \
                 INSN " %6, %6, %8, %8\n\t" INSN " %7, %7, %8, %8"                            \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                 : "v"(b))

#define KERNEL(NAME, STMT)                                                        \
    __global__ void NAME(uint32_t* out, uint32_t s) {                             \
        uint32_t a0 = s + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7;     \
        uint32_t a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19, b = s;   \
        for (int it = 0; it < ITERS; ++it) { STMT; }                              \
        if ((a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) == 0x12345678u) out[0] = 1;   \
    }

KERNEL(k_add, BODY8("v_add_u32"))
KERNEL(k_and, BODY8("v_and_b32"))
KERNEL(k_lshl, BODY8("v_lshlrev_b32"))
KERNEL(k_pkadd, BODY8("v_pk_add_u16"))
KERNEL(k_pkmax, BODY8("v_pk_max_u16"))
KERNEL(k_lerp, BODY8_3("v_lerp_u8"))
KERNEL(k_align, BODY8_3("v_alignbyte_b32"))
KERNEL(k_perm, BODY8_3("v_perm_b32"))
KERNEL(k_bfi, BODY8_3("v_bfi_b32"))
KERNEL(k_or3, BODY8_3("v_or3_b32"))
KERNEL(k_add3, BODY8_3("v_add3_u32"))
KERNEL(k_sad, BODY8_3("v_sad_u8"))
KERNEL(k_max3, BODY8_3("v_max3_u32"))
KERNEL(k_bitop3, asm volatile("v_bitop3_b32 %0, %0, %8, %8 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %8, %8 bitop3:0x96\n\tv_bitop3_b32 %2, %2, %8, %8 bitop3:0x96\n\tv_bitop3_b32 %3, %3, %8, %8 bitop3:0x96\n\tv_bitop3_b32 %4, %4, %8, %8 bitop3:0x96\n\tv_bitop3_b32 %5, %5, %8, %8 bitop3:0x96\n\tv_bitop3_b32 %6, %6, %8, %8 bitop3:0x96\n\tv_bitop3_b32 %7, %7, %8, %8 bitop3:0x96" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b)))
KERNEL(k_xor, BODY8("v_xor_b32"))
KERNEL(k_not, asm volatile("v_not_b32 %0, %0\n\tv_not_b32 %1, %1\n\tv_not_b32 %2, %2\n\tv_not_b32 %3, %3\n\tv_not_b32 %4, %4\n\tv_not_b32 %5, %5\n\tv_not_b32 %6, %6\n\tv_not_b32 %7, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b)))
KERNEL(k_and_or, BODY8_3("v_and_or_b32"))
KERNEL(k_lshr, BODY8("v_lshrrev_b32"))

typedef void (*Fn)(uint32_t*, uint32_t);
double run(Fn f) {
    uint32_t* d;
    hipMalloc(&d, 4);
    hipEvent_t s, e;
    hipEventCreate(&s);
    hipEventCreate(&e);
    const int blocks = 256 * 8, threads = 256;
    hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, 3u);
    hipDeviceSynchronize();
    hipEventRecord(s);
    hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, 3u);
    hipEventRecord(e);
    hipEventSynchronize(e);
    float ms;
    hipEventElapsedTime(&ms, s, e);
    hipFree(d);
    return (double)blocks * threads / 64 * ITERS * 8 / (ms * 1e-3) / 1e9;
}

int main() {
    struct { const char* n; Fn f; } ks[] = {
        {"v_add_u32", k_add}, {"v_and_b32", k_and}, {"v_lshlrev_b32", k_lshl},
        {"v_pk_add_u16", k_pkadd}, {"v_pk_max_u16", k_pkmax}, {"v_lerp_u8", k_lerp},
        {"v_alignbyte_b32", k_align}, {"v_perm_b32", k_perm}, {"v_bfi_b32", k_bfi},
        {"v_or3_b32", k_or3}, {"v_add3_u32", k_add3}, {"v_sad_u8", k_sad},
        {"v_max3_u32", k_max3}, {"v_bitop3_b32", k_bitop3}, {"v_xor_b32", k_xor},
        {"v_not_b32", k_not}, {"v_and_or_b32", k_and_or}, {"v_lshrrev_b32", k_lshr}};
    for (auto& k : ks) {
        const double r = run(k.f);
        printf("%-16s %7.1f G wave-instr/s  %.3f per CU-cycle @2.4GHz\n", k.n, r, r / 256 / 2.4);
    }
    return 0;
}
