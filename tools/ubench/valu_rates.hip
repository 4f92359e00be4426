// Micro-benchmark: issue cost (cycles per wave-instruction per SIMD, 8 waves/SIMD) of the
// VALU instructions the pixel kernel is made of.  One kernel per instruction, independent
// chains per lane, s_memtime around the loop.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench/valu_rates.hip -o tools/ubench/valu_rates
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define N_IT 256
#define BODY(ASM) \
    _Pragma("unroll") for (int i = 0; i < 16; i++) asm volatile(ASM : "+v"(r[i]) : "v"(s0), "v"(s1));

template <int OP>
__global__ __launch_bounds__(512) void k(uint32_t* out, uint32_t s0, uint32_t s1, uint64_t* cyc) {
    uint32_t r[16];
    for (int i = 0; i < 16; i++) r[i] = threadIdx.x * 7 + i;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < N_IT; it++) {
        if constexpr (OP == 0) { BODY("v_add_u32 %0, %0, %1") }
        if constexpr (OP == 1) { BODY("v_dot4_u32_u8 %0, %1, %2, %0") }
        if constexpr (OP == 2) { BODY("v_dot2_u32_u16 %0, %1, %2, %0") }
        if constexpr (OP == 3) { BODY("v_perm_b32 %0, %0, %1, %2") }
        if constexpr (OP == 4) { BODY("v_alignbyte_b32 %0, %0, %1, 2") }
        if constexpr (OP == 5) { BODY("v_mad_u32_u24 %0, %0, %1, %2") }
        if constexpr (OP == 6) { BODY("v_sad_u8 %0, %0, %1, %2") }
        if constexpr (OP == 7) { BODY("v_cvt_pk_u8_f32 %0, %1, 2, %0") }
        if constexpr (OP == 8) { BODY("v_mov_b32_dpp %0, %0 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1") }
        if constexpr (OP == 9) { BODY("v_bfe_u32 %0, %0, 8, %1") }
        if constexpr (OP == 10) { BODY("v_lshl_or_b32 %0, %0, 16, %1") }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
    for (int i = 0; i < 16; i++) acc ^= r[i];
    out[blockIdx.x * 512 + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// NV v_dot4 + NS s_add per iteration in one wave's stream (VALU/SALU co-issue)
template <int NS>
__global__ __launch_bounds__(512) void km(uint32_t* out, uint32_t s0, uint32_t s1, uint64_t* cyc) {
    uint32_t r[16];
    for (int i = 0; i < 16; i++) r[i] = threadIdx.x * 7 + i;
    uint32_t sa = __builtin_amdgcn_readfirstlane(s0), sb = __builtin_amdgcn_readfirstlane(s1), sc = sa ^ 5, sd = sb ^ 9;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < N_IT; it++) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            asm volatile("v_dot4_u32_u8 %0, %1, %2, %0" : "+v"(r[i]) : "v"(s0), "v"(s1));
            if (i < NS) {
                if (i & 1) asm volatile("s_add_u32 %0, %0, %1" : "+s"(sa) : "s"(sb));
                else asm volatile("s_xor_b32 %0, %0, %1" : "+s"(sc) : "s"(sd));
            }
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = sa ^ sc;
    for (int i = 0; i < 16; i++) acc ^= r[i];
    out[blockIdx.x * 512 + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
__global__ __launch_bounds__(512) void kd(double* out, double s0, uint64_t* cyc) {
    double r[8];
    for (int i = 0; i < 8; i++) r[i] = threadIdx.x * 0.5 + i;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < N_IT; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if constexpr (OP == 0) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(r[i]) : "v"(s0));
            if constexpr (OP == 1) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(r[i]) : "v"(s0));
            if constexpr (OP == 2) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(r[i]) : "v"((uint32_t)it));
            if constexpr (OP == 3) {
                float f;
                asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f) : "v"(r[i]));
                asm volatile("" ::"v"(f));
            }
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    double acc = 0;
    for (int i = 0; i < 8; i++) acc += r[i];
    out[blockIdx.x * 512 + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <typename F>
static void run(const char* name, F launch, int per_it) {
    uint64_t* cyc;
    (void)hipMalloc(&cyc, 4096 * 8);
    launch(cyc);
    (void)hipDeviceSynchronize();
    launch(cyc);
    (void)hipDeviceSynchronize();
    static uint64_t h[1024];
    (void)hipMemcpy(h, cyc, 1024 * 8, hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < 1024; i++) m += (double)h[i];
    m /= 1024;
    // 1024 workgroups of 8 waves on 256 CUs = 4 per CU = 8 waves per SIMD, all resident
    printf("%-18s %.2f cycles per wave-instruction per SIMD\n", name, m / (8.0 * N_IT * per_it));
    (void)hipFree(cyc);
}

int main() {
    uint32_t* o;
    double* od;
    (void)hipMalloc(&o, 1024 * 512 * 4);
    (void)hipMalloc(&od, 1024 * 512 * 8);
    const char* names[] = {"v_add_u32", "v_dot4_u32_u8", "v_dot2_u32_u16", "v_perm_b32", "v_alignbyte_b32", "v_mad_u32_u24",
                           "v_sad_u8", "v_cvt_pk_u8_f32", "v_mov_b32_dpp", "v_bfe_u32", "v_lshl_or_b32"};
#define R(I) run(names[I], [&](uint64_t* c) { hipLaunchKernelGGL(k<I>, dim3(1024), dim3(512), 0, 0, o, 0x01020304u, 0x05060708u, c); }, 16);
    R(0) R(1) R(2) R(3) R(4) R(5) R(6) R(7) R(8) R(9) R(10)
    const char* dn[] = {"v_fma_f64", "v_mul_f64", "v_cvt_f64_u32", "v_cvt_f32_f64"};
#define D(I) run(dn[I], [&](uint64_t* c) { hipLaunchKernelGGL(kd<I>, dim3(1024), dim3(512), 0, 0, od, 1.0000001, c); }, 8);
    D(0) D(1) D(2) D(3)
    const char* mn[] = {"16 dot4 + 0 salu", "16 dot4 + 8 salu", "16 dot4 + 16 salu"};
#define M(I, NS) run(mn[I], [&](uint64_t* c) { hipLaunchKernelGGL(km<NS>, dim3(1024), dim3(512), 0, 0, o, 0x01020304u, 0x05060708u, c); }, 16);
    M(0, 0) M(1, 8) M(2, 16)
    return 0;
}
