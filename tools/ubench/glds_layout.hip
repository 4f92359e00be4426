// Which LDS bytes does one global_load_lds_dwordx3 / dwordx4 fill (lane-linear at 12 / 16 B per lane?)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
template <int SZ>
__global__ void k(const uint32_t* src, uint32_t* out) {
    __shared__ uint32_t lds[64 * 4 + 64];
    for (int i = threadIdx.x; i < 64 * 4 + 64; i += 64) lds[i] = 0xDEADBEEFu;
    __syncthreads();
    const int ln = threadIdx.x;
    const uint32_t* g = src + ln * (SZ / 4);
    uint32_t keep;
    const uint32_t base = (uint32_t)(uintptr_t)lds;
    if (SZ == 12)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx3 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(base) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(base) : "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * 4 + 64; i += 64) out[i] = lds[i];
}
int main() {
    uint32_t *s, *o;
    hipMalloc(&s, 4096);
    hipMalloc(&o, 4096);
    uint32_t h[1024];
    for (int i = 0; i < 1024; i++) h[i] = 0x1000 + i;
    hipMemcpy(s, h, 4096, hipMemcpyHostToDevice);
    for (int sz : {12, 16}) {
        if (sz == 12) hipLaunchKernelGGL(k<12>, dim3(1), dim3(64), 0, 0, s, o);
        else hipLaunchKernelGGL(k<16>, dim3(1), dim3(64), 0, 0, s, o);
        hipMemcpy(h, o, 4 * 320, hipMemcpyDeviceToHost);
        printf("size %d: ", sz);
        for (int i = 0; i < 24; i++) printf("%x ", h[i]);
        printf("... [190..200]: ");
        for (int i = 188; i < 200; i++) printf("%x ", h[i]);
        printf("\n");
    }
    return 0;
}
