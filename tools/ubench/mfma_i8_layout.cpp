// Probe: the operand / accumulator lane maps of the gfx950 i8 MFMAs, checked with exact integer data.
// 32x32x32 (hypothesis: the bf16 32x32x16 map at twice the K): lane l (r = l & 31, h = l >> 5) holds A[r][16h + j]
//   and B[16h + j][r] in byte j = 0..15 of its 4-dword operand; C/D: lane l, register i -> C[(i & 3) + 8 (i >> 2) + 4h][r].
// 16x16x64 (the bf16 16x16x32 map at twice the K): lane l (r = l & 15, q = l >> 4) holds A[r][16q + j], B[16q + j][r];
//   C/D: lane l, register i -> C[4q + i][r].
// Build: hipcc --offload-arch=gfx950 -O2 tools/ubench/mfma_i8_layout.cpp -o tools/ubench/mfma_i8_layout
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
__global__ void k32(const v4i* a, const v4i* b, v16i* c) {
    v16i acc = {};
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[threadIdx.x], b[threadIdx.x], acc, 0, 0, 0);
    c[threadIdx.x] = acc;
}
__global__ void k16(const v4i* a, const v4i* b, v4i* c) {
    v4i acc = {};
    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[threadIdx.x], b[threadIdx.x], acc, 0, 0, 0);
    c[threadIdx.x] = acc;
}
static int check(bool big) {
    const int M = big ? 32 : 16, K = big ? 32 : 64, NR = big ? 16 : 4;
    static int8_t A[32][64], B[64][32];
    for (int i = 0; i < M; i++)
        for (int k = 0; k < K; k++) A[i][k] = (int8_t)(rand() % 256 - 128);
    for (int k = 0; k < K; k++)
        for (int j = 0; j < M; j++) B[k][j] = (int8_t)(rand() % 256 - 128);
    int8_t ha[64][16], hb[64][16];
    for (int l = 0; l < 64; l++)
        for (int j = 0; j < 16; j++) {
            const int r = big ? (l & 31) : (l & 15), q = big ? (l >> 5) : (l >> 4);
            ha[l][j] = A[r][16 * q + j];
            hb[l][j] = B[16 * q + j][r];
        }
    void *da, *db, *dc;
    (void)hipMalloc(&da, sizeof ha); (void)hipMalloc(&db, sizeof hb); (void)hipMalloc(&dc, 64 * 64);
    (void)hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    if (big) hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, (const v4i*)da, (const v4i*)db, (v16i*)dc);
    else hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, (const v4i*)da, (const v4i*)db, (v4i*)dc);
    int32_t hc[64][16];
    (void)hipMemcpy(hc, dc, 64 * NR * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; l++)
        for (int i = 0; i < NR; i++) {
            const int row = big ? (i & 3) + 8 * (i >> 2) + 4 * (l >> 5) : 4 * (l >> 4) + i, col = big ? (l & 31) : (l & 15);
            int s = 0;
            for (int k = 0; k < K; k++) s += A[row][k] * B[k][col];
            if (reinterpret_cast<int32_t*>(hc)[l * NR + i] != s) bad++;
        }
    (void)hipFree(da); (void)hipFree(db); (void)hipFree(dc);
    printf("mfma_i32_%s_i8: %d of %d results differ from the hypothesised map\n", big ? "32x32x32" : "16x16x64", bad, 64 * NR);
    return bad;
}
int main() {
    srand(7);
    int bad = check(true) + check(false);
    return bad != 0;
}
