// Decode-time linear layer on gfx950:  y[M, N] = x[M, K] W[N, K]^T (+ b)  for M <= 4 input rows.
//
// Token-by-token generation runs every linear layer at M = 1: the layer is a weight stream (2 bytes of W per
// 2 FLOPs), and hipBLASLt's GEMM tiles move it at ~1.1 TB/s on the 7B decode step.  Here W is streamed once at
// full width (cdna_hip_programming.md, "GEMV / M <= 16 decode weights": straight to VGPRs, deep unroll, late wait):
//  * one wave per output row n, all M inputs at once; lanes split K in 16-byte pieces (8 elements), four pieces
//    per lane in flight per trip (4 KiB per wave), fp32 FMAs;
//  * x is tiny (M x K) and re-read by every wave from L1/L2 (at M <= 4 its L1 traffic stays within the CU's
//    load bandwidth);
//  * one wave reduction per (row, input) at the end; bias added in fp32, one rounding to the output type.
#include "common.h"
#include "launch.h"

using namespace sa;

namespace {

template <int M, typename E>
__global__ __launch_bounds__(256) void gemv_kernel(const E* __restrict__ x, int64_t ldx, const E* __restrict__ W,
                                                   int64_t ldw, const E* __restrict__ bias, E* __restrict__ y,
                                                   int64_t ldy, int N, int K) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= N) return;  // wave-uniform
    const E* w = W + (int64_t)row * ldw;
    float acc[M];
#pragma unroll
    for (int m = 0; m < M; ++m) acc[m] = 0.f;
    constexpr int U = 4;
    const int G = K >> 3;  // 8-element pieces per row
    int g = lane;
    for (; g + 64 * (U - 1) < G; g += 64 * U) {
        float wv[U][8];
#pragma unroll
        for (int u = 0; u < U; ++u) V8<E>::ld(w + 8 * (g + 64 * u), wv[u]);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int m = 0; m < M; ++m) {
                float xv[8];
                V8<E>::ld(x + m * ldx + 8 * (g + 64 * u), xv);
#pragma unroll
                for (int i = 0; i < 8; ++i) acc[m] = __builtin_fmaf(wv[u][i], xv[i], acc[m]);
            }
    }
    for (; g < G; g += 64) {
        float wv[8];
        V8<E>::ld(w + 8 * g, wv);
#pragma unroll
        for (int m = 0; m < M; ++m) {
            float xv[8];
            V8<E>::ld(x + m * ldx + 8 * g, xv);
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[m] = __builtin_fmaf(wv[i], xv[i], acc[m]);
        }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) acc[m] = wave_sum(acc[m]);
    if (lane < M) {
        float v = acc[0];
#pragma unroll
        for (int m = 1; m < M; ++m)
            if (lane == m) v = acc[m];
        if (bias != nullptr) v += IO<E>::ld(bias, row);
        IO<E>::st(y, (int64_t)lane * ldy + row, v);
    }
}

template <typename E>
void launch(int M, const void* x, int64_t ldx, const void* W, int64_t ldw, const void* b, void* y, int64_t ldy, int N,
            int K, hipStream_t st) {
    const dim3 grid((unsigned)((N + 3) / 4)), block(256);
    const E *xp = (const E*)x, *wp = (const E*)W, *bp = (const E*)b;
    E* yp = (E*)y;
    switch (M) {
        case 1: hipLaunchKernelGGL((gemv_kernel<1, E>), grid, block, 0, st, xp, ldx, wp, ldw, bp, yp, ldy, N, K); break;
        case 2: hipLaunchKernelGGL((gemv_kernel<2, E>), grid, block, 0, st, xp, ldx, wp, ldw, bp, yp, ldy, N, K); break;
        case 3: hipLaunchKernelGGL((gemv_kernel<3, E>), grid, block, 0, st, xp, ldx, wp, ldw, bp, yp, ldy, N, K); break;
        default: hipLaunchKernelGGL((gemv_kernel<4, E>), grid, block, 0, st, xp, ldx, wp, ldw, bp, yp, ldy, N, K); break;
    }
}

}  // namespace

namespace sa_launch {
void gemv(int dtype, int M, const void* x, int64_t ldx, const void* W, int64_t ldw, const void* b, void* y, int64_t ldy,
          int N, int K, hipStream_t st) {
    if (dtype == DT_F16) launch<_Float16>(M, x, ldx, W, ldw, b, y, ldy, N, K, st);
    else launch<u16>(M, x, ldx, W, ldw, b, y, ldy, N, K, st);
}
}  // namespace sa_launch
