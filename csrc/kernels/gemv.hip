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
// Decode epilogues (each removes one latency-bound launch per layer and token from the graph-decode step):
//  * RES: y = rnd(rnd(x W^T) + res)   -- the residual add after the MLP down projection (torch's bf16 add order);
//  * SWIGLU: W holds [gate; up] (2F rows); the wave streams rows n and F + n and writes
//    y[:, n] = rnd(rnd(silu(g)) * u) with g, u rounded as the unfused GEMV stores them -- bit-identical to
//    gemv + swiglu_fwd_kernel.
#include "common.h"
#include "launch.h"

using namespace sa;

namespace {

enum { EPI_NONE = 0, EPI_RES = 1, EPI_SWIGLU = 2 };

template <int M, int NR, typename E>
__device__ __forceinline__ void gemv_rows(const E* __restrict__ x, int64_t ldx, const E* const (&w)[NR], int K,
                                          int lane, float (&acc)[NR][M]) {
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int m = 0; m < M; ++m) acc[r][m] = 0.f;
    constexpr int U = 4 / NR;
    const int G = K >> 3;  // 8-element pieces per row
    int g = lane;
    for (; g + 64 * (U - 1) < G; g += 64 * U) {
        float wv[NR][U][8];
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u) V8<E>::ld(w[r] + 8 * (g + 64 * u), wv[r][u]);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int m = 0; m < M; ++m) {
                float xv[8];
                V8<E>::ld(x + m * ldx + 8 * (g + 64 * u), xv);
#pragma unroll
                for (int r = 0; r < NR; ++r)
#pragma unroll
                    for (int i = 0; i < 8; ++i) acc[r][m] = __builtin_fmaf(wv[r][u][i], xv[i], acc[r][m]);
            }
    }
    for (; g < G; g += 64) {
        float wv[NR][8];
#pragma unroll
        for (int r = 0; r < NR; ++r) V8<E>::ld(w[r] + 8 * g, wv[r]);
#pragma unroll
        for (int m = 0; m < M; ++m) {
            float xv[8];
            V8<E>::ld(x + m * ldx + 8 * g, xv);
#pragma unroll
            for (int r = 0; r < NR; ++r)
#pragma unroll
                for (int i = 0; i < 8; ++i) acc[r][m] = __builtin_fmaf(wv[r][i], xv[i], acc[r][m]);
        }
    }
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int m = 0; m < M; ++m) acc[r][m] = wave_sum(acc[r][m]);
}

// lane m < M picks input m's value out of the per-input accumulators (all lanes hold every sum after wave_sum)
template <int M>
__device__ __forceinline__ float pick(const float (&a)[M], int lane) {
    float v = a[0];
#pragma unroll
    for (int m = 1; m < M; ++m)
        if (lane == m) v = a[m];
    return v;
}

template <int M, int EPI, typename E>
__global__ __launch_bounds__(256) void gemv_kernel(const E* __restrict__ x, int64_t ldx, const E* __restrict__ W,
                                                   int64_t ldw, const E* __restrict__ bias, const E* __restrict__ res,
                                                   int64_t ldr, E* __restrict__ y, int64_t ldy, int N, int K) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= N) return;  // wave-uniform
    constexpr int NR = EPI == EPI_SWIGLU ? 2 : 1;
    const E* w[NR];
    w[0] = W + (int64_t)row * ldw;
    if constexpr (NR == 2) w[NR - 1] = W + (int64_t)(row + N) * ldw;  // up row F + n
    float acc[NR][M];
    gemv_rows<M, NR, E>(x, ldx, w, K, lane, acc);
    if (lane < M) {
        float v = pick<M>(acc[0], lane);
        if constexpr (EPI == EPI_SWIGLU) {
            const float a = rnd<E>(v), b = rnd<E>(pick<M>(acc[NR - 1], lane));
            v = rnd<E>(a / (1.f + __expf(-a))) * b;
        } else {
            if (bias != nullptr) v += IO<E>::ld(bias, row);
            if constexpr (EPI == EPI_RES) v = rnd<E>(v) + IO<E>::ld(res, (int64_t)lane * ldr + row);
        }
        IO<E>::st(y, (int64_t)lane * ldy + row, v);
    }
}

template <int EPI, typename E>
void launch(int M, const void* x, int64_t ldx, const void* W, int64_t ldw, const void* b, const void* r, int64_t ldr,
            void* y, int64_t ldy, int N, int K, hipStream_t st) {
    const dim3 grid((unsigned)((N + 3) / 4)), block(256);
    const E *xp = (const E*)x, *wp = (const E*)W, *bp = (const E*)b, *rp = (const E*)r;
    E* yp = (E*)y;
    switch (M) {
        case 1: hipLaunchKernelGGL((gemv_kernel<1, EPI, E>), grid, block, 0, st, xp, ldx, wp, ldw, bp, rp, ldr, yp, ldy, N, K); break;
        case 2: hipLaunchKernelGGL((gemv_kernel<2, EPI, E>), grid, block, 0, st, xp, ldx, wp, ldw, bp, rp, ldr, yp, ldy, N, K); break;
        case 3: hipLaunchKernelGGL((gemv_kernel<3, EPI, E>), grid, block, 0, st, xp, ldx, wp, ldw, bp, rp, ldr, yp, ldy, N, K); break;
        default: hipLaunchKernelGGL((gemv_kernel<4, EPI, E>), grid, block, 0, st, xp, ldx, wp, ldw, bp, rp, ldr, yp, ldy, N, K); break;
    }
}

template <typename E>
void launch_epi(int epi, int M, const void* x, int64_t ldx, const void* W, int64_t ldw, const void* b, const void* r,
                int64_t ldr, void* y, int64_t ldy, int N, int K, hipStream_t st) {
    if (epi == EPI_SWIGLU) launch<EPI_SWIGLU, E>(M, x, ldx, W, ldw, b, r, ldr, y, ldy, N, K, st);
    else if (epi == EPI_RES) launch<EPI_RES, E>(M, x, ldx, W, ldw, b, r, ldr, y, ldy, N, K, st);
    else launch<EPI_NONE, E>(M, x, ldx, W, ldw, b, r, ldr, y, ldy, N, K, st);
}

}  // namespace

namespace sa_launch {
// epi 0: y = x W^T (+ b); 1: y = rnd(x W^T (+ b)) + res; 2: SwiGLU over W = [gate; up] (N = F output columns)
void gemv(int dtype, int M, const void* x, int64_t ldx, const void* W, int64_t ldw, const void* b, void* y, int64_t ldy,
          int N, int K, hipStream_t st, int epi, const void* res, int64_t ldr) {
    if (dtype == DT_F16) launch_epi<_Float16>(epi, M, x, ldx, W, ldw, b, res, ldr, y, ldy, N, K, st);
    else launch_epi<u16>(epi, M, x, ldx, W, ldw, b, res, ldr, y, ldy, N, K, st);
}
}  // namespace sa_launch
