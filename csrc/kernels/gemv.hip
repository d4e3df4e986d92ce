// Decode-time linear layer on gfx950:  y[M, N] = x[M, K] W[N, K]^T (+ b)  for M <= 4 input rows.
//
// Token-by-token generation runs every linear layer at M = 1: the layer is a weight stream (2 bytes of W per
// 2 FLOPs), and hipBLASLt's GEMM tiles move it at ~1.1 TB/s on the 7B decode step.  Here W is streamed once at
// full width (cdna_hip_programming.md, "GEMV / M <= 16 decode weights": straight to VGPRs, deep unroll, late wait):
//  * one wave per output row n (or four waves splitting K, see gemv_kernel), all M inputs at once; lanes split K
//    in 16-byte pieces (8 elements), four pieces per lane in flight per trip (4 KiB per wave), fp32 FMAs;
//  * x is tiny (M x K) and re-read by every wave from L1/L2 (at M <= 4 its L1 traffic stays within the CU's
//    load bandwidth);
//  * one wave reduction per (row, input) at the end; bias added in fp32, one rounding to the output type.
// Decode epilogues (each removes one latency-bound launch per layer and token from the graph-decode step):
//  * RES: y = rnd(rnd(x W^T) + res)   -- the residual add after the MLP down projection (torch's bf16 add order);
//  * SWIGLU: W holds [gate; up] (2F rows); the wave streams rows n and F + n and writes
//    y[:, n] = rnd(rnd(silu(g)) * u) with g, u rounded as the unfused GEMV stores them -- bit-identical to
//    gemv + swiglu_fwd_kernel.
// Decode prologue (NORM): the RMSNorm in front of the projection (optionally after the residual add
// s = rnd(x + add)) runs inside the same single pass over the weights.  Every wave already reads all of x, so it
// also accumulates sum(s^2) and dots the weights with s * gamma; the row's rstd scales the dot product at the end:
//     y = rstd * sum_k w_k s_k gamma_k      (fp32; the unfused path rounds s * rstd and * gamma to bf16 first)
// No prologue pass, no barrier, no extra launch: the two latency-bound norm launches per layer and token go away.
// The wave that owns output row 0 also writes s (the new residual stream).  Eager and graph decoding both run this
// kernel, so their tokens stay identical; against norm + GEMV it differs by the two skipped bf16 roundings.
#include "common.h"
#include "launch.h"

#include <cstdlib>

using namespace sa;

namespace {

enum { EPI_NONE = 0, EPI_RES = 1, EPI_SWIGLU = 2, EPI_ROPE = 3 };

template <typename E>
struct NormArgs {
    const E* g;      // RMSNorm weight [K]; nullptr: no norm
    const E* add;    // residual added before the norm ([M, K] contiguous) or nullptr
    E* sum;          // rnd(x + add), written by the wave of output row 0 when add != nullptr
    float eps;
    // EPI_ROPE (one token, W = [q; k; v] heads of hd rows, interleaved rotary pairs = the wave's two rows):
    // rotate q -> q_out, rotate k -> kc row pos, copy v -> vc row pos (rope_kv_append_kernel's arithmetic)
    const float* cosb;
    const float* sinb;
    const int64_t* pos;
    E* q_out;
    E* kc;
    E* vc;
    int nq, nkv, hd, rd;
    int64_t lim;  // position bound: min(cache rows, rotary table rows)
    int* err;     // set when the position is out of [0, lim): nothing is written to the caches
};

// Streams this wave's share of K -- pieces g0, g0 + GS, ... (GS = 64 x waves per row) -- of NR weight rows against
// all M inputs; returns the wave-reduced dot products acc and (NORM) sums of squares ss.
template <int M, int NR, typename E, bool NORM>
__device__ __forceinline__ void gemv_rows(const E* __restrict__ x, int64_t ldx, const E* const (&w)[NR], int K,
                                          int g0, int GS, float (&acc)[NR][M], float (&ss)[M], const NormArgs<E>& na,
                                          bool write_sum) {
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int m = 0; m < M; ++m) acc[r][m] = 0.f;
#pragma unroll
    for (int m = 0; m < M; ++m) ss[m] = 0.f;
    // one 8-element piece p of every input row against the weight pieces wv (NR rows)
    auto piece = [&](int p, const float (&wv)[NR][8]) {
        float gv[8];
        if constexpr (NORM) V8<E>::ld(na.g + 8 * p, gv);
#pragma unroll
        for (int m = 0; m < M; ++m) {
            float xv[8];
            V8<E>::ld(x + m * ldx + 8 * p, xv);
            if constexpr (NORM) {
                if (na.add != nullptr) {
                    float av[8];
                    V8<E>::ld(na.add + (int64_t)m * K + 8 * p, av);
#pragma unroll
                    for (int i = 0; i < 8; ++i) xv[i] = rnd<E>(xv[i] + av[i]);
                    if (write_sum) V8<E>::st(na.sum + (int64_t)m * K + 8 * p, xv);
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    ss[m] = __builtin_fmaf(xv[i], xv[i], ss[m]);
                    xv[i] *= gv[i];
                }
            }
#pragma unroll
            for (int r = 0; r < NR; ++r)
#pragma unroll
                for (int i = 0; i < 8; ++i) acc[r][m] = __builtin_fmaf(wv[r][i], xv[i], acc[r][m]);
        }
    };
    constexpr int U = 4 / NR > 0 ? 4 / NR : 1;  // pieces per weight row per trip (4 KiB per wave)
    const int G = K >> 3;                        // 8-element pieces per row
    int g = g0;
    for (; g + GS * (U - 1) < G; g += GS * U) {
        float wv[U][NR][8];
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u) V8<E>::ld(w[r] + 8 * (g + GS * u), wv[u][r]);
#pragma unroll
        for (int u = 0; u < U; ++u) piece(g + GS * u, wv[u]);
    }
    if (g < G) {  // the ragged tail as ONE predicated trip
        float wv[U][NR][8];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (g + GS * u < G) {
#pragma unroll
                for (int r = 0; r < NR; ++r) V8<E>::ld(w[r] + 8 * (g + GS * u), wv[u][r]);
            }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (g + GS * u < G) piece(g + GS * u, wv[u]);
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
        if constexpr (NORM) ss[m] = wave_sum(ss[m]);
#pragma unroll
        for (int r = 0; r < NR; ++r) acc[r][m] = wave_sum(acc[r][m]);
    }
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

// RPW output rows per wave (consecutive rows r, r + 1): the NORM kernels take 2, which halves the per-weight-byte
// work on x / add / gamma (every wave recomputes the normalised row for the pieces it streams).
// KS waves per row (1 or 4): with few output rows (N = 4096: o / down projections) one wave per row leaves the CUs
// a quarter occupied, so the workgroup's four waves split K (interleaved 1 KiB slices, the workgroup streams
// contiguous 4 KiB) and reduce through LDS in a fixed order.
template <int M, int EPI, typename E, bool NORM, int RPW, int KS>
__global__ __launch_bounds__(256) void gemv_kernel(const E* __restrict__ x, int64_t ldx, const E* __restrict__ W,
                                                   int64_t ldw, const E* __restrict__ bias, const E* __restrict__ res,
                                                   int64_t ldr, E* __restrict__ y, int64_t ldy, int N, int K,
                                                   NormArgs<E> na) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int row = (blockIdx.x * (4 / KS) + wv / KS) * RPW;
    const int kw = wv % KS;  // this wave's K slice
    if (row >= N) return;    // wave-uniform (N % RPW == 0); workgroup-uniform when KS == 4
    constexpr int NS = EPI == EPI_SWIGLU ? 2 : 1;  // weight rows per output row
    constexpr int NR = NS * RPW;
    const E* w[NR];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        w[q] = W + (int64_t)(row + q) * ldw;
        if constexpr (NS == 2) w[RPW + q] = W + (int64_t)(row + q + N) * ldw;  // up row F + n
    }
    float acc[NR][M], ss[M];
    gemv_rows<M, NR, E, NORM>(x, ldx, w, K, lane + 64 * kw, 64 * KS, acc, ss, na, NORM && row == 0);  // row 0's waves write s
    if constexpr (KS > 1) {
        // partial sums of the K slices: waves 1..KS-1 -> LDS, wave 0 adds them in slice order
        __shared__ float red[KS][NR + 1][M];
        if (kw > 0 && lane == 0) {
#pragma unroll
            for (int m = 0; m < M; ++m) {
#pragma unroll
                for (int r = 0; r < NR; ++r) red[kw][r][m] = acc[r][m];
                red[kw][NR][m] = ss[m];
            }
        }
        __syncthreads();
        if (kw > 0) return;
#pragma unroll
        for (int k = 1; k < KS; ++k)
#pragma unroll
            for (int m = 0; m < M; ++m) {
#pragma unroll
                for (int r = 0; r < NR; ++r) acc[r][m] += red[k][r][m];
                ss[m] += red[k][NR][m];
            }
    }
    if constexpr (NORM) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const float rstd = rsqrtf(ss[m] / K + na.eps);
#pragma unroll
            for (int r = 0; r < NR; ++r) acc[r][m] *= rstd;
        }
    }
    if constexpr (EPI == EPI_ROPE) {
        static_assert(RPW == 2, "EPI_ROPE: a wave's two rows are one rotary pair");
        if (lane == 0) {
            const float v0 = rnd<E>(acc[0][0]), v1 = rnd<E>(acc[1][0]);  // the projection's bf16 outputs
            const int h = row / na.hd, d = row - h * na.hd;
            const int64_t ps = na.pos[0];
            if (ps < 0 || ps >= na.lim) {  // out-of-range position: no cache write, q zeroed, error word set
                if (row == 0) *na.err = 1;
                if (h < na.nq) {
                    IO<E>::st(na.q_out + (int64_t)h * na.hd, d, 0.f);
                    IO<E>::st(na.q_out + (int64_t)h * na.hd, d + 1, 0.f);
                }
                return;
            }
            float o0 = v0, o1 = v1;
            E* dst;
            if (h < na.nq + na.nkv) {
                if (d < na.rd) {
                    const float cs = na.cosb[ps * (na.rd / 2) + d / 2], sn = na.sinb[ps * (na.rd / 2) + d / 2];
                    rot_pair(v0, v1, cs, sn, o0, o1);
                }
                dst = h < na.nq ? na.q_out + (int64_t)h * na.hd : na.kc + (ps * na.nkv + (h - na.nq)) * na.hd;
            } else {
                dst = na.vc + (ps * na.nkv + (h - na.nq - na.nkv)) * na.hd;
            }
            IO<E>::st(dst, d, o0);
            IO<E>::st(dst, d + 1, o1);
        }
        return;
    }
    if (lane < M) {
#pragma unroll
        for (int q = 0; q < RPW; ++q) {
            float v = pick<M>(acc[q], lane);
            if constexpr (EPI == EPI_SWIGLU) {
                const float a = rnd<E>(v), b = rnd<E>(pick<M>(acc[RPW + q], lane));
                v = rnd<E>(a / (1.f + __expf(-a))) * b;
            } else {
                if (bias != nullptr) v += IO<E>::ld(bias, row + q);
                if constexpr (EPI == EPI_RES) v = rnd<E>(v) + IO<E>::ld(res, (int64_t)lane * ldr + row + q);
            }
            IO<E>::st(y, (int64_t)lane * ldy + row + q, v);
        }
    }
}

int rows_per_wave(bool norm, int N) {
    const int r = norm ? 2 : 1;  // two rows per wave amortise the folded norm's pass over x (profiles/decode_r3b.log)
    return (r == 2 && N % 2 == 0) ? 2 : 1;
}

// waves per output row (cold-cache micro-benchmark, tools/gemv_bench.py): 4 for the NORM and SwiGLU kernels (their
// per-piece work on x / gamma / two weight rows wants more waves in flight) and for long rows over few outputs
// (the 4096 x 11008 down projection), 1 for the plain projections
int waves_per_row(bool split) { return split ? 4 : 1; }

template <int EPI, typename E, bool NORM, int RPW, int KS>
void launch_k(int M, const void* x, int64_t ldx, const void* W, int64_t ldw, const void* b, const void* r, int64_t ldr,
              void* y, int64_t ldy, int N, int K, hipStream_t st, NormArgs<E> na) {
    constexpr int RB = 4 / KS * RPW;  // output rows per workgroup
    const dim3 grid((unsigned)((N + RB - 1) / RB)), block(256);
    const E *xp = (const E*)x, *wp = (const E*)W, *bp = (const E*)b, *rp = (const E*)r;
    E* yp = (E*)y;
    if constexpr (EPI == EPI_ROPE) {
        hipLaunchKernelGGL((gemv_kernel<1, EPI, E, NORM, RPW, KS>), grid, block, 0, st, xp, ldx, wp, ldw, bp, rp, ldr, yp, ldy, N, K, na);
        return;
    }
    switch (M) {
        case 1: hipLaunchKernelGGL((gemv_kernel<1, EPI, E, NORM, RPW, KS>), grid, block, 0, st, xp, ldx, wp, ldw, bp, rp, ldr, yp, ldy, N, K, na); break;
        case 2: hipLaunchKernelGGL((gemv_kernel<2, EPI, E, NORM, RPW, KS>), grid, block, 0, st, xp, ldx, wp, ldw, bp, rp, ldr, yp, ldy, N, K, na); break;
        case 3: hipLaunchKernelGGL((gemv_kernel<3, EPI, E, NORM, RPW, KS>), grid, block, 0, st, xp, ldx, wp, ldw, bp, rp, ldr, yp, ldy, N, K, na); break;
        default: hipLaunchKernelGGL((gemv_kernel<4, EPI, E, NORM, RPW, KS>), grid, block, 0, st, xp, ldx, wp, ldw, bp, rp, ldr, yp, ldy, N, K, na); break;
    }
}

template <int EPI, typename E, bool NORM, int RPW>
void launch_r(int M, const void* x, int64_t ldx, const void* W, int64_t ldw, const void* b, const void* r, int64_t ldr,
              void* y, int64_t ldy, int N, int K, hipStream_t st, NormArgs<E> na) {
    if (waves_per_row(NORM || EPI == EPI_SWIGLU || (N <= 8192 && K >= 2 * N)) == 4) launch_k<EPI, E, NORM, RPW, 4>(M, x, ldx, W, ldw, b, r, ldr, y, ldy, N, K, st, na);
    else launch_k<EPI, E, NORM, RPW, 1>(M, x, ldx, W, ldw, b, r, ldr, y, ldy, N, K, st, na);
}

template <int EPI, typename E, bool NORM>
void launch(int M, const void* x, int64_t ldx, const void* W, int64_t ldw, const void* b, const void* r, int64_t ldr,
            void* y, int64_t ldy, int N, int K, hipStream_t st, NormArgs<E> na) {
    if constexpr (EPI == EPI_ROPE) {
        if constexpr (NORM) launch_r<EPI, E, NORM, 2>(M, x, ldx, W, ldw, b, r, ldr, y, ldy, N, K, st, na);
    } else if (rows_per_wave(NORM, N) == 2) {
        launch_r<EPI, E, NORM, 2>(M, x, ldx, W, ldw, b, r, ldr, y, ldy, N, K, st, na);
    } else {
        launch_r<EPI, E, NORM, 1>(M, x, ldx, W, ldw, b, r, ldr, y, ldy, N, K, st, na);
    }
}

template <int EPI, typename E>
void launch_n(int M, const void* x, int64_t ldx, const void* W, int64_t ldw, const void* b, const void* r, int64_t ldr,
              void* y, int64_t ldy, int N, int K, hipStream_t st, const NormArgs<E>& na) {
    if (na.g != nullptr) launch<EPI, E, true>(M, x, ldx, W, ldw, b, r, ldr, y, ldy, N, K, st, na);
    else launch<EPI, E, false>(M, x, ldx, W, ldw, b, r, ldr, y, ldy, N, K, st, na);
}

template <typename E>
void launch_epi(int epi, int M, const void* x, int64_t ldx, const void* W, int64_t ldw, const void* b, const void* r,
                int64_t ldr, void* y, int64_t ldy, int N, int K, hipStream_t st, const NormArgs<E>& na) {
    if (epi == EPI_ROPE) launch_n<EPI_ROPE, E>(1, x, ldx, W, ldw, b, r, ldr, y, ldy, N, K, st, na);
    else if (epi == EPI_SWIGLU) launch_n<EPI_SWIGLU, E>(M, x, ldx, W, ldw, b, r, ldr, y, ldy, N, K, st, na);
    else if (epi == EPI_RES) launch_n<EPI_RES, E>(M, x, ldx, W, ldw, b, r, ldr, y, ldy, N, K, st, na);
    else launch_n<EPI_NONE, E>(M, x, ldx, W, ldw, b, r, ldr, y, ldy, N, K, st, na);
}

}  // namespace

namespace sa_launch {
// epi 0: y = x W^T (+ b); 1: y = rnd(x W^T (+ b)) + res; 2: SwiGLU over W = [gate; up] (N = F output columns);
// 3 (with norm_w, one token): q/k/v projection + interleaved RoPE + K/V cache append (rope; y unused).
// norm_w != nullptr: x is first replaced by rms_norm(x (+ norm_add), norm_w, eps) inside the same pass
// (norm_add / norm_sum [M, K] contiguous; norm_sum receives x + norm_add).
void gemv(int dtype, int M, const void* x, int64_t ldx, const void* W, int64_t ldw, const void* b, void* y, int64_t ldy,
          int N, int K, hipStream_t st, int epi, const void* res, int64_t ldr, const void* norm_w, const void* norm_add,
          void* norm_sum, float eps, const GemvRope* rope) {
    const GemvRope z{};
    const GemvRope& rp = rope ? *rope : z;
    if (dtype == DT_F16) {
        const NormArgs<_Float16> na{(const _Float16*)norm_w, (const _Float16*)norm_add, (_Float16*)norm_sum, eps,
                                    rp.cosb, rp.sinb, rp.pos, (_Float16*)rp.q_out, (_Float16*)rp.kc, (_Float16*)rp.vc,
                                    rp.nq, rp.nkv, rp.hd, rp.rd, rp.lim, rp.err};
        launch_epi<_Float16>(epi, M, x, ldx, W, ldw, b, res, ldr, y, ldy, N, K, st, na);
    } else {
        const NormArgs<u16> na{(const u16*)norm_w, (const u16*)norm_add, (u16*)norm_sum, eps,
                               rp.cosb, rp.sinb, rp.pos, (u16*)rp.q_out, (u16*)rp.kc, (u16*)rp.vc,
                               rp.nq, rp.nkv, rp.hd, rp.rd, rp.lim, rp.err};
        launch_epi<u16>(epi, M, x, ldx, W, ldw, b, res, ldr, y, ldy, N, K, st, na);
    }
}
}  // namespace sa_launch
