// RMSNorm / LayerNorm forward + backward for gfx950.
// One wave64 per row, 8 elements (16 B for 16-bit types) per lane per step, the row cached in VGPRs
// (NV steps of 512 columns), fp32 statistics. dgamma/dbeta are reduced deterministically:
// every block writes an fp32 partial row, two column-parallel passes sum them in fixed order.
// Optional fusions: forward normalises x + residual (and writes the sum), backward adds the gradient
// that reaches the normalised input through the residual stream.
#include "common.h"
#include "launch.h"

#include <cstdlib>

using namespace sa;

template <typename T, int NV, bool LAYER>
__global__ __launch_bounds__(256) void norm_fwd_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                       const T* __restrict__ b, T* __restrict__ y,
                                                       float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                       int64_t rows, int H, float eps, const T* __restrict__ res,
                                                       T* __restrict__ sum_out) {
    // res != nullptr: normalise s = x + res (rounded to T like the unfused add) and also write s
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform => scalar row addressing
    if (row >= rows) return;
    const T* xr = x + row * H;
    float v[NV][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int c = (i * 64 + lane) * 8;
        if (c < H) {
            V8<T>::ld(xr + c, v[i]);
            if (res != nullptr) {
                float rv[8];
                V8<T>::ld(res + row * H + c, rv);
#pragma unroll
                for (int j = 0; j < 8; ++j) v[i][j] = rnd<T>(v[i][j] + rv[j]);
                V8<T>::st(sum_out + row * H + c, v[i]);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) s += LAYER ? v[i][j] : v[i][j] * v[i][j];
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
        }
    }
    s = wave_sum(s);
    float mean = 0.f, rstd;
    if (LAYER) {
        mean = s / H;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int c = (i * 64 + lane) * 8;
            if (c < H) {
#pragma unroll
                for (int j = 0; j < 8; ++j) { const float d = v[i][j] - mean; q += d * d; }
            }
        }
        q = wave_sum(q);
        rstd = rsqrtf(q / H + eps);
    } else {
        rstd = rsqrtf(s / H + eps);
    }
    T* yr = y + row * H;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int c = (i * 64 + lane) * 8;
        if (c < H) {
            float wv[8], o[8];
            V8<T>::ld(w + c, wv);
            if (LAYER) {
                float bv[8];
                V8<T>::ld(b + c, bv);
#pragma unroll
                for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rstd * wv[j] + bv[j];
            } else {
                // torch reference: (x * rstd).type_as(x) * weight
#pragma unroll
                for (int j = 0; j < 8; ++j) o[j] = rnd<T>(v[i][j] * rstd) * wv[j];
            }
            V8<T>::st(yr + c, o);
        }
    }
    if (lane == 0) {
        rstd_out[row] = rstd;
        if (LAYER) mean_out[row] = mean;
    }
}

// Decode-sized forward (rows <= 4, one token per sequence): one wave per row as in norm_fwd_kernel (same lane ->
// element assignment and summation order, so results are bit-identical to it), but the weight (and bias) loads are
// issued together with x before the reduction: one memory round trip instead of two on a latency-bound launch.
template <typename T, int NV, bool LAYER>
__global__ __launch_bounds__(64) void norm_fwd_row_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                          const T* __restrict__ b, T* __restrict__ y,
                                                          float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                          int H, float eps, const T* __restrict__ res,
                                                          T* __restrict__ sum_out) {
    const int lane = threadIdx.x;
    const int64_t row = blockIdx.x;
    const T* xr = x + row * H;
    float v[NV][8], wr[NV][8], br[NV][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int c = (i * 64 + lane) * 8;
        if (c < H) {
            V8<T>::ld(xr + c, v[i]);
            V8<T>::ld(w + c, wr[i]);
            if (LAYER) V8<T>::ld(b + c, br[i]);
            if (res != nullptr) {
                float rv[8];
                V8<T>::ld(res + row * H + c, rv);
#pragma unroll
                for (int j = 0; j < 8; ++j) v[i][j] = rnd<T>(v[i][j] + rv[j]);
                V8<T>::st(sum_out + row * H + c, v[i]);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) s += LAYER ? v[i][j] : v[i][j] * v[i][j];
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
        }
    }
    s = wave_sum(s);
    float mean = 0.f, rstd;
    if (LAYER) {
        mean = s / H;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int c = (i * 64 + lane) * 8;
            if (c < H) {
#pragma unroll
                for (int j = 0; j < 8; ++j) { const float d = v[i][j] - mean; q += d * d; }
            }
        }
        q = wave_sum(q);
        rstd = rsqrtf(q / H + eps);
    } else {
        rstd = rsqrtf(s / H + eps);
    }
    T* yr = y + row * H;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int c = (i * 64 + lane) * 8;
        if (c < H) {
            float o[8];
            if (LAYER) {
#pragma unroll
                for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rstd * wr[i][j] + br[i][j];
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) o[j] = rnd<T>(v[i][j] * rstd) * wr[i][j];
            }
            V8<T>::st(yr + c, o);
        }
    }
    if (lane == 0) {
        rstd_out[row] = rstd;
        if (LAYER) mean_out[row] = mean;
    }
}

// Raw 8-element vector of T kept packed in registers (halves the VGPRs of a cached bf16 row).
template <typename T> struct Raw8 { float v[8]; };
template <> struct Raw8<u16> { u16x8 v; };
template <typename T> __device__ __forceinline__ void raw_ld(const T* p, Raw8<T>& r) { V8<T>::ld(p, r.v); }
template <> __device__ __forceinline__ void raw_ld<u16>(const u16* p, Raw8<u16>& r) { r.v = *reinterpret_cast<const u16x8*>(p); }
template <typename T> __device__ __forceinline__ float raw_get(const Raw8<T>& r, int j) { return r.v[j]; }
template <> __device__ __forceinline__ float raw_get<u16>(const Raw8<u16>& r, int j) { return bf2f(r.v[j]); }
// Opaque register barrier: forces the fp32 conversions of a packed row to be recomputed after this point
// instead of being kept live (the compiler otherwise CSEs them and doubles the register footprint).
template <typename T> __device__ __forceinline__ void raw_opaque(Raw8<T>& r) {
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(r.v[j]));
}
template <> __device__ __forceinline__ void raw_opaque<u16>(Raw8<u16>& r) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4 t = __builtin_bit_cast(u32x4, r.v);
    asm volatile("" : "+v"(t));
    r.v = __builtin_bit_cast(u16x8, t);
}
template <typename T> __device__ __forceinline__ void raw_zero(Raw8<T>& r) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r.v[j] = 0;
}

// WAVES (8, or 4 for rows wider than 4096 so a lane may hold 512 VGPRs) waves per block, one row per wave per iteration.  Per-lane fp32 dgamma/dbeta accumulators are reduced
// across the block's waves through LDS (fixed pairwise tree => deterministic) and one partial row per
// BLOCK is written, so the grid can be 8x wider than with per-wave partials at the same scratch size.
constexpr int kRedSteps = 4;  // column steps (of 512) reduced per LDS round: 4 slots x 4 x 512 floats = 32 KB
template <typename T, int NV, bool LAYER, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void norm_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                       const T* __restrict__ w, const float* __restrict__ mean_in,
                                                       const float* __restrict__ rstd_in, T* __restrict__ dx,
                                                       float* __restrict__ dw_part, float* __restrict__ db_part,
                                                       int64_t rows, int H, const T* __restrict__ dadd) {
    // dadd != nullptr: dx += dadd (gradient reaching the normalised input through a residual path)
    __shared__ float red[WAVES / 2][kRedSteps * 512];
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t wave = (int64_t)blockIdx.x * WAVES + wid;
    const int64_t nwaves = (int64_t)gridDim.x * WAVES;
    float dwa[NV][8], dba[NV][8];
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) { dwa[i][j] = 0.f; dba[i][j] = 0.f; }
    Raw8<T> wr[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int c = (i * 64 + lane) * 8;
        if (c < H) raw_ld(w + c, wr[i]);
        else raw_zero(wr[i]);
    }
    for (int64_t row = wave; row < rows; row += nwaves) {
        const float rstd = rstd_in[row];
        const float mean = LAYER ? mean_in[row] : 0.f;
        Raw8<T> xr[NV], gr[NV];
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int c = (i * 64 + lane) * 8;
            if (c < H) {
                raw_ld(x + row * H + c, xr[i]);
                raw_ld(dy + row * H + c, gr[i]);
            } else {
                raw_zero(xr[i]);
                raw_zero(gr[i]);
            }
        }
        float sg = 0.f, sgx = 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float xh = (raw_get(xr[i], j) - mean) * rstd;
                const float dv = raw_get(gr[i], j);
                const float g = dv * raw_get(wr[i], j);
                sg += g;
                sgx += g * xh;
            }
        sgx = wave_sum(sgx) / H;
        sg = LAYER ? wave_sum(sg) / H : 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            raw_opaque(xr[i]);
            raw_opaque(gr[i]);
            raw_opaque(wr[i]);
        }
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int c = (i * 64 + lane) * 8;
            if (c < H) {
                float o[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    // second pass re-expands the packed row: only the accumulators stay live across rows
                    const float xh = (raw_get(xr[i], j) - mean) * rstd;
                    const float dv = raw_get(gr[i], j);
                    o[j] = rstd * (dv * raw_get(wr[i], j) - sg - xh * sgx);
                    dwa[i][j] += dv * (LAYER ? xh : rnd<T>(xh));
                    dba[i][j] += dv;
                }
                if (dadd != nullptr) {
                    float av[8];
                    V8<T>::ld(dadd + row * H + c, av);
#pragma unroll
                    for (int j = 0; j < 8; ++j) o[j] += av[j];
                }
                V8<T>::st(dx + row * H + c, o);
            }
        }
    }
    // block reduction: waves w and w + half pair up (half = 4, 2, 1); wave 0 ends with the block sum
#pragma unroll
    for (int q = 0; q < (LAYER ? 2 : 1); ++q) {
        float (&acc)[NV][8] = q == 0 ? dwa : dba;
        float* outp = q == 0 ? dw_part : db_part;
#pragma unroll
        for (int i0 = 0; i0 < NV; i0 += kRedSteps) {
#pragma unroll
            for (int half = WAVES / 2; half >= 1; half >>= 1) {
                __syncthreads();
                if (wid >= half && wid < 2 * half) {
#pragma unroll
                    for (int i = i0; i < i0 + kRedSteps && i < NV; ++i) {
                        float* d = &red[wid - half][((i - i0) * 64 + lane) * 8];
                        *reinterpret_cast<f32x4*>(d) = f32x4{acc[i][0], acc[i][1], acc[i][2], acc[i][3]};
                        *reinterpret_cast<f32x4*>(d + 4) = f32x4{acc[i][4], acc[i][5], acc[i][6], acc[i][7]};
                    }
                }
                __syncthreads();
                if (wid < half) {
#pragma unroll
                    for (int i = i0; i < i0 + kRedSteps && i < NV; ++i) {
                        const float* d = &red[wid][((i - i0) * 64 + lane) * 8];
                        const f32x4 a = *reinterpret_cast<const f32x4*>(d), b = *reinterpret_cast<const f32x4*>(d + 4);
#pragma unroll
                        for (int j = 0; j < 4; ++j) { acc[i][j] += a[j]; acc[i][j + 4] += b[j]; }
                    }
                }
            }
            if (wid == 0) {
#pragma unroll
                for (int i = i0; i < i0 + kRedSteps && i < NV; ++i) {
                    const int c = (i * 64 + lane) * 8;
                    if (c < H) V8<float>::st(outp + (int64_t)blockIdx.x * H + c, acc[i]);
                }
            }
        }
    }
}

// Column sums of the per-wave partials in two fixed-order levels (bitwise reproducible):
//   level 1: grid (H/64, S) — block (c-block, s) sums rows s, s+S, ... into part2[s, c] (4 waves split rows)
//   level 2: out[c] = sum_s part2[s, c]
constexpr int kColSplit = 32;
constexpr int bwd_waves(int nv) { return nv <= 8 ? 8 : 4; }
__global__ __launch_bounds__(256) void colsum1_kernel(const float* __restrict__ part, float* __restrict__ part2, int R, int H) {
    __shared__ float red[4][64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + lane, sidx = blockIdx.y;
    float s = 0.f;
    if (c < H)
        for (int r = sidx + kColSplit * wid; r < R; r += 4 * kColSplit) s += part[(int64_t)r * H + c];
    red[wid][lane] = s;
    __syncthreads();
    if (wid == 0 && c < H) part2[(int64_t)sidx * H + c] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}
template <typename T>
__global__ __launch_bounds__(256) void colsum2_kernel(const float* __restrict__ part2, T* __restrict__ out, int H) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= H) return;
    float s = 0.f;
#pragma unroll 8
    for (int k = 0; k < kColSplit; ++k) s += part2[(int64_t)k * H + c];
    IO<T>::st(out, c, s);
}

template <typename T, bool LAYER>
static void fwd_dispatch(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd, int64_t rows,
                         int H, float eps, const void* res, void* sum_out, hipStream_t st) {
    const int nv = (H + 511) / 512;
    dim3 grid(cdiv(rows, 4)), block(256);
    if (rows <= 4 && H <= 4096) {  // decode-sized (NV <= 8): one wave per row (profiles/decode_norm_row_ab_r2.log)
#define SA_NR(N)                                                                                                   \
    hipLaunchKernelGGL((norm_fwd_row_kernel<T, N, LAYER>), dim3((unsigned)rows), dim3(64), 0, st, (const T*)x,      \
                       (const T*)w, (const T*)b, (T*)y, mean, rstd, H, eps, (const T*)res, (T*)sum_out)
        if (nv <= 1) SA_NR(1);
        else if (nv <= 2) SA_NR(2);
        else if (nv <= 4) SA_NR(4);
        else SA_NR(8);
#undef SA_NR
        return;
    }
#define SA_NF(N)                                                                                               \
    hipLaunchKernelGGL((norm_fwd_kernel<T, N, LAYER>), grid, block, 0, st, (const T*)x, (const T*)w, (const T*)b, \
                       (T*)y, mean, rstd, rows, H, eps, (const T*)res, (T*)sum_out)
    if (nv <= 1) SA_NF(1);
    else if (nv <= 2) SA_NF(2);
    else if (nv <= 4) SA_NF(4);
    else if (nv <= 8) SA_NF(8);
    else if (nv <= 16) SA_NF(16);
    else SA_NF(32);
#undef SA_NF
}

template <typename T, bool LAYER>
static void bwd_dispatch(const void* dy, const void* x, const void* w, const float* mean, const float* rstd, void* dx,
                         void* dw, void* db, float* part, int64_t rows, int H, int nwaves, const void* dadd,
                         hipStream_t st) {
    const int nv = (H + 511) / 512;
    dim3 grid(nwaves);  // nwaves = number of partial rows = blocks
    float* dwp = part;
    float* dbp = part + (int64_t)nwaves * H;
#define SA_NB(N)                                                                                                   \
    hipLaunchKernelGGL((norm_bwd_kernel<T, N, LAYER, bwd_waves(N)>), grid, dim3(64 * bwd_waves(N)), 0, st, (const T*)dy, (const T*)x, (const T*)w, \
                       mean, rstd, (T*)dx, dwp, dbp, rows, H, (const T*)dadd)
    if (nv <= 1) SA_NB(1);
    else if (nv <= 2) SA_NB(2);
    else if (nv <= 4) SA_NB(4);
    else if (nv <= 8) SA_NB(8);
    else if (nv <= 16) SA_NB(16);
    else SA_NB(32);
#undef SA_NB
    float* p2 = part + (int64_t)(LAYER ? 2 : 1) * nwaves * H;  // kColSplit x H scratch after the partials
    hipLaunchKernelGGL(colsum1_kernel, dim3(cdiv(H, 64), kColSplit), dim3(256), 0, st, dwp, p2, nwaves, H);
    hipLaunchKernelGGL((colsum2_kernel<T>), dim3(cdiv(H, 256)), dim3(256), 0, st, p2, (T*)dw, H);
    if (LAYER) {
        hipLaunchKernelGGL(colsum1_kernel, dim3(cdiv(H, 64), kColSplit), dim3(256), 0, st, dbp, p2, nwaves, H);
        hipLaunchKernelGGL((colsum2_kernel<T>), dim3(cdiv(H, 256)), dim3(256), 0, st, p2, (T*)db, H);
    }
}

namespace sa_launch {
void norm_fwd(int dtype, bool layer, const void* x, const void* w, const void* b, void* y, float* mean, float* rstd,
              int64_t rows, int H, float eps, hipStream_t st, const void* res, void* sum_out) {
#define SA_F(T, L) fwd_dispatch<T, L>(x, w, b, y, mean, rstd, rows, H, eps, res, sum_out, st)
    if (dtype == DT_BF16) { if (layer) SA_F(u16, true); else SA_F(u16, false); }
    else if (dtype == DT_F16) { if (layer) SA_F(f16, true); else SA_F(f16, false); }
    else { if (layer) SA_F(float, true); else SA_F(float, false); }
#undef SA_F
}
int norm_bwd_waves(int64_t rows, int H) {  // = blocks of the backward kernel = fp32 partial rows
    const int wv = bwd_waves((H + 511) / 512);
    const int64_t b = (rows + wv - 1) / wv;
    return (int)(b < 512 ? b : 512);
}
int64_t norm_bwd_scratch(int64_t rows, int H, bool layer) {
    return (int64_t)(layer ? 2 : 1) * norm_bwd_waves(rows, H) * H + (int64_t)kColSplit * H;
}
void norm_bwd(int dtype, bool layer, const void* dy, const void* x, const void* w, const float* mean,
              const float* rstd, void* dx, void* dw, void* db, float* part, int64_t rows, int H, hipStream_t st,
              const void* dadd) {
    const int nw = norm_bwd_waves(rows, H);
#define SA_B(T, L) bwd_dispatch<T, L>(dy, x, w, mean, rstd, dx, dw, db, part, rows, H, nw, dadd, st)
    if (dtype == DT_BF16) { if (layer) SA_B(u16, true); else SA_B(u16, false); }
    else if (dtype == DT_F16) { if (layer) SA_B(f16, true); else SA_B(f16, false); }
    else { if (layer) SA_B(float, true); else SA_B(float, false); }
#undef SA_B
}
}  // namespace sa_launch
