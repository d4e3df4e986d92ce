// RMSNorm / LayerNorm forward + backward for gfx950.
// One wave64 per row, 8 elements (16 B for 16-bit types) per lane per step, the row cached in VGPRs
// (NV steps of 512 columns), fp32 statistics. dgamma/dbeta are reduced deterministically:
// every wave writes an fp32 partial row, a column-parallel kernel sums them in fixed order.
#include "common.h"
#include "launch.h"

using namespace sa;

template <typename T, int NV, bool LAYER>
__global__ __launch_bounds__(256) void norm_fwd_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                       const T* __restrict__ b, T* __restrict__ y,
                                                       float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                       int64_t rows, int H, float eps) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (row >= rows) return;
    const T* xr = x + row * H;
    float v[NV][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int c = (i * 64 + lane) * 8;
        if (c < H) {
            V8<T>::ld(xr + c, v[i]);
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

template <typename T, int NV, bool LAYER>
__global__ __launch_bounds__(256) void norm_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                       const T* __restrict__ w, const float* __restrict__ mean_in,
                                                       const float* __restrict__ rstd_in, T* __restrict__ dx,
                                                       float* __restrict__ dw_part, float* __restrict__ db_part,
                                                       int64_t rows, int H) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    float dwa[NV][8], dba[NV][8];
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) { dwa[i][j] = 0.f; dba[i][j] = 0.f; }
    float wv[NV][8];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int c = (i * 64 + lane) * 8;
        if (c < H) V8<T>::ld(w + c, wv[i]);
        else
#pragma unroll
            for (int j = 0; j < 8; ++j) wv[i][j] = 0.f;
    }
    for (int64_t row = wave; row < rows; row += nwaves) {
        const float rstd = rstd_in[row];
        const float mean = LAYER ? mean_in[row] : 0.f;
        float xh[NV][8], g[NV][8];
        float sg = 0.f, sgx = 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int c = (i * 64 + lane) * 8;
            if (c < H) {
                float xv[8], dv[8];
                V8<T>::ld(x + row * H + c, xv);
                V8<T>::ld(dy + row * H + c, dv);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    xh[i][j] = (xv[j] - mean) * rstd;
                    g[i][j] = dv[j] * wv[i][j];
                    sg += g[i][j];
                    sgx += g[i][j] * xh[i][j];
                    dwa[i][j] += dv[j] * (LAYER ? xh[i][j] : rnd<T>(xh[i][j]));
                    dba[i][j] += dv[j];
                }
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) { xh[i][j] = 0.f; g[i][j] = 0.f; }
            }
        }
        sgx = wave_sum(sgx) / H;
        sg = LAYER ? wave_sum(sg) / H : 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int c = (i * 64 + lane) * 8;
            if (c < H) {
                float o[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) o[j] = rstd * (g[i][j] - sg - xh[i][j] * sgx);
                V8<T>::st(dx + row * H + c, o);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int c = (i * 64 + lane) * 8;
        if (c < H) {
            V8<float>::st(dw_part + wave * H + c, dwa[i]);
            if (LAYER) V8<float>::st(db_part + wave * H + c, dba[i]);
        }
    }
}

// out[c] = sum_r part[r, c]  (fixed order => bitwise reproducible)
template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ part, T* __restrict__ out, int R, int H) {
    __shared__ float red[4][64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + lane;
    float s = 0.f;
    if (c < H)
        for (int r = wid; r < R; r += 4) s += part[(int64_t)r * H + c];
    red[wid][lane] = s;
    __syncthreads();
    if (wid == 0 && c < H) IO<T>::st(out, c, red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane]);
}

template <typename T, bool LAYER>
static void fwd_dispatch(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd, int64_t rows,
                         int H, float eps, hipStream_t st) {
    const int nv = (H + 511) / 512;
    dim3 grid(cdiv(rows, 4)), block(256);
#define SA_NF(N)                                                                                               \
    hipLaunchKernelGGL((norm_fwd_kernel<T, N, LAYER>), grid, block, 0, st, (const T*)x, (const T*)w, (const T*)b, \
                       (T*)y, mean, rstd, rows, H, eps)
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
                         void* dw, void* db, float* part, int64_t rows, int H, int nwaves, hipStream_t st) {
    const int nv = (H + 511) / 512;
    dim3 grid(nwaves / 4), block(256);
    float* dwp = part;
    float* dbp = part + (int64_t)nwaves * H;
#define SA_NB(N)                                                                                                   \
    hipLaunchKernelGGL((norm_bwd_kernel<T, N, LAYER>), grid, block, 0, st, (const T*)dy, (const T*)x, (const T*)w, \
                       mean, rstd, (T*)dx, dwp, dbp, rows, H)
    if (nv <= 1) SA_NB(1);
    else if (nv <= 2) SA_NB(2);
    else if (nv <= 4) SA_NB(4);
    else if (nv <= 8) SA_NB(8);
    else if (nv <= 16) SA_NB(16);
    else SA_NB(32);
#undef SA_NB
    hipLaunchKernelGGL((colsum_kernel<T>), dim3(cdiv(H, 64)), dim3(256), 0, st, dwp, (T*)dw, nwaves, H);
    if (LAYER) hipLaunchKernelGGL((colsum_kernel<T>), dim3(cdiv(H, 64)), dim3(256), 0, st, dbp, (T*)db, nwaves, H);
}

namespace sa_launch {
void norm_fwd(int dtype, bool layer, const void* x, const void* w, const void* b, void* y, float* mean, float* rstd,
              int64_t rows, int H, float eps, hipStream_t st) {
    if (dtype == DT_BF16) layer ? fwd_dispatch<u16, true>(x, w, b, y, mean, rstd, rows, H, eps, st)
                                : fwd_dispatch<u16, false>(x, w, b, y, mean, rstd, rows, H, eps, st);
    else if (dtype == DT_F16) layer ? fwd_dispatch<f16, true>(x, w, b, y, mean, rstd, rows, H, eps, st)
                                    : fwd_dispatch<f16, false>(x, w, b, y, mean, rstd, rows, H, eps, st);
    else layer ? fwd_dispatch<float, true>(x, w, b, y, mean, rstd, rows, H, eps, st)
               : fwd_dispatch<float, false>(x, w, b, y, mean, rstd, rows, H, eps, st);
}
int norm_bwd_waves(int64_t rows) {
    int64_t w = rows < 1024 ? rows : 1024;
    return (int)((w + 3) / 4 * 4);
}
void norm_bwd(int dtype, bool layer, const void* dy, const void* x, const void* w, const float* mean,
              const float* rstd, void* dx, void* dw, void* db, float* part, int64_t rows, int H, hipStream_t st) {
    const int nw = norm_bwd_waves(rows);
    if (dtype == DT_BF16) layer ? bwd_dispatch<u16, true>(dy, x, w, mean, rstd, dx, dw, db, part, rows, H, nw, st)
                                : bwd_dispatch<u16, false>(dy, x, w, mean, rstd, dx, dw, db, part, rows, H, nw, st);
    else if (dtype == DT_F16) layer ? bwd_dispatch<f16, true>(dy, x, w, mean, rstd, dx, dw, db, part, rows, H, nw, st)
                                    : bwd_dispatch<f16, false>(dy, x, w, mean, rstd, dx, dw, db, part, rows, H, nw, st);
    else layer ? bwd_dispatch<float, true>(dy, x, w, mean, rstd, dx, dw, db, part, rows, H, nw, st)
               : bwd_dispatch<float, false>(dy, x, w, mean, rstd, dx, dw, db, part, rows, H, nw, st);
}
}  // namespace sa_launch
