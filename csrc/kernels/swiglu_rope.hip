// SwiGLU and rotary-embedding kernels (memory-bound; 16 B per lane per access).
#include "common.h"
#include "launch.h"

using namespace sa;

// ------------------------------------------------------------------ SwiGLU
// out[t, j] = rnd(silu(a[t, j])) * b[t, j]  (torch: silu(x) then * y, each rounded to the storage type)
template <typename T>
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const T* __restrict__ a, const T* __restrict__ b, int64_t lda,
                                                         T* __restrict__ out, int64_t rows, int F) {
    const int vpr = F / 8;
    const int64_t n = rows * vpr;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / vpr;
        const int c = (int)(i - r * vpr) * 8;
        float av[8], bv[8], o[8];
        V8<T>::ld(a + r * lda + c, av);
        V8<T>::ld(b + r * lda + c, bv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float s = av[j] / (1.f + __expf(-av[j]));
            o[j] = rnd<T>(s) * bv[j];
        }
        V8<T>::st(out + r * F + c, o);
    }
}

template <typename T>
__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ a,
                                                         const T* __restrict__ b, int64_t lda, T* __restrict__ da,
                                                         T* __restrict__ db, int64_t ldd, int64_t rows, int F) {
    const int vpr = F / 8;
    const int64_t n = rows * vpr;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / vpr;
        const int c = (int)(i - r * vpr) * 8;
        float g[8], av[8], bv[8], oa[8], ob[8];
        V8<T>::ld(dy + r * F + c, g);
        V8<T>::ld(a + r * lda + c, av);
        V8<T>::ld(b + r * lda + c, bv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float sig = 1.f / (1.f + __expf(-av[j]));
            const float s = av[j] * sig;
            ob[j] = g[j] * rnd<T>(s);
            const float ds = g[j] * bv[j];
            oa[j] = ds * (sig * (1.f + av[j] * (1.f - sig)));
        }
        V8<T>::st(da + r * ldd + c, oa);
        V8<T>::st(db + r * ldd + c, ob);
    }
}

// ------------------------------------------------------------------ RoPE
// x: [T, nh, hd] with arbitrary token/head strides (elements); out: contiguous [T, nh, hd].
// table: fp32 cos/sin [max_pos, rd/2] (NeoX: pair (i, i+rd/2); complex: pair (2i, 2i+1)).
// sign = +1 forward, -1 backward (rotation transpose). Dims >= rd are copied through.
template <typename T, bool INTERLEAVED>
__global__ __launch_bounds__(256) void rope_kernel(const T* __restrict__ x, int64_t tok_stride, int64_t head_stride,
                                                   T* __restrict__ out, const float* __restrict__ cosb,
                                                   const float* __restrict__ sinb, const int64_t* __restrict__ pos,
                                                   int64_t T_, int nh, int hd, int rd, int seq_len, float sign) {
    // one thread per (token, head, pair)
    const int half = rd / 2;
    const int pairs = half + (hd - rd + 1) / 2;  // rotated pairs + pass-through element pairs
    const int64_t n = T_ * nh * pairs;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int p = (int)(i % pairs);
        const int64_t th = i / pairs;
        const int h = (int)(th % nh);
        const int64_t t = th / nh;
        const T* xr = x + t * tok_stride + (int64_t)h * head_stride;
        T* orow = out + (t * nh + h) * hd;
        if (p < half) {
            const int64_t ps = pos ? pos[t] : (t % seq_len);
            const float c = cosb[ps * half + p];
            const float s = sinb[ps * half + p] * sign;
            const int i0 = INTERLEAVED ? 2 * p : p;
            const int i1 = INTERLEAVED ? 2 * p + 1 : p + half;
            const float x0 = IO<T>::ld(xr, i0), x1 = IO<T>::ld(xr, i1);
            IO<T>::st(orow, i0, x0 * c - x1 * s);
            IO<T>::st(orow, i1, x1 * c + x0 * s);
        } else {
            const int j = rd + 2 * (p - half);
            orow[j] = xr[j];
            if (j + 1 < hd) orow[j + 1] = xr[j + 1];
        }
    }
}

static int grid_for(int64_t n) {
    int64_t g = (n + 255) / 256;
    return (int)(g < 8192 ? (g < 1 ? 1 : g) : 8192);
}

namespace sa_launch {
void swiglu_fwd(int dtype, const void* a, const void* b, int64_t lda, void* out, int64_t rows, int F, hipStream_t st) {
    const int g = grid_for(rows * (F / 8));
    if (dtype == DT_BF16) hipLaunchKernelGGL(swiglu_fwd_kernel<u16>, g, 256, 0, st, (const u16*)a, (const u16*)b, lda, (u16*)out, rows, F);
    else if (dtype == DT_F16) hipLaunchKernelGGL(swiglu_fwd_kernel<f16>, g, 256, 0, st, (const f16*)a, (const f16*)b, lda, (f16*)out, rows, F);
    else hipLaunchKernelGGL(swiglu_fwd_kernel<float>, g, 256, 0, st, (const float*)a, (const float*)b, lda, (float*)out, rows, F);
}
void swiglu_bwd(int dtype, const void* dy, const void* a, const void* b, int64_t lda, void* da, void* db, int64_t ldd,
                int64_t rows, int F, hipStream_t st) {
    const int g = grid_for(rows * (F / 8));
    if (dtype == DT_BF16) hipLaunchKernelGGL(swiglu_bwd_kernel<u16>, g, 256, 0, st, (const u16*)dy, (const u16*)a, (const u16*)b, lda, (u16*)da, (u16*)db, ldd, rows, F);
    else if (dtype == DT_F16) hipLaunchKernelGGL(swiglu_bwd_kernel<f16>, g, 256, 0, st, (const f16*)dy, (const f16*)a, (const f16*)b, lda, (f16*)da, (f16*)db, ldd, rows, F);
    else hipLaunchKernelGGL(swiglu_bwd_kernel<float>, g, 256, 0, st, (const float*)dy, (const float*)a, (const float*)b, lda, (float*)da, (float*)db, ldd, rows, F);
}
void rope(int dtype, bool interleaved, const void* x, int64_t tok_stride, int64_t head_stride, void* out,
          const float* cosb, const float* sinb, const int64_t* pos, int64_t T_, int nh, int hd, int rd, int seq_len,
          float sign, hipStream_t st) {
    const int pairs = rd / 2 + (hd - rd + 1) / 2;
    const int g = grid_for(T_ * nh * pairs);
#define SA_ROPE(TT, IL) hipLaunchKernelGGL((rope_kernel<TT, IL>), g, 256, 0, st, (const TT*)x, tok_stride, head_stride, (TT*)out, cosb, sinb, pos, T_, nh, hd, rd, seq_len, sign)
    if (dtype == DT_BF16) { if (interleaved) SA_ROPE(u16, true); else SA_ROPE(u16, false); }
    else if (dtype == DT_F16) { if (interleaved) SA_ROPE(f16, true); else SA_ROPE(f16, false); }
    else { if (interleaved) SA_ROPE(float, true); else SA_ROPE(float, false); }
#undef SA_ROPE
}
}  // namespace sa_launch
