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
// x, out: [T, nh, hd] with arbitrary token/head strides (elements, unit element stride); out may alias x
// (every work item reads its elements before writing the same elements), which the fused attention
// backward uses to rotate dq/dk in place inside the dQKV buffer.
// table: fp32 cos/sin [max_pos, rd/2] (NeoX: pair (i, i+rd/2); complex: pair (2i, 2i+1)).
// sign = +1 forward, -1 backward (rotation transpose). Dims >= rd are copied through.
struct RopeArgs {
    int64_t xt, xh, ot, oh;  // token / head strides of x and out
    const float* cosb;
    const float* sinb;
    const int64_t* pos;
    int T, nh, hd, rd, seq_len;
    float sign;
};

// Vector path: one work item = 8 pair slots of one (token, head) row — NeoX: elements p..p+7 and
// half+p..half+p+7 (two 16 B loads); complex: elements e..e+7 (four pairs, one 16 B load); the
// pass-through tail [rd, hd) moves in 8-element chunks.  Needs 16 B aligned rows (checked on host).
template <typename T, bool IL>
__global__ __launch_bounds__(256) void rope_v8_kernel(const T* __restrict__ x, T* __restrict__ out, RopeArgs a) {
    const int half = a.rd / 2;
    const int rc = IL ? a.rd / 8 : half / 8;  // rotating chunks per row
    const int CR = rc + (a.hd - a.rd) / 8;
    const int n = a.T * a.nh * CR;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int row = i / CR, c = i - row * CR;
        const int t = row / a.nh, h = row - t * a.nh;
        const T* xr = x + t * a.xt + h * a.xh;
        T* orow = out + t * a.ot + h * a.oh;
        if (c < rc) {
            const int64_t ps = a.pos ? a.pos[t] : (t % a.seq_len);
            const float* cb = a.cosb + ps * half;
            const float* sb = a.sinb + ps * half;
            if (!IL) {
                const int p = c * 8;
                float x0[8], x1[8], cs[8], sn[8], o0[8], o1[8];
                V8<T>::ld(xr + p, x0);
                V8<T>::ld(xr + half + p, x1);
                V8<float>::ld(cb + p, cs);
                V8<float>::ld(sb + p, sn);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float sj = sn[j] * a.sign;
                    rot_pair(x0[j], x1[j], cs[j], sj, o0[j], o1[j]);
                }
                V8<T>::st(orow + p, o0);
                V8<T>::st(orow + half + p, o1);
            } else {
                const int e = c * 8;
                float v[8], o[8];
                V8<T>::ld(xr + e, v);
                const f32x4 cs = *reinterpret_cast<const f32x4*>(cb + e / 2);
                const f32x4 sn = *reinterpret_cast<const f32x4*>(sb + e / 2);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float sj = sn[j] * a.sign;
                    rot_pair(v[2 * j], v[2 * j + 1], cs[j], sj, o[2 * j], o[2 * j + 1]);
                }
                V8<T>::st(orow + e, o);
            }
        } else {
            const int e = a.rd + (c - rc) * 8;
            float v[8];
            V8<T>::ld(xr + e, v);
            V8<T>::st(orow + e, v);
        }
    }
}

// Scalar fallback (odd rotary dims / unaligned views): one thread per (token, head, pair).
template <typename T, bool INTERLEAVED>
__global__ __launch_bounds__(256) void rope_kernel(const T* __restrict__ x, T* __restrict__ out, RopeArgs a) {
    const int half = a.rd / 2;
    const int pairs = half + (a.hd - a.rd + 1) / 2;  // rotated pairs + pass-through element pairs
    const int64_t n = (int64_t)a.T * a.nh * pairs;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int p = (int)(i % pairs);
        const int64_t th = i / pairs;
        const int h = (int)(th % a.nh);
        const int64_t t = th / a.nh;
        const T* xr = x + t * a.xt + (int64_t)h * a.xh;
        T* orow = out + t * a.ot + (int64_t)h * a.oh;
        if (p < half) {
            const int64_t ps = a.pos ? a.pos[t] : (t % a.seq_len);
            const float c = a.cosb[ps * half + p];
            const float s = a.sinb[ps * half + p] * a.sign;
            const int i0 = INTERLEAVED ? 2 * p : p;
            const int i1 = INTERLEAVED ? 2 * p + 1 : p + half;
            const float x0 = IO<T>::ld(xr, i0), x1 = IO<T>::ld(xr, i1);
            float r0, r1;
            rot_pair(x0, x1, c, s, r0, r1);
            IO<T>::st(orow, i0, r0);
            IO<T>::st(orow, i1, r1);
        } else {
            const int j = a.rd + 2 * (p - half);
            const T v0 = xr[j];
            const T v1 = j + 1 < a.hd ? xr[j + 1] : v0;
            orow[j] = v0;
            if (j + 1 < a.hd) orow[j + 1] = v1;
        }
    }
}

// Graph-decode step (one token): RoPE of the q and k heads and the K/V cache append in ONE launch.  x is the QKV
// projection row [nq + 2 nkv heads][hd] (contiguous); q heads are rotated into q_out [nq][hd]; k heads are rotated
// straight into row *pos of the K cache and v heads copied into row *pos of the V cache ([cap][nkv][hd] each) --
// replacing rope(q), rope(k) and two index_copy launches.  One work item = 8 pair slots (as rope_v8_kernel).
// lim = min(cache rows, rotary table rows): a position outside [0, lim) writes no cache row, zeros q and sets *err
// (the caller checks the word on the host; an out-of-range row index would otherwise write past the cache silently).
template <typename T, bool IL>
__global__ __launch_bounds__(256) void rope_kv_append_kernel(const T* __restrict__ x, T* __restrict__ q_out,
                                                             T* __restrict__ kc, T* __restrict__ vc,
                                                             const int64_t* __restrict__ pos, const float* cosb,
                                                             const float* sinb, int nq, int nkv, int hd, int rd,
                                                             int64_t lim, int* __restrict__ err) {
    const int half = rd / 2;
    const int rc = IL ? rd / 8 : half / 8;
    const int CR = rc + (hd - rd) / 8;
    const int nh = nq + 2 * nkv;
    const int64_t ps = pos[0];
    if (ps < 0 || ps >= lim) {
        if (blockIdx.x == 0 && threadIdx.x == 0) *err = 1;
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nq * hd / 8; i += gridDim.x * blockDim.x) {
            const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            V8<T>::st(q_out + 8 * i, z);
        }
        return;
    }
    const int n = nh * CR;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int h = i / CR, c = i - h * CR;
        const T* xr = x + (int64_t)h * hd;
        T* orow;
        if (h < nq) orow = q_out + (int64_t)h * hd;
        else if (h < nq + nkv) orow = kc + (ps * nkv + (h - nq)) * hd;
        else orow = vc + (ps * nkv + (h - nq - nkv)) * hd;
        if (h >= nq + nkv) {  // v: plain copy of the row's chunks
            for (int e = 8 * c; e < hd; e += 8 * CR) {
                float v[8];
                V8<T>::ld(xr + e, v);
                V8<T>::st(orow + e, v);
            }
            continue;
        }
        if (c < rc) {
            const float* cb = cosb + ps * half;
            const float* sb = sinb + ps * half;
            if (!IL) {
                const int p = c * 8;
                float x0[8], x1[8], cs[8], sn[8], o0[8], o1[8];
                V8<T>::ld(xr + p, x0);
                V8<T>::ld(xr + half + p, x1);
                V8<float>::ld(cb + p, cs);
                V8<float>::ld(sb + p, sn);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    rot_pair(x0[j], x1[j], cs[j], sn[j], o0[j], o1[j]);
                }
                V8<T>::st(orow + p, o0);
                V8<T>::st(orow + half + p, o1);
            } else {
                const int e = c * 8;
                float v[8], o[8];
                V8<T>::ld(xr + e, v);
                const f32x4 cs = *reinterpret_cast<const f32x4*>(cb + e / 2);
                const f32x4 sn = *reinterpret_cast<const f32x4*>(sb + e / 2);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    rot_pair(v[2 * j], v[2 * j + 1], cs[j], sn[j], o[2 * j], o[2 * j + 1]);
                }
                V8<T>::st(orow + e, o);
            }
        } else {
            const int e = rd + (c - rc) * 8;
            float v[8];
            V8<T>::ld(xr + e, v);
            V8<T>::st(orow + e, v);
        }
    }
}

static int grid_for(int64_t n) {
    int64_t g = (n + 255) / 256;
    return (int)(g < 8192 ? (g < 1 ? 1 : g) : 8192);
}

namespace sa_launch {
bool rope_kv_append(int dtype, bool interleaved, const void* x, void* q_out, void* kc, void* vc, const int64_t* pos,
                    const float* cosb, const float* sinb, int nq, int nkv, int hd, int rd, int64_t lim, int* err,
                    hipStream_t st) {
    if (dtype == DT_F32 || hd % 8 || (interleaved ? rd % 8 : rd % 16)) return false;
    const int CR = (interleaved ? rd / 8 : rd / 16) + (hd - rd) / 8;
    const int g = grid_for((int64_t)(nq + 2 * nkv) * CR);
#define SA_RKV(TT, IL)                                                                                            \
    hipLaunchKernelGGL((rope_kv_append_kernel<TT, IL>), g, 256, 0, st, (const TT*)x, (TT*)q_out, (TT*)kc, (TT*)vc, \
                       pos, cosb, sinb, nq, nkv, hd, rd, lim, err)
    if (dtype == DT_BF16) { if (interleaved) SA_RKV(u16, true); else SA_RKV(u16, false); }
    else { if (interleaved) SA_RKV(f16, true); else SA_RKV(f16, false); }
#undef SA_RKV
    return true;
}
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
void rope(int dtype, bool interleaved, const void* x, int64_t x_tok, int64_t x_head, void* out, int64_t o_tok,
          int64_t o_head, const float* cosb, const float* sinb, const int64_t* pos, int64_t T_, int nh, int hd, int rd,
          int seq_len, float sign, hipStream_t st) {
    const RopeArgs a{x_tok, x_head, o_tok, o_head, cosb, sinb, pos, (int)T_, nh, hd, rd, seq_len, sign};
    const int vec_elems = dtype == DT_F32 ? 4 : 8;  // 16 B
    const bool aligned = ((uintptr_t)x % 16 == 0) && ((uintptr_t)out % 16 == 0) && x_tok % vec_elems == 0 &&
                         x_head % vec_elems == 0 && o_tok % vec_elems == 0 && o_head % vec_elems == 0;
    const bool vec = aligned && hd % 8 == 0 && (interleaved ? rd % 8 == 0 : rd % 16 == 0) &&
                     T_ * nh * (hd / 8) < (int64_t)INT32_MAX;
    if (vec) {
        const int CR = (interleaved ? rd / 8 : rd / 16) + (hd - rd) / 8;
        const int g = grid_for(T_ * nh * CR);
#define SA_ROPE(TT, IL) hipLaunchKernelGGL((rope_v8_kernel<TT, IL>), g, 256, 0, st, (const TT*)x, (TT*)out, a)
        if (dtype == DT_BF16) { if (interleaved) SA_ROPE(u16, true); else SA_ROPE(u16, false); }
        else if (dtype == DT_F16) { if (interleaved) SA_ROPE(f16, true); else SA_ROPE(f16, false); }
        else { if (interleaved) SA_ROPE(float, true); else SA_ROPE(float, false); }
#undef SA_ROPE
        return;
    }
    const int pairs = rd / 2 + (hd - rd + 1) / 2;
    const int g = grid_for(T_ * nh * pairs);
#define SA_ROPE(TT, IL) hipLaunchKernelGGL((rope_kernel<TT, IL>), g, 256, 0, st, (const TT*)x, (TT*)out, a)
    if (dtype == DT_BF16) { if (interleaved) SA_ROPE(u16, true); else SA_ROPE(u16, false); }
    else if (dtype == DT_F16) { if (interleaved) SA_ROPE(f16, true); else SA_ROPE(f16, false); }
    else { if (interleaved) SA_ROPE(float, true); else SA_ROPE(float, false); }
#undef SA_ROPE
}
}  // namespace sa_launch
