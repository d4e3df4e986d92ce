// Fused cross-entropy, vocab-parallel embedding, fused AdamW and multi-tensor L2/inf reductions.
#include "common.h"
#include "launch.h"

using namespace sa;

// ------------------------------------------------------------------ cross entropy
// One 256-thread block per row. Online (max, sum-exp) in fp32 over 8-wide vector loads.
// Outputs per row: m (row max), s (sum exp(x - m)), tgt (target logit or 0 if target outside
// [v0, v0+V)), amax (argmax index, global vocab id). For tp=1 lse = m + log(s).
template <typename T>
__global__ __launch_bounds__(256) void xent_stats_kernel(const T* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                         int64_t rows, int V, int64_t v0, float* __restrict__ m_out,
                                                         float* __restrict__ s_out, float* __restrict__ t_out,
                                                         int64_t* __restrict__ amax_out, int vec) {
    __shared__ float sm[4], ss[4];
    __shared__ int si[4];
    const int64_t row = blockIdx.x;
    const T* x = logits + row * (int64_t)V;
    float m = -INFINITY, s = 0.f;
    int am = 0;
    const int nv = vec ? V / 8 : 0;  // 16-byte vector path only for aligned rows (V % 8 == 0, aligned base)
    for (int i = threadIdx.x; i < nv; i += 256) {
        float v[8];
        V8<T>::ld(x + i * 8, v);
        float lm = v[0];
        int li = 0;
#pragma unroll
        for (int j = 1; j < 8; ++j)
            if (v[j] > lm) { lm = v[j]; li = j; }
        if (lm > m) {
            s = s * __expf(m - lm);
            m = lm;
            am = i * 8 + li;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) s += __expf(v[j] - m);
    }
    for (int i = nv * 8 + threadIdx.x; i < V; i += 256) {  // tail
        const float v = IO<T>::ld(x, i);
        if (v > m) { s = s * __expf(m - v); m = v; am = i; }
        s += __expf(v - m);
    }
    // wave reduce (max, then rescaled sum); argmax ties -> lowest index
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
        const int oi = __shfl_xor(am, o, 64);
        const float nm = fmaxf(m, om);
        s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
        if (om > m || (om == m && oi < am)) am = oi;
        m = nm;
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) { sm[wid] = m; ss[wid] = s; si[wid] = am; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float M = sm[0], S = ss[0];
        int I = si[0];
        for (int w = 1; w < 4; ++w) {
            const float nm = fmaxf(M, sm[w]);
            S = S * __expf(M - nm) + ss[w] * __expf(sm[w] - nm);
            if (sm[w] > M || (sm[w] == M && si[w] < I)) I = si[w];
            M = nm;
        }
        m_out[row] = M;
        s_out[row] = S;
        const int64_t t = tgt[row] - v0;
        t_out[row] = (t >= 0 && t < V) ? IO<T>::ld(x, t) : 0.f;
        amax_out[row] = I + v0;
    }
}

// dlogits[r, j] = (exp(x - lse[r]) - [j == tgt]) * gscale[r]; may alias logits (in-place).
template <typename T>
__global__ __launch_bounds__(256) void xent_bwd_kernel(const T* logits, const int64_t* __restrict__ tgt,
                                                       const float* __restrict__ lse, const float* __restrict__ gscale,
                                                       T* dlogits, int64_t rows, int V, int64_t v0, int vec) {
    const int64_t row = blockIdx.x;
    const T* x = logits + row * (int64_t)V;
    T* d = dlogits + row * (int64_t)V;
    const float L = lse[row], g = gscale[row];
    const int64_t t = tgt[row] - v0;
    const int nv = vec ? V / 8 : 0;
    for (int i = threadIdx.x; i < nv; i += 256) {
        float v[8];
        V8<T>::ld(x + i * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (__expf(v[j] - L) - ((int64_t)(i * 8 + j) == t ? 1.f : 0.f)) * g;
        V8<T>::st(d + i * 8, v);
    }
    for (int i = nv * 8 + threadIdx.x; i < V; i += 256) {
        const float v = IO<T>::ld(x, i);
        IO<T>::st(d, i, (__expf(v - L) - ((int64_t)i == t ? 1.f : 0.f)) * g);
    }
}

// ------------------------------------------------------------------ embedding
// out[t] = W[id - v0] if v0 <= id < v0 + Vp else 0; one wave per token row, 16 B per lane.
template <typename T>
__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ ids, const T* __restrict__ W,
                                                        T* __restrict__ out, int64_t ntok, int H, int64_t v0, int64_t Vp) {
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= ntok) return;
    const int64_t id = ids[t] - v0;
    const bool ok = id >= 0 && id < Vp;
    for (int c = lane * 8; c < H; c += 512) {
        float v[8];
        if (ok) V8<T>::ld(W + id * H + c, v);
        else
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = 0.f;
        V8<T>::st(out + t * H + c, v);
    }
}

// dW[id] = sum of dy rows whose token is id, over the token positions sorted by id (stable, so the sum runs in token
// order and the result is deterministic): one wave per sorted position; the wave at the first position of each id's
// run adds the run's rows and writes the row.  Rows of ids outside this rank's shard are skipped; rows with no token
// keep the caller's zeros.  Run boundaries are found on the device, so the host never reads the number of distinct
// ids back (a device sync per backward in the unique / count formulation).
template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_kernel(const T* __restrict__ dy, const int64_t* __restrict__ order,
                                                        const int64_t* __restrict__ sid, int64_t ntok, T* __restrict__ dW,
                                                        int H, int64_t v0, int64_t Vp) {
    const int lane = threadIdx.x & 63;
    const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (k >= ntok) return;
    const int64_t s = sid[k];
    if (k > 0 && sid[k - 1] == s) return;  // not the first position of its run
    const int64_t id = s - v0;
    if (id < 0 || id >= Vp) return;
    int64_t e = k + 1;
    while (e < ntok && sid[e] == s) ++e;
    for (int c = lane * 8; c < H; c += 512) {
        float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int64_t r = k; r < e; ++r) {
            float v[8];
            V8<T>::ld(dy + order[r] * H + c, v);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] += v[j];
        }
        V8<T>::st(dW + id * H + c, acc);
    }
}

// ------------------------------------------------------------------ AdamW (flat fp32 master buffers)
// torch.optim.AdamW semantics: p *= 1 - lr*wd; m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
// p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps).  g = grad * gscale (loss-scale and clip folded in).
// Optionally writes the updated parameter in the model dtype (bf16/f16) in the same pass.
template <typename G, typename P>
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const G* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, P* __restrict__ pout,
                                                    int64_t n, float lr, float b1, float b2, float eps, float wd,
                                                    float bc1, float bc2_sqrt, float gscale, int vec) {
    const float step = lr / bc1;
    const float decay = 1.f - lr * wd;
    const int64_t n4 = vec ? n / 4 : 0;  // f32x4 path only when p/m/v are 16-byte aligned
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        f32x4 pv = reinterpret_cast<f32x4*>(p)[i];
        f32x4 mv = reinterpret_cast<f32x4*>(m)[i];
        f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
        const auto gv = reinterpret_cast<const typename Vec4<G>::type*>(g)[i];  // one 8-B (16-B for f32) load
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float gr = to_f32(gv[j]) * gscale;
            float pp = pv[j] * decay;
            const float mm = b1 * mv[j] + (1.f - b1) * gr;
            const float vvv = b2 * vv[j] + (1.f - b2) * gr * gr;
            pp -= step * mm / (sqrtf(vvv) / bc2_sqrt + eps);
            pv[j] = pp; mv[j] = mm; vv[j] = vvv; o[j] = pp;
        }
        reinterpret_cast<f32x4*>(p)[i] = pv;
        reinterpret_cast<f32x4*>(m)[i] = mv;
        reinterpret_cast<f32x4*>(v)[i] = vv;
        if (pout) {
            typename Vec4<P>::type ov;
#pragma unroll
            for (int j = 0; j < 4; ++j) ov[j] = from_f32<P>(o[j]);
            reinterpret_cast<typename Vec4<P>::type*>(pout)[i] = ov;
        }
    }
    // tail
    for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float gr = IO<G>::ld(g, i) * gscale;
        float pp = p[i] * decay;
        const float mm = b1 * m[i] + (1.f - b1) * gr;
        const float vvv = b2 * v[i] + (1.f - b2) * gr * gr;
        pp -= step * mm / (sqrtf(vvv) / bc2_sqrt + eps);
        p[i] = pp; m[i] = mm; v[i] = vvv;
        if (pout) IO<P>::st(pout, i, pp);
    }
}

// ------------------------------------------------------------------ L2 norm^2 + non-finite count
// Stage 1: per-block partial (sum of squares in fp32, per-thread then fixed-order block reduce).
template <typename G>
__global__ __launch_bounds__(256) void sumsq_kernel(const G* __restrict__ x, int64_t n, float scale,
                                                    float* __restrict__ part_sq, float* __restrict__ part_bad) {
    // x is 16-B aligned here (host peels the unaligned head): 8 elements per thread per trip
    __shared__ float scratch[4];
    float s = 0.f, bad = 0.f;
    const int64_t n8 = n / 8, stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
        float v[8];
        V8<G>::ld(x + 8 * i, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float t = v[j] * scale;
            const bool fin = isfinite(t);
            bad += fin ? 0.f : 1.f;
            s += fin ? t * t : 0.f;
        }
    }
    if (blockIdx.x == 0) {
        for (int64_t i = 8 * n8 + threadIdx.x; i < n; i += blockDim.x) {
            const float t = IO<G>::ld(x, i) * scale;
            if (!isfinite(t)) bad += 1.f;
            else s += t * t;
        }
    }
    s = block_sum(s, scratch);
    bad = block_sum(bad, scratch);
    if (threadIdx.x == 0) { part_sq[blockIdx.x] = s; part_bad[blockIdx.x] = bad; }
}

__global__ __launch_bounds__(256) void finalize_sum_kernel(const float* __restrict__ part, int n, float* __restrict__ out,
                                                           int accumulate) {
    __shared__ float scratch[4];
    float s = 0.f;
    for (int i = threadIdx.x; i < n; i += 256) s += part[i];
    s = block_sum(s, scratch);
    if (threadIdx.x == 0) out[0] = accumulate ? out[0] + s : s;
}

template <typename Src, typename Dst>
__global__ __launch_bounds__(256) void cast_scale_kernel(const Src* __restrict__ x, Dst* __restrict__ y, int64_t n, float scale) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        IO<Dst>::st(y, i, IO<Src>::ld(x, i) * scale);
}
// both pointers 16-B aligned: 8 elements per thread per trip, scalar tail
template <typename Src, typename Dst>
__global__ __launch_bounds__(256) void cast_scale_v8_kernel(const Src* __restrict__ x, Dst* __restrict__ y, int64_t n, float scale) {
    const int64_t n8 = n / 8;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
        float v[8];
        V8<Src>::ld(x + 8 * i, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= scale;
        V8<Dst>::st(y + 8 * i, v);
    }
    if (blockIdx.x == 0)
        for (int64_t i = 8 * n8 + threadIdx.x; i < n; i += blockDim.x) IO<Dst>::st(y, i, IO<Src>::ld(x, i) * scale);
}

static int gridn(int64_t n, int per = 256, int cap = 4096) {
    int64_t g = (n + per - 1) / per;
    return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

namespace sa_launch {
static inline int xent_vec_ok(const void* a, const void* b, int V) {
    return (V % 8 == 0) && ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) % 16 == 0);
}
void xent_stats(int dtype, const void* logits, const int64_t* tgt, int64_t rows, int V, int64_t v0, float* m, float* s,
                float* t, int64_t* amax, hipStream_t st) {
    if (rows == 0) return;
    const int vec = xent_vec_ok(logits, logits, V);
    if (dtype == DT_BF16) hipLaunchKernelGGL(xent_stats_kernel<u16>, dim3(rows), 256, 0, st, (const u16*)logits, tgt, rows, V, v0, m, s, t, amax, vec);
    else if (dtype == DT_F16) hipLaunchKernelGGL(xent_stats_kernel<f16>, dim3(rows), 256, 0, st, (const f16*)logits, tgt, rows, V, v0, m, s, t, amax, vec);
    else hipLaunchKernelGGL(xent_stats_kernel<float>, dim3(rows), 256, 0, st, (const float*)logits, tgt, rows, V, v0, m, s, t, amax, vec);
}
void xent_bwd(int dtype, const void* logits, const int64_t* tgt, const float* lse, const float* gscale, void* dlogits,
              int64_t rows, int V, int64_t v0, hipStream_t st) {
    if (rows == 0) return;
    const int vec = xent_vec_ok(logits, dlogits, V);
    if (dtype == DT_BF16) hipLaunchKernelGGL(xent_bwd_kernel<u16>, dim3(rows), 256, 0, st, (const u16*)logits, tgt, lse, gscale, (u16*)dlogits, rows, V, v0, vec);
    else if (dtype == DT_F16) hipLaunchKernelGGL(xent_bwd_kernel<f16>, dim3(rows), 256, 0, st, (const f16*)logits, tgt, lse, gscale, (f16*)dlogits, rows, V, v0, vec);
    else hipLaunchKernelGGL(xent_bwd_kernel<float>, dim3(rows), 256, 0, st, (const float*)logits, tgt, lse, gscale, (float*)dlogits, rows, V, v0, vec);
}
void embed_fwd(int dtype, const int64_t* ids, const void* W, void* out, int64_t ntok, int H, int64_t v0, int64_t Vp,
               hipStream_t st) {
    if (ntok == 0) return;
    const int g = (int)((ntok + 3) / 4);
    if (dtype == DT_BF16) hipLaunchKernelGGL(embed_fwd_kernel<u16>, g, 256, 0, st, ids, (const u16*)W, (u16*)out, ntok, H, v0, Vp);
    else if (dtype == DT_F16) hipLaunchKernelGGL(embed_fwd_kernel<f16>, g, 256, 0, st, ids, (const f16*)W, (f16*)out, ntok, H, v0, Vp);
    else hipLaunchKernelGGL(embed_fwd_kernel<float>, g, 256, 0, st, ids, (const float*)W, (float*)out, ntok, H, v0, Vp);
}
void embed_bwd(int dtype, const void* dy, const int64_t* order, const int64_t* sid, int64_t ntok, void* dW, int H,
               int64_t v0, int64_t Vp, hipStream_t st) {
    if (ntok == 0) return;
    const int g = (int)((ntok + 3) / 4);
    if (dtype == DT_BF16) hipLaunchKernelGGL(embed_bwd_kernel<u16>, g, 256, 0, st, (const u16*)dy, order, sid, ntok, (u16*)dW, H, v0, Vp);
    else if (dtype == DT_F16) hipLaunchKernelGGL(embed_bwd_kernel<f16>, g, 256, 0, st, (const f16*)dy, order, sid, ntok, (f16*)dW, H, v0, Vp);
    else hipLaunchKernelGGL(embed_bwd_kernel<float>, g, 256, 0, st, (const float*)dy, order, sid, ntok, (float*)dW, H, v0, Vp);
}
void adamw(int gdtype, int pdtype, float* p, const void* g, float* m, float* v, void* pout, int64_t n, float lr,
           float b1, float b2, float eps, float wd, float bc1, float bc2_sqrt, float gscale, hipStream_t st) {
    if (n == 0) return;
    // the vector path also loads 4 gradients / stores 4 parameters per access: g and pout 4-element aligned too
    const int gsz = gdtype == DT_F32 ? 4 : 2, psz = pdtype == DT_F32 ? 4 : 2;
    const int vec = ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v)) % 16) == 0 &&
                    reinterpret_cast<uintptr_t>(g) % (4 * gsz) == 0 && reinterpret_cast<uintptr_t>(pout) % (4 * psz) == 0;
    const int grid = gridn(vec ? n / 4 + 1 : n, 256, 8192);
#define SA_ADAM(GT, PT) hipLaunchKernelGGL((adamw_kernel<GT, PT>), grid, 256, 0, st, p, (const GT*)g, m, v, (PT*)pout, n, lr, b1, b2, eps, wd, bc1, bc2_sqrt, gscale, vec)
    if (gdtype == DT_F32) {
        if (pdtype == DT_BF16) SA_ADAM(float, u16); else if (pdtype == DT_F16) SA_ADAM(float, f16); else SA_ADAM(float, float);
    } else if (gdtype == DT_BF16) {
        if (pdtype == DT_BF16) SA_ADAM(u16, u16); else if (pdtype == DT_F16) SA_ADAM(u16, f16); else SA_ADAM(u16, float);
    } else {
        if (pdtype == DT_BF16) SA_ADAM(f16, u16); else if (pdtype == DT_F16) SA_ADAM(f16, f16); else SA_ADAM(f16, float);
    }
#undef SA_ADAM
}
int sumsq_blocks(int64_t n) { return gridn(n, 256 * 16, 2048) + 1; }
// bytes of x before its first 16-B boundary, in elements (the scalar head handled by the extra block)
static int64_t head_elems(const void* x, int esz, int64_t n) {
    const uintptr_t mis = reinterpret_cast<uintptr_t>(x) & 15;
    if (mis == 0) return 0;
    const int64_t h = (int64_t)((16 - mis) / esz);
    return h < n ? h : n;
}
void sumsq(int dtype, const void* x, int64_t n, float scale, float* part_sq, float* part_bad, float* out_sq,
           float* out_bad, int accumulate, hipStream_t st) {
    const int nb = sumsq_blocks(n);
    const int esz = dtype == DT_F32 ? 4 : 2;
    const int64_t h = head_elems(x, esz, n);
    // block nb-1 sums the unaligned head [0, h); blocks [0, nb-1) the aligned rest
    const char* xb = static_cast<const char*>(x);
#define SA_SQ(G)                                                                                                       \
    do {                                                                                                               \
        hipLaunchKernelGGL(sumsq_kernel<G>, nb - 1, 256, 0, st, (const G*)(xb + h * esz), n - h, scale, part_sq, part_bad); \
        hipLaunchKernelGGL(sumsq_kernel<G>, 1, 256, 0, st, (const G*)x, h, scale, part_sq + nb - 1, part_bad + nb - 1); \
    } while (0)
    if (dtype == DT_BF16) SA_SQ(u16);
    else if (dtype == DT_F16) SA_SQ(f16);
    else SA_SQ(float);
#undef SA_SQ
    hipLaunchKernelGGL(finalize_sum_kernel, 1, 256, 0, st, part_sq, nb, out_sq, accumulate);
    hipLaunchKernelGGL(finalize_sum_kernel, 1, 256, 0, st, part_bad, nb, out_bad, accumulate);
}
void cast_scale(int sdt, int ddt, const void* x, void* y, int64_t n, float scale, hipStream_t st) {
    if (n == 0) return;
    const bool vec = (reinterpret_cast<uintptr_t>(x) % 16) == 0 && (reinterpret_cast<uintptr_t>(y) % 16) == 0;
    const int g = vec ? gridn(n, 256 * 8, 8192) : gridn(n, 256, 8192);
#define SA_CS(S, D)                                                                                   \
    do {                                                                                              \
        if (vec) hipLaunchKernelGGL((cast_scale_v8_kernel<S, D>), g, 256, 0, st, (const S*)x, (D*)y, n, scale); \
        else hipLaunchKernelGGL((cast_scale_kernel<S, D>), g, 256, 0, st, (const S*)x, (D*)y, n, scale);        \
    } while (0)
    if (sdt == DT_BF16) { if (ddt == DT_F32) SA_CS(u16, float); else if (ddt == DT_BF16) SA_CS(u16, u16); else SA_CS(u16, f16); }
    else if (sdt == DT_F16) { if (ddt == DT_F32) SA_CS(f16, float); else if (ddt == DT_BF16) SA_CS(f16, u16); else SA_CS(f16, f16); }
    else { if (ddt == DT_F32) SA_CS(float, float); else if (ddt == DT_BF16) SA_CS(float, u16); else SA_CS(float, f16); }
#undef SA_CS
}
}  // namespace sa_launch
