// Row-softmax, activation and dropout kernels for gfx950 (wave64):
//   * masked softmax fwd/bwd — the reference's unfused "torch" attention kernel
//     (src/scaling/core/nn/masked_softmax/masked_softmax.py:14-30: x*scale, masked_fill(-10000),
//     softmax over the last dim; optional rounding of x*scale through the storage dtype when the
//     softmax is not forced to fp32).  One wave per row, online (max, sum) in one read pass, a second
//     pass writes the probabilities; 16-B vector accesses when the row length allows.
//   * GELU (erf / tanh) and SiLU fwd/bwd (reference nn/activation_function.py) — 8 elements per lane.
//   * dropout(+residual add) fwd/bwd with a counter-based keep mask (hash of seed and element index),
//     regenerated in the backward instead of stored (reference layer.py:211-233 dropout + residual).
#include "common.h"
#include "launch.h"

using namespace sa;

namespace {

__device__ __forceinline__ uint32_t hmix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// ------------------------------------------------------------------ masked softmax
struct MsmArgs {
    const void* x;
    const void* dy;
    const void* y;
    const uint8_t* mask;  // may be null
    void* out;
    int64_t rows, mb, mh, mq;  // mask strides of the [B, H, Sq, Sk] (possibly expanded) view
    int N, H, Sq;
    float scale, fill;
};

__device__ __forceinline__ const uint8_t* mask_row(const MsmArgs& a, int64_t row) {
    if (a.mask == nullptr) return nullptr;
    const int q = (int)(row % a.Sq);
    const int64_t bh = row / a.Sq;
    const int hh = (int)(bh % a.H);
    const int64_t bb = bh / a.H;
    return a.mask + bb * a.mb + hh * a.mh + (int64_t)q * a.mq;
}

template <typename T, bool ROUND>
__device__ __forceinline__ float msm_in(float v, float scale, bool masked, float fill) {
    float s = v * scale;
    if constexpr (ROUND) s = rnd<T>(s);
    return masked ? fill : s;
}

__device__ __forceinline__ void online(float& m, float& l, float v) {
    if (v > m) {
        l = l * __expf(m - v) + 1.f;
        m = v;
    } else {
        l += __expf(v - m);
    }
}

__device__ __forceinline__ void wave_merge(float& m, float& l) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float m2 = __shfl_xor(m, o, 64), l2 = __shfl_xor(l, o, 64);
        const float mn = fmaxf(m, m2);
        l = (m == -INFINITY ? 0.f : l * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : l2 * __expf(m2 - mn));
        m = mn;
    }
}

template <typename T, bool ROUND, bool VEC>
__global__ __launch_bounds__(256) void msm_fwd_kernel(MsmArgs a) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= a.rows) return;
    const int lane = threadIdx.x & 63;
    const T* xr = reinterpret_cast<const T*>(a.x) + row * a.N;
    T* yr = reinterpret_cast<T*>(a.out) + row * a.N;
    const uint8_t* mr = mask_row(a, row);
    float m = -INFINITY, l = 0.f;
    if constexpr (VEC) {
        for (int j = lane * 8; j < a.N; j += 512) {
            float v[8];
            V8<T>::ld(xr + j, v);
#pragma unroll
            for (int i = 0; i < 8; ++i) online(m, l, msm_in<T, ROUND>(v[i], a.scale, mr != nullptr && mr[j + i], a.fill));
        }
    } else {
        for (int j = lane; j < a.N; j += 64) online(m, l, msm_in<T, ROUND>(IO<T>::ld(xr, j), a.scale, mr != nullptr && mr[j], a.fill));
    }
    wave_merge(m, l);
    const float inv = 1.f / l;
    if constexpr (VEC) {
        for (int j = lane * 8; j < a.N; j += 512) {
            float v[8];
            V8<T>::ld(xr + j, v);
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = __expf(msm_in<T, ROUND>(v[i], a.scale, mr != nullptr && mr[j + i], a.fill) - m) * inv;
            V8<T>::st(yr + j, v);
        }
    } else {
        for (int j = lane; j < a.N; j += 64)
            IO<T>::st(yr, j, __expf(msm_in<T, ROUND>(IO<T>::ld(xr, j), a.scale, mr != nullptr && mr[j], a.fill) - m) * inv);
    }
}

// dx = masked ? 0 : scale * y * (dy - sum(dy * y))
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void msm_bwd_kernel(MsmArgs a) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= a.rows) return;
    const int lane = threadIdx.x & 63;
    const T* yr = reinterpret_cast<const T*>(a.y) + row * a.N;
    const T* gr = reinterpret_cast<const T*>(a.dy) + row * a.N;
    T* dr = reinterpret_cast<T*>(a.out) + row * a.N;
    const uint8_t* mr = mask_row(a, row);
    float dot = 0.f;
    if constexpr (VEC) {
        for (int j = lane * 8; j < a.N; j += 512) {
            float y[8], g[8];
            V8<T>::ld(yr + j, y);
            V8<T>::ld(gr + j, g);
#pragma unroll
            for (int i = 0; i < 8; ++i) dot += y[i] * g[i];
        }
    } else {
        for (int j = lane; j < a.N; j += 64) dot += IO<T>::ld(yr, j) * IO<T>::ld(gr, j);
    }
    dot = wave_sum(dot);
    if constexpr (VEC) {
        for (int j = lane * 8; j < a.N; j += 512) {
            float y[8], g[8];
            V8<T>::ld(yr + j, y);
            V8<T>::ld(gr + j, g);
#pragma unroll
            for (int i = 0; i < 8; ++i) y[i] = (mr != nullptr && mr[j + i]) ? 0.f : a.scale * y[i] * (g[i] - dot);
            V8<T>::st(dr + j, y);
        }
    } else {
        for (int j = lane; j < a.N; j += 64) {
            const float y = IO<T>::ld(yr, j), g = IO<T>::ld(gr, j);
            IO<T>::st(dr, j, (mr != nullptr && mr[j]) ? 0.f : a.scale * y * (g - dot));
        }
    }
}

// ------------------------------------------------------------------ activations
// kind: 0 = gelu (erf), 1 = silu, 2 = gelu (tanh approximation)
__device__ __forceinline__ float act_f(float x, int kind) {
    if (kind == 1) return x / (1.f + __expf(-x));
    if (kind == 2) {
        const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
        return 0.5f * x * (1.f + tanhf(u));
    }
    return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
}
__device__ __forceinline__ float act_df(float x, int kind) {
    if (kind == 1) {
        const float s = 1.f / (1.f + __expf(-x));
        return s * (1.f + x * (1.f - s));
    }
    if (kind == 2) {
        const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
        const float t = tanhf(u);
        return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * 0.7978845608028654f * (1.f + 3.f * 0.044715f * x * x);
    }
    return 0.5f * (1.f + erff(x * 0.7071067811865476f)) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
}

template <typename T>
__global__ __launch_bounds__(256) void act_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n, int kind) {
    const int64_t nv = n / 8;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
        float v[8];
        V8<T>::ld(x + 8 * i, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = act_f(v[j], kind);
        V8<T>::st(y + 8 * i, v);
    }
    if (blockIdx.x == 0)
        for (int64_t i = 8 * nv + threadIdx.x; i < n; i += blockDim.x) IO<T>::st(y, i, act_f(IO<T>::ld(x, i), kind));
}

template <typename T>
__global__ __launch_bounds__(256) void act_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x, T* __restrict__ dx,
                                                      int64_t n, int kind) {
    const int64_t nv = n / 8;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
        float v[8], g[8];
        V8<T>::ld(x + 8 * i, v);
        V8<T>::ld(dy + 8 * i, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = g[j] * act_df(v[j], kind);
        V8<T>::st(dx + 8 * i, v);
    }
    if (blockIdx.x == 0)
        for (int64_t i = 8 * nv + threadIdx.x; i < n; i += blockDim.x)
            IO<T>::st(dx, i, IO<T>::ld(dy, i) * act_df(IO<T>::ld(x, i), kind));
}

// ------------------------------------------------------------------ dropout (+ residual)
__device__ __forceinline__ bool keep_elem(uint32_t hs, int64_t i, uint32_t thr) {
    return hmix(hs ^ ((uint32_t)i * 0x9e3779b9u) ^ ((uint32_t)(i >> 32) * 0x85ebca6bu)) >= thr;
}

// out = res + x * keep / (1 - p)   (res may be null); backward: dx = g * keep / (1 - p)
template <typename T>
__global__ __launch_bounds__(256) void dropout_kernel(const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ out,
                                                      int64_t n, uint32_t seed, uint32_t thr, float rp) {
    const uint32_t hs = hmix(seed);
    const int64_t nv = n / 8;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
        float v[8], r[8];
        V8<T>::ld(x + 8 * i, v);
        if (res != nullptr) V8<T>::ld(res + 8 * i, r);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float d = keep_elem(hs, 8 * i + j, thr) ? v[j] * rp : 0.f;
            v[j] = res != nullptr ? r[j] + d : d;
        }
        V8<T>::st(out + 8 * i, v);
    }
    if (blockIdx.x == 0)
        for (int64_t i = 8 * nv + threadIdx.x; i < n; i += blockDim.x) {
            const float d = keep_elem(hs, i, thr) ? IO<T>::ld(x, i) * rp : 0.f;
            IO<T>::st(out, i, res != nullptr ? IO<T>::ld(res, i) + d : d);
        }
}

// debug: one wave that busy-waits `ticks` of the constant 100 MHz wall clock (s_memrealtime), so a stream carrying
// it runs ~late; used to delay the DP communication stream in race checks (SCALING_AMD_COMM_DELAY_US)
__global__ __launch_bounds__(64) void spin_kernel(uint64_t ticks) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(16);
}

// per-rank proxy with emulated communication (bench.py --shard-proxy ... --proxy-comm emulate): a collective's
// footprint on THIS GPU.  `nwg` workgroups (RCCL's channels hold as many CUs) stream its per-rank send volume from the
// collective's tensor (wrapping) into a scratch ring (local HBM read + write), then hold their CUs until the modelled
// xGMI time `ticks` (100 MHz wall clock) has passed since the kernel started.  Every loop is bounded by n16 / ticks.
__global__ __launch_bounds__(256) void xgmi_emu_kernel(const uint4* __restrict__ src, int64_t src16, uint4* __restrict__ dst,
                                                       int64_t dst16, int64_t n16, uint64_t ticks) {
    const uint64_t t0 = wall_clock64();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i % dst16] = src[i % src16];
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

int ew_grid(int64_t n) {
    const int64_t blocks = (n / 8 + 255) / 256;
    return (int)std::max<int64_t>(1, std::min<int64_t>(blocks, 256 * 16));
}

template <typename T>
void msm_fwd_t(const MsmArgs& a, bool round, hipStream_t st) {
    const int grid = (int)((a.rows + 3) / 4);
    const bool vec = a.N % 8 == 0;
    if (round) {
        if (vec) hipLaunchKernelGGL((msm_fwd_kernel<T, true, true>), grid, 256, 0, st, a);
        else hipLaunchKernelGGL((msm_fwd_kernel<T, true, false>), grid, 256, 0, st, a);
    } else {
        if (vec) hipLaunchKernelGGL((msm_fwd_kernel<T, false, true>), grid, 256, 0, st, a);
        else hipLaunchKernelGGL((msm_fwd_kernel<T, false, false>), grid, 256, 0, st, a);
    }
}

template <typename T>
void msm_bwd_t(const MsmArgs& a, hipStream_t st) {
    const int grid = (int)((a.rows + 3) / 4);
    if (a.N % 8 == 0) hipLaunchKernelGGL((msm_bwd_kernel<T, true>), grid, 256, 0, st, a);
    else hipLaunchKernelGGL((msm_bwd_kernel<T, false>), grid, 256, 0, st, a);
}

MsmArgs msm_args(const void* mask, int64_t rows, int N, int H, int Sq, int64_t mb, int64_t mh, int64_t mq, float scale,
                 float fill) {
    MsmArgs a{};
    a.mask = reinterpret_cast<const uint8_t*>(mask);
    a.rows = rows; a.N = N; a.H = H; a.Sq = Sq; a.mb = mb; a.mh = mh; a.mq = mq; a.scale = scale; a.fill = fill;
    return a;
}

}  // namespace

namespace sa_launch {
void masked_softmax_fwd(int dtype, const void* x, const void* mask, void* y, int64_t rows, int N, int H, int Sq, int64_t mb,
                        int64_t mh, int64_t mq, float scale, float fill, bool round, hipStream_t st) {
    MsmArgs a = msm_args(mask, rows, N, H, Sq, mb, mh, mq, scale, fill);
    a.x = x;
    a.out = y;
    if (dtype == DT_BF16) msm_fwd_t<u16>(a, round, st);
    else if (dtype == DT_F16) msm_fwd_t<_Float16>(a, round, st);
    else msm_fwd_t<float>(a, false, st);
}
void masked_softmax_bwd(int dtype, const void* dy, const void* y, const void* mask, void* dx, int64_t rows, int N, int H,
                        int Sq, int64_t mb, int64_t mh, int64_t mq, float scale, hipStream_t st) {
    MsmArgs a = msm_args(mask, rows, N, H, Sq, mb, mh, mq, scale, 0.f);
    a.dy = dy;
    a.y = y;
    a.out = dx;
    if (dtype == DT_BF16) msm_bwd_t<u16>(a, st);
    else if (dtype == DT_F16) msm_bwd_t<_Float16>(a, st);
    else msm_bwd_t<float>(a, st);
}
void act_fwd(int dtype, const void* x, void* y, int64_t n, int kind, hipStream_t st) {
    const int g = ew_grid(n);
    if (dtype == DT_BF16) hipLaunchKernelGGL(act_fwd_kernel<u16>, g, 256, 0, st, (const u16*)x, (u16*)y, n, kind);
    else if (dtype == DT_F16) hipLaunchKernelGGL(act_fwd_kernel<_Float16>, g, 256, 0, st, (const _Float16*)x, (_Float16*)y, n, kind);
    else hipLaunchKernelGGL(act_fwd_kernel<float>, g, 256, 0, st, (const float*)x, (float*)y, n, kind);
}
void act_bwd(int dtype, const void* dy, const void* x, void* dx, int64_t n, int kind, hipStream_t st) {
    const int g = ew_grid(n);
    if (dtype == DT_BF16)
        hipLaunchKernelGGL(act_bwd_kernel<u16>, g, 256, 0, st, (const u16*)dy, (const u16*)x, (u16*)dx, n, kind);
    else if (dtype == DT_F16)
        hipLaunchKernelGGL(act_bwd_kernel<_Float16>, g, 256, 0, st, (const _Float16*)dy, (const _Float16*)x, (_Float16*)dx, n, kind);
    else hipLaunchKernelGGL(act_bwd_kernel<float>, g, 256, 0, st, (const float*)dy, (const float*)x, (float*)dx, n, kind);
}
void spin(int64_t us, hipStream_t st) {
    if (us > 0) hipLaunchKernelGGL(spin_kernel, 1, 64, 0, st, (uint64_t)us * 100);
}
void xgmi_emulate(const void* src, int64_t src_bytes, void* scratch, int64_t scratch_bytes, int64_t bytes, double us,
                  int nwg, hipStream_t st) {
    const int64_t src16 = src_bytes / 16, dst16 = scratch_bytes / 16;
    const int64_t n16 = (src16 > 0 && dst16 > 0) ? bytes / 16 : 0;
    const uint64_t ticks = us > 0 ? (uint64_t)(us * 100.0) : 0;
    if (n16 == 0 && ticks == 0) return;
    hipLaunchKernelGGL(xgmi_emu_kernel, std::max(1, nwg), 256, 0, st, (const uint4*)src, std::max<int64_t>(src16, 1),
                       (uint4*)scratch, std::max<int64_t>(dst16, 1), n16, ticks);
}
void dropout(int dtype, const void* x, const void* res, void* out, int64_t n, uint32_t seed, uint32_t thr, float rp,
             hipStream_t st) {
    const int g = ew_grid(n);
    if (dtype == DT_BF16)
        hipLaunchKernelGGL(dropout_kernel<u16>, g, 256, 0, st, (const u16*)x, (const u16*)res, (u16*)out, n, seed, thr, rp);
    else if (dtype == DT_F16)
        hipLaunchKernelGGL(dropout_kernel<_Float16>, g, 256, 0, st, (const _Float16*)x, (const _Float16*)res, (_Float16*)out, n,
                           seed, thr, rp);
    else
        hipLaunchKernelGGL(dropout_kernel<float>, g, 256, 0, st, (const float*)x, (const float*)res, (float*)out, n, seed, thr, rp);
}
}  // namespace sa_launch
