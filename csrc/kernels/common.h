// Shared device helpers for the scaling_amd CDNA4 (gfx950) kernels.
// Wave64 everywhere: reductions use 64-lane xor-shuffles; vector memory is 16 B/lane (8 x bf16).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sa {

constexpr int kWave = 64;

typedef __bf16 bf16;
typedef unsigned short u16;
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(u16 v) {
    return __uint_as_float(((uint32_t)v) << 16);
}
// round-to-nearest-even; NaN-preserving through the hardware cvt (plain cast to __bf16)
__device__ __forceinline__ u16 f2bf(float f) {
    bf16 h = (bf16)f;
    return __builtin_bit_cast(u16, h);
}
__device__ __forceinline__ float round_bf(float f) { return bf2f(f2bf(f)); }

template <typename T> struct IO;
template <> struct IO<float> {
    __device__ static __forceinline__ float ld(const float* p, int64_t i) { return p[i]; }
    __device__ static __forceinline__ void st(float* p, int64_t i, float v) { p[i] = v; }
};
template <> struct IO<u16> {
    __device__ static __forceinline__ float ld(const u16* p, int64_t i) { return bf2f(p[i]); }
    __device__ static __forceinline__ void st(u16* p, int64_t i, float v) { p[i] = f2bf(v); }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Block-wide sum of one float per thread; `scratch` needs blockDim/64 floats.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) scratch[wid] = v;
    __syncthreads();
    float r = 0.f;
    for (int i = 0; i < nw; ++i) r += scratch[i];
    return r;
}
__device__ __forceinline__ float block_max(float v, float* scratch) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    v = wave_max(v);
    __syncthreads();
    if (lane == 0) scratch[wid] = v;
    __syncthreads();
    float r = -INFINITY;
    for (int i = 0; i < nw; ++i) r = fmaxf(r, scratch[i]);
    return r;
}

inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective"): consecutive logical tiles land on the same XCD so they share its L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// Rotates the pair (x0, x1) by the angle with cosine c and sine s (RoPE).  ONE spelled-out contraction shared by every
// rotating kernel -- the training RoPE (forward and the transposed backward rotation), the graph-decode RoPE + K/V
// append step and the GEMV RoPE epilogue -- so all of them round identically whatever hipcc would contract.
__device__ __forceinline__ void rot_pair(float x0, float x1, float c, float s, float& o0, float& o1) {
    o0 = __builtin_fmaf(x0, c, -(x1 * s));
    o1 = __builtin_fmaf(x1, c, x0 * s);
}

}  // namespace sa

#define SA_CHECK_LAUNCH() (void)hipGetLastError()

namespace sa {
typedef _Float16 f16;
template <> struct IO<_Float16> {
    __device__ static __forceinline__ float ld(const _Float16* p, int64_t i) { return (float)p[i]; }
    __device__ static __forceinline__ void st(_Float16* p, int64_t i, float v) { p[i] = (_Float16)v; }
};

// 4-element vectors of a storage type and scalar conversions (bf16 as u16 bits, round to nearest even)
template <typename T> struct Vec4 { typedef T type __attribute__((ext_vector_type(4))); };
__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(u16 x) { return bf2f(x); }
__device__ __forceinline__ float to_f32(_Float16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ u16 from_f32<u16>(float x) { return f2bf(x); }
template <> __device__ __forceinline__ _Float16 from_f32<_Float16>(float x) { return (_Float16)x; }

// 8 contiguous elements <-> 8 floats, 16 B (bf16/f16) or 32 B (f32) per lane.
template <typename T> struct V8;
template <> struct V8<u16> {
    __device__ static __forceinline__ void ld(const u16* p, float (&v)[8]) {
        u16x8 r = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = bf2f(r[i]);
    }
    __device__ static __forceinline__ void st(u16* p, const float (&v)[8]) {
        u16x8 r;
#pragma unroll
        for (int i = 0; i < 8; ++i) r[i] = f2bf(v[i]);
        *reinterpret_cast<u16x8*>(p) = r;
    }
};
template <> struct V8<_Float16> {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    __device__ static __forceinline__ void ld(const _Float16* p, float (&v)[8]) {
        h8 r = *reinterpret_cast<const h8*>(p);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = (float)r[i];
    }
    __device__ static __forceinline__ void st(_Float16* p, const float (&v)[8]) {
        h8 r;
#pragma unroll
        for (int i = 0; i < 8; ++i) r[i] = (_Float16)v[i];
        *reinterpret_cast<h8*>(p) = r;
    }
};
template <> struct V8<float> {
    __device__ static __forceinline__ void ld(const float* p, float (&v)[8]) {
        f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) { v[i] = a[i]; v[i + 4] = b[i]; }
    }
    __device__ static __forceinline__ void st(float* p, const float (&v)[8]) {
        f32x4 a, b;
#pragma unroll
        for (int i = 0; i < 4; ++i) { a[i] = v[i]; b[i] = v[i + 4]; }
        *reinterpret_cast<f32x4*>(p) = a;
        *reinterpret_cast<f32x4*>(p + 4) = b;
    }
};
// round a float through the storage type (emulates torch's per-op rounding)
template <typename T> __device__ __forceinline__ float rnd(float v);
template <> __device__ __forceinline__ float rnd<float>(float v) { return v; }
template <> __device__ __forceinline__ float rnd<u16>(float v) { return round_bf(v); }
template <> __device__ __forceinline__ float rnd<_Float16>(float v) { return (float)(_Float16)v; }
}  // namespace sa
