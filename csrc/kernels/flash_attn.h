// Flash-attention building blocks for gfx950 (MFMA 32x32x16 bf16, wave64).
//
// Conventions (cdna_hip_programming.md §3, "An accumulator tile as the next MFMA's operand"):
//  * mfma_f32_32x32x16_bf16 operands: lane l (r = l&31, h = l>>5) holds A[r][8h+j], B[8h+j][r];
//    C/D: col = l&31, row = (reg&3) + 8*(reg>>2) + 4*h.
//  * "swapped" products keep the query (fwd, dQ) or the key (dK/dV) on the lane, so every softmax
//    row statistic is lane-local and an accumulator feeds the next MFMA as its B operand with no
//    lane movement (k order inside a step permuted: element j <-> row 16s + 8(j>>2) + 4h + (j&3)).
//  * The transposed operand of that next product is read with ds_read_b64_tr_b16.
//  * One LDS image per tile serves both row reads (ds_read_b128) and transposed reads: the
//    16-B chunk swizzle of §5.5 T10 "One image for row reads AND transposed reads" (b), extended
//    to 64/32-wide heads (see SWZ below) — conflict-free for both read kinds.
#pragma once
#include "common.h"

namespace sa {
namespace fa {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <int D>
__device__ __forceinline__ int swz(int r, int c) {
    if constexpr (D == 128) return c ^ (((r & 3) << 2) | ((r >> 2) & 3));
    else if constexpr (D == 64) return c ^ ((((r >> 1) & 1) << 2) | ((r >> 2) & 3));
    else return c ^ ((r >> 2) & 3);  // D == 32
}

// byte offset of element (r, d) in a [rows][D] bf16 LDS image
template <int D>
__device__ __forceinline__ int lds_off(int r, int d) {
    return r * D * 2 + 16 * swz<D>(r, d >> 3) + ((d & 7) << 1);
}

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// row read: 8 bf16 of row r starting at column d (d multiple of 8)
template <int D>
__device__ __forceinline__ bf16x8 ld_row(const char* lds, int r, int d) {
    return *reinterpret_cast<const bf16x8*>(lds + lds_off<D>(r, d));
}

// transposed A-operand fragment of X^T where X is a [rows][D] tile: lane receives
// X[kb + 4h + q][col] (q=0..3) and X[kb + 8 + 4h + q][col] for col = c0 + (l&31).
template <int D>
__device__ __forceinline__ bf16x8 ld_tr(const char* lds, int kb, int c0) {
    const int l = threadIdx.x & 63;
    const int h = l >> 5, g = (l >> 4) & 1, i = l & 15;
    const int row = kb + 4 * h + (i >> 2);
    const int col = c0 + 16 * g + 4 * (i & 3);
    s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + lds_off<D>(row, col)));
    s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + lds_off<D>(row + 8, col)));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

// pack accumulator registers 8s..8s+7 into a bf16 B-operand fragment
__device__ __forceinline__ bf16x8 pack_acc(const f32x16& acc, int s) {
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (__bf16)acc[8 * s + j];
    return r;
}

// global -> register staging of a [64][D] tile (rows beyond `valid` read as zero), 256 threads.
template <int D>
struct Stage {
    static constexpr int NPT = 64 * D / 8 / 256;
    u16x8 r[NPT];
    __device__ __forceinline__ void load(const u16* base, int64_t tok_stride, int valid) {
#pragma unroll
        for (int i = 0; i < NPT; ++i) {
            const int id = threadIdx.x + i * 256;
            const int row = id / (D / 8), c = id % (D / 8);
            if (row < valid) r[i] = *reinterpret_cast<const u16x8*>(base + (int64_t)row * tok_stride + c * 8);
            else r[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
    }
    __device__ __forceinline__ void store(char* lds) {
#pragma unroll
        for (int i = 0; i < NPT; ++i) {
            const int id = threadIdx.x + i * 256;
            const int row = id / (D / 8), c = id % (D / 8);
            *reinterpret_cast<u16x8*>(lds + row * D * 2 + 16 * swz<D>(row, c)) = r[i];
        }
    }
};

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
// Placed at the top of a rarely taken, wave-uniform block (boundary-tile mask, lazy rescale): an empty volatile asm
// cannot be speculated, so the optimiser keeps the block behind its scalar branch instead of if-converting it into
// per-element compares + selects that every tile would execute.
__device__ __forceinline__ void mask_fence() { asm volatile(""); }

// dword 3 of a raw buffer resource on gfx9/CDNA (32-bit data format, no swizzle); out-of-range
// loads return 0
constexpr int kBufFlags = 0x00020000;

// buffer resource from values the compiler cannot prove wave-uniform (they are): readfirstlane
// keeps the descriptor in SGPRs instead of a per-load waterfall loop
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, uint32_t nbytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const uint64_t u = ((uint64_t)hi << 32) | lo;
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(u), (short)0, __builtin_amdgcn_readfirstlane(nbytes),
                                             kBufFlags);
}

// LDS-DMA of a 64-row x D bf16 tile into its swizzled LDS image by the W waves of a workgroup:
// buffer_load_dwordx4 ... lds writes 64 lanes x 16 B = 1 KiB linearly at M0, so each lane reads the
// global chunk that belongs at its linear LDS position (source-permuted swizzle).  Rows past the
// resource range land as zeros.  No staging registers, no ds_write; completion is the vmcnt(0)
// the compiler places before the next __syncthreads().
typedef __attribute__((address_space(3))) void lds_void;
template <int D, int W, int ROWS = 64>
struct DmaTile {
    static constexpr int PIECES = ROWS * D * 2 / 1024;
    static constexpr int NPW = (PIECES + W - 1) / W;
    static_assert(PIECES >= 1, "empty tile");
    int voff[NPW];
    __device__ __forceinline__ void init(int wave, int lane, int64_t tok) {
#pragma unroll
        for (int i = 0; i < NPW; ++i) {
            const int p = (wave + W * i) * 1024 + lane * 16;
            const int row = p / (2 * D), slot = (p % (2 * D)) / 16;
            voff[i] = row * (int)tok * 2 + 16 * (slot ^ swz<D>(row, 0));
        }
    }
    __device__ __forceinline__ void load(const void* base, int64_t tok, int rows, char* tile, int wave_u) const {
        const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(base, (uint32_t)max(rows, 0) * (uint32_t)tok * 2u);
#pragma unroll
        for (int i = 0; i < NPW; ++i)
            if (PIECES % W == 0 || wave_u + W * i < PIECES)  // wave-uniform
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(tile + (wave_u + W * i) * 1024), 16, voff[i], 0, 0, 0);
    }
};

template <int D, int W, int R>
__device__ __forceinline__ void dma_load(const DmaTile<D, W, R>& t, const void* base, int64_t tok, int rows, char* tile,
                                         int wave_u) {
    t.load(base, tok, rows, tile, wave_u);
}

// Workgroup barrier after which every wave may read what ANY wave staged by LDS-DMA: each wave first waits for its own
// pieces (s_waitcnt vmcnt(0)), then the barrier.  A plain __syncthreads() is not enough inside a loop: hipcc emits only
// lgkmcnt(0) there and puts the vmcnt wait in front of the wave's next ds_read, which covers only its OWN pieces -- a
// wave could read a slower peer's piece of the next tile before it landed (the stale bytes of two tiles ago).  That
// happened rarely, under load (cdna_hip_programming.md §5 "Read a staged buffer one phase AFTER the wait that retires
// it"; found by the race check's gradient trace, tools/race_trace.py).
__device__ __forceinline__ void dma_barrier() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// 3-way max without the canonicalising v_max the compiler wraps around fmaxf
__device__ __forceinline__ float vmax3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// max of 16 floats as ONE statement of 8 dependent v_max3: hipcc pads every inline-asm boundary whose output the next
// VALU reads with an s_nop, so 16 single-instruction vmax3 statements cost 16 extra issue slots per row max
__device__ __forceinline__ float vmax16(const f32x16& x) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3\n\t"
        "v_max3_f32 %0, %0, %4, %5\n\t"
        "v_max3_f32 %0, %0, %6, %7\n\t"
        "v_max3_f32 %0, %0, %8, %9\n\t"
        "v_max3_f32 %0, %0, %10, %11\n\t"
        "v_max3_f32 %0, %0, %12, %13\n\t"
        "v_max3_f32 %0, %0, %14, %15\n\t"
        "v_max_f32 %0, %0, %16"
        : "=&v"(r)
        : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(x[7]), "v"(x[8]),
          "v"(x[9]), "v"(x[10]), "v"(x[11]), "v"(x[12]), "v"(x[13]), "v"(x[14]), "v"(x[15]));
    return r;
}
// lane l and lane l^32 combined with one v_permlane32_swap: returns {x_l, x_(l^32)} in some order
__device__ __forceinline__ void xchg32(float x, float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
__device__ __forceinline__ float max_xchg32(float x) {
    float a, b;
    xchg32(x, a, b);
    return vmax3(a, b, a);
}
__device__ __forceinline__ float sum_xchg32(float x) {
    float a, b;
    xchg32(x, a, b);
    return a + b;
}
// ---- element type: bf16 or fp16 operands (same 16-bit layouts; MFMA variant + conversions differ)
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
template <bool F16>
__device__ __forceinline__ f32x16 mma(bf16x8 a, bf16x8 b, f32x16 c) {
    if constexpr (F16)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
template <bool F16>
__device__ __forceinline__ bf16x8 pack_acc_t(const f32x16& acc, int s) {
    if constexpr (F16) {
        f16x8 r;
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = (_Float16)acc[8 * s + j];
        return __builtin_bit_cast(bf16x8, r);
    } else {
        return pack_acc(acc, s);
    }
}
template <bool F16>
__device__ __forceinline__ u16 f2t(float f) {
    if constexpr (F16) return __builtin_bit_cast(u16, (_Float16)f);
    else return f2bf(f);
}
template <bool F16>
__device__ __forceinline__ float t2f(u16 v) {
    if constexpr (F16) return (float)__builtin_bit_cast(_Float16, v);
    else return bf2f(v);
}

// ---- attention dropout: counter-based keep mask, a pure function of (seed, q head, query token, key
// token), so the forward and both backward kernels (different lane <-> element layouts) regenerate the
// identical mask without storing it.  mix32 is the "lowbias32" integer finaliser (bijective).
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ uint32_t drop_head(uint32_t seed, int head) { return mix32(seed ^ ((uint32_t)head * 0x9e3779b9u)); }
__device__ __forceinline__ uint32_t drop_row(uint32_t hs, int qtok) { return mix32(hs + (uint32_t)qtok); }
__device__ __forceinline__ bool drop_keep(uint32_t row, int ktok, uint32_t thr) {
    return mix32(row ^ ((uint32_t)ktok * 0x85ebca6bu)) >= thr;
}

// q head of grid column x (grid x = Hq, walked fastest, so x mod 8 is the workgroup's XCD: blockIdx round-robins
// over the 8 XCDs).  With SA_ATTN_XCD each XCD takes Hq/8 CONSECUTIVE q heads, i.e. whole GQA groups, so the K / V
// stream of a kv head is fetched into one XCD's L2 instead of Hq/Hkv of them (cdna_hip_programming.md T1).
#ifndef SA_ATTN_XCD
#define SA_ATTN_XCD 1
#endif
__device__ __forceinline__ int xcd_head(int x, int Hq) {
    if constexpr (SA_ATTN_XCD) {
        if ((Hq & 7) == 0) return (x & 7) * (Hq >> 3) + (x >> 3);
    }
    return x;
}

// Grid of the query-tiled kernels (forward, dQ): x = q head (xcd_head), and (SA_ATTN_SEGMAJOR, default) y = query
// tile, z = segment, so the workgroups resident on an XCD at once are mostly the q tiles of few segments: they stream
// the same K / V tiles in lockstep (one L2 fetch, many readers).  Otherwise y = segment, z = query tile (tile slowest).
// Causal work is issued heaviest tile first either way (within a segment for the segment-major order).
#ifndef SA_ATTN_SEGMAJOR
#define SA_ATTN_SEGMAJOR 1
#endif
__host__ __device__ inline dim3 attn_grid(int hq, int nseg, int qtiles) {
    return SA_ATTN_SEGMAJOR ? dim3(hq, qtiles, nseg) : dim3(hq, nseg, qtiles);
}
__device__ __forceinline__ int attn_seg() { return SA_ATTN_SEGMAJOR ? (int)blockIdx.z : (int)blockIdx.y; }
__device__ __forceinline__ int attn_qtile(bool causal) {
    const int n = SA_ATTN_SEGMAJOR ? (int)gridDim.y : (int)gridDim.z, i = SA_ATTN_SEGMAJOR ? (int)blockIdx.y : (int)blockIdx.z;
    return causal ? n - 1 - i : i;
}

// Shared by the attention kernels: per-lane LDS offsets of row fragments (row lk, cols 16ks + 8h) and of
// transposed fragments (rows 4h + i/4 (+8), cols 32t + 16g + 4(i&3)); tile bases and the 32/16-row
// block offsets are compile-time immediates (loops unrolled per buffer).
template <int D>
struct LdsOffsets {
    // swz(r, c) = c ^ F(r): a chunk index 2ks + h (row reads) or 4t + low (transposed reads) XOR F(r)
    // splits into a per-lane base plus (const ^ per-lane high bits), so 6 registers replace 16 offsets
    int row_base, row_hi;
    int tr_base[2], tr_hi[2];
    __device__ __forceinline__ void init(int lane) {
        const int h = lane >> 5, r = lane & 31, g = (lane >> 4) & 1, i = lane & 15;
        const int fr = swz<D>(r, 0);
        row_base = r * D * 2 + 16 * (h ^ (fr & 1));
        row_hi = 16 * (fr & ~1);
        const int low = 2 * g + ((i & 3) >> 1);
#pragma unroll
        for (int x = 0; x < 2; ++x) {
            const int tr_row = 4 * h + (i >> 2) + 8 * x;
            const int ft = swz<D>(tr_row, 0);
            tr_base[x] = tr_row * D * 2 + 16 * (low ^ (ft & 3)) + (((4 * (i & 3)) & 7) << 1);
            tr_hi[x] = 16 * (ft & ~3);
        }
    }
    __device__ __forceinline__ int row(int ks) const { return row_base + ((32 * ks) ^ row_hi); }
    __device__ __forceinline__ int tr(int t, int x) const { return tr_base[x] + ((64 * t) ^ tr_hi[x]); }
};
template <int D>
__device__ __forceinline__ bf16x8 rd_row(const char* tile, int imm, int off) {
    return *reinterpret_cast<const bf16x8*>(tile + imm + off);
}
template <int D>
__device__ __forceinline__ bf16x8 rd_tr(const char* tile, int imm, const LdsOffsets<D>& lo, int t) {
    const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + imm + lo.tr(t, 0)));
    const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + imm + lo.tr(t, 1)));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
}

// row offset (r) of accumulator register j in a 32x32 MFMA C tile, excluding the 4h lane term
__host__ __device__ constexpr int crow(int j) { return (j & 3) + 8 * (j >> 2); }

}  // namespace fa
}  // namespace sa
