// Forward / input-gradient GEMM of a linear layer on gfx950:  C[M, N] = A[M, K] B[N, K]^T, both operands
// k-contiguous (A: activations or the output gradient, B: the weight [out, in] for the forward, its cached transpose
// W^T for the input gradient), bf16 in, fp32 accumulate, with fused epilogues:
//   EPI_STORE       C = acc
//   EPI_SWIGLU      the fused gate/up projection of a SwiGLU MLP: B = [W_gate; W_up] ([2F, K]); each 256-column tile
//                   covers 128 features (gate and up rows interleaved in 16-row blocks as they are staged), so every
//                   lane holds gate and up of the same (token, feature): z = [g | u] (the backward's input, optional)
//                   and h = silu(g) * u are written directly (no separate SwiGLU pass over z)
//   EPI_SWIGLU_BWD  the input gradient of the MLP's down projection, dh = dY W_down, consumed in registers: reads
//                   g, u from z and writes dz = [dh u silu'(g) | dh silu(g)] (dh never goes to memory)
// Numerics: every epilogue rounds the GEMM result to bf16 first and then applies exactly the arithmetic of the
// stand-alone SwiGLU kernels (swiglu_rope.hip), so the fused and unfused paths agree.
//
// Structure (persistent: one workgroup per CU walks its 256x256 tiles; 4 waves = one per SIMD, each 128x128 of
// 16x16x32 MFMAs in AGPRs):
//  * 64-deep k-stages in five 32-KiB LDS images of [256 rows][64 k] bf16: A in two, B in three (see below);
//  * LDS-DMA pieces (buffer_load ... lds) of 8 rows x 128 B: every lane group of 8 reads ONE full 128-B line
//    (the previous 16-rows x 64-B pieces read half lines: twice the cache-line requests per byte);
//  * image swizzle: 16-B chunk c of row r at c ^ ((r >> 1) & 7) -- every ds_read_b128 lane group of a fragment
//    read hits 16 distinct 16-B bank slots (conflict-free), and the DMA source is permuted to match;
//  * per stage t: sub-step 0 multiplies k 0-31 (registers F0) while reading k 32-63 (F1) and issuing stage t+2's B
//    pieces; wait for own reads and stage t+1, ONE barrier; sub-step 1 multiplies F1 while reading F0 of stage t+1
//    and issuing stage t+2's A pieces.  One barrier per 128 MFMAs, 8 DMA pieces per sub-step (a schedule with two
//    stage buffers had to issue all 16 in one sub-step: 1.25-1.30 PF against 1.37-1.46 for this one,
//    profiles/gemm_nt_split5_ab_r4.log).
//  * grid: XCD-aware bijective remap, then 4-row groups of tiles (the 32 tiles resident on one XCD share A/B panels
//    in its L2);
//  * the k-stage pipeline runs on across a workgroup's tiles: a tile's last two stages stage the next tile's first
//    two, so neither the pipeline fill nor the epilogue's stores leave the MFMAs idle between tiles.
// Reference op: F.linear at src/scaling/core/nn/linear/column_parallel_linear.py:151 / row_parallel_linear.py:158,
// SwiGLU at src/scaling/core/nn/mlp.py:157-161.
#include "common.h"
#include "flash_attn.h"
#include "launch.h"

using namespace sa;

namespace sa_gemm_nt {

using fa::bf16x8;
using fa::lds_void;

constexpr int kImg = 256 * 64 * 2;  // one operand's stage image [256][64] bf16
constexpr int kLds = 5 * kImg;      // A[0..1] + B[0..2]: all 160 KiB of LDS

__device__ __forceinline__ void mfma(f32x4& c, const bf16x8& a, const bf16x8& b) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void hard_barrier() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ float silu_f(float a) { return a / (1.f + __expf(-a)); }

template <int EPI>
__global__ __launch_bounds__(256, 1) void gemm_nt_kernel(const u16* __restrict__ A, int lda, uint32_t a_bytes,
                                                         const u16* __restrict__ B, int ldb, uint32_t b_bytes, int M,
                                                         int N, int K, NtEpi ep) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int tm = M / 256, tn = N / 256, ntiles = tm * tn;
    const int T = K / 64;
    // persistent: workgroup b takes virtual blocks b, b + G, ... (G = gridDim.x, a multiple of 8, so all on b's XCD);
    // a virtual block maps to its tile as a one-tile-per-workgroup grid would: XCD-aware bijective remap, then groups
    // of GM M-tiles sweeping N together (4 beat 8 / 16: profiles/gemm_nt_group_ab_r4.log)
    constexpr int GM = 4;
    auto tile_of = [&](int vb, int& tm0, int& tnt) {
        const int v = xcd_remap(vb, ntiles);
        const int group = GM * tn;
        const int first_m = (v / group) * GM;
        const int gm = min(tm - first_m, GM);
        const int within = v % group;
        tm0 = (first_m + within % gm) * 256;
        tnt = within / gm;
    };
    int tile = blockIdx.x, m0, nt;
    tile_of(tile, m0, nt);

    // ---- LDS-DMA: wave w stages pieces P = w + 4i (image rows 8P .. 8P+7) of each operand; lane -> (row lane >> 3,
    // 16-B slot lane & 7), source chunk = slot ^ f(row), f = (row >> 1) & 7 = 4 (P & 1) + (lane >> 4) (piece-invariant)
    const int prow = lane >> 3;
    const int pch = (lane & 7) ^ ((((wave & 1) << 2) | (lane >> 4)) & 7);
    const int va = (prow * lda + 8 * pch) * 2;
    const int vb = (prow * ldb + 8 * pch) * 2;
    auto a_base = [&](int tm0) { return __builtin_amdgcn_readfirstlane((tm0 + 8 * wave) * lda * 2); };
    auto b_base = [&](int tnt) {
        // SWIGLU: image rows 16 jb .. +15: jb even = gate rows, jb odd = up rows of features f0 + 16 (jb >> 1) ..;
        // piece P = w + 4i has jb = P >> 1: gate/up by (w >> 1) & 1, feature block i, half (w & 1)
        const int brow0 =
            EPI == EPI_SWIGLU ? ((wave >> 1) & 1) * ep.F + tnt * 128 + (wave & 1) * 8 : tnt * 256 + 8 * wave;
        return __builtin_amdgcn_readfirstlane(brow0 * ldb * 2);
    };
    int abase = a_base(m0), bbase = b_base(nt);
    const int astep = __builtin_amdgcn_readfirstlane(32 * lda * 2);
    const int bstep = __builtin_amdgcn_readfirstlane((EPI == EPI_SWIGLU ? 16 : 32) * ldb * 2);
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    const i32x4 rsa = {(int)__builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uint64_t>(A)),
                       (int)(__builtin_amdgcn_readfirstlane((uint32_t)(reinterpret_cast<uint64_t>(A) >> 32)) & 0xffff),
                       (int)__builtin_amdgcn_readfirstlane(a_bytes), fa::kBufFlags};
    const i32x4 rsb = {(int)__builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uint64_t>(B)),
                       (int)(__builtin_amdgcn_readfirstlane((uint32_t)(reinterpret_cast<uint64_t>(B) >> 32)) & 0xffff),
                       (int)__builtin_amdgcn_readfirstlane(b_bytes), fa::kBufFlags};
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>((lds_void*)smem));
    // piece I of operand A / B (ISB) of k-stage KU of the tile whose operand base is BASE, into the image at LBASE.
    // Inline asm so the waitcnt pass does not drain the pipeline in front of every ds_read (it cannot tell which LDS
    // bytes a compiler-visible LDS-DMA writes); m0 is written in the statement that reads it.
#define NT_PIECE_AT(ISB, I, LBASE, KU, BASE)                                                                      \
    {                                                                                                             \
        const uint32_t l_ = (LBASE) + (wave + 4 * (I)) * 1024;                                                    \
        if (ISB)                                                                                                  \
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(l_),     \
                         "v"(vb), "s"(rsb), "s"((BASE) + (I) * bstep + (KU) * 128)                                 \
                         : "m0");                                                                                 \
        else                                                                                                      \
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(l_),     \
                         "v"(va), "s"(rsa), "s"((BASE) + (I) * astep + (KU) * 128)                                 \
                         : "m0");                                                                                 \
    }
    // in the loop: the piece together with the MFMA before it, in one statement -- the MFMA is the wait state between
    // the M0 write and the LDS-DMA instead of an s_nop issue slot (+1.6-3 %, profiles/gemm_nt_mfma_piece_ab_r4.log).
    // ZC "%0" accumulates, "0" starts the accumulator (first k-slice of a tile)
#define NT_MFMA_PIECE_AT(C_, A_, B_, ISB, I, LBASE, KU, BASE, ZC)                                                   \
    {                                                                                                             \
        const uint32_t l_ = (LBASE) + (wave + 4 * (I)) * 1024;                                                    \
        if (ISB)                                                                                                  \
            asm volatile("s_mov_b32 m0, %3\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, " ZC "\n\t"                  \
                         "buffer_load_dwordx4 %4, %5, %6 offen lds"                                               \
                         : "+a"(C_) : "v"(A_), "v"(B_), "s"(l_), "v"(vb), "s"(rsb),                               \
                           "s"((BASE) + (I) * bstep + (KU) * 128) : "m0");                                         \
        else                                                                                                      \
            asm volatile("s_mov_b32 m0, %3\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, " ZC "\n\t"                  \
                         "buffer_load_dwordx4 %4, %5, %6 offen lds"                                               \
                         : "+a"(C_) : "v"(A_), "v"(B_), "s"(l_), "v"(va), "s"(rsa),                               \
                           "s"((BASE) + (I) * astep + (KU) * 128) : "m0");                                         \
    }

    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
    auto frag = [&](int off, int i) -> bf16x8 { return *reinterpret_cast<const bf16x8*>(smem + off + i * 2048); };
    const int fr = lane & 15, fg = lane >> 4, ff = fr >> 1;
    // lane l holds row 16i + (l & 15) of its wave's 128 rows, k chunk 4h + (l >> 4) of the stage; stored chunk
    // = c ^ f(r), f = ((l & 15) >> 1)
    const int lo0 = fr * 128 + 16 * (fg ^ ff), lo1 = fr * 128 + 16 * ((fg ^ ff) ^ 4);
    // ---- five 32-KiB images: A[0..1] at 0 / 32 KiB, B[0..2] at 64 / 96 / 128 KiB (all 160 KiB of LDS).  Stage s
    // lives in A[s % 2] and B[s % 3]; B's third buffer lets stage t+2's B image be staged during sub-step (t, 0)
    // (B[(t+2) % 3] was last read before barrier t-1) and its A image during (t, 1) (A[t % 2] was last read before
    // barrier t), so every sub-step carries 8 DMA pieces + 16 fragment reads beside its 64 MFMAs instead of one
    // sub-step carrying all 16 pieces.  End of (t, 0): own reads retired, vmcnt(8) (stage t+1 landed, the 8 B pieces
    // of stage t+2 just issued stay in flight), barrier t.  The B buffer roles rotate in registers (cur, next,
    // next-next), the A buffers by the 2-stage unroll.  Stages count on across the tiles of a workgroup: the last two
    // stages of a tile stage the next tile's first two (the pipeline never drains between tiles, and the epilogue's
    // stores overlap those loads); after the last tile they re-stage the tile's own first two (never read).
    int oa[2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        oa[s][0] = s * kImg + wm * 128 * 128 + lo0;
        oa[s][1] = s * kImg + wm * 128 * 128 + lo1;
        asm volatile("" : "+v"(oa[s][0]), "+v"(oa[s][1]));
    }
    int obc0 = 2 * kImg + wn * 128 * 128 + lo0, obc1 = obc0 - lo0 + lo1;
    int obn0 = obc0 + kImg, obn1 = obc1 + kImg;
    int obnn0 = obc0 + 2 * kImg, obnn1 = obc1 + 2 * kImg;
    uint32_t lbnn = lds0 + 4 * kImg;  // LDS byte address of B[(t+2) % 3]
    uint32_t lbc = lds0 + 2 * kImg;
    uint32_t lbn = lds0 + 3 * kImg;
#define NT5_ROTATE()                                                                                              \
    {                                                                                                             \
        const int t0_ = obc0, t1_ = obc1;                                                                         \
        obc0 = obn0; obc1 = obn1; obn0 = obnn0; obn1 = obnn1; obnn0 = t0_; obnn1 = t1_;                           \
        const uint32_t tl_ = lbc;                                                                                 \
        lbc = lbn; lbn = lbnn; lbnn = tl_;                                                                        \
        asm volatile("" : "+v"(obc0), "+v"(obc1), "+v"(obn0), "+v"(obn1), "+v"(obnn0), "+v"(obnn1));             \
    }
    // sub-step (t, 0), A buffer SA: MFMAs on F0, F1 read one fragment per 3 MFMAs over the first 48, the B pieces of
    // k-stage KU (= t + 2, or 0 / 1 of the next tile) from operand base BB one per 8 MFMAs; retire own reads + stage
    // t+1, barrier.  ZC "0": first k-slice of the tile (starts the accumulators)
#define NT5_SUB0(SA, KU, BB, ZC)                                                                                  \
    {                                                                                                             \
        _Pragma("unroll") for (int i = 0; i < 8; ++i) _Pragma("unroll") for (int j = 0; j < 8; ++j) {             \
            const int m_ = i * 8 + j;                                                                             \
            if ((m_ & 7) == 7)                                                                   \
                NT_MFMA_PIECE_AT(acc[i][j], fb0[j], fa0[i], true, m_ >> 3, lbnn, KU, BB, ZC)                      \
            else asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, " ZC : "+a"(acc[i][j]) : "v"(fb0[j]), "v"(fa0[i]));\
            if (m_ % 3 == 1 && m_ < 48) {                                                                         \
                const int f_ = m_ / 3;                                                                            \
                if (f_ < 8) fb1[f_] = frag(obc1, f_);                                                             \
                else fa1[f_ - 8] = frag(oa[SA][1], f_ - 8);                                                       \
            }                                                                                                     \
        }                                                                                                         \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                        \
        wait_vm<8>();                                                                                             \
        hard_barrier();                                                                                           \
    }
    // sub-step (t, 1): MFMAs on F1, F0 of stage t+1 read one per 3 MFMAs over the first 48, the A pieces of k-stage
    // KU from operand base AB into A[SA] one per 8 MFMAs (one per 4 over the first 32: 0-1.6 % slower,
    // profiles/gemm_nt_apiece_ab_r4.log)
#define NT5_SUB1(SA, KU, AB)                                                                                      \
    {                                                                                                             \
        _Pragma("unroll") for (int i = 0; i < 8; ++i) _Pragma("unroll") for (int j = 0; j < 8; ++j) {             \
            const int m_ = i * 8 + j;                                                                             \
            if ((m_ & 7) == 3)                                                                   \
                NT_MFMA_PIECE_AT(acc[i][j], fb1[j], fa1[i], false, m_ >> 3, lds0 + (SA) * kImg, KU, AB, "%0")     \
            else mfma(acc[i][j], fb1[j], fa1[i]);                                                                 \
            if (m_ % 3 == 1 && m_ < 48) {                                                                         \
                const int f_ = m_ / 3;                                                                            \
                if (f_ < 8) fb0[f_] = frag(obn0, f_);                                                             \
                else fa0[f_ - 8] = frag(oa[(SA) ^ 1][0], f_ - 8);                                                 \
            }                                                                                                     \
        }                                                                                                         \
        NT5_ROTATE()                                                                                              \
    }
    // prologue: stages 0 and 1 of the first tile in flight (A[0] B[0], A[1] B[1]), stage 0 landed, barrier, F0
    // the DMA descriptors / offsets may be fresh from v_readfirstlane (a VALU write of an SGPR that an inline-asm
    // buffer_load reads needs 5 wait states the compiler cannot see)
    asm volatile("s_nop 4" ::: "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        NT_PIECE_AT(false, i, lds0, 0, abase)
        NT_PIECE_AT(true, i, lds0 + 2 * kImg, 0, bbase)
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        NT_PIECE_AT(false, i, lds0 + kImg, 1, abase)
        NT_PIECE_AT(true, i, lds0 + 3 * kImg, 1, bbase)
    }
    wait_vm<16>();
    hard_barrier();
#pragma unroll
    for (int f = 0; f < 16; ++f) {
        if (f < 8) fb0[f] = frag(obc0, f);
        else fa0[f - 8] = frag(oa[0][0], f - 8);
    }
    for (;;) {
        const int next = tile + (int)gridDim.x;
        const bool more = next < ntiles;  // workgroup-uniform
        int nm0, nnt;
        tile_of(more ? next : tile, nm0, nnt);
        const int nab = a_base(nm0), nbb = b_base(nnt);
        asm volatile("s_nop 4" ::: "memory");
        NT5_SUB0(0, 2, bbase, "0")
        NT5_SUB1(0, 2, abase)
        NT5_SUB0(1, 3, bbase, "%0")
        NT5_SUB1(1, 3, abase)
        for (int u = 2; u < T - 2; u += 2) {  // T even and >= 4 (checked by the dispatcher)
            NT5_SUB0(0, u + 2, bbase, "%0")
            NT5_SUB1(0, u + 2, abase)
            NT5_SUB0(1, u + 3, bbase, "%0")
            NT5_SUB1(1, u + 3, abase)
        }
        NT5_SUB0(0, 0, nbb, "%0")
        NT5_SUB1(0, 0, nab)
        NT5_SUB0(1, 1, nbb, "%0")
        NT5_SUB1(1, 1, nab)
        // the MFMAs are inline asm, invisible to the hazard recognizer: cover the MFMA -> VALU read of the
        // accumulators, and pin every accumulator read behind that cover (an empty "+a" asm per accumulator: without
        // it hipcc hoists the first v_accvgpr_reads in among the last MFMAs, which then read stale AGPRs)
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));

        // ---- epilogue: acc[i][j][e] = C[m0 + 128 wm + 16 i + (lane & 15)][tile col 128 wn + 16 j + 4 (lane >> 4) + e]
        const int r = lane & 15, q4 = 4 * (lane >> 4);
        if constexpr (EPI == EPI_STORE) {
    #pragma unroll
            for (int i = 0; i < 8; ++i) {
                u16* cp = ep.C + (int64_t)(m0 + 128 * wm + 16 * i + r) * ep.ldc + nt * 256 + 128 * wn + q4;
    #pragma unroll
                for (int j = 0; j < 8; ++j) {
                    u16x4 o;
    #pragma unroll
                    for (int e = 0; e < 4; ++e) o[e] = f2bf(acc[i][j][e]);
                    *reinterpret_cast<u16x4*>(cp + 16 * j) = o;
                }
            }
        } else if constexpr (EPI == EPI_SWIGLU) {
            // j = 2 jj: gate, j = 2 jj + 1: up of features nt * 128 + 64 wn + 16 jj + q4 + e
    #pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int64_t row = m0 + 128 * wm + 16 * i + r;
                const int f = nt * 128 + 64 * wn + q4;
    #pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    u16x4 gz, uz, hz;
    #pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        gz[e] = f2bf(acc[i][2 * jj][e]);
                        uz[e] = f2bf(acc[i][2 * jj + 1][e]);
                        hz[e] = f2bf(round_bf(silu_f(bf2f(gz[e]))) * bf2f(uz[e]));
                    }
                    if (ep.C) {
                        *reinterpret_cast<u16x4*>(ep.C + row * ep.ldc + f + 16 * jj) = gz;
                        *reinterpret_cast<u16x4*>(ep.C + row * ep.ldc + ep.F + f + 16 * jj) = uz;
                    }
                    *reinterpret_cast<u16x4*>(ep.H + row * ep.ldh + f + 16 * jj) = hz;
                }
            }
        } else {  // EPI_SWIGLU_BWD: tile column = feature
            // z of row block i + 1 is loaded before row block i is computed and stored: every wait is for loads
            // issued one block earlier, not for a full memory round trip per block
            const u16* zrow = ep.Z + (int64_t)(m0 + 128 * wm + r) * ep.ldz + nt * 256 + 128 * wn + q4;
            u16x4 gz[2][8], uz[2][8];
            auto zload = [&](int bb, int i) {
                const u16* zp = zrow + (int64_t)(16 * i) * ep.ldz;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    gz[bb][j] = *reinterpret_cast<const u16x4*>(zp + 16 * j);
                    uz[bb][j] = *reinterpret_cast<const u16x4*>(zp + ep.F + 16 * j);
                }
            };
            zload(0, 0);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (i + 1 < 8) zload((i + 1) & 1, i + 1);
                const int64_t row = m0 + 128 * wm + 16 * i + r;
                u16* dp = ep.C + row * ep.ldc + nt * 256 + 128 * wn + q4;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    u16x4 da, db;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float g = round_bf(acc[i][j][e]);
                        const float av = bf2f(gz[i & 1][j][e]), bv = bf2f(uz[i & 1][j][e]);
                        const float sig = 1.f / (1.f + __expf(-av));
                        const float s = av * sig;
                        db[e] = f2bf(g * round_bf(s));
                        const float ds = g * bv;
                        da[e] = f2bf(ds * (sig * (1.f + av * (1.f - sig))));
                    }
                    *reinterpret_cast<u16x4*>(dp + 16 * j) = da;
                    *reinterpret_cast<u16x4*>(dp + ep.F + 16 * j) = db;
                }
            }
        }
        // the next tile's first MFMAs overwrite the accumulators the epilogue just read
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
        asm volatile("s_nop 4" ::: "memory");
        if (!more) break;
        tile = next;
        m0 = nm0;
        nt = nnt;
        abase = nab;
        bbase = nbb;
    }
    wait_vm<0>();  // the re-staged pieces of the last tile land before the workgroup's LDS is released
}
#define SA_NT_INST(E)                                                                                          \
    template __global__ void gemm_nt_kernel<E>(const u16* __restrict__, int, uint32_t, const u16* __restrict__, int, \
                                               uint32_t, int, int, int, NtEpi);
SA_NT_INST(EPI_STORE) SA_NT_INST(EPI_SWIGLU) SA_NT_INST(EPI_SWIGLU_BWD)
#undef SA_NT_INST

}  // namespace sa_gemm_nt

namespace sa_launch {
bool gemm_nt_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb) {
    return M % 256 == 0 && N % 256 == 0 && K % 128 == 0 && K >= 256 && M > 0 && N > 0 && lda % 8 == 0 &&
           ldb % 8 == 0 && lda >= K && ldb >= K && M * lda * 2 < (int64_t(1) << 31) &&
           N * ldb * 2 < (int64_t(1) << 31) && (M / 256) * (N / 256) < (int64_t(1) << 31);
}
void gemm_nt(int epi, const void* A, int64_t lda, const void* B, int64_t ldb, int64_t M, int64_t N, int64_t K,
               const NtEpi& ep, hipStream_t st) {
    using namespace sa_gemm_nt;
    static const int ncu = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 8)
            n = 256;
        return n - n % 8;
    }();
    const int ntiles = (int)((M / 256) * (N / 256));
    const int nwg = ntiles < ncu ? ntiles : ncu;  // persistent: one workgroup per CU (160 KiB of LDS each)
    const uint32_t ab = (uint32_t)(M * lda * 2), bb = (uint32_t)(N * ldb * 2);
#define SA_NT_LAUNCH(E)                                                                                         \
    hipLaunchKernelGGL((gemm_nt_kernel<E>), dim3(nwg), dim3(256), kLds, st, (const u16*)A, (int)lda, ab,         \
                       (const u16*)B, (int)ldb, bb, (int)M, (int)N, (int)K, ep)
    if (epi == EPI_SWIGLU) SA_NT_LAUNCH(EPI_SWIGLU);
    else if (epi == EPI_SWIGLU_BWD) SA_NT_LAUNCH(EPI_SWIGLU_BWD);
    else SA_NT_LAUNCH(EPI_STORE);
#undef SA_NT_LAUNCH
}
}  // namespace sa_launch
