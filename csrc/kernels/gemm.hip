// bf16 GEMM for the weight gradient of a linear layer on gfx950:  C[M, N] (+)= A^T B  with A: [K, M] and B: [K, N]
// both stored k-major (row = reduction index), i.e. dW = dY^T X over the token dimension.  Both operands are staged
// exactly as they lie in memory and the MFMA fragments come from the hardware transposing LDS read.
//
//  * 256x256 output tile per workgroup, 4 waves (one per SIMD) as 2 (M) x 2 (N), 128x128 per wave = 8x8 MFMA
//    16x16x32 tiles accumulated in place in AGPRs (inline-asm MFMAs);
//  * four-slot LDS ring of 32-deep k-steps: A and B images [32][256] bf16 (512-B rows) per slot, filled by LDS-DMA
//    (buffer_load ... lds, 16 B per lane, source-permuted so the lane-linear destination IS the swizzled image);
//  * during k-step t each wave multiplies F_t (in registers), reads F_{t+1} from slot (t+1)%4 (one fragment = two
//    transposing reads per 4 MFMAs) and stages k-step t+4 into slot t%4 (one 1-KiB piece per 8 MFMAs); one barrier
//    per k-step: every wave's reads of slot (t+1)%4 retired and k-step t+2 landed (16 pieces of k-steps t+3 / t+4
//    stay in flight), so each piece has 2-3 k-steps to land;
//  * image swizzle: 16-B slot ^ sw16(row) keeps every half-wave's 32 8-B transposing reads in 16 distinct 16-B bank
//    windows (conflict-free);
//  * grid: XCD-aware bijective remap, then 8-row groups of tiles so the 32 tiles resident on one XCD share A/B panels
//    in its L2; the ragged last round of tiles runs split over K (fp32 partials + a combine pass);
//  * epilogue: C = acc (+ C) with one bf16 rounding (beta = 1 accumulates into a main-grad buffer).
// Ragged M / N (multiples of 16, e.g. the tensor-parallel shards 5504 = 21.5 x 256, 2752, 16000): the edge tiles load
// past the last row / column like full ones -- those bytes are either another row of the same operand (only the
// output rows / columns past M / N see them) or past the buffer resource's byte range, which the LDS-DMA reads as
// zeros -- and the epilogue stores only the 16 x 16 accumulator blocks inside C (wave-uniform tests).  Shapes this kernel
// does not tile (M/N not multiples of 16, K not a multiple of 128) run on hipBLASLt (scaling_amd/ops/gemm.py).  The pipeline variants measured against this one (ping-pong 8-wave, 2-stage BK 64,
// interleaved, register-staged, other ring schedules) are in git history before commit "Delete losing GEMM variants"
// with their A/B logs in profiles/gemm_variants_*.log and profiles/gemm_ring_variants_r3*.log.
// Reference op: the weight gradient of F.linear at src/scaling/core/nn/linear/column_parallel_linear.py:151.
#include <algorithm>

#include "common.h"
#include "flash_attn.h"
#include "launch.h"

using namespace sa;

namespace sa_gemm {

using fa::bf16x8;
using fa::lds_s16x4;
using fa::lds_void;

// M-tiles per tile group (the 32 tiles resident on one XCD are group_m x 32/group_m, sharing A / B panels in its L2):
// 4 for tall outputs (tm >= 2 tn: gate/up 86 x 16 tiles +2.6 %, LM head 125 x 16 +1.6 %), 8 otherwise (down 16 x 43:
// 8 beats 4 by 1.2 %; 16 loses everywhere), profiles/wgrad_group_ab_r5.log.  SA_WGRAD_GROUPM pins it for an A/B.
__host__ __device__ __forceinline__ int group_m(int tm, int tn) {
#ifdef SA_WGRAD_GROUPM
    (void)tm;
    (void)tn;
    return SA_WGRAD_GROUPM;
#else
    return tm >= 2 * tn ? 4 : 8;
#endif
}
constexpr int BK = 32;                  // k rows per ring slot
constexpr int kImg = BK * 256 * 2;      // one operand image [32][256] bf16 = 16 KiB
constexpr int kSlot = 2 * kImg;         // A + B
constexpr int kSlots = 4;
constexpr int NW = 4;                   // waves
constexpr int NP = kImg / 1024 / NW;    // LDS-DMA pieces per wave per image (4)

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// workgroup barrier that neither the compiler's memory ordering nor its scheduler moves anything across
__device__ __forceinline__ void hard_barrier() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void mfma16_acc(f32x4& c, const bf16x8& a, const bf16x8& b) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
// image swizzle: the four 16-lane groups of a fragment read the SAME 16 columns at different k rows, so rows r and
// r+4 are separated too: 16-B slot ^ ((r&3)<<2 ^ ((r>>2)&1)<<1)
__device__ __forceinline__ int sw16(int r) { return ((r & 3) << 2) ^ (((r >> 2) & 1) << 1); }
__device__ __forceinline__ int koff16(int r, int c) { return r * 512 + 16 * ((c >> 3) ^ sw16(r)) + ((c & 7) << 1); }

// Workgroup -> virtual tile id (the tile order of group_m above).  SA_WGRAD_ROUND (default): round-major -- the 256
// workgroups resident at once (one per CU) take the contiguous range [256 r, 256 r + 256) of the tile order, a
// compact chip-wide block whose panels shared across XCDs are served by the MALL, and XCD c (workgroups b % 8 == c)
// its 32-tile sub-range, a compact block in that XCD's L2.  Otherwise the XCD-contiguous remap over the whole grid.
#ifndef SA_WGRAD_ROUND
#define SA_WGRAD_ROUND 1
#endif
__device__ __forceinline__ int round_remap(int b, int nwg) {
    if constexpr (SA_WGRAD_ROUND) {
        constexpr int R = 256;
        const int full = nwg / R * R;
        if (b >= full) return full + xcd_remap(b - full, nwg - full);
        return b / R * R + xcd_remap(b % R, R);
    }
    return xcd_remap(b, nwg);
}

template <bool BETA>
__global__ __launch_bounds__(256, 1) void gemm_tn_ring_kernel(const u16* __restrict__ A, int lda, uint32_t a_bytes,
                                                              const u16* __restrict__ B, int ldb, uint32_t b_bytes,
                                                              u16* __restrict__ C, int ldc, int M, int N, int K,
                                                              int full_blocks, int tail_split, float* __restrict__ ws) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 1, wn = wave & 1;

    // tile coordinates.  Blocks [0, full_blocks) own whole tiles (XCD remap over them); with a split tail the
    // remaining tiles run as tail_split K-slices each (one block per slice) writing fp32 partials that
    // gemm_tn_combine_kernel adds into C: the last round is full instead of ragged.
    const int tm = (M + 255) / 256, tn = (N + 255) / 256;
    int v, k_lo = 0, nk = K / 64, unit = -1;  // 64-deep tiles (the split plan's unit)
    if ((int)blockIdx.x < full_blocks) {
        v = round_remap(blockIdx.x, full_blocks);
    } else {
        unit = (int)blockIdx.x - full_blocks;
        v = full_blocks + unit / tail_split;
        nk /= tail_split;
        k_lo = (unit % tail_split) * nk;
    }
    const int ns = 2 * nk, s_lo = 2 * k_lo;  // 32-deep k-steps of this block
    const int gM = group_m(tm, tn);
    const int group = gM * tn;
    const int first_m = (v / group) * gM;
    const int gm = min(tm - first_m, gM);
    const int within = v % group;
    const int m0 = (first_m + within % gm) * 256, n0 = (within / gm) * 256;

    // LDS-DMA: piece i of this wave covers image rows 2 (wave + NW i) + {0, 1} (lane >> 5), 16-B slot (lane & 31);
    // the row advances by 2 NW (a multiple of 8), so the swizzle is piece-invariant: one VGPR offset per operand
    int voff_a, voff_b, step_a, step_b;
    {
        const int row = 2 * wave + (lane >> 5);
        const int slot = (lane & 31) ^ sw16(row);
        voff_a = (row * lda + slot * 8) * 2;
        voff_b = (row * ldb + slot * 8) * 2;
        step_a = __builtin_amdgcn_readfirstlane(4 * NW * lda);  // bytes: 2 NW rows of 2-B elements
        step_b = __builtin_amdgcn_readfirstlane(4 * NW * ldb);
    }
    auto soff_a = [&](int u) { return __builtin_amdgcn_readfirstlane(((s_lo + min(u, ns - 1)) * BK * lda + m0) * 2); };
    auto soff_b = [&](int u) { return __builtin_amdgcn_readfirstlane(((s_lo + min(u, ns - 1)) * BK * ldb + n0) * 2); };
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    const i32x4 rsa = {(int)__builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uint64_t>(A)),
                       (int)(__builtin_amdgcn_readfirstlane((uint32_t)(reinterpret_cast<uint64_t>(A) >> 32)) & 0xffff),
                       (int)__builtin_amdgcn_readfirstlane(a_bytes), fa::kBufFlags};
    const i32x4 rsb = {(int)__builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uint64_t>(B)),
                       (int)(__builtin_amdgcn_readfirstlane((uint32_t)(reinterpret_cast<uint64_t>(B) >> 32)) & 0xffff),
                       (int)__builtin_amdgcn_readfirstlane(b_bytes), fa::kBufFlags};
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>((lds_void*)smem));
    // piece P (0..7: even = A piece P/2, odd = B piece P/2) with scalar k-step offsets (SA, SB) into slot SLOT.
    // Inline asm on purpose: for a compiler-visible LDS-DMA the waitcnt pass cannot tell which LDS bytes are pending
    // and puts s_waitcnt vmcnt(0) in front of every later ds_read; the kernel counts these loads itself (wait_vm).
    // m0 is written in the statement that reads it (the compiler emits no other m0 use in this kernel).
#define SA_RING_PIECE(P, SLOT, SA, SB)                                                                           \
    {                                                                                                            \
        const int i_ = (P) >> 1;                                                                                 \
        const uint32_t l_ = lds0 + (SLOT) * kSlot + (((P) & 1) ? kImg : 0) + (wave + NW * i_) * 1024;            \
        if ((P) & 1)                                                                                             \
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(l_),    \
                         "v"(voff_b), "s"(rsb), "s"((SB) + i_ * step_b)                                       \
                         : "m0");                                                                                \
        else                                                                                                     \
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(l_),    \
                         "v"(voff_a), "s"(rsa), "s"((SA) + i_ * step_a)                                       \
                         : "m0");                                                                                \
    }
    // in the loop: the piece in one statement with the MFMA before it -- the MFMA is the wait state between the M0
    // write and the LDS-DMA, where an s_nop would take an issue slot (the same change gained 1.6-3 % on the NT kernel,
    // profiles/gemm_nt_mfma_piece_ab_r4.log)
#define SA_RING_MFMA_PIECE(C_, A_, B_, P, SLOT, SA, SB)                                                          \
    {                                                                                                            \
        const int i_ = (P) >> 1;                                                                                 \
        const uint32_t l_ = lds0 + (SLOT) * kSlot + (((P) & 1) ? kImg : 0) + (wave + NW * i_) * 1024;            \
        if ((P) & 1)                                                                                             \
            asm volatile("s_mov_b32 m0, %3\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\t"                     \
                         "buffer_load_dwordx4 %4, %5, %6 offen lds"                                              \
                         : "+a"(C_) : "v"(A_), "v"(B_), "s"(l_), "v"(voff_b), "s"(rsb), "s"((SB) + i_ * step_b)  \
                         : "m0");                                                                                \
        else                                                                                                     \
            asm volatile("s_mov_b32 m0, %3\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\t"                     \
                         "buffer_load_dwordx4 %4, %5, %6 offen lds"                                              \
                         : "+a"(C_) : "v"(A_), "v"(B_), "s"(l_), "v"(voff_a), "s"(rsa), "s"((SA) + i_ * step_a)  \
                         : "m0");                                                                                \
    }

    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // per-lane fragment offsets for slot pairs {0,1} and {2,3}; slot parity (32 KiB), B image (16 KiB) and the second
    // transposing read (+16 rows = 8 KiB) ride in the ds_read immediate (< 64 KiB)
    int oa[2][8], ob[2][8];
    {
        const int g = lane >> 4, i16 = lane & 15;
        const int row = 4 * g + (i16 >> 2), cl = 4 * (i16 & 3);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                oa[h][i] = h * 2 * kSlot + koff16(row, 128 * wm + 16 * i + cl);
                ob[h][i] = h * 2 * kSlot + kImg + koff16(row, 128 * wn + 16 * i + cl);
            }
    }
    auto frag = [&](int off, int slot) -> bf16x8 {
        const char* p = smem + off + (slot & 1) * kSlot;
        const s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
        const s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 16 * 512));
        return __builtin_bit_cast(bf16x8, __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
#define SA_RING_READ(SLOT, FA, FB, F)                                         \
    {                                                                         \
        if ((F) < 8) FB[(F)] = frag(ob[(SLOT) >> 1][(F)], (SLOT));            \
        else FA[(F) - 8] = frag(oa[(SLOT) >> 1][(F) - 8], (SLOT));            \
    }
    // k-step T in slot SLOT with fragments (FA, FB); next fragments into (NA, NB) one per 4 MFMAs, k-step T+4's
    // pieces into slot SLOT one per 8 MFMAs (every issue slot evenly loaded)
#define SA_RING_STEP(SLOT, T, FA, FB, NA, NB)                                                                   \
    {                                                                                                           \
        const int sa_ = soff_a((T) + 4), sb_ = soff_b((T) + 4);                                                 \
        _Pragma("unroll") for (int i = 0; i < 8; ++i)                                                           \
            _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                                     \
                const int m_ = i * 8 + j;                                                                       \
                if ((m_ & 7) == 3) SA_RING_MFMA_PIECE(acc[i][j], FB[j], FA[i], m_ >> 3, SLOT, sa_, sb_)         \
                else mfma16_acc(acc[i][j], FB[j], FA[i]);                                                       \
                if ((m_ & 3) == 1) SA_RING_READ(((SLOT) + 1) & 3, NA, NB, m_ >> 2)                              \
            }                                                                                                   \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                      \
        wait_vm<4 * NP>();                                                                                      \
        hard_barrier();                                                                                         \
    }

    // prologue: k-steps 0-3 in flight (clamped: a short block re-stages its last k-step), 0 and 1 landed, F_0 read,
    // then a barrier so slot 0 may be restaged during k-step 0
    // the DMA descriptors / offsets may be fresh from v_readfirstlane (a VALU write of an SGPR that an inline-asm
    // buffer_load reads needs 5 wait states the compiler cannot see)
    asm volatile("s_nop 4" ::: "memory");
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int sa_ = soff_a(u), sb_ = soff_b(u);
#pragma unroll
        for (int p = 0; p < 8; ++p) SA_RING_PIECE(p, u, sa_, sb_)
    }
    wait_vm<4 * NP>();
    hard_barrier();
#pragma unroll
    for (int f = 0; f < 16; ++f) SA_RING_READ(0, fa0, fb0, f)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    hard_barrier();
    for (int t = 0; t + 3 < ns; t += 4) {  // ns % 4 == 0: whole pairs of 64-deep tiles per block (dispatcher)
        SA_RING_STEP(0, t, fa0, fb0, fa1, fb1)
        SA_RING_STEP(1, t + 1, fa1, fb1, fa0, fb0)
        SA_RING_STEP(2, t + 2, fa0, fb0, fa1, fb1)
        SA_RING_STEP(3, t + 3, fa1, fb1, fa0, fb0)
    }
#undef SA_RING_STEP
#undef SA_RING_READ
#undef SA_RING_PIECE
#undef SA_RING_MFMA_PIECE
    wait_vm<0>();
    // the MFMAs are inline asm, invisible to the hazard recognizer: cover the MFMA -> VALU read of the accumulators,
    // and pin every accumulator read behind that cover (an empty "+a" asm per accumulator: without it hipcc hoists
    // the first v_accvgpr_reads in among the last MFMAs, which then read stale AGPRs)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));

    // epilogue: acc[i][j][e] = C[m0 + 128wm + 16i + (lane & 15)][n0 + 128wn + 16j + 4(lane >> 4) + e]
    const int r = lane & 15, q4 = 4 * (lane >> 4);
    if (unit >= 0) {  // K-slice of a tail tile: fp32 partial [256][256] at ws + unit * 65536
        float* wp = ws + (int64_t)unit * 65536;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float* rp = wp + (128 * wm + 16 * i + r) * 256 + 128 * wn + q4;
#pragma unroll
            for (int j = 0; j < 8; ++j) *reinterpret_cast<f32x4*>(rp + 16 * j) = acc[i][j];
        }
        return;
    }
    const bool edge = m0 + 256 > M || n0 + 256 > N;  // ragged last tile row / column: store the blocks inside C
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (edge && m0 + 128 * wm + 16 * i >= M) continue;  // wave-uniform (M % 16 == 0)
        u16* crow_p = C + (int64_t)(m0 + 128 * wm + 16 * i + r) * ldc + n0 + 128 * wn + q4;
        u16x4 old[8];
        if (BETA) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (!edge || n0 + 128 * wn + 16 * j < N) old[j] = *reinterpret_cast<const u16x4*>(crow_p + 16 * j);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (edge && n0 + 128 * wn + 16 * j >= N) continue;
            u16x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float x = acc[i][j][e];
                if (BETA) x += bf2f(old[j][e]);
                o[e] = f2bf(x);
            }
            *reinterpret_cast<u16x4*>(crow_p + 16 * j) = o;
        }
    }
}
template __global__ void gemm_tn_ring_kernel<true>(const u16* __restrict__, int, uint32_t, const u16* __restrict__, int,
                                                   uint32_t, u16* __restrict__, int, int, int, int, int, int,
                                                   float* __restrict__);
template __global__ void gemm_tn_ring_kernel<false>(const u16* __restrict__, int, uint32_t, const u16* __restrict__, int,
                                                    uint32_t, u16* __restrict__, int, int, int, int, int, int,
                                                    float* __restrict__);

// tail tile v (>= full_blocks): C[m0 + r][n0 + c] = (beta ? C : 0) + sum of its K-slice partials; block (tile, 4 rows)
__global__ __launch_bounds__(256) void gemm_tn_combine_kernel(const float* __restrict__ ws, u16* __restrict__ C, int ldc,
                                                              int M, int N, int full_blocks, int split, int beta) {
    const int tm = (M + 255) / 256, tn = (N + 255) / 256;
    const int v = full_blocks + (int)blockIdx.x;
    const int gM = group_m(tm, tn);
    const int group = gM * tn;
    const int first_m = (v / group) * gM;
    const int gm = min(tm - first_m, gM);
    const int within = v % group;
    const int m0 = (first_m + within % gm) * 256, n0 = (within / gm) * 256;
    const int row = 4 * (int)blockIdx.y + (threadIdx.x >> 6), col = (threadIdx.x & 63) * 4;
    if (m0 + row >= M || n0 + col >= N) return;  // ragged edge tile
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* wp = ws + (int64_t)blockIdx.x * split * 65536 + row * 256 + col;
    for (int p = 0; p < split; ++p) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(wp + (int64_t)p * 65536);
        acc += x;
    }
    u16* cp = C + (int64_t)(m0 + row) * ldc + n0 + col;
    u16x4 o;
    const u16x4 old = beta ? *reinterpret_cast<const u16x4*>(cp) : u16x4{0, 0, 0, 0};
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = f2bf(acc[e] + (beta ? bf2f(old[e]) : 0.f));
    *reinterpret_cast<u16x4*>(cp) = o;
}

}  // namespace sa_gemm
using namespace sa_gemm;

namespace sa_launch {
bool gemm_tn_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc) {
    return M % 16 == 0 && N % 16 == 0 && K % 128 == 0 && M > 0 && N > 0 && K > 0 && lda % 8 == 0 &&
           ldb % 8 == 0 && ldc % 4 == 0 && K * lda * 2 < (int64_t(1) << 31) && K * ldb * 2 < (int64_t(1) << 31) &&
           ldc < (1 << 30);
}
// Split plan for the ragged last round: with nwg tiles on `slots` workgroup slots (one 256x256 tile per CU), the
// r = nwg % slots tiles of the last round leave slots - r CUs idle; those tiles run as `split` K-slices each
// (2..4, >= 4 64-deep tiles per slice and an even number of them, chosen to minimise the tail's rounds x slice
// length) and a combine pass adds the fp32 partials into C.  Returns the fp32 workspace floats needed (0: no split).
int64_t gemm_tn_plan(int64_t M, int64_t N, int64_t K, int slots, int& full_blocks, int& split) {
    const int nwg = (int)(((M + 255) / 256) * ((N + 255) / 256));
    full_blocks = nwg;
    split = 1;
    if (slots <= 0) return 0;
    const int r = nwg % slots, nk = (int)(K / 64);
    if (r == 0 || nk % 2 != 0) return 0;
    // the split tail costs ceil(r * s / slots) rounds of 1/s of a tile: pick the cheapest s (fewest on ties)
    int s = 1;
    double best = 1.0;
    for (int c = 2; c <= 4; ++c) {
        if (nk % c != 0 || nk / c < 4 || (nk / c) % 2 != 0) continue;
        const double cost = (double)((r * c + slots - 1) / slots) / c;
        if (cost < best - 1e-9) { best = cost; s = c; }
    }
    if (s <= 1 || best > 0.8) return 0;
    split = s;
    full_blocks = nwg - r;
    return (int64_t)r * s * 65536;
}
void gemm_tn(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int64_t N,
             int64_t K, bool beta, hipStream_t st, int full_blocks, int split, float* ws) {
    const int nwg = (int)(((M + 255) / 256) * ((N + 255) / 256));
    if (full_blocks < 0 || split <= 1) { full_blocks = nwg; split = 1; }
    const int grid = full_blocks + (nwg - full_blocks) * split;
    const uint32_t ab = (uint32_t)(K * lda * 2), bb = (uint32_t)(K * ldb * 2);
    if (beta)
        hipLaunchKernelGGL((gemm_tn_ring_kernel<true>), dim3(grid), dim3(256), kSlots * kSlot, st, (const u16*)A,
                           (int)lda, ab, (const u16*)B, (int)ldb, bb, (u16*)C, (int)ldc, (int)M, (int)N, (int)K,
                           full_blocks, split, ws);
    else
        hipLaunchKernelGGL((gemm_tn_ring_kernel<false>), dim3(grid), dim3(256), kSlots * kSlot, st, (const u16*)A,
                           (int)lda, ab, (const u16*)B, (int)ldb, bb, (u16*)C, (int)ldc, (int)M, (int)N, (int)K,
                           full_blocks, split, ws);
    if (split > 1)
        hipLaunchKernelGGL(gemm_tn_combine_kernel, dim3(nwg - full_blocks, 64), dim3(256), 0, st, (const float*)ws,
                           (u16*)C, (int)ldc, (int)M, (int)N, full_blocks, split, beta ? 1 : 0);
}
}  // namespace sa_launch
