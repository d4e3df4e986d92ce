// bf16 GEMM for the weight gradient of a linear layer on gfx950:  C[M, N] (+)= A^T B  with
// A: [K, M] and B: [K, N] both stored k-major (row = reduction index), i.e. dW = dY^T X over the
// token dimension.  hipBLASLt runs this "TN with both operands k-strided" shape at ~1.0 PF in the
// 7B model (vs ~1.5 PF for the forward); here both operands are staged exactly as they lie in
// memory and the MFMA fragments are produced by the hardware transposing LDS read.
//
//  * 256x256 output tile per workgroup, 8 waves as 2 (M) x 4 (N), 128x64 per wave = 4x2 MFMA
//    32x32x16 tiles (128 fp32 accumulators per lane).
//  * K-tiles of 64 rows: A and B images [64][256] bf16 (512-B rows) filled by LDS-DMA
//    (buffer_load ... lds, 16 B per lane, source-permuted so the lane-linear destination IS the
//    swizzled image), two stages, the load of K-tile t+1 in flight while t is multiplied.
//  * Image swizzle: 16-B slot index XOR ((row & 3) << 2) puts the four rows of every
//    ds_read_b64_tr_b16 lane group in four different 64-B bank windows (conflict-free).
//  * Operand fragments: ds_read_b64_tr_b16 pairs (k rows kb+4h..+3 and kb+8+4h..+3) give each lane 8
//    k-values of its column; A and B use the same k permutation, so the MFMA sum is exact.
//  * Grid: XCD-aware bijective remap, then 8-row groups of tiles so the 32 tiles resident on one XCD
//    cover an 8x4 block and share A/B panels in its L2.
//  * Epilogue: C = acc (+ C) with one bf16 rounding (beta = 1 accumulates into a main-grad buffer).
#include <algorithm>

#include "common.h"
#include "flash_attn.h"
#include "launch.h"

using namespace sa;

namespace sa_gemm {

using fa::bf16x8;
using fa::lds_s16x4;
using fa::lds_void;

constexpr int kWaves = 8;
constexpr int kGroupM = 8;

__device__ __forceinline__ int koff(int r, int c) {
    return r * 512 + 16 * ((c >> 3) ^ ((r & 3) << 2)) + ((c & 7) << 1);
}

__device__ __forceinline__ bf16x8 frag_tr(const char* img, int kb, int c0, int lane) {
    const int h = lane >> 5, g = (lane >> 4) & 1, i = lane & 15;
    const int row = kb + 4 * h + (i >> 2);
    const int col = c0 + 16 * g + 4 * (i & 3);
    const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + koff(row, col)));
    const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + koff(row + 8, col)));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int BK>
struct Cfg {
    static constexpr int kImg = BK * 256 * 2;           // one operand's K-tile image [BK][256] bf16
    static constexpr int kStage = 2 * kImg;             // A + B
    static constexpr int kPieces = kImg / 1024 / kWaves;  // LDS-DMA instructions per wave per image
};

// this wave's LDS-DMA pieces of one [BK][256] operand image: a per-lane byte offset relative to the K-tile's
// first element (source-permuted swizzle), issued with the tile offset as the scalar soffset.  Piece i covers rows
// 2 (wave + NW i) + {0, 1}: the row advances by 2 NW (a multiple of 8), so the swizzle is the same for every piece
// and piece i only adds i * step bytes to the scalar offset (one VGPR per operand instead of NP).
template <int NP, int NW = kWaves>
struct Dma {
    static_assert(NW % 4 == 0, "piece rows must advance by a multiple of 8 for a piece-invariant swizzle");
    int voff;
    int step;
    __device__ __forceinline__ void init(int wave, int lane, int ld) {
        const int row = 2 * wave + (lane >> 5);
        const int slot = (lane & 31) ^ ((row & 3) << 2);
        voff = (row * ld + slot * 8) * 2;
        step = __builtin_amdgcn_readfirstlane(4 * NW * ld);
    }
    // Issued as inline asm on purpose: for a compiler-visible LDS-DMA the waitcnt pass cannot tell which LDS
    // bytes are pending and puts s_waitcnt vmcnt(0) in front of every later ds_read, draining the whole
    // prefetch pipeline each phase.  The kernel counts these loads itself (wait_vm) and retires them all
    // before the epilogue.
    // one piece (i must be a compile-time constant after unrolling)
    __device__ __forceinline__ void load_piece(int i, const void* base, uint32_t nbytes, int soff, char* img,
                                               int wave_u) const {
        typedef int i32x4 __attribute__((ext_vector_type(4)));
        const uint64_t a = reinterpret_cast<uint64_t>(base);
        const i32x4 rs = {(int)__builtin_amdgcn_readfirstlane((uint32_t)a),
                          (int)(__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) & 0xffff),
                          (int)__builtin_amdgcn_readfirstlane(nbytes), fa::kBufFlags};
        const uint32_t lds = __builtin_amdgcn_readfirstlane(
            (uint32_t)reinterpret_cast<uintptr_t>((lds_void*)(img + (wave_u + NW * i) * 1024)));
        int saved;
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %1\n\t"
            "s_nop 0\n\t"
            "buffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(saved)
            : "s"(lds), "v"(voff), "s"(rs), "s"(soff + i * step)
            : "memory");
    }
    // the same piece without a "memory" clobber, for a caller whose barriers (asm with a memory clobber) already
    // order it after the last reads of its destination: with the clobber the waitcnt pass drains every pending LDS
    // read (lgkmcnt(0)) right behind the asm
    __device__ __forceinline__ void load_piece_nc(int i, const void* base, uint32_t nbytes, int soff, char* img,
                                                  int wave_u) const {
        typedef int i32x4 __attribute__((ext_vector_type(4)));
        const uint64_t a = reinterpret_cast<uint64_t>(base);
        const i32x4 rs = {(int)__builtin_amdgcn_readfirstlane((uint32_t)a),
                          (int)(__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) & 0xffff),
                          (int)__builtin_amdgcn_readfirstlane(nbytes), fa::kBufFlags};
        const uint32_t lds = __builtin_amdgcn_readfirstlane(
            (uint32_t)reinterpret_cast<uintptr_t>((lds_void*)(img + (wave_u + NW * i) * 1024)));
        int saved;
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %1\n\t"
            "s_nop 0\n\t"
            "buffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(saved)
            : "s"(lds), "v"(voff), "s"(rs), "s"(soff + i * step));
    }
    __device__ __forceinline__ void load(const void* base, uint32_t nbytes, int soff, char* img, int wave_u) const {
        typedef int i32x4 __attribute__((ext_vector_type(4)));
        const uint64_t a = reinterpret_cast<uint64_t>(base);
        const i32x4 rs = {(int)__builtin_amdgcn_readfirstlane((uint32_t)a),
                          (int)(__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) & 0xffff),
                          (int)__builtin_amdgcn_readfirstlane(nbytes), fa::kBufFlags};
        const uint32_t lds0 = __builtin_amdgcn_readfirstlane(
            (uint32_t)reinterpret_cast<uintptr_t>((lds_void*)(img + wave_u * 1024)));
#pragma unroll
        for (int i = 0; i < NP; ++i)
        {
            int saved;
            asm volatile(
                "s_mov_b32 %0, m0\n\t"
                "s_mov_b32 m0, %1\n\t"
                "s_nop 0\n\t"
                "buffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
                "s_mov_b32 m0, %0"
                : "=&s"(saved)
                : "s"(lds0 + i * NW * 1024), "v"(voff), "s"(rs), "s"(soff + i * step)
                : "memory");
        }
    }
};

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

// Ping-pong schedule.  Waves 0-3 (group 0) and 4-7 (group 1) share the four SIMDs pairwise.  Each K-tile of BK
// rows is one phase per group:
//     [fragment reads of the tile, LDS-DMA of tile t+LEAD, lgkmcnt(0)]  barrier  [MFMAs, vmcnt: tile t+1 landed]  barrier
// Group 1 runs one barrier behind group 0, so on every SIMD one wave multiplies while its partner reads and stages.
// Reads are retired before the first barrier, so a buffer can be restaged in the phase after its last read
// (LEAD = STAGES - 1).  Tile t+1 must be retired by every wave before barrier event 2t+2, where group 0 starts
// reading it: that is group 0's second barrier of phase t (LATEWAIT: its wait sits behind its MFMAs) but group
// 1's FIRST barrier.  With two stages (LEAD 1) group 1 could not overlap its own DMA at all, so group 0 stages
// every piece (DMA0) and group 1 never waits.
constexpr int kDbgTiles = 8, kDbgT0 = 32, kDbgEv = 5;
template <bool BETA, int BK, int STAGES, bool LATEWAIT, bool TIMING = false>
__global__ __launch_bounds__(512, 1) void gemm_tn_kernel(const u16* __restrict__ A, int lda, uint32_t a_bytes,
                                                         const u16* __restrict__ B, int ldb, uint32_t b_bytes,
                                                         u16* __restrict__ C, int ldc, int M, int N, int K,
                                                         uint64_t* __restrict__ dbg, int full_blocks, int tail_split,
                                                         float* __restrict__ ws) {
    using G = Cfg<BK>;
    constexpr int KS = BK / 16;                   // MFMA k-steps per K-tile
    constexpr bool B3 = STAGES == 3;              // two A buffers + three B buffers (160 KiB): see below
    constexpr bool SPLIT = STAGES == 2 || B3;     // group 0 stages A images, group 1 stages B images
    constexpr int NW = SPLIT ? kWaves / 2 : kWaves;  // waves staging one image
    constexpr int NP = G::kImg / 1024 / NW;       // LDS-DMA instructions per staging wave per operand image
    constexpr int PT = SPLIT ? NP : 2 * NP;       // ... per K-tile
    constexpr int LEAD = STAGES - 1;              // K-tiles in flight ahead of the one being read
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 2, wn = wave & 3;  // wm doubles as the ping-pong group

    // tile coordinates.  Blocks [0, full_blocks) own whole tiles (XCD remap over them); with a split tail the
    // remaining tiles [full_blocks, nwg) run as tail_split K-slices each (one block per slice, the grid's last
    // round) writing fp32 partials that gemm_tn_combine adds into C — the last round is full instead of ragged.
    const int tm = M / 256, tn = N / 256;
    int v, k_lo = 0, nk = K / BK, unit = -1;
    if ((int)blockIdx.x < full_blocks) {
        v = xcd_remap(blockIdx.x, full_blocks);
    } else {
        unit = (int)blockIdx.x - full_blocks;
        v = full_blocks + unit / tail_split;
        nk /= tail_split;
        k_lo = (unit % tail_split) * nk;
    }
    const int group = kGroupM * tn;
    const int first_m = (v / group) * kGroupM;
    const int gm = min(tm - first_m, kGroupM);
    const int within = v % group;
    const int m0 = (first_m + within % gm) * 256, n0 = (within / gm) * 256;

    Dma<NP, NW> da, db;
    const bool stager = true;
    const int swave = SPLIT ? wave & 3 : wave;
    da.init(swave, lane, lda);
    db.init(swave, lane, ldb);

    f32x16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

#define SA_ISSUE(t_)                                                                                      \
    if (stager) {                                                                                         \
        char* st_ = smem + ((t_) % STAGES) * G::kStage;                                                   \
        const int k0_ = (k_lo + (t_)) * BK;                                                                        \
        da.load(A, a_bytes, __builtin_amdgcn_readfirstlane((k0_ * lda + m0) * 2), st_, swave);          \
        db.load(B, b_bytes, __builtin_amdgcn_readfirstlane((k0_ * ldb + n0) * 2), st_ + G::kImg, swave); \
    }
    // retire tile `need` given that tiles up to `last` have been issued
#define SA_RETIRE(need_, last_)                                                                           \
    if (stager) {                                                                                         \
        const int after_ = (last_) - (need_);                                                             \
        if (after_ >= 3) wait_vm<PT * 3>();                                                               \
        else if (after_ == 2) wait_vm<PT * 2>();                                                          \
        else if (after_ == 1) wait_vm<PT>();                                                              \
        else wait_vm<0>();                                                                                \
    }
    if constexpr (SPLIT) {
        // B3 (variant 5): A images rotate over two buffers, B images over three (2 x 32 + 3 x 32 KiB = all of LDS).
        // Group 1 then stages tile t+2's B image in its READ window of phase t (buffer (t+2) % 3 = (t-1) % 3, whose
        // last reads retired before event 2t) and retires it one read window later (before event 2t+4, where group
        // 0 starts reading it): no LDS-DMA issue inside any MFMA window, and B gets two phases of latency cover.
        // Two stages.  Group 0 stages tile t+1's A image at the start of its read window of phase t and retires
        // it behind its MFMAs (before barrier event 2t+2); group 1 stages tile t+2's B image inside its MFMA
        // window of phase t (event 2t+2 onward: both groups' reads of tile t are retired by then) and retires it
        // in its read window of phase t+1 (before event 2t+4).  Each wave has at most one image in flight.
#define SA_ABUF(t_) (B3 ? smem + ((t_) & 1) * G::kImg : smem + ((t_) & 1) * G::kStage)
#define SA_BBUF(t_) (B3 ? smem + (2 + (t_) % 3) * G::kImg : smem + ((t_) & 1) * G::kStage + G::kImg)
#define SA_ISSUE_G(t_)                                                                                    \
        {                                                                                                 \
            const int k0_ = (k_lo + (t_)) * BK;                                                                    \
            if (wm == 0) da.load(A, a_bytes, __builtin_amdgcn_readfirstlane((k0_ * lda + m0) * 2), SA_ABUF(t_), swave); \
            else db.load(B, b_bytes, __builtin_amdgcn_readfirstlane((k0_ * ldb + n0) * 2), SA_BBUF(t_), swave); \
        }
        SA_ISSUE_G(0)
        if (wm == 1 && nk > 1) {
            SA_ISSUE_G(1)
            wait_vm<NP>();
        } else {
            wait_vm<0>();
        }
        hard_barrier();
        if (wm == 1) hard_barrier();
        for (int t = 0; t < nk; ++t) {
            const char* ia = SA_ABUF(t);
            const char* ib = SA_BBUF(t);
            uint64_t* stamp = reinterpret_cast<uint64_t*>(smem + STAGES * G::kStage) +
                              (wave * kDbgTiles + (t - kDbgT0)) * kDbgEv;
            const bool rec = TIMING && blockIdx.x == 0 && t >= kDbgT0 && t < kDbgT0 + kDbgTiles && lane == 0;
#define SA_STAMP(e_) \
            if (rec) stamp[e_] = __builtin_amdgcn_s_memtime();
            SA_STAMP(0)
            bf16x8 a[KS][4], b[KS][2];
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
                for (int i = 0; i < 4; ++i) a[ks][i] = frag_tr(ia, 16 * ks, 128 * wm + 32 * i, lane);
#pragma unroll
                for (int j = 0; j < 2; ++j) b[ks][j] = frag_tr(ib, 16 * ks, 64 * wn + 32 * j, lane);
            }
            if constexpr (B3) {
                if (wm == 0) {
                    if (t + 1 < nk) SA_ISSUE_G(t + 1)
                } else if (t + 2 < nk) {
                    SA_ISSUE_G(t + 2)
                    wait_vm<NP>();  // B(t+1) retired, B(t+2) stays in flight
                } else {
                    wait_vm<0>();
                }
            } else if (t + 1 < nk) {
                if (wm == 0) SA_ISSUE_G(t + 1)
                else wait_vm<0>();
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            SA_STAMP(1)
            hard_barrier();
            SA_STAMP(2)
            __builtin_amdgcn_s_setprio(1);
            // group 1 threads its B-image pieces for tile t+2 between the MFMAs (one per 32 / NP MFMAs) so
            // they issue in the matrix pipe's shadow
            const bool stage_b = !B3 && wm == 1 && t + 2 < nk;
            const int soff_b = __builtin_amdgcn_readfirstlane(((k_lo + t + 2) * BK * ldb + n0) * 2);
            char* st_b = smem + (t & 1) * G::kStage + G::kImg;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        acc[i][j] = fa::mfma(b[ks][j], a[ks][i], acc[i][j]);
                        constexpr int every = (KS * 8) / NP;
                        const int m = ks * 8 + i * 2 + j;
                        if (m % every == every - 1 && stage_b) {
                            __builtin_amdgcn_sched_barrier(0);
                            db.load_piece(m / every, B, b_bytes, soff_b, st_b, swave);
                            __builtin_amdgcn_sched_barrier(0);
                        }
                    }
            }
            __builtin_amdgcn_s_setprio(0);
            if (wm == 0 && t + 1 < nk) wait_vm<0>();
            SA_STAMP(3)
            hard_barrier();
            SA_STAMP(4)
        }
#undef SA_STAMP
#undef SA_ISSUE_G
#undef SA_ABUF
#undef SA_BBUF
    } else {
    // prologue: LEAD K-tiles in flight, tile 0 retired, group 1 one barrier behind
#pragma unroll
    for (int t = 0; t < LEAD; ++t)
        if (t < nk) SA_ISSUE(t)
    SA_RETIRE(0, min(LEAD, nk) - 1)
    hard_barrier();
    if (wm == 1) hard_barrier();
    for (int t = 0; t < nk; ++t) {
        const char* ia = smem + (t % STAGES) * G::kStage;
        const char* ib = ia + G::kImg;
        uint64_t* stamp = reinterpret_cast<uint64_t*>(smem + STAGES * G::kStage) +
                          (wave * kDbgTiles + (t - kDbgT0)) * kDbgEv;
        const bool rec = TIMING && blockIdx.x == 0 && t >= kDbgT0 && t < kDbgT0 + kDbgTiles && lane == 0;
#define SA_STAMP(e_) \
        if (rec) stamp[e_] = __builtin_amdgcn_s_memtime();
        SA_STAMP(0)
        bf16x8 a[KS][4], b[KS][2];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
            for (int i = 0; i < 4; ++i) a[ks][i] = frag_tr(ia, 16 * ks, 128 * wm + 32 * i, lane);
#pragma unroll
            for (int j = 0; j < 2; ++j) b[ks][j] = frag_tr(ib, 16 * ks, 64 * wn + 32 * j, lane);
        }
        const int last = min(t + LEAD, nk - 1);  // last tile issued once this phase has staged
        if (t + LEAD < nk) SA_ISSUE(t + LEAD)
        if ((!LATEWAIT || wm == 1) && t + 1 < nk) SA_RETIRE(t + 1, last)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        SA_STAMP(1)
        hard_barrier();
        SA_STAMP(2)
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = fa::mfma(b[ks][j], a[ks][i], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
        if (LATEWAIT && wm == 0 && t + 1 < nk) SA_RETIRE(t + 1, last)
        SA_STAMP(3)
        hard_barrier();
        SA_STAMP(4)
    }
#undef SA_STAMP
    }
#undef SA_RETIRE
#undef SA_ISSUE
    if (wm == 0) hard_barrier();  // equal barrier counts for both groups
    if (TIMING && blockIdx.x == 0) {
        __syncthreads();
        const uint64_t* src = reinterpret_cast<const uint64_t*>(smem + STAGES * G::kStage);
        for (int i = threadIdx.x; i < kWaves * kDbgTiles * kDbgEv; i += blockDim.x) dbg[i] = src[i];
    }

    // epilogue: acc[i][j][4q + e] = C[m0 + 128wm + 32i + (lane & 31)][n0 + 64wn + 32j + 8q + 4h + e]
    const int h = lane >> 5, c = lane & 31;
    if (unit >= 0) {  // K-slice of a tail tile: fp32 partial [256][256] at ws + unit * 65536
        float* wp = ws + (int64_t)unit * 65536;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float* rp = wp + (128 * wm + 32 * i + c) * 256 + 64 * wn + 4 * h;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    f32x4 o;
#pragma unroll
                    for (int e = 0; e < 4; ++e) o[e] = acc[i][j][4 * q + e];
                    *reinterpret_cast<f32x4*>(rp + 32 * j + 8 * q) = o;
                }
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        u16* crow_p = C + (int64_t)(m0 + 128 * wm + 32 * i + c) * ldc + n0 + 64 * wn + 4 * h;
        u16x4 old[2][4];
        if (BETA) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) old[j][q] = *reinterpret_cast<const u16x4*>(crow_p + 32 * j + 8 * q);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                u16x4 o;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float x = acc[i][j][4 * q + e];
                    if (BETA) x += bf2f(old[j][q][e]);
                    o[e] = f2bf(x);
                }
                *reinterpret_cast<u16x4*>(crow_p + 32 * j + 8 * q) = o;
            }
    }
}

// ---------------------------------------------------------------------------------------------------------------
// Variant 4: the same ping-pong pipeline (BK 64, two stages, group 0 stages A images, group 1 stages B images in its
// MFMA window) on v_mfma_f32_16x16x32_bf16 — 64 MFMAs of 16 cycles per K-tile per wave instead of 32 of 32 cycles:
// the same cycles per FLOP, but the chip holds a higher clock on the 16x16 shape on random data
// (MI355X_MICROARCH.md 'DVFS give-back' item 7).
//  * fragment: lane (g = lane>>4, i = lane&15) holds column c0+i of the operand with k rows
//    {kb+4g .. +3} and {kb+16+4g .. +3} (two ds_read_b64_tr_b16); A and B use the same k permutation;
//  * the four 16-lane groups read the SAME 16 columns at different k rows, so the image swizzle also separates
//    rows r and r+4: 16-B slot ^ ((r&3)<<2 ^ ((r>>2)&1)<<1) keeps every half-wave's 32 8-B reads in 16 distinct
//    16-B bank windows (conflict-free); the LDS-DMA source addresses carry the same permutation.
__device__ __forceinline__ int sw16(int r) { return ((r & 3) << 2) ^ (((r >> 2) & 1) << 1); }
__device__ __forceinline__ int koff16(int r, int c) { return r * 512 + 16 * ((c >> 3) ^ sw16(r)) + ((c & 7) << 1); }

__device__ __forceinline__ bf16x8 frag16_tr(const char* img, int kb, int c0, int lane) {
    const int g = lane >> 4, i = lane & 15;
    const int row = kb + 4 * g + (i >> 2);
    const int col = c0 + 4 * (i & 3);
    const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + koff16(row, col)));
    const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + koff16(row + 16, col)));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int NP, int NW>
struct Dma16 : Dma<NP, NW> {
    __device__ __forceinline__ void init(int wave, int lane, int ld) {
        const int row = 2 * wave + (lane >> 5);
        const int slot = (lane & 31) ^ sw16(row);
        this->voff = (row * ld + slot * 8) * 2;
        this->step = __builtin_amdgcn_readfirstlane(4 * NW * ld);
    }
};

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <bool BETA>
__global__ __launch_bounds__(512, 1) void gemm_tn16_kernel(const u16* __restrict__ A, int lda, uint32_t a_bytes,
                                                           const u16* __restrict__ B, int ldb, uint32_t b_bytes,
                                                           u16* __restrict__ C, int ldc, int M, int N, int K) {
    constexpr int BK = 64;
    using G = Cfg<BK>;
    constexpr int KS = BK / 32;                  // 16x16x32 k-steps per K-tile
    constexpr int NW = kWaves / 2;               // waves staging one image
    constexpr int NP = G::kImg / 1024 / NW;      // LDS-DMA instructions per staging wave per image
    constexpr int NMF = KS * 8 * 4;              // MFMAs per wave per K-tile
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 2, wn = wave & 3;  // wm doubles as the ping-pong group

    const int tm = M / 256, tn = N / 256, nwg = tm * tn;
    const int v = xcd_remap(blockIdx.x, nwg);
    const int group = kGroupM * tn;
    const int first_m = (v / group) * kGroupM;
    const int gm = min(tm - first_m, kGroupM);
    const int within = v % group;
    const int m0 = (first_m + within % gm) * 256, n0 = (within / gm) * 256;

    Dma16<NP, NW> da, db;
    const int swave = wave & 3;
    da.init(swave, lane, lda);
    db.init(swave, lane, ldb);

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = K / BK;
#define SA_ISSUE_G(t_)                                                                                        \
    {                                                                                                         \
        char* st_ = smem + ((t_) & 1) * G::kStage;                                                            \
        const int k0_ = (t_) * BK;                                                                            \
        if (wm == 0) da.load(A, a_bytes, __builtin_amdgcn_readfirstlane((k0_ * lda + m0) * 2), st_, swave);       \
        else db.load(B, b_bytes, __builtin_amdgcn_readfirstlane((k0_ * ldb + n0) * 2), st_ + G::kImg, swave);     \
    }
    SA_ISSUE_G(0)
    if (wm == 1 && nk > 1) {
        SA_ISSUE_G(1)
        wait_vm<NP>();
    } else {
        wait_vm<0>();
    }
    hard_barrier();
    if (wm == 1) hard_barrier();
    for (int t = 0; t < nk; ++t) {
        const char* ia = smem + (t & 1) * G::kStage;
        const char* ib = ia + G::kImg;
        bf16x8 a[KS][8], b[KS][4];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
            for (int i = 0; i < 8; ++i) a[ks][i] = frag16_tr(ia, 32 * ks, 128 * wm + 16 * i, lane);
#pragma unroll
            for (int j = 0; j < 4; ++j) b[ks][j] = frag16_tr(ib, 32 * ks, 64 * wn + 16 * j, lane);
        }
        if (t + 1 < nk) {
            if (wm == 0) SA_ISSUE_G(t + 1)
            else wait_vm<0>();
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        hard_barrier();
        __builtin_amdgcn_s_setprio(1);
        const bool stage_b = wm == 1 && t + 2 < nk;
        const int soff_b = __builtin_amdgcn_readfirstlane(((t + 2) * BK * ldb + n0) * 2);
        char* st_b = smem + (t & 1) * G::kStage + G::kImg;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc[i][j] = mfma16(b[ks][j], a[ks][i], acc[i][j]);
                    constexpr int every = NMF / NP;
                    const int m = ks * 32 + i * 4 + j;
                    if (m % every == every - 1 && stage_b) {
                        __builtin_amdgcn_sched_barrier(0);
                        db.load_piece(m / every, B, b_bytes, soff_b, st_b, swave);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
        }
        __builtin_amdgcn_s_setprio(0);
        if (wm == 0 && t + 1 < nk) wait_vm<0>();
        hard_barrier();
    }
#undef SA_ISSUE_G
    if (wm == 0) hard_barrier();  // equal barrier counts for both groups

    // epilogue: acc[i][j][e] = C[m0 + 128wm + 16i + (lane & 15)][n0 + 64wn + 16j + 4(lane >> 4) + e]
    const int r = lane & 15, q = lane >> 4;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        u16* crow_p = C + (int64_t)(m0 + 128 * wm + 16 * i + r) * ldc + n0 + 64 * wn + 4 * q;
        u16x4 old[4];
        if (BETA) {
#pragma unroll
            for (int j = 0; j < 4; ++j) old[j] = *reinterpret_cast<const u16x4*>(crow_p + 16 * j);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
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
template __global__ void gemm_tn16_kernel<true>(const u16* __restrict__, int, uint32_t, const u16* __restrict__, int,
                                                uint32_t, u16* __restrict__, int, int, int, int);
template __global__ void gemm_tn16_kernel<false>(const u16* __restrict__, int, uint32_t, const u16* __restrict__, int,
                                                 uint32_t, u16* __restrict__, int, int, int, int);

// ---------------------------------------------------------------------------------------------------------------
// Variant 6: no ping-pong.  Every wave interleaves its own fragment reads with its MFMAs (the reads of k-step ks+1
// issue in the shadow of k-step ks's 8 MFMAs), so both waves of a SIMD feed the matrix pipe all the time instead of
// alternating a 32-MFMA window with a read window.  One barrier per 64-deep K-tile, placed before the tile's last
// k-step: by then every wave has retired its reads of the tile and its LDS-DMA pieces of the next one, so right after
// it each wave (a) reads the next tile's first fragments and (b) threads its pieces of tile t+2 (into the buffer
// just released) between the last k-step's MFMAs — the barrier's read latency hides behind those MFMAs.
//   LDS 2 x 64 KiB; every wave stages NP = 4 pieces of each operand image per K-tile.
template <bool BETA, bool TIMING = false>
__global__ __launch_bounds__(512, 1) void gemm_tn_il_kernel(const u16* __restrict__ A, int lda, uint32_t a_bytes,
                                                            const u16* __restrict__ B, int ldb, uint32_t b_bytes,
                                                            u16* __restrict__ C, int ldc, int M, int N, int K,
                                                            int full_blocks, int tail_split, float* __restrict__ ws,
                                                            uint64_t* __restrict__ dbg = nullptr) {
    constexpr int BK = 64;
    using G = Cfg<BK>;
    constexpr int NP = G::kImg / 1024 / kWaves;  // LDS-DMA pieces per wave per operand image (4)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 2, wn = wave & 3;

    const int tm = M / 256, tn = N / 256;
    int v, k_lo = 0, nk = K / BK, unit = -1;
    if ((int)blockIdx.x < full_blocks) {
        v = xcd_remap(blockIdx.x, full_blocks);
    } else {
        unit = (int)blockIdx.x - full_blocks;
        v = full_blocks + unit / tail_split;
        nk /= tail_split;
        k_lo = (unit % tail_split) * nk;
    }
    const int group = kGroupM * tn;
    const int first_m = (v / group) * kGroupM;
    const int gm = min(tm - first_m, kGroupM);
    const int within = v % group;
    const int m0 = (first_m + within % gm) * 256, n0 = (within / gm) * 256;

    Dma<NP, kWaves> da, db;
    da.init(wave, lane, lda);
    db.init(wave, lane, ldb);

    f32x16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    bf16x8 fa[2][4], fb[2][2];
#define SA_IL_READ(IA, IB, KS, SET)                                                                     \
    {                                                                                                   \
        _Pragma("unroll") for (int i = 0; i < 4; ++i) fa[SET][i] = frag_tr((IA), 16 * (KS), 128 * wm + 32 * i, lane); \
        _Pragma("unroll") for (int j = 0; j < 2; ++j) fb[SET][j] = frag_tr((IB), 16 * (KS), 64 * wn + 32 * j, lane);  \
    }
#define SA_IL_MFMA(SET)                                                                                 \
    {                                                                                                   \
        _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                   \
            _Pragma("unroll") for (int j = 0; j < 2; ++j) acc[i][j] = fa::mfma(fb[SET][j], fa[SET][i], acc[i][j]); \
    }
    // 8 MFMAs of the current k-step with the 12 reads of the next one threaded between them
#define SA_IL_SCHED()                                                       \
    {                                                                       \
        _Pragma("unroll") for (int q = 0; q < 4; ++q) {                     \
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);              \
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);              \
        }                                                                   \
        _Pragma("unroll") for (int q = 0; q < 4; ++q) {                     \
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);              \
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);              \
        }                                                                   \
    }
    auto soff_a = [&](int t) { return __builtin_amdgcn_readfirstlane(((k_lo + t) * BK * lda + m0) * 2); };
    auto soff_b = [&](int t) { return __builtin_amdgcn_readfirstlane(((k_lo + t) * BK * ldb + n0) * 2); };

    // prologue: tiles 0 and 1 in flight, tile 0 retired, its first fragments requested
    da.load(A, a_bytes, soff_a(0), smem, wave);
    db.load(B, b_bytes, soff_b(0), smem + G::kImg, wave);
    if (nk > 1) {
        da.load(A, a_bytes, soff_a(1), smem + G::kStage, wave);
        db.load(B, b_bytes, soff_b(1), smem + G::kStage + G::kImg, wave);
        wait_vm<2 * NP>();
    } else {
        wait_vm<0>();
    }
    hard_barrier();
    SA_IL_READ(smem, smem + G::kImg, 0, 0)
    for (int t = 0; t < nk; ++t) {
        const char* ia = smem + (t & 1) * G::kStage;
        const char* ib = ia + G::kImg;
        // timing build: events per K-tile 0 top, 1 k-steps 0-2 issued, 2 reads + DMA retired, 3 past the barrier,
        // 4 last k-step issued (stamps of workgroup 0 in LDS past the two stages)
        uint64_t* stamp = reinterpret_cast<uint64_t*>(smem + 2 * G::kStage) + (wave * kDbgTiles + (t - kDbgT0)) * kDbgEv;
        const bool rec = TIMING && blockIdx.x == 0 && t >= kDbgT0 && t < kDbgT0 + kDbgTiles && lane == 0;
#define SA_IL_STAMP(e_) \
        if (rec) stamp[e_] = __builtin_amdgcn_s_memtime();
        SA_IL_STAMP(0)
        SA_IL_READ(ia, ib, 1, 1)
        SA_IL_MFMA(0)
        SA_IL_SCHED()
        SA_IL_READ(ia, ib, 2, 0)
        SA_IL_MFMA(1)
        SA_IL_SCHED()
        SA_IL_READ(ia, ib, 3, 1)
        SA_IL_MFMA(0)
        SA_IL_SCHED()
        // every read of buffer t&1 retired (compiler-visible wait, so its own lgkm bookkeeping stays exact), this
        // wave's pieces of tile t+1 landed -> publish
        SA_IL_STAMP(1)
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        wait_vm<0>();
        SA_IL_STAMP(2)
        hard_barrier();
        SA_IL_STAMP(3)
        {  // next tile's first fragments (after the last tile: a harmless read of the other buffer, never used)
            const char* na = smem + ((t + 1) & 1) * G::kStage;
            SA_IL_READ(na, na + G::kImg, 0, 0)
        }
        // last k-step of tile t; tile t+2's pieces (into the buffer just released) threaded between its MFMAs
        const bool stage = t + 2 < nk;
        char* st = smem + (t & 1) * G::kStage;
        const int sa = soff_a(t + 2), sb = soff_b(t + 2);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                acc[i][j] = fa::mfma(fb[1][j], fa[1][i], acc[i][j]);
                const int m = i * 2 + j;  // 8 MFMAs, 8 pieces: A pieces after even, B pieces after odd MFMAs
                if (stage) {
                    __builtin_amdgcn_sched_barrier(0);
                    if ((m & 1) == 0) da.load_piece_nc(m >> 1, A, a_bytes, sa, st, wave);
                    else db.load_piece_nc(m >> 1, B, b_bytes, sb, st + G::kImg, wave);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        SA_IL_STAMP(4)
#undef SA_IL_STAMP
    }
    if (TIMING && blockIdx.x == 0) {
        __syncthreads();
        const uint64_t* src = reinterpret_cast<const uint64_t*>(smem + 2 * G::kStage);
        for (int i = threadIdx.x; i < kWaves * kDbgTiles * kDbgEv; i += blockDim.x) dbg[i] = src[i];
    }
#undef SA_IL_READ
#undef SA_IL_MFMA
#undef SA_IL_SCHED

    const int h = lane >> 5, c = lane & 31;
    if (unit >= 0) {  // K-slice of a tail tile: fp32 partial [256][256] at ws + unit * 65536
        float* wp = ws + (int64_t)unit * 65536;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float* rp = wp + (128 * wm + 32 * i + c) * 256 + 64 * wn + 4 * h;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    f32x4 o;
#pragma unroll
                    for (int e = 0; e < 4; ++e) o[e] = acc[i][j][4 * q + e];
                    *reinterpret_cast<f32x4*>(rp + 32 * j + 8 * q) = o;
                }
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        u16* crow_p = C + (int64_t)(m0 + 128 * wm + 32 * i + c) * ldc + n0 + 64 * wn + 4 * h;
        u16x4 old[2][4];
        if (BETA) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) old[j][q] = *reinterpret_cast<const u16x4*>(crow_p + 32 * j + 8 * q);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                u16x4 o;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float x = acc[i][j][4 * q + e];
                    if (BETA) x += bf2f(old[j][q][e]);
                    o[e] = f2bf(x);
                }
                *reinterpret_cast<u16x4*>(crow_p + 32 * j + 8 * q) = o;
            }
    }
}
template __global__ void gemm_tn_il_kernel<true, false>(const u16* __restrict__, int, uint32_t, const u16* __restrict__,
                                                        int, uint32_t, u16* __restrict__, int, int, int, int, int, int,
                                                        float* __restrict__, uint64_t* __restrict__);
template __global__ void gemm_tn_il_kernel<false, false>(const u16* __restrict__, int, uint32_t, const u16* __restrict__,
                                                         int, uint32_t, u16* __restrict__, int, int, int, int, int, int,
                                                         float* __restrict__, uint64_t* __restrict__);
template __global__ void gemm_tn_il_kernel<false, true>(const u16* __restrict__, int, uint32_t, const u16* __restrict__,
                                                        int, uint32_t, u16* __restrict__, int, int, int, int, int, int,
                                                        float* __restrict__, uint64_t* __restrict__);

// ---------------------------------------------------------------------------------------------------------------
// Variant 7: one wave per SIMD, register-staged.  The ping-pong kernels above pay for their LDS-DMA pieces in the
// issue stream (~60 cycles per 1-KiB piece among MFMAs, 100-185 inside a read phase: MI355X_MICROARCH.md cycle
// constants) and for 1.5 transposing LDS reads per MFMA at a 128x64 wave tile.  Here:
//  * 4 waves x 128x128 (4 x 4 MFMA 32x32x16 tiles, 256 fp32 accumulators per lane in the unified register file):
//    one transposing read per MFMA;
//  * the next K-tile travels global -> VGPRs (16 B per lane per load, 64 staging VGPRs) and is written into the
//    other LDS buffer with ds_write_b128 in the MFMA gaps of k-step 2; the global loads of the tile after it are
//    issued right behind, so each load has about two K-tiles of latency cover;
//  * one barrier per 64-deep K-tile, placed before the last k-step: right after it the wave reads the next tile's
//    first fragments, whose latency hides behind the last k-step's 16 MFMAs.
// LDS images and fragment reads are those of variant 2 (koff swizzle, frag_tr), written directly (no source
// permutation: register staging writes any layout).
template <bool BETA>
__global__ __launch_bounds__(256, 1) void gemm_tn_w4_kernel(const u16* __restrict__ A, int lda,
                                                            const u16* __restrict__ B, int ldb, u16* __restrict__ C,
                                                            int ldc, int M, int N, int K, int full_blocks, int tail_split,
                                                            float* __restrict__ ws) {
    constexpr int BK = 64, IMG = BK * 256 * 2, STAGE = 2 * IMG;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int tm = M / 256, tn = N / 256;
    int v, k_lo = 0, nk = K / BK, unit = -1;
    if ((int)blockIdx.x < full_blocks) {
        v = xcd_remap(blockIdx.x, full_blocks);
    } else {
        unit = (int)blockIdx.x - full_blocks;
        v = full_blocks + unit / tail_split;
        nk /= tail_split;
        k_lo = (unit % tail_split) * nk;
    }
    const int group = kGroupM * tn;
    const int first_m = (v / group) * kGroupM;
    const int gm = min(tm - first_m, kGroupM);
    const int within = v % group;
    const int m0 = (first_m + within % gm) * 256, n0 = (within / gm) * 256;

    // staging: this wave moves image rows 16 wave + 2 i + (lane >> 5), i < 8, 16 B (8 columns) per lane
    const int srow = 16 * wave + (lane >> 5), scol = 8 * (lane & 31);
    // buffer loads: one 32-bit lane offset per operand, the row / K-tile steps in scalar offsets (64-bit per-load
    // addresses would cost 32 VGPRs the staging registers need)
    const __amdgpu_buffer_rsrc_t ra = fa::uniform_rsrc(A + (int64_t)k_lo * BK * lda + m0, (uint32_t)(nk * BK * lda * 2));
    const __amdgpu_buffer_rsrc_t rb = fa::uniform_rsrc(B + (int64_t)k_lo * BK * ldb + n0, (uint32_t)(nk * BK * ldb * 2));
    const int va = (srow * lda + scol) * 2, vb = (srow * ldb + scol) * 2;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 sa[8], sb[8];
    auto load = [&](int t) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            sa[i] = __builtin_amdgcn_raw_buffer_load_b128(ra, va, __builtin_amdgcn_readfirstlane((t * BK + 2 * i) * lda * 2), 0);
            sb[i] = __builtin_amdgcn_raw_buffer_load_b128(rb, vb, __builtin_amdgcn_readfirstlane((t * BK + 2 * i) * ldb * 2), 0);
        }
    };
    auto store = [&](char* st) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            *reinterpret_cast<u32x4*>(st + koff(srow + 2 * i, scol)) = sa[i];
            *reinterpret_cast<u32x4*>(st + IMG + koff(srow + 2 * i, scol)) = sb[i];
        }
    };
    bf16x8 fa_[4], fb_[4], ga_[4], gb_[4];  // fragments of the current / next k-step
    auto read = [&](const char* st, int ks, bf16x8 (&a)[4], bf16x8 (&b)[4]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = frag_tr(st, 16 * ks, 128 * wm + 32 * i, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = frag_tr(st + IMG, 16 * ks, 128 * wn + 32 * j, lane);
    };
    f32x16 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    auto mfmas = [&](const bf16x8 (&a)[4], const bf16x8 (&b)[4]) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = fa::mfma(b[j], a[i], acc[i][j]);
    };

    // prologue: tile 0 in LDS buffer 0, tile 1 in flight in the staging registers, k-step 0 fragments read
    load(0);
    store(smem);
    if (nk > 1) load(1);
    __syncthreads();
    read(smem, 0, fa_, fb_);
    // issue order inside a k-step: one fragment read (and in k-step 2 one ds_write + one global load) per MFMA gap
    auto interleave = [&](int extra) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
            if (extra) {
                __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
            }
        }
    };
    for (int t = 0; t < nk; ++t) {
        const char* cur = smem + (t & 1) * STAGE;
        char* nxt = smem + ((t + 1) & 1) * STAGE;
        read(cur, 1, ga_, gb_);
        mfmas(fa_, fb_);  // k-step 0
        interleave(0);
        __builtin_amdgcn_sched_barrier(0);
        read(cur, 2, fa_, fb_);
        mfmas(ga_, gb_);  // k-step 1
        interleave(0);
        __builtin_amdgcn_sched_barrier(0);
        read(cur, 3, ga_, gb_);
        if (t + 1 < nk) store(nxt);  // tile t+1 (staged during tile t-1) -> the buffer tile t-1 used
        if (t + 2 < nk) load(t + 2);
        mfmas(fa_, fb_);  // k-step 2
        interleave(1);
        __builtin_amdgcn_sched_barrier(0);
        // tile t+1's image complete and every wave done reading tile t's k-steps (k-step 3 is in registers)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (t + 1 < nk) read(nxt, 0, fa_, fb_);
        mfmas(ga_, gb_);  // k-step 3
        interleave(0);
        __builtin_amdgcn_sched_barrier(0);
    }

    const int h = lane >> 5, c = lane & 31;
    if (unit >= 0) {  // K-slice of a tail tile: fp32 partial [256][256] at ws + unit * 65536
        float* wp = ws + (int64_t)unit * 65536;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float* rp = wp + (128 * wm + 32 * i + c) * 256 + 128 * wn + 4 * h;
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    f32x4 o;
#pragma unroll
                    for (int e = 0; e < 4; ++e) o[e] = acc[i][j][4 * q + e];
                    *reinterpret_cast<f32x4*>(rp + 32 * j + 8 * q) = o;
                }
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        u16* crow_p = C + (int64_t)(m0 + 128 * wm + 32 * i + c) * ldc + n0 + 128 * wn + 4 * h;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            u16x4 old[4];
            if (BETA) {
#pragma unroll
                for (int q = 0; q < 4; ++q) old[q] = *reinterpret_cast<const u16x4*>(crow_p + 32 * j + 8 * q);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                u16x4 o;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float x = acc[i][j][4 * q + e];
                    if (BETA) x += bf2f(old[q][e]);
                    o[e] = f2bf(x);
                }
                *reinterpret_cast<u16x4*>(crow_p + 32 * j + 8 * q) = o;
            }
        }
    }
}
template __global__ void gemm_tn_w4_kernel<true>(const u16* __restrict__, int, const u16* __restrict__, int,
                                                 u16* __restrict__, int, int, int, int, int, int, float* __restrict__);
template __global__ void gemm_tn_w4_kernel<false>(const u16* __restrict__, int, const u16* __restrict__, int,
                                                  u16* __restrict__, int, int, int, int, int, int, float* __restrict__);

// ---------------------------------------------------------------------------------------------------------------
// Variant 8: one wave per SIMD on v_mfma_f32_16x16x32_bf16, both operands by LDS-DMA.  The shape of the vendor
// library's fastest forward kernel on this chip (256x256x64 macro tile, 4 waves x 128x128, 16x16x32 MFMAs, DMA pieces
// threaded between the MFMAs, one barrier per K-tile), with the operand fragments produced by transposing LDS reads
// because both wgrad operands are k-strided.
//  * 64 MFMAs of 16 cycles per 32-deep k-step per wave (8 x 8 tiles of 16x16, 256 fp32 accumulators per lane in the
//    unified register file); 16 fragments per k-step = 32 ds_read_b64_tr_b16 (0.5 per MFMA);
//  * per 64-deep K-tile each wave stages 8 one-KiB pieces of the A image and 8 of the B image (koff16 swizzle, the
//    images of variant 4);
//  * fragment addresses are per-lane offsets precomputed for both stages (the loop is unrolled by two tiles so the
//    stage is a constant); k-step, second read and image offsets ride in the ds_read immediate.
// in-place accumulate in AGPRs: with 256 live fp32 accumulators per lane the register allocator otherwise
// rotates them through copies (v_accvgpr_read/write/mov per MFMA) and spills the fragments
__device__ __forceinline__ void mfma16_acc(f32x4& c, const bf16x8& a, const bf16x8& b) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

template <bool BETA>
__global__ __launch_bounds__(256, 1) void gemm_tn_w4m16_kernel(const u16* __restrict__ A, int lda, uint32_t a_bytes,
                                                               const u16* __restrict__ B, int ldb, uint32_t b_bytes,
                                                               u16* __restrict__ C, int ldc, int M, int N, int K,
                                                               int full_blocks, int tail_split, float* __restrict__ ws) {
    constexpr int BK = 64;
    using G = Cfg<BK>;
    constexpr int NW = 4;                         // every wave stages both images
    constexpr int NP = G::kImg / 1024 / NW;       // 8 pieces per wave per image
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 1, wn = wave & 1;

    const int tm = M / 256, tn = N / 256;
    int v, k_lo = 0, nk = K / BK, unit = -1;
    if ((int)blockIdx.x < full_blocks) {
        v = xcd_remap(blockIdx.x, full_blocks);
    } else {
        unit = (int)blockIdx.x - full_blocks;
        v = full_blocks + unit / tail_split;
        nk /= tail_split;
        k_lo = (unit % tail_split) * nk;
    }
    const int group = kGroupM * tn;
    const int first_m = (v / group) * kGroupM;
    const int gm = min(tm - first_m, kGroupM);
    const int within = v % group;
    const int m0 = (first_m + within % gm) * 256, n0 = (within / gm) * 256;

    Dma16<NP, NW> da, db;
    da.init(wave, lane, lda);
    db.init(wave, lane, ldb);
    auto soff_a = [&](int t) { return __builtin_amdgcn_readfirstlane(((k_lo + t) * BK * lda + m0) * 2); };
    auto soff_b = [&](int t) { return __builtin_amdgcn_readfirstlane(((k_lo + t) * BK * ldb + n0) * 2); };

    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // per-lane LDS byte offsets of the 16 fragments (k-step 0, first transposing read) in each stage
    int oa[2][8], ob[2][8];
    {
        const int g = lane >> 4, i16 = lane & 15;
        const int row = 4 * g + (i16 >> 2), cl = 4 * (i16 & 3);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                oa[s][i] = s * G::kStage + koff16(row, 128 * wm + 16 * i + cl);
                ob[s][i] = s * G::kStage + G::kImg + koff16(row, 128 * wn + 16 * i + cl);
            }
    }
    auto frag = [&](int off, int ks) -> bf16x8 {
        const char* p = smem + off + ks * 32 * 512;
        const s16x4 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
        const s16x4 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 16 * 512));
        return __builtin_bit_cast(bf16x8, __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7));
    };

    bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
#define SA_W16_READ(S, KS, FA, FB)                                                \
    {                                                                             \
        _Pragma("unroll") for (int j = 0; j < 8; ++j) FB[j] = frag(ob[S][j], KS); \
        _Pragma("unroll") for (int i = 0; i < 8; ++i) FA[i] = frag(oa[S][i], KS); \
    }
    // One 64-deep K-tile t in LDS stage S (tile t+1 in flight into stage 1-S).  k-step 0 multiplies beside the
    // k-step 1 fragment reads (one per two MFMAs); one barrier (every read of stage S retired, this wave's pieces of
    // tile t+1 landed); k-step 1 multiplies beside tile t+1's k-step 0 reads (first half, one per MFMA) and tile t+2's
    // pieces into stage S (second half, one per two MFMAs).  Branch-free: after the last tile the reads hit the other
    // stage harmlessly and the last two tiles re-stage tile nk-1 into a stage never read again.
#define SA_W16_TILE(S, T)                                                                                       \
    {                                                                                                           \
        _Pragma("unroll") for (int i = 0; i < 8; ++i)                                                           \
            _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                                     \
                mfma16_acc(acc[i][j], fb0[j], fa0[i]);                                                          \
                const int m_ = i * 8 + j;                                                                       \
                if ((m_ & 3) == 3) {                                                                            \
                    const int f_ = m_ >> 2;                                                                     \
                    if (f_ < 8) fb1[f_] = frag(ob[S][f_], 1);                                                   \
                    else fa1[f_ - 8] = frag(oa[S][f_ - 8], 1);                                                  \
                }                                                                                               \
            }                                                                                                   \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                      \
        wait_vm<0>();                                                                                           \
        hard_barrier();                                                                                         \
        _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                           \
            _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                                     \
                mfma16_acc(acc[i][j], fb1[j], fa1[i]);                                                          \
                const int m_ = i * 8 + j;                                                                       \
                if ((m_ & 1) == 1) {                                                                            \
                    const int f_ = m_ >> 1;                                                                     \
                    if (f_ < 8) fb0[f_] = frag(ob[1 - (S)][f_], 0);                                             \
                    else fa0[f_ - 8] = frag(oa[1 - (S)][f_ - 8], 0);                                            \
                }                                                                                               \
            }                                                                                                   \
        {                                                                                                       \
            const int t2_ = min((T) + 2, nk - 1);                                                               \
            const int sa_ = soff_a(t2_), sb_ = soff_b(t2_);                                                     \
            char* st_ = smem + (S) * G::kStage;                                                                 \
            _Pragma("unroll") for (int i = 4; i < 8; ++i)                                                       \
                _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                                 \
                    mfma16_acc(acc[i][j], fb1[j], fa1[i]);                                                      \
                    const int m_ = (i - 4) * 8 + j;                                                             \
                    if ((m_ & 1) == 1) {                                                                        \
                        const int p_ = m_ >> 1;                                                                 \
                        if ((p_ & 1) == 0) da.load_piece_nc(p_ >> 1, A, a_bytes, sa_, st_, wave);               \
                        else db.load_piece_nc(p_ >> 1, B, b_bytes, sb_, st_ + G::kImg, wave);                   \
                    }                                                                                           \
                }                                                                                               \
        }                                                                                                       \
    }

    // prologue: tiles 0 and 1 in flight, tile 0 landed everywhere, its k-step 0 fragments read
    da.load(A, a_bytes, soff_a(0), smem, wave);
    db.load(B, b_bytes, soff_b(0), smem + G::kImg, wave);
    if (nk > 1) {
        da.load(A, a_bytes, soff_a(1), smem + G::kStage, wave);
        db.load(B, b_bytes, soff_b(1), smem + G::kStage + G::kImg, wave);
        wait_vm<2 * NP>();
    } else {
        wait_vm<0>();
    }
    hard_barrier();
    SA_W16_READ(0, 0, fa0, fb0)
    int t = 0;
    for (; t + 1 < nk; t += 2) {
        SA_W16_TILE(0, t)
        SA_W16_TILE(1, t + 1)
    }
    if (t < nk) SA_W16_TILE(0, t)
#undef SA_W16_TILE
#undef SA_W16_READ
    wait_vm<0>();
    // the MFMAs are inline asm, invisible to the hazard recognizer: cover the MFMA -> VALU read of the accumulators
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

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
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        u16* crow_p = C + (int64_t)(m0 + 128 * wm + 16 * i + r) * ldc + n0 + 128 * wn + q4;
        u16x4 old[8];
        if (BETA) {
#pragma unroll
            for (int j = 0; j < 8; ++j) old[j] = *reinterpret_cast<const u16x4*>(crow_p + 16 * j);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
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
template __global__ void gemm_tn_w4m16_kernel<true>(const u16* __restrict__, int, uint32_t, const u16* __restrict__,
                                                    int, uint32_t, u16* __restrict__, int, int, int, int, int, int,
                                                    float* __restrict__);
template __global__ void gemm_tn_w4m16_kernel<false>(const u16* __restrict__, int, uint32_t, const u16* __restrict__,
                                                     int, uint32_t, u16* __restrict__, int, int, int, int, int, int,
                                                     float* __restrict__);

// ---------------------------------------------------------------------------------------------------------------
// Variant 9: variant 8's wave layout (4 waves x 128x128, 16x16x32 MFMAs, in-place AGPR accumulators) on a four-slot
// LDS ring of 32-deep k-steps (A and B images [32][256] bf16 per slot, 4 x 32 KiB) instead of two 64-deep stages:
//  * during k-step t each wave multiplies F_t (in registers), reads F_{t+1} from slot (t+1)%4 (16 fragments over the
//    first 48 MFMAs) and stages k-step t+4 into slot t%4 (8 one-KiB pieces, one per 8 MFMAs);
//  * one barrier per k-step: every wave's reads of slot (t+1)%4 retired and k-step t+2 landed (vmcnt leaves the
//    16 pieces of k-steps t+3 and t+4 in flight), so each piece has 2-3 k-steps (2-3k cycles) to land instead of 1-2.
//  SCHED: 0 = F_{t+1} reads one per 3 MFMAs over the first 48, pieces one per 8 MFMAs; 1 = reads one per 2 MFMAs over
//  the first 32, pieces one per 4 over the last 32; 2 = one fragment (two transposing reads) per 4 MFMAs and one piece
//  per 8 over the whole k-step (the default: every issue slot evenly loaded, +2-4 % over 1); 5 = like 2 with the two
//  reads of a fragment in separate MFMA gaps.
//  FASTDMA: 0 = Dma::load_piece_nc (descriptor rebuilt per piece, m0 saved / restored); 1 = descriptors built once,
//  m0 clobbered (the compiler emits no other m0 use in this kernel, but an m0 clobber is only a warning to it);
//  2 = descriptors built once, m0 saved / restored around each piece.
//  SCHED 3 = SCHED 1 with the pieces one per 2 MFMAs over MFMAs 32-47 (they land earlier).
//  TIMING: s_memtime stamps of workgroup 0, k-steps 32-39, events 0 top, 1 MFMA stream issued, 2 reads retired,
//  3 pieces landed, 4 past the barrier (LDS past the ring, then dbg[wave][step][event]).
template <bool BETA, int SCHED = 0, int FASTDMA = 0, bool TIMING = false>
__global__ __launch_bounds__(256, 1) void gemm_tn_ring_kernel(const u16* __restrict__ A, int lda, uint32_t a_bytes,
                                                              const u16* __restrict__ B, int ldb, uint32_t b_bytes,
                                                              u16* __restrict__ C, int ldc, int M, int N, int K,
                                                              int full_blocks, int tail_split, float* __restrict__ ws,
                                                              uint64_t* __restrict__ dbg = nullptr) {
    constexpr int BK = 32;
    using G = Cfg<BK>;                            // kImg 16 KiB, kStage 32 KiB
    constexpr int NW = 4;
    constexpr int NP = G::kImg / 1024 / NW;       // 4 pieces per wave per image
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 1, wn = wave & 1;

    const int tm = M / 256, tn = N / 256;
    int v, k_lo = 0, nk = K / 64, unit = -1;      // 64-deep tiles (the split plan's unit)
    if ((int)blockIdx.x < full_blocks) {
        v = xcd_remap(blockIdx.x, full_blocks);
    } else {
        unit = (int)blockIdx.x - full_blocks;
        v = full_blocks + unit / tail_split;
        nk /= tail_split;
        k_lo = (unit % tail_split) * nk;
    }
    const int ns = 2 * nk, s_lo = 2 * k_lo;      // 32-deep k-steps of this block
    const int group = kGroupM * tn;
    const int first_m = (v / group) * kGroupM;
    const int gm = min(tm - first_m, kGroupM);
    const int within = v % group;
    const int m0 = (first_m + within % gm) * 256, n0 = (within / gm) * 256;

    Dma16<NP, NW> da, db;
    da.init(wave, lane, lda);
    db.init(wave, lane, ldb);
    auto soff_a = [&](int u) { return __builtin_amdgcn_readfirstlane(((s_lo + min(u, ns - 1)) * BK * lda + m0) * 2); };
    auto soff_b = [&](int u) { return __builtin_amdgcn_readfirstlane(((s_lo + min(u, ns - 1)) * BK * ldb + n0) * 2); };
    auto stage_all = [&](int u, int slot) {
        da.load(A, a_bytes, soff_a(u), smem + slot * G::kStage, wave);
        db.load(B, b_bytes, soff_b(u), smem + slot * G::kStage + G::kImg, wave);
    };

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
                oa[h][i] = h * 2 * G::kStage + koff16(row, 128 * wm + 16 * i + cl);
                ob[h][i] = h * 2 * G::kStage + G::kImg + koff16(row, 128 * wn + 16 * i + cl);
            }
    }
    auto frag = [&](int off, int slot) -> bf16x8 {
        const char* p = smem + off + (slot & 1) * G::kStage;
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
    // one of the two transposing reads of fragment F (H = 0: k rows 0-15 half, 1: the +16 rows half), written into
    // that half of the fragment register in place
    auto half = [&](int off, int slot, int h) -> s16x4 {
        return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + off + (slot & 1) * G::kStage + h * 16 * 512));
    };
#define SA_RING_HALF(SLOT, FA, FB, F, H)                                                                        \
    {                                                                                                           \
        bf16x8& d_ = (F) < 8 ? FB[(F)] : FA[(F) - 8];                                                           \
        const s16x4 x_ = half((F) < 8 ? ob[(SLOT) >> 1][(F)] : oa[(SLOT) >> 1][(F) - 8], (SLOT), (H));          \
        s16x8 w_ = __builtin_bit_cast(s16x8, d_);                                                               \
        if ((H) == 0) w_ = __builtin_shufflevector(w_, __builtin_shufflevector(x_, x_, 0, 1, 2, 3, 0, 1, 2, 3), \
                                                   8, 9, 10, 11, 4, 5, 6, 7);                                   \
        else w_ = __builtin_shufflevector(w_, __builtin_shufflevector(x_, x_, 0, 1, 2, 3, 0, 1, 2, 3),          \
                                          0, 1, 2, 3, 8, 9, 10, 11);                                            \
        d_ = __builtin_bit_cast(bf16x8, w_);                                                                    \
    }
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    const i32x4 rsa = {(int)__builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uint64_t>(A)),
                       (int)(__builtin_amdgcn_readfirstlane((uint32_t)(reinterpret_cast<uint64_t>(A) >> 32)) & 0xffff),
                       (int)__builtin_amdgcn_readfirstlane(a_bytes), fa::kBufFlags};
    const i32x4 rsb = {(int)__builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uint64_t>(B)),
                       (int)(__builtin_amdgcn_readfirstlane((uint32_t)(reinterpret_cast<uint64_t>(B) >> 32)) & 0xffff),
                       (int)__builtin_amdgcn_readfirstlane(b_bytes), fa::kBufFlags};
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>((lds_void*)smem));
    // piece P (0..7: even = A piece P/2, odd = B piece P/2) of k-step U into slot SLOT
#define SA_RING_PIECE(P, SLOT, SA, SB, ST)                                                                       \
    {                                                                                                            \
        if constexpr (FASTDMA != 0) {                                                                            \
            const bool isb_ = ((P) & 1) != 0;                                                                    \
            const int i_ = (P) >> 1;                                                                             \
            const uint32_t l_ = lds0 + (SLOT) * G::kStage + (isb_ ? G::kImg : 0) + (wave + NW * i_) * 1024;    \
            if constexpr (FASTDMA == 1) {                                                                        \
                if (isb_)                                                                                        \
                    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"      \
                                 ::"s"(l_), "v"(db.voff), "s"(rsb), "s"((SB) + i_ * db.step) : "m0");           \
                else                                                                                             \
                    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"      \
                                 ::"s"(l_), "v"(da.voff), "s"(rsa), "s"((SA) + i_ * da.step) : "m0");           \
            } else {                                                                                             \
                int keep_;                                                                                       \
                asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"                              \
                             "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0"                     \
                             : "=&s"(keep_)                                                                      \
                             : "s"(l_), "v"(isb_ ? db.voff : da.voff), "s"(isb_ ? rsb : rsa),                   \
                               "s"(isb_ ? (SB) + i_ * db.step : (SA) + i_ * da.step));                          \
            }                                                                                                    \
        } else {                                                                                                 \
            if (((P) & 1) == 0) da.load_piece_nc((P) >> 1, A, a_bytes, (SA), (ST), wave);                      \
            else db.load_piece_nc((P) >> 1, B, b_bytes, (SB), (ST) + G::kImg, wave);                            \
        }                                                                                                        \
    }
    uint64_t* stamp = reinterpret_cast<uint64_t*>(smem + 4 * G::kStage);
#define SA_RING_STAMP(T, E)                                                                                      \
    if (TIMING && blockIdx.x == 0 && lane == 0 && (T) >= 32 && (T) < 40)                                         \
        stamp[(wave * 8 + ((T) - 32)) * 5 + (E)] = __builtin_amdgcn_s_memtime();
    // k-step T in slot SLOT with fragments (FA, FB); next fragments into (NA, NB)
#define SA_RING_STEP(SLOT, T, FA, FB, NA, NB)                                                                   \
    {                                                                                                           \
        SA_RING_STAMP(T, 0)                                                                                     \
        const int sa_ = soff_a((T) + 4), sb_ = soff_b((T) + 4);                                                 \
        char* st_ = smem + (SLOT) * G::kStage;                                                                  \
        _Pragma("unroll") for (int i = 0; i < 8; ++i)                                                           \
            _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                                     \
                mfma16_acc(acc[i][j], FB[j], FA[i]);                                                            \
                const int m_ = i * 8 + j;                                                                       \
                if (SCHED == 0) {                                                                               \
                    if (m_ % 3 == 2 && m_ < 48) SA_RING_READ(((SLOT) + 1) & 3, NA, NB, m_ / 3)                  \
                    if ((m_ & 7) == 7) SA_RING_PIECE(m_ >> 3, SLOT, sa_, sb_, st_)                              \
                } else if (SCHED == 1) {                                                                        \
                    if ((m_ & 1) == 1 && m_ < 32) SA_RING_READ(((SLOT) + 1) & 3, NA, NB, m_ >> 1)               \
                    if ((m_ & 3) == 3 && m_ >= 32) SA_RING_PIECE((m_ - 32) >> 2, SLOT, sa_, sb_, st_)           \
                } else if (SCHED == 3) {                                                                        \
                    if ((m_ & 1) == 1 && m_ < 32) SA_RING_READ(((SLOT) + 1) & 3, NA, NB, m_ >> 1)               \
                    if ((m_ & 1) == 1 && m_ >= 32 && m_ < 48) SA_RING_PIECE((m_ - 32) >> 1, SLOT, sa_, sb_, st_) \
                } else if (SCHED == 2) {                                                                        \
                    if ((m_ & 3) == 1) SA_RING_READ(((SLOT) + 1) & 3, NA, NB, m_ >> 2)                          \
                    if ((m_ & 7) == 3) SA_RING_PIECE(m_ >> 3, SLOT, sa_, sb_, st_)                              \
                } else {                                                                                        \
                    if ((m_ & 1) == 0) SA_RING_HALF(((SLOT) + 1) & 3, NA, NB, m_ >> 2, (m_ >> 1) & 1)           \
                    if ((m_ & 7) == 5) SA_RING_PIECE(m_ >> 3, SLOT, sa_, sb_, st_)                              \
                }                                                                                               \
            }                                                                                                   \
        SA_RING_STAMP(T, 1)                                                                                     \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                      \
        SA_RING_STAMP(T, 2)                                                                                     \
        wait_vm<4 * NP>();                                                                                      \
        SA_RING_STAMP(T, 3)                                                                                     \
        hard_barrier();                                                                                         \
        SA_RING_STAMP(T, 4)                                                                                     \
    }

    // prologue: k-steps 0-3 in flight (clamped: a short block re-stages its last k-step), 0 and 1 landed, F_0 read,
    // then a barrier so slot 0 may be restaged during k-step 0
    stage_all(0, 0);
    stage_all(1, 1);
    stage_all(2, 2);
    stage_all(3, 3);
    wait_vm<4 * NP>();
    hard_barrier();
#pragma unroll
    for (int f = 0; f < 16; ++f) SA_RING_READ(0, fa0, fb0, f)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    hard_barrier();
    int t = 0;
    for (; t + 3 < ns; t += 4) {
        SA_RING_STEP(0, t, fa0, fb0, fa1, fb1)
        SA_RING_STEP(1, t + 1, fa1, fb1, fa0, fb0)
        SA_RING_STEP(2, t + 2, fa0, fb0, fa1, fb1)
        SA_RING_STEP(3, t + 3, fa1, fb1, fa0, fb0)
    }
    // no remainder: the dispatcher gives this kernel whole pairs of 64-deep tiles per block (ns % 4 == 0)
#undef SA_RING_STEP
#undef SA_RING_READ
#undef SA_RING_HALF
#undef SA_RING_PIECE
#undef SA_RING_STAMP
    wait_vm<0>();
    if (TIMING && blockIdx.x == 0) {
        __syncthreads();
        for (int i = threadIdx.x; i < 4 * 8 * 5; i += blockDim.x) dbg[i] = stamp[i];
    }
    // the MFMAs are inline asm, invisible to the hazard recognizer: cover the MFMA -> VALU read of the accumulators
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

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
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        u16* crow_p = C + (int64_t)(m0 + 128 * wm + 16 * i + r) * ldc + n0 + 128 * wn + q4;
        u16x4 old[8];
        if (BETA) {
#pragma unroll
            for (int j = 0; j < 8; ++j) old[j] = *reinterpret_cast<const u16x4*>(crow_p + 16 * j);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
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
#define SA_RING_INST(BETA, SCHED, FD, TM)                                                                        \
    template __global__ void gemm_tn_ring_kernel<BETA, SCHED, FD, TM>(                                           \
        const u16* __restrict__, int, uint32_t, const u16* __restrict__, int, uint32_t, u16* __restrict__, int, int, \
        int, int, int, int, float* __restrict__, uint64_t* __restrict__);
#define SA_RING_INST2(SCHED, FD) SA_RING_INST(true, SCHED, FD, false) SA_RING_INST(false, SCHED, FD, false) \
    SA_RING_INST(false, SCHED, FD, true)
SA_RING_INST2(0, 0) SA_RING_INST2(1, 1) SA_RING_INST2(1, 2) SA_RING_INST2(3, 2) SA_RING_INST2(2, 1)
SA_RING_INST2(5, 1)
#undef SA_RING_INST2
#undef SA_RING_INST

// ---------------------------------------------------------------------------------------------------------------
// Forward / input-gradient GEMM  C[M, N] (+)= A[M, K] B[N, K]^T  with both operands k-contiguous (row-major A, and B
// stored [N][K]: a linear layer's weight for the forward, its cached transpose for dgrad) on the wgrad ring's
// structure: 256x256 macro tile, 4 waves x 128x128 (16x16x32 MFMAs, in-place AGPR accumulators), four-slot LDS ring of
// 32-deep k-steps filled by LDS-DMA, one barrier per k-step.  Here the operand rows are k-contiguous, so a fragment
// (row l & 15, k 8(l >> 4) .. +7) is ONE ds_read_b128 instead of two transposing reads.
//  * image per operand and slot: [256 rows][32 k] bf16, 64-B rows; the 16-B chunk c of row r sits at chunk
//    c ^ f(r), f = (-(r >> 2)) & 3, which makes every ds_read_b128 lane group of a fragment read hit 16 distinct
//    16-B bank windows (conflict-free);
//  * LDS-DMA piece = 16 rows x 64 B; the source is permuted so the lane-linear destination is the swizzled image;
//  * all fragment addresses are one per-lane VGPR per slot pair + a compile-time immediate.
__device__ __forceinline__ int nt_sw(int r) { return (-(r >> 2)) & 3; }

template <bool BETA, bool TIMING = false>
__global__ __launch_bounds__(256, 1) void gemm_nt_ring_kernel(const u16* __restrict__ A, int lda, uint32_t a_bytes,
                                                              const u16* __restrict__ B, int ldb, uint32_t b_bytes,
                                                              u16* __restrict__ C, int ldc, int M, int N, int K,
                                                              uint64_t* __restrict__ dbg = nullptr) {
    constexpr int BK = 32, IMG = 256 * BK * 2, STAGE = 2 * IMG;  // 16 KiB per image, 32 KiB per slot
    constexpr int NW = 4;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int tm = M / 256, tn = N / 256, nwg = tm * tn;
    const int v = xcd_remap(blockIdx.x, nwg);
    const int group = kGroupM * tn;
    const int first_m = (v / group) * kGroupM;
    const int gm = min(tm - first_m, kGroupM);
    const int within = v % group;
    const int m0 = (first_m + within % gm) * 256, n0 = (within / gm) * 256;
    const int ns = K / BK;

    // DMA: lane -> (row lane >> 2 of the piece, chunk slot lane & 3), source chunk = slot ^ f(row); piece i of this
    // wave covers rows 16 (wave + 4 i) .. +15 (f depends on row & 15 only: piece-invariant)
    const int prow = lane >> 2, pchunk = (lane & 3) ^ nt_sw(prow);
    const int va = ((16 * wave + prow) * lda + 8 * pchunk) * 2;
    const int vb = ((16 * wave + prow) * ldb + 8 * pchunk) * 2;
    const int stepa = __builtin_amdgcn_readfirstlane(64 * lda * 2), stepb = __builtin_amdgcn_readfirstlane(64 * ldb * 2);
    const int basea = __builtin_amdgcn_readfirstlane(m0 * lda * 2), baseb = __builtin_amdgcn_readfirstlane(n0 * ldb * 2);
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    const i32x4 rsa = {(int)__builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uint64_t>(A)),
                       (int)(__builtin_amdgcn_readfirstlane((uint32_t)(reinterpret_cast<uint64_t>(A) >> 32)) & 0xffff),
                       (int)__builtin_amdgcn_readfirstlane(a_bytes), fa::kBufFlags};
    const i32x4 rsb = {(int)__builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uint64_t>(B)),
                       (int)(__builtin_amdgcn_readfirstlane((uint32_t)(reinterpret_cast<uint64_t>(B) >> 32)) & 0xffff),
                       (int)__builtin_amdgcn_readfirstlane(b_bytes), fa::kBufFlags};
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>((lds_void*)smem));
    // piece P (even: A piece P/2, odd: B piece P/2) of k-step U into slot SLOT.  m0 is written in the statement that
    // reads it (the compiler emits no other m0 use in this kernel; its clobber is only a warning to hipcc).
#define SA_NT_PIECE(P, SLOT, U)                                                                                     \
    {                                                                                                               \
        const bool isb_ = ((P) & 1) != 0;                                                                           \
        const int i_ = (P) >> 1;                                                                                    \
        const uint32_t l_ = lds0 + (SLOT) * STAGE + (isb_ ? IMG : 0) + (wave + NW * i_) * 1024;                   \
        const int ku_ = min((U), ns - 1) * BK * 2;                                                                  \
        if (isb_)                                                                                                   \
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"                 \
                         ::"s"(l_), "v"(vb), "s"(rsb), "s"(baseb + i_ * stepb + ku_) : "m0");                     \
        else                                                                                                        \
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"                 \
                         ::"s"(l_), "v"(va), "s"(rsa), "s"(basea + i_ * stepa + ku_) : "m0");                     \
    }

    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // fragment addresses: per-lane part + (slot pair) + wave rows; fragment i / slot parity in the immediate
    int oa[2], ob[2];
    {
        const int r = lane & 15, g = lane >> 4;
        const int lo = r * 64 + 16 * (g ^ nt_sw(r));
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            oa[h] = h * 2 * STAGE + 128 * wm * 64 + lo;
            ob[h] = h * 2 * STAGE + IMG + 128 * wn * 64 + lo;
            // opaque: otherwise hipcc rebuilds the slot-pair-1 bases as base + 0x1xxxx with a v_add per read
            asm volatile("" : "+v"(oa[h]), "+v"(ob[h]));
        }
    }
    auto frag = [&](int base, int slot, int i) -> bf16x8 {
        return *reinterpret_cast<const bf16x8*>(smem + base + (slot & 1) * STAGE + i * 16 * 64);
    };
    bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
#define SA_NT_READ(SLOT, FA, FB, F)                                                 \
    {                                                                               \
        if ((F) < 8) FB[(F)] = frag(ob[(SLOT) >> 1], (SLOT), (F));                  \
        else FA[(F) - 8] = frag(oa[(SLOT) >> 1], (SLOT), (F) - 8);                  \
    }
    // k-step T in slot SLOT: MFMAs on (FA, FB), next fragments into (NA, NB) one per 4 MFMAs, k-step T+4's pieces
    // into slot SLOT one per 8 MFMAs; then every read of the next slot retired, k-step T+2 landed, barrier
    uint64_t* stamp = reinterpret_cast<uint64_t*>(smem + 4 * STAGE);
#define SA_NT_STAMP(T, E)                                                                                        \
    if (TIMING && blockIdx.x == 0 && lane == 0 && (T) >= 32 && (T) < 40)                                         \
        stamp[(wave * 8 + ((T) - 32)) * 5 + (E)] = __builtin_amdgcn_s_memtime();
#define SA_NT_STEP(SLOT, T, FA, FB, NA, NB)                                                                     \
    {                                                                                                           \
        SA_NT_STAMP(T, 0)                                                                                       \
        _Pragma("unroll") for (int i = 0; i < 8; ++i)                                                           \
            _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                                     \
                mfma16_acc(acc[i][j], FB[j], FA[i]);                                                            \
                const int m_ = i * 8 + j;                                                                       \
                if ((m_ & 3) == 1) SA_NT_READ(((SLOT) + 1) & 3, NA, NB, m_ >> 2)                                \
                if ((m_ & 7) == 3) SA_NT_PIECE(m_ >> 3, SLOT, (T) + 4)                                          \
            }                                                                                                   \
        SA_NT_STAMP(T, 1)                                                                                       \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                      \
        SA_NT_STAMP(T, 2)                                                                                       \
        wait_vm<16>();                                                                                          \
        SA_NT_STAMP(T, 3)                                                                                       \
        hard_barrier();                                                                                         \
        SA_NT_STAMP(T, 4)                                                                                       \
    }

    // prologue: k-steps 0-3 in flight, 0 and 1 landed, F_0 read, then a barrier (slot 0 is restaged in k-step 0)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int p = 0; p < 8; ++p) SA_NT_PIECE(p, u, u)
    wait_vm<16>();
    hard_barrier();
#pragma unroll
    for (int f = 0; f < 16; ++f) SA_NT_READ(0, fa0, fb0, f)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    hard_barrier();
    for (int t = 0; t < ns; t += 4) {  // ns % 4 == 0 (the dispatcher checks K % 128)
        SA_NT_STEP(0, t, fa0, fb0, fa1, fb1)
        SA_NT_STEP(1, t + 1, fa1, fb1, fa0, fb0)
        SA_NT_STEP(2, t + 2, fa0, fb0, fa1, fb1)
        SA_NT_STEP(3, t + 3, fa1, fb1, fa0, fb0)
    }
#undef SA_NT_STEP
#undef SA_NT_READ
#undef SA_NT_PIECE
#undef SA_NT_STAMP
    wait_vm<0>();
    if (TIMING && blockIdx.x == 0) {
        __syncthreads();
        for (int i = threadIdx.x; i < 4 * 8 * 5; i += blockDim.x) dbg[i] = stamp[i];
    }
    // the MFMAs are inline asm, invisible to the hazard recognizer: cover the MFMA -> VALU read of the accumulators
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

    // epilogue: acc[i][j][e] = C[m0 + 128wm + 16i + (lane & 15)][n0 + 128wn + 16j + 4(lane >> 4) + e]
    const int r = lane & 15, q4 = 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        u16* crow_p = C + (int64_t)(m0 + 128 * wm + 16 * i + r) * ldc + n0 + 128 * wn + q4;
        u16x4 old[8];
        if (BETA) {
#pragma unroll
            for (int j = 0; j < 8; ++j) old[j] = *reinterpret_cast<const u16x4*>(crow_p + 16 * j);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
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
template __global__ void gemm_nt_ring_kernel<true, false>(const u16* __restrict__, int, uint32_t, const u16* __restrict__,
                                                          int, uint32_t, u16* __restrict__, int, int, int, int,
                                                          uint64_t* __restrict__);
template __global__ void gemm_nt_ring_kernel<false, false>(const u16* __restrict__, int, uint32_t, const u16* __restrict__,
                                                           int, uint32_t, u16* __restrict__, int, int, int, int,
                                                           uint64_t* __restrict__);
template __global__ void gemm_nt_ring_kernel<false, true>(const u16* __restrict__, int, uint32_t, const u16* __restrict__,
                                                          int, uint32_t, u16* __restrict__, int, int, int, int,
                                                          uint64_t* __restrict__);

// explicit instantiations: hipcc otherwise silently drops the host stubs of some instances of this kernel
// template (the build's stub check catches that)
#define SA_GEMM_INST(BETA, BK, S, LW, TM)                                                                          \
    template __global__ void gemm_tn_kernel<BETA, BK, S, LW, TM>(const u16* __restrict__, int, uint32_t,            \
                                                                 const u16* __restrict__, int, uint32_t,            \
                                                                 u16* __restrict__, int, int, int, int,             \
                                                                 uint64_t* __restrict__, int, int, float* __restrict__);
#define SA_GEMM_INST2(BK, S, LW) SA_GEMM_INST(true, BK, S, LW, false) SA_GEMM_INST(false, BK, S, LW, false)
SA_GEMM_INST2(32, 4, false) SA_GEMM_INST2(32, 4, true) SA_GEMM_INST2(64, 2, true) SA_GEMM_INST2(32, 5, true)
SA_GEMM_INST2(64, 3, true)
SA_GEMM_INST(false, 32, 4, true, true) SA_GEMM_INST(false, 64, 2, true, true)
#undef SA_GEMM_INST2
#undef SA_GEMM_INST

// tail tile v (>= full_blocks): C[m0 + r][n0 + c] = (beta ? C : 0) + sum of its K-slice partials; block (tile, 4 rows)
__global__ __launch_bounds__(256) void gemm_tn_combine_kernel(const float* __restrict__ ws, u16* __restrict__ C, int ldc,
                                                              int M, int N, int full_blocks, int split, int beta) {
    const int tm = M / 256, tn = N / 256;
    const int v = full_blocks + (int)blockIdx.x;
    const int group = kGroupM * tn;
    const int first_m = (v / group) * kGroupM;
    const int gm = min(tm - first_m, kGroupM);
    const int within = v % group;
    const int m0 = (first_m + within % gm) * 256, n0 = (within / gm) * 256;
    const int row = 4 * (int)blockIdx.y + (threadIdx.x >> 6), col = (threadIdx.x & 63) * 4;
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

template <bool BETA>
void launch_tn_il(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int64_t N,
                  int64_t K, hipStream_t st, int full_blocks, int split, float* ws) {
    const int nwg = (int)((M / 256) * (N / 256));
    if (full_blocks < 0 || split <= 1) { full_blocks = nwg; split = 1; }
    const int grid = full_blocks + (nwg - full_blocks) * split;
    const uint32_t ab = (uint32_t)(K * lda * 2), bb = (uint32_t)(K * ldb * 2);
    hipLaunchKernelGGL((gemm_tn_il_kernel<BETA, false>), dim3(grid), dim3(512), 2 * Cfg<64>::kStage, st, (const u16*)A,
                       (int)lda, ab, (const u16*)B, (int)ldb, bb, (u16*)C, (int)ldc, (int)M, (int)N, (int)K, full_blocks,
                       split, ws, nullptr);
    if (split > 1)
        hipLaunchKernelGGL(gemm_tn_combine_kernel, dim3(nwg - full_blocks, 64), dim3(256), 0, st, (const float*)ws, (u16*)C,
                           (int)ldc, (int)M, (int)N, full_blocks, split, BETA ? 1 : 0);
}

template <bool BETA>
void launch_tn_w4(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int64_t N,
                  int64_t K, hipStream_t st, int full_blocks, int split, float* ws) {
    const int nwg = (int)((M / 256) * (N / 256));
    if (full_blocks < 0 || split <= 1) { full_blocks = nwg; split = 1; }
    const int grid = full_blocks + (nwg - full_blocks) * split;
    hipLaunchKernelGGL((gemm_tn_w4_kernel<BETA>), dim3(grid), dim3(256), 2 * Cfg<64>::kStage, st, (const u16*)A,
                       (int)lda, (const u16*)B, (int)ldb, (u16*)C, (int)ldc, (int)M, (int)N, (int)K, full_blocks, split,
                       ws);
    if (split > 1)
        hipLaunchKernelGGL(gemm_tn_combine_kernel, dim3(nwg - full_blocks, 64), dim3(256), 0, st, (const float*)ws, (u16*)C,
                           (int)ldc, (int)M, (int)N, full_blocks, split, BETA ? 1 : 0);
}

template <bool BETA>
void launch_tn_w4m16(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M,
                     int64_t N, int64_t K, hipStream_t st, int full_blocks, int split, float* ws) {
    const int nwg = (int)((M / 256) * (N / 256));
    if (full_blocks < 0 || split <= 1) { full_blocks = nwg; split = 1; }
    const int grid = full_blocks + (nwg - full_blocks) * split;
    const uint32_t ab = (uint32_t)(K * lda * 2), bb = (uint32_t)(K * ldb * 2);
    hipLaunchKernelGGL((gemm_tn_w4m16_kernel<BETA>), dim3(grid), dim3(256), 2 * Cfg<64>::kStage, st, (const u16*)A,
                       (int)lda, ab, (const u16*)B, (int)ldb, bb, (u16*)C, (int)ldc, (int)M, (int)N, (int)K, full_blocks,
                       split, ws);
    if (split > 1)
        hipLaunchKernelGGL(gemm_tn_combine_kernel, dim3(nwg - full_blocks, 64), dim3(256), 0, st, (const float*)ws, (u16*)C,
                           (int)ldc, (int)M, (int)N, full_blocks, split, BETA ? 1 : 0);
}

template <bool BETA, int SCHED, int FD>
void launch_tn_ring(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M,
                    int64_t N, int64_t K, hipStream_t st, int full_blocks, int split, float* ws) {
    const int nwg = (int)((M / 256) * (N / 256));
    if (full_blocks < 0 || split <= 1) { full_blocks = nwg; split = 1; }
    const int grid = full_blocks + (nwg - full_blocks) * split;
    const uint32_t ab = (uint32_t)(K * lda * 2), bb = (uint32_t)(K * ldb * 2);
    hipLaunchKernelGGL((gemm_tn_ring_kernel<BETA, SCHED, FD, false>), dim3(grid), dim3(256), 4 * Cfg<32>::kStage, st,
                       (const u16*)A, (int)lda, ab, (const u16*)B, (int)ldb, bb, (u16*)C, (int)ldc, (int)M, (int)N,
                       (int)K, full_blocks, split, ws, nullptr);
    if (split > 1)
        hipLaunchKernelGGL(gemm_tn_combine_kernel, dim3(nwg - full_blocks, 64), dim3(256), 0, st, (const float*)ws, (u16*)C,
                           (int)ldc, (int)M, (int)N, full_blocks, split, BETA ? 1 : 0);
}

template <bool BETA, int BK, int STAGES, bool LW>
void launch_tn(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int64_t N,
               int64_t K, hipStream_t st, int full_blocks = -1, int split = 1, float* ws = nullptr) {
    const int nwg = (int)((M / 256) * (N / 256));
    if (full_blocks < 0 || split <= 1) { full_blocks = nwg; split = 1; }
    const int grid = full_blocks + (nwg - full_blocks) * split;
    const uint32_t ab = (uint32_t)(K * lda * 2), bb = (uint32_t)(K * ldb * 2);
    const int lds = (BK == 64 && STAGES == 3) ? 5 * Cfg<BK>::kImg : STAGES * Cfg<BK>::kStage;
    hipLaunchKernelGGL((gemm_tn_kernel<BETA, BK, STAGES, LW>), dim3(grid), dim3(512), lds, st,
                       (const u16*)A, (int)lda, ab, (const u16*)B, (int)ldb, bb, (u16*)C, (int)ldc, (int)M, (int)N,
                       (int)K, nullptr, full_blocks, split, ws);
    if (split > 1)
        hipLaunchKernelGGL(gemm_tn_combine_kernel, dim3(nwg - full_blocks, 64), dim3(256), 0, st, (const float*)ws, (u16*)C,
                           (int)ldc, (int)M, (int)N, full_blocks, split, BETA ? 1 : 0);
}

}  // namespace sa_gemm
using namespace sa_gemm;

namespace sa_launch {
// pipeline variants (benchmarking hook): 13 (default) = four-slot ring, one wave per SIMD (gemm_tn_ring_kernel) with
// fragment reads and LDS-DMA pieces spread over the whole k-step; 9-12 / 14 = the ring with other schedules / LDS-DMA
// issue forms (profiles/gemm_ring_variants_r3*.log); 8 = one wave per SIMD on two 64-deep stages;
// 2 = BK 64 x 2 stages, split staging (one 32-MFMA block per
// phase); 5 = the same with three B buffers (B staged in group 1's read window); 0 = BK 32 x 4 stages, wait behind
// the MFMAs; 1 = same, wait before the first barrier; 3 = BK 32 x 5 stages; 4 = 16x16x32 MFMA form of 2;
// 6 = no ping-pong, reads interleaved with each wave's own MFMAs (gemm_tn_il_kernel); 7 = one wave per SIMD,
// 128x128 wave tiles, register-staged (gemm_tn_w4_kernel)
static int g_gemm_variant = 13;
void gemm_set_variant(int v) { g_gemm_variant = v; }
int gemm_get_variant() { return g_gemm_variant; }
// profiling hook: one launch of the timing build (variant 0 or 2), stamps of workgroup 0 to dbg (8 x 8 x 5 uint64)
void gemm_tn_timing(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int64_t N,
                    int64_t K, uint64_t* dbg, hipStream_t st) {
    const int nwg = (int)((M / 256) * (N / 256));
    const uint32_t ab = (uint32_t)(K * lda * 2), bb = (uint32_t)(K * ldb * 2);
    const int extra = kWaves * kDbgTiles * kDbgEv * 8;
#define SA_RING_T(SCHED, FD)                                                                                    \
    hipLaunchKernelGGL((gemm_tn_ring_kernel<false, SCHED, FD, true>), dim3(nwg), dim3(256), 4 * Cfg<32>::kStage + 4096, \
                       st, (const u16*)A, (int)lda, ab, (const u16*)B, (int)ldb, bb, (u16*)C, (int)ldc, (int)M, (int)N, \
                       (int)K, nwg, 1, nullptr, dbg);
    if (g_gemm_variant == 9) { SA_RING_T(0, 0) return; }
    if (g_gemm_variant == 10) { SA_RING_T(1, 1) return; }
    if (g_gemm_variant == 11) { SA_RING_T(1, 2) return; }
    if (g_gemm_variant == 12) { SA_RING_T(3, 2) return; }
    if (g_gemm_variant == 13) { SA_RING_T(2, 1) return; }
    if (g_gemm_variant == 14) { SA_RING_T(5, 1) return; }
#undef SA_RING_T
    if (g_gemm_variant == 6)
        hipLaunchKernelGGL((gemm_tn_il_kernel<false, true>), dim3(nwg), dim3(512), 2 * Cfg<64>::kStage + extra, st,
                           (const u16*)A, (int)lda, ab, (const u16*)B, (int)ldb, bb, (u16*)C, (int)ldc, (int)M, (int)N,
                           (int)K, nwg, 1, nullptr, dbg);
    else if (g_gemm_variant == 2)
        hipLaunchKernelGGL((gemm_tn_kernel<false, 64, 2, true, true>), dim3(nwg), dim3(512), 2 * Cfg<64>::kStage + extra,
                           st, (const u16*)A, (int)lda, ab, (const u16*)B, (int)ldb, bb, (u16*)C, (int)ldc, (int)M,
                           (int)N, (int)K, dbg, nwg, 1, nullptr);
    else
        hipLaunchKernelGGL((gemm_tn_kernel<false, 32, 4, true, true>), dim3(nwg), dim3(512), 4 * Cfg<32>::kStage + extra,
                           st, (const u16*)A, (int)lda, ab, (const u16*)B, (int)ldb, bb, (u16*)C, (int)ldc, (int)M,
                           (int)N, (int)K, dbg, nwg, 1, nullptr);
}
bool gemm_tn_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc) {
    return M % 256 == 0 && N % 256 == 0 && K % 64 == 0 && M > 0 && N > 0 && K > 0 && lda % 8 == 0 &&
           ldb % 8 == 0 && ldc % 4 == 0 && K * lda * 2 < (int64_t(1) << 31) && K * ldb * 2 < (int64_t(1) << 31) &&
           ldc < (1 << 30);
}
// Split plan for the ragged last round: with nwg tiles on `slots` workgroup slots (one 256x256 tile per CU), the
// r = nwg % slots tiles of the last round leave slots - r CUs idle; those tiles run as `split` K-slices each
// (2..4, >= 4 K-tiles per slice, chosen to minimise the tail's rounds x slice length) and a combine pass adds the
// fp32 partials into C.
// Variant 2 only.  Returns the fp32 workspace floats needed (0: no split).
int64_t gemm_tn_plan(int64_t M, int64_t N, int64_t K, int slots, int& full_blocks, int& split) {
    const int nwg = (int)((M / 256) * (N / 256));
    full_blocks = nwg;
    split = 1;
    if ((g_gemm_variant != 2 && g_gemm_variant != 5 && g_gemm_variant != 6 && g_gemm_variant != 7 &&
         g_gemm_variant != 8 && (g_gemm_variant < 9 || g_gemm_variant > 14)) ||
        slots <= 0)
        return 0;
    const int r = nwg % slots, nk = (int)(K / 64);
    if (r == 0) return 0;
    // the split tail costs ceil(r * s / slots) rounds of 1/s of a tile: pick the cheapest s (fewest on ties)
    int s = 1;
    double best = 1.0;
    const bool ring = g_gemm_variant >= 9 && g_gemm_variant <= 14;
    if (ring && nk % 2 != 0) return 0;  // the ring kernels run whole pairs of 64-deep tiles (gemm_tn falls back)
    for (int c = 2; c <= 4; ++c) {
        if (nk % c != 0 || nk / c < 4 || (ring && (nk / c) % 2 != 0)) continue;
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
    // the ring kernels (9-13) take whole pairs of 64-deep tiles per block only (K % 128): anything else runs variant 2
    int v = g_gemm_variant;
    if (v >= 9 && v <= 14 && (K / 64) % 2 != 0) v = 2;
    if (v == 2 && split > 1) {
        if (beta) launch_tn<true, 64, 2, true>(A, lda, B, ldb, C, ldc, M, N, K, st, full_blocks, split, ws);
        else launch_tn<false, 64, 2, true>(A, lda, B, ldb, C, ldc, M, N, K, st, full_blocks, split, ws);
        return;
    }
    if (v >= 9 && v <= 14) {
#define SA_RING(SCHED, FD)                                                                                 \
    if (beta) launch_tn_ring<true, SCHED, FD>(A, lda, B, ldb, C, ldc, M, N, K, st, full_blocks, split, ws); \
    else launch_tn_ring<false, SCHED, FD>(A, lda, B, ldb, C, ldc, M, N, K, st, full_blocks, split, ws);
        switch (v) {
            case 9: SA_RING(0, 0) break;
            case 10: SA_RING(1, 1) break;
            case 11: SA_RING(1, 2) break;
            case 12: SA_RING(3, 2) break;
            case 13: SA_RING(2, 1) break;
            default: SA_RING(5, 1) break;
        }
#undef SA_RING
        return;
    }
    if (v == 8) {
        if (beta) launch_tn_w4m16<true>(A, lda, B, ldb, C, ldc, M, N, K, st, full_blocks, split, ws);
        else launch_tn_w4m16<false>(A, lda, B, ldb, C, ldc, M, N, K, st, full_blocks, split, ws);
        return;
    }
    if (v == 7) {
        if (beta) launch_tn_w4<true>(A, lda, B, ldb, C, ldc, M, N, K, st, full_blocks, split, ws);
        else launch_tn_w4<false>(A, lda, B, ldb, C, ldc, M, N, K, st, full_blocks, split, ws);
        return;
    }
    if (v == 6) {
        if (beta) launch_tn_il<true>(A, lda, B, ldb, C, ldc, M, N, K, st, full_blocks, split, ws);
        else launch_tn_il<false>(A, lda, B, ldb, C, ldc, M, N, K, st, full_blocks, split, ws);
        return;
    }
    if (v == 5) {
        if (beta) launch_tn<true, 64, 3, true>(A, lda, B, ldb, C, ldc, M, N, K, st, full_blocks, split, ws);
        else launch_tn<false, 64, 3, true>(A, lda, B, ldb, C, ldc, M, N, K, st, full_blocks, split, ws);
        return;
    }
#define SA_TN(BK, S, LW)                                                                      \
    if (beta) launch_tn<true, BK, S, LW>(A, lda, B, ldb, C, ldc, M, N, K, st);                \
    else launch_tn<false, BK, S, LW>(A, lda, B, ldb, C, ldc, M, N, K, st);
    if (v == 4) {
        const int nwg = (int)((M / 256) * (N / 256));
        const uint32_t ab = (uint32_t)(K * lda * 2), bb = (uint32_t)(K * ldb * 2);
        if (beta)
            hipLaunchKernelGGL((gemm_tn16_kernel<true>), dim3(nwg), dim3(512), 2 * Cfg<64>::kStage, st, (const u16*)A,
                               (int)lda, ab, (const u16*)B, (int)ldb, bb, (u16*)C, (int)ldc, (int)M, (int)N, (int)K);
        else
            hipLaunchKernelGGL((gemm_tn16_kernel<false>), dim3(nwg), dim3(512), 2 * Cfg<64>::kStage, st, (const u16*)A,
                               (int)lda, ab, (const u16*)B, (int)ldb, bb, (u16*)C, (int)ldc, (int)M, (int)N, (int)K);
        return;
    }
    switch (v) {
        case 1: SA_TN(32, 4, false) break;
        case 2: SA_TN(64, 2, true) break;
        case 3: SA_TN(32, 5, true) break;
        default: SA_TN(32, 4, true) break;
    }
#undef SA_TN
}
bool gemm_nt_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc) {
    return M % 256 == 0 && N % 256 == 0 && K % 128 == 0 && M > 0 && N > 0 && K > 0 && lda % 8 == 0 && ldb % 8 == 0 &&
           ldc % 4 == 0 && M * lda * 2 < (int64_t(1) << 31) && N * ldb * 2 < (int64_t(1) << 31) &&
           (M / 256) * (N / 256) < (int64_t(1) << 31) && ldc < (1 << 30);
}
void gemm_nt(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int64_t N,
             int64_t K, bool beta, hipStream_t st, uint64_t* timing_dbg) {
    const int nwg = (int)((M / 256) * (N / 256));
    const uint32_t ab = (uint32_t)(M * lda * 2), bb = (uint32_t)(N * ldb * 2);
    if (timing_dbg)
        hipLaunchKernelGGL((gemm_nt_ring_kernel<false, true>), dim3(nwg), dim3(256), 128 * 1024 + 4096, st, (const u16*)A,
                           (int)lda, ab, (const u16*)B, (int)ldb, bb, (u16*)C, (int)ldc, (int)M, (int)N, (int)K, timing_dbg);
    else if (beta)
        hipLaunchKernelGGL((gemm_nt_ring_kernel<true, false>), dim3(nwg), dim3(256), 128 * 1024, st, (const u16*)A,
                           (int)lda, ab, (const u16*)B, (int)ldb, bb, (u16*)C, (int)ldc, (int)M, (int)N, (int)K, nullptr);
    else
        hipLaunchKernelGGL((gemm_nt_ring_kernel<false, false>), dim3(nwg), dim3(256), 128 * 1024, st, (const u16*)A,
                           (int)lda, ab, (const u16*)B, (int)ldb, bb, (u16*)C, (int)ldc, (int)M, (int)N, (int)K, nullptr);
}
}  // namespace sa_launch
