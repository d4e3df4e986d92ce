// Flash-attention forward, gfx950.  Workgroup = 4 waves x 32 query rows (BM = 128) of one
// (segment, q-head); K/V tiles of 64 keys double-buffered in LDS (register-staged: issue the next
// tile's global loads before the MFMA phase, write them to LDS after it — T14).  Per wave:
//   S^T = K Q^T   (query on the lane; 2 x 32x32 accumulators per 64 keys)
//   online softmax in base 2, lane-local row statistics (+1 exchange with lane^32)
//   O^T += V^T P^T (P^T accumulators reused as B operands; V^T via ds_read_b64_tr_b16)
// GQA is native (kv head = q head / group); varlen via cu_seqlens; causal (bottom-right aligned,
// flash-attn convention) and sliding window.

#include "flash_attn.h"
#include "launch.h"

using namespace sa;
using namespace sa::fa;

template <int D, bool F16, bool DROP>
__global__ __launch_bounds__(256, 2) void fa_fwd_kernel(FwdArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)  // the host pass only needs the signature for the launch stub
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int TILE = 64 * D * 2;  // bytes per K or V tile
    // buffer b: K at smem + 2*b*TILE, V at smem + (2*b+1)*TILE

    const int seg = blockIdx.z, hq = blockIdx.y;
    const int q0s = a.cu_q[seg], k0s = a.cu_k[seg];
    const int Lq = a.cu_q[seg + 1] - q0s, Lk = a.cu_k[seg + 1] - k0s;
    const int ntiles_q = (Lq + 127) / 128;
    const int qt = a.causal ? (int)gridDim.x - 1 - (int)blockIdx.x : (int)blockIdx.x;
    if (qt >= ntiles_q) return;
    const int hk = hq / (a.Hq / a.Hkv);
    const int win = hq < a.local_heads ? a.window : -1;  // per-head window (mixed local/global heads)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, lq = lane & 31;
    const int off = Lk - Lq;  // bottom-right causal alignment
    const int qwg0 = qt * 128;
    const int qw0 = qwg0 + wave * 32;
    const int myq = qw0 + lq;

    // key range for the workgroup
    const int qlast = min(qwg0 + 127, Lq - 1);
    int khi = Lk;
    if (a.causal) khi = min(Lk, qlast + off + 1);
    else if (win >= 0) khi = min(Lk, qlast + off + win + 1);
    int klo = 0;
    if (win >= 0) klo = max(0, qwg0 + off - win);
    klo = (klo / 64) * 64;

    // Q fragments (B operand of S^T = K Q^T): lane holds Q[myq][16 ks + 8h .. +7]
    bf16x8 qf[D / 16];
    {
        const u16* qp = a.q + (int64_t)(q0s + min(myq, Lq - 1)) * a.q_tok + (int64_t)hq * a.q_head;
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) {
            u16x8 v = *reinterpret_cast<const u16x8*>(qp + 16 * ks + 8 * h);
            qf[ks] = __builtin_bit_cast(bf16x8, v);
        }
    }
    f32x16 o[D / 32];
#pragma unroll
    for (int t = 0; t < D / 32; ++t) o[t] = f32x16{};
    float m = -INFINITY, lsum = 0.f;
    uint32_t drow = 0;
    if constexpr (DROP) drow = drop_row(drop_head(a.seed, hq), q0s + myq);

    const u16* kbase = a.k + (int64_t)k0s * a.k_tok + (int64_t)hk * a.k_head;
    const u16* vbase = a.v + (int64_t)k0s * a.v_tok + (int64_t)hk * a.v_head;
    Stage<D> sk, sv;
    int cur = 0;
    if (klo < khi) {
        sk.load(kbase + (int64_t)klo * a.k_tok, a.k_tok, min(64, Lk - klo));
        sv.load(vbase + (int64_t)klo * a.v_tok, a.v_tok, min(64, Lk - klo));
        sk.store(smem);
        sv.store(smem + TILE);
    }
    __syncthreads();
    for (int kt = klo; kt < khi; kt += 64) {
        const bool has_next = kt + 64 < khi;
        if (has_next) {
            sk.load(kbase + (int64_t)(kt + 64) * a.k_tok, a.k_tok, min(64, Lk - kt - 64));
            sv.load(vbase + (int64_t)(kt + 64) * a.v_tok, a.v_tok, min(64, Lk - kt - 64));
        }
        const char* K = smem + 2 * cur * TILE;
        const char* V = K + TILE;
        // ---- S^T = K Q^T
        f32x16 s[2] = {f32x16{}, f32x16{}};
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) {
#pragma unroll
            for (int b = 0; b < 2; ++b) s[b] = mma<F16>(ld_row<D>(K, 32 * b + lq, 16 * ks + 8 * h), qf[ks], s[b]);
        }
        // ---- scale + mask (mask only on boundary tiles; wave-uniform decision)
        const bool need_mask = (kt + 64 > Lk) || (a.causal && kt + 63 > qw0 + off) ||
                               (win >= 0 && (kt < qw0 + 31 + off - win || (!a.causal && kt + 63 > qw0 + off + win)));
        float mloc = -INFINITY;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float x = s[b][r] * a.scale_log2;
                if (need_mask) {
                    const int key = kt + 32 * b + (r & 3) + 8 * (r >> 2) + 4 * h;
                    bool ok = key < Lk && myq < Lq;
                    if (a.causal) ok = ok && key <= myq + off;
                    if (win >= 0) ok = ok && key >= myq + off - win && (a.causal || key <= myq + off + win);
                    x = ok ? x : -INFINITY;
                }
                s[b][r] = x;
                mloc = fmaxf(mloc, x);
            }
        }
        mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
        const float mnew = fmaxf(m, mloc);
        const float msafe = mnew == -INFINITY ? 0.f : mnew;
        const float alpha = fast_exp2(m - msafe);
        float rs = 0.f;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float p = fast_exp2(s[b][r] - msafe);
                s[b][r] = p;
                rs += p;
            }
        rs += __shfl_xor(rs, 32, 64);
        lsum = lsum * alpha + rs;
        m = mnew;
        if constexpr (DROP) {  // normaliser uses every p; only the P.V product sees the dropped ones
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (!drop_keep(drow, k0s + kt + 32 * b + 4 * h + crow(r), a.drop_thr)) s[b][r] = 0.f;
        }
#pragma unroll
        for (int t = 0; t < D / 32; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
        // ---- O^T += V^T P^T
        bf16x8 pf[2][2];
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) pf[b][ss] = pack_acc_t<F16>(s[b], ss);
#pragma unroll
        for (int t = 0; t < D / 32; ++t)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) o[t] = mma<F16>(ld_tr<D>(V, 32 * b + 16 * ss, 32 * t), pf[b][ss], o[t]);
        if (has_next) {
            sk.store(smem + 2 * (cur ^ 1) * TILE);
            sv.store(smem + (2 * (cur ^ 1) + 1) * TILE);
        }
        __syncthreads();
        cur ^= 1;
    }
    // ---- epilogue: O = O^T / l, lse = (m + log2 l) * ln2
    if (myq < Lq) {
        const float inv = (lsum > 0.f ? 1.f / lsum : 0.f) * (DROP ? a.rp_drop : 1.f);
        u16* op = a.o + (int64_t)(q0s + myq) * a.o_tok + (int64_t)hq * a.o_head;
#pragma unroll
        for (int t = 0; t < D / 32; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                u16x4 w;
#pragma unroll
                for (int j = 0; j < 4; ++j) w[j] = f2t<F16>(o[t][4 * g + j] * inv);
                *reinterpret_cast<u16x4*>(op + 32 * t + 8 * g + 4 * h) = w;
            }
        if (h == 0) a.lse[(int64_t)hq * a.lse_stride + q0s + myq] = lsum > 0.f ? (m + __log2f(lsum)) * 0.69314718055994530942f : INFINITY;
    }
#endif
}


// ---------------------------------------------------------------------------------------------
// v2 (D = 64, 128): 4 waves x 32 query rows (BM = 128) share each K/V tile; two independent 256-thread workgroups
// per CU (their phases drift apart, so one workgroup's softmax overlaps the other's MFMAs on a SIMD).  VALU per MFMA
// is the limiter of the v1 loop (rocprof: 10.9 VALU/MFMA), so:
//  * every LDS address is a per-lane register computed once (swizzle folded in) + a compile-time
//    immediate: the K/V loop is unrolled x2 so both buffer bases are constants;
//  * row max on raw scores with v_max3 (no canonicalising max), scale folded into one FMA;
//  * lazy rescale: the running max only moves when a row max exceeds it by > 8 (log2 units), and
//    the O / l rescale is skipped by a wave-uniform test otherwise (P <= 2^8 stays exact in fp32,
//    representable in bf16);
//  * lane^32 exchanges through v_permlane32_swap;
//  * masking only on boundary tiles, as 1-2 compares against per-lane bounds.
template <int D, int NW_ = 4>
struct FwdV2 {
    static constexpr int NW = NW_, BM = 32 * NW, KT = 64, TILE = KT * D * 2, NKS = D / 16, NT = D / 32;
    static constexpr float TH = 8.f;
};

// Variants measured against this one and dropped (8 waves per workgroup, inline-asm LDS-DMA, pinned read-ahead, an
// 8-wave ping-pong schedule): profiles/attn_fwd_waves_ab_r2.log, attn_fwd_pingpong_ab_r3.log, attn_ab_r2_asyncdma.log;
// their code is in git history before commit "Delete losing attention variants".  128-key tiles (8 waves x 32 queries,
// 128 KiB of LDS, one workgroup per CU, causal tiles past a wave's queries skipped): 1.28 vs 1.13 ms at the 7B shape,
// profiles/attn_fwd_kt128_ab_r6.log (code in git history, commit "Drop the race-forensics build switches").
// K / V staged through registers (buffer loads issued before a tile's MFMAs, ds_write after them, T14) instead of
// LDS-DMA: 1.22-1.26 vs 1.13-1.16 ms, profiles/attn_fwd_regstage_ab_r6.log.
// Half 1's exponentials scheduled into the gaps of half 0's P.V MFMAs (sched_group_barrier, bit-identical): 1.19-1.21
// vs 1.17 ms, profiles/attn_fwd_pipe_ab_r6.log -- the loop is issue-bound at two waves per SIMD, not latency-bound.
// NW = 4: 2 workgroups / CU = 2 waves / SIMD; NW = 6 (BM = 192): 2 workgroups / CU = 3 waves / SIMD (<= 168 VGPRs)
#ifndef SA_FWD_NW
#define SA_FWD_NW 4
#endif
template <int D, bool F16, bool DROP, int NW>
__global__ __launch_bounds__(64 * NW, NW / 2) void fa_fwd_v2_kernel(FwdArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)  // the host pass only needs the signature for the launch stub
    using C = FwdV2<D, NW>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // grid (Hq, nseg, q tiles): the dispatcher walks x fastest, so the tile index is the slowest
    // dimension and causal work is issued heaviest-first across all heads (LPT balance)
    const int seg = attn_seg(), hq = xcd_head(blockIdx.x, a.Hq);  // see attn_grid
    const int q0s = a.cu_q[seg], k0s = a.cu_k[seg];
    const int Lq = a.cu_q[seg + 1] - q0s, Lk = a.cu_k[seg + 1] - k0s;
    const int ntiles_q = (Lq + C::BM - 1) / C::BM;
    const int qt = attn_qtile(a.causal);
    if (qt >= ntiles_q) return;
    const int hk = hq / (a.Hq / a.Hkv);
    const int win = hq < a.local_heads ? a.window : -1;  // per-head window (mixed local/global heads)
    // wave index through readfirstlane: everything derived from it (qw0, the mask test) is provably
    // wave-uniform, so the boundary-tile mask is a real branch instead of per-element selects
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5,
              lq = lane & 31;
    const int off = Lk - Lq;
    const int qwg0 = qt * C::BM, qw0 = qwg0 + 32 * wave, myq = qw0 + lq;
    const int qlast = min(qwg0 + C::BM - 1, Lq - 1);
    int khi = Lk;
    if (a.causal) khi = min(Lk, qlast + off + 1);
    else if (win >= 0) khi = min(Lk, qlast + off + win + 1);
    int klo = 0;
    if (win >= 0) klo = max(0, qwg0 + off - win);
    klo = (klo / C::KT) * C::KT;

    // ---- per-lane LDS offsets (bytes, relative to a tile base) ----
    // per-lane LDS offsets: K row fragments (row lq, cols 16ks + 8h) and V^T fragments (rows 4h + i/4 (+8), cols
    // 32t + 16g + 4(i&3)) as 6 registers + per-use XORs (a 16-register table spilled at 3 waves / SIMD)
    LdsOffsets<D> lo;
    lo.init(lane);
    // K / V tiles by LDS-DMA (no staging registers); rows past the segment land as zeros
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    DmaTile<D, C::NW> tk, tv;
    tk.init(wave_u, lane, a.k_tok);
    tv.init(wave_u, lane, a.v_tok);
    const u16* kbase = a.k + (int64_t)k0s * a.k_tok + (int64_t)hk * a.k_head;
    const u16* vbase = a.v + (int64_t)k0s * a.v_tok + (int64_t)hk * a.v_head;
#define SA_FWD_ISSUE(KT, BUFP)                                                                          \
    do {                                                                                                \
        const int kp_ = (KT);                                                                           \
        dma_load(tk, kbase + (int64_t)kp_ * a.k_tok, a.k_tok, Lk - kp_, (BUFP), wave_u);                    \
        dma_load(tv, vbase + (int64_t)kp_ * a.v_tok, a.v_tok, Lk - kp_, (BUFP) + C::TILE, wave_u);          \
    } while (0)

    bf16x8 qf[C::NKS];
    {
        const u16* qp = a.q + (int64_t)(q0s + min(myq, Lq - 1)) * a.q_tok + (int64_t)hq * a.q_head;
#pragma unroll
        for (int ks = 0; ks < C::NKS; ++ks)
            qf[ks] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u16x8*>(qp + 16 * ks + 8 * h));
        // consume Q here: hipcc then retires its loads before the loop instead of inside it, where its vmcnt would
        // also wait for the asm LDS-DMA in flight
#pragma unroll
        for (int ks = 0; ks < C::NKS; ++ks) asm volatile("" ::"v"(qf[ks]));
    }
    f32x16 o[C::NT];
#pragma unroll
    for (int t = 0; t < C::NT; ++t) o[t] = f32x16{};
    float m = -INFINITY, l = 0.f;
    const float c2 = a.scale_log2;
    uint32_t drow = 0;
    if constexpr (DROP) drow = drop_row(drop_head(a.seed, hq), q0s + myq);

    auto tile = [&](const char* K, int kt) {
        const char* V = K + C::TILE;
        f32x16 s[2] = {f32x16{}, f32x16{}};
        {
#pragma unroll
            for (int ks = 0; ks < C::NKS; ++ks)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    s[b] = mma<F16>(*reinterpret_cast<const bf16x8*>(K + 32 * b * D * 2 + lo.row(ks)), qf[ks], s[b]);
            // one K fragment read per MFMA.  Reading them 4 MFMAs ahead (or interleaving the softmax of the previous
            // tile into these MFMAs) was measured slower: at two waves per SIMD the loop is bound by the SIMD's issue
            // slots, not by LDS latency (profiles/attn_sched_ab_r4.log)
#pragma unroll
            for (int i = 0; i < 2 * C::NKS; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
            }
        }
        // wave-uniform: does any element of this wave's 32 x 64 block need a mask?
        const bool need_mask = (kt + C::KT > Lk) || (a.causal && kt + C::KT - 1 > qw0 + off) ||
                               (win >= 0 && (kt < qw0 + 31 + off - win ||
                                                  (!a.causal && kt + C::KT - 1 > qw0 + off + win)));
        if (need_mask) {
            mask_fence();
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const int base = kt + 32 * b + 4 * h;  // key of register j = base + crow(j)
                int hi = Lk - 1 - base;
                if (a.causal) hi = min(hi, myq + off - base);
                else if (win >= 0) hi = min(hi, myq + off + win - base);
                const int lo = win >= 0 ? myq + off - win - base : -1;
#pragma unroll
                for (int j = 0; j < 16; ++j) s[b][j] = (crow(j) <= hi && crow(j) >= lo) ? s[b][j] : -INFINITY;
            }
        }
        // two independent 16-element chains, one statement each (no hazard pads inside)
        const float m0 = vmax16(s[0]), m1 = vmax16(s[1]);
        const float mx = vmax3(m0, m1, m1);
        const float mrow = max_xchg32(mx) * c2;
        if (__builtin_amdgcn_ballot_w64(mrow > m + C::TH) != 0) {  // rare after the first tiles
            mask_fence();
            const float mnew = fmaxf(m, mrow);
            const float alpha = mnew == -INFINITY ? 1.f : fast_exp2(m - mnew);
            l *= alpha;
#pragma unroll
            for (int t = 0; t < C::NT; ++t)
#pragma unroll
                for (int j = 0; j < 16; ++j) o[t][j] *= alpha;
            m = mnew;
        }
        const float nm = m == -INFINITY ? 0.f : -m;
        float rs[4] = {0.f, 0.f, 0.f, 0.f};  // four independent add chains instead of one 32-deep one
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const float p = fast_exp2(__builtin_fmaf(s[b][j], c2, nm));
                s[b][j] = p;
                rs[j & 3] += p;
            }
        // (the row sum as a fifth P.V product against all-ones was measured slower: profiles/attn_rowsum_mfma_ab_r4.log)
        l += sum_xchg32((rs[0] + rs[1]) + (rs[2] + rs[3]));
        if constexpr (DROP) {  // normaliser uses every p; only the P.V product sees the dropped ones
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    if (!drop_keep(drow, k0s + kt + 32 * b + 4 * h + crow(j), a.drop_thr)) s[b][j] = 0.f;
        }
        bf16x8 pf[2][2];
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) pf[b][ss] = pack_acc_t<F16>(s[b], ss);
        {
#pragma unroll
            for (int t = 0; t < C::NT; ++t)
#pragma unroll
                for (int b = 0; b < 2; ++b)
#pragma unroll
                    for (int ss = 0; ss < 2; ++ss) {
                        const int kb = (32 * b + 16 * ss) * D * 2;
                        const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(V + kb + lo.tr(t, 0)));
                        const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(V + kb + lo.tr(t, 1)));
                        o[t] = mma<F16>(__builtin_bit_cast(bf16x8, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7)), pf[b][ss], o[t]);
                    }
#pragma unroll
            for (int i = 0; i < 4 * C::NT; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);  // 2 x ds_read_b64_tr_b16
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);  // MFMA
            }
        }
    };

    char* buf0 = smem;
    char* buf1 = smem + 2 * C::TILE;
    if (klo < khi) SA_FWD_ISSUE(klo, buf0);
    dma_barrier();
    // pairs of tiles (buffer 0 then 1) so every LDS address is register + immediate; odd tail peeled
    const int ntiles = khi > klo ? (khi - klo + C::KT - 1) / C::KT : 0;
    int kt = klo;
    for (int pr = 0; pr < ntiles / 2; ++pr, kt += 2 * C::KT) {
        SA_FWD_ISSUE(kt + C::KT, buf1);
        tile(buf0, kt);
        dma_barrier();  // every wave's pieces of tile kt + KT landed (see dma_barrier)
        if (kt + 2 * C::KT < khi) SA_FWD_ISSUE(kt + 2 * C::KT, buf0);
        tile(buf1, kt + C::KT);
        dma_barrier();
    }
    if (ntiles & 1) tile(buf0, kt);
#undef SA_FWD_ISSUE
    if (myq < Lq) {
        const float inv = (l > 0.f ? 1.f / l : 0.f) * (DROP ? a.rp_drop : 1.f);
        u16* op = a.o + (int64_t)(q0s + myq) * a.o_tok + (int64_t)hq * a.o_head;
#pragma unroll
        for (int t = 0; t < C::NT; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                u16x4 w;
#pragma unroll
                for (int j = 0; j < 4; ++j) w[j] = f2t<F16>(o[t][4 * g + j] * inv);
                *reinterpret_cast<u16x4*>(op + 32 * t + 8 * g + 4 * h) = w;
            }
        if (h == 0)
            a.lse[(int64_t)hq * a.lse_stride + q0s + myq] = l > 0.f ? (m + __log2f(l)) * 0.69314718055994530942f : INFINITY;
    }
#endif
}

template <bool F16, bool DROP>
static void launch_fwd(const FwdArgs& a, int D, int max_q, hipStream_t st) {
    if (D == 128 || D == 64) {
        constexpr int NW = SA_FWD_NW;
        constexpr int BM = FwdV2<128, NW>::BM;
        dim3 grid = attn_grid(a.Hq, a.nseg, (max_q + BM - 1) / BM), block(64 * NW);
        if (D == 128) hipLaunchKernelGGL((fa_fwd_v2_kernel<128, F16, DROP, NW>), grid, block, (4 * FwdV2<128, NW>::TILE), st, a);
        else hipLaunchKernelGGL((fa_fwd_v2_kernel<64, F16, DROP, NW>), grid, block, (4 * FwdV2<64, NW>::TILE), st, a);
        return;
    }
    dim3 grid((max_q + 127) / 128, a.Hq, a.nseg), block(256);
    hipLaunchKernelGGL((fa_fwd_kernel<32, F16, DROP>), grid, block, 4 * 64 * 32 * 2, st, a);
}

namespace sa_launch {
void fa_fwd(const FwdArgs& a, int D, int max_q, bool f16, hipStream_t st) {
    const bool drop = a.p_drop > 0.f;
    if (f16) {
        if (drop) launch_fwd<true, true>(a, D, max_q, st);
        else launch_fwd<true, false>(a, D, max_q, st);
    } else {
        if (drop) launch_fwd<false, true>(a, D, max_q, st);
        else launch_fwd<false, false>(a, D, max_q, st);
    }
}
}  // namespace sa_launch
