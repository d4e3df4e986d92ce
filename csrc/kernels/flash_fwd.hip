// Flash-attention forward, gfx950.  Workgroup = 4 waves x 32 query rows (BM = 128) of one
// (segment, q-head); K/V tiles of 64 keys double-buffered in LDS (register-staged: issue the next
// tile's global loads before the MFMA phase, write them to LDS after it — T14).  Per wave:
//   S^T = K Q^T   (query on the lane; 2 x 32x32 accumulators per 64 keys)
//   online softmax in base 2, lane-local row statistics (+1 exchange with lane^32)
//   O^T += V^T P^T (P^T accumulators reused as B operands; V^T via ds_read_b64_tr_b16)
// GQA is native (kv head = q head / group); varlen via cu_seqlens; causal (bottom-right aligned,
// flash-attn convention) and sliding window.
#include <cstdlib>
#include <type_traits>

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
// their code is in git history before commit "Delete losing attention variants".
template <int D, bool F16, bool DROP>
__global__ __launch_bounds__(256, 2) void fa_fwd_v2_kernel(FwdArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)  // the host pass only needs the signature for the launch stub
    using C = FwdV2<D>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // grid (Hq, nseg, q tiles): the dispatcher walks x fastest, so the tile index is the slowest
    // dimension and causal work is issued heaviest-first across all heads (LPT balance)
    const int seg = blockIdx.y, hq = blockIdx.x;
    const int q0s = a.cu_q[seg], k0s = a.cu_k[seg];
    const int Lq = a.cu_q[seg + 1] - q0s, Lk = a.cu_k[seg + 1] - k0s;
    const int ntiles_q = (Lq + C::BM - 1) / C::BM;
    const int qt = a.causal ? (int)gridDim.z - 1 - (int)blockIdx.z : (int)blockIdx.z;
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
    int rowoff[C::NKS];  // K row fragment: row lq, cols 16ks + 8h
#pragma unroll
    for (int ks = 0; ks < C::NKS; ++ks) rowoff[ks] = lds_off<D>(lq, 16 * ks + 8 * h);
    int troff[C::NT][2];  // V^T fragment (ld_tr): rows 4h + i/4 (+8), cols 32t + 16g + 4(i&3)
    {
        const int g = (lane >> 4) & 1, i = lane & 15;
#pragma unroll
        for (int t = 0; t < C::NT; ++t) {
            troff[t][0] = lds_off<D>(4 * h + (i >> 2), 32 * t + 16 * g + 4 * (i & 3));
            troff[t][1] = lds_off<D>(4 * h + (i >> 2) + 8, 32 * t + 16 * g + 4 * (i & 3));
        }
    }
    // K / V tiles by LDS-DMA (no staging registers); rows past the segment land as zeros
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    DmaTile<D, C::NW> tk, tv;
    tk.init(wave_u, lane, a.k_tok);
    tv.init(wave_u, lane, a.v_tok);
    const u16* kbase = a.k + (int64_t)k0s * a.k_tok + (int64_t)hk * a.k_head;
    const u16* vbase = a.v + (int64_t)k0s * a.v_tok + (int64_t)hk * a.v_head;
#define SA_FWD_ISSUE(KT, BUFP)                                                                          \
    do {                                                                                                \
        dma_load(tk, kbase + (int64_t)(KT) * a.k_tok, a.k_tok, Lk - (KT), (BUFP), wave_u);                   \
        dma_load(tv, vbase + (int64_t)(KT) * a.v_tok, a.v_tok, Lk - (KT), (BUFP) + C::TILE, wave_u);         \
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
                    s[b] = mma<F16>(*reinterpret_cast<const bf16x8*>(K + 32 * b * D * 2 + rowoff[ks]), qf[ks], s[b]);
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
                        const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(V + kb + troff[t][0]));
                        const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(V + kb + troff[t][1]));
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

// ---------------------------------------------------------------------------------------------
// v3 (D = 128, no dropout, no window): ONE wave per SIMD, two independent 32-row query blocks per wave.
// Workgroup = 4 waves x 64 query rows (BM = 256) of one (segment, q head), one workgroup per CU (512 registers per
// lane).  With a single wave on its SIMD, the only VALU that can hide under an MFMA stream is the wave's own, so the
// two query blocks A (rows 0-31 of the wave) and B (rows 32-63) are software-pipelined against each other: per 64-key
// tile j the wave issues four 16-MFMA phases, each carrying the other block's softmax work as fillers:
//   1. S_A(j)   = K_j Q_A^T        || second half of block B's softmax of tile j-1 (exp, row sum, bf16 pack)
//   2. O_B     += V_{j-1}^T P_B    || block A's row max / lazy-rescale decision / first half of its exps
//   3. S_B(j)   = K_j Q_B^T        || second half of block A's softmax of tile j
//   4. O_A     += V_j^T P_A        || block B's row max / rescale decision / first half of its exps
// (the cdna_hip_programming.md Appendix B "4-wave, one-wave-per-SIMD" structure).  Phase 2 still reads V_{j-1}, so
// K/V tiles rotate over a 3-slot LDS ring (96 KiB): the DMA of tile j+1 is issued into the slot of tile j-2 right after
// the per-tile barrier, a whole tile ahead of its use.  The loop is unrolled x3 so every LDS address is a per-lane
// register + a compile-time immediate.  The O rescale of the lazy online softmax (running max moves only when a row
// max exceeds it by > 8 in log2 units) is decided in the block's max phase and applied as a wave-uniform branch right
// before its next P.V phase, after every P.V of the older tiles (the T13 ordering).  Tiles that need a mask (the causal
// diagonal, a ragged last key tile) run a serial, unpipelined per-block step; tiles past a wave's last row are skipped
// by that wave (it still joins the barrier and its share of the DMA).
struct FwdV3 {
    static constexpr int D = 128, NW = 4, BM = 64 * NW, KT = 64, TILE = KT * D * 2, NKS = D / 16, NT = D / 32;
    static constexpr int SLOT = 2 * TILE, QOFF = 3 * SLOT, LDS = QOFF + BM * D * 2;  // 96 KiB ring + 64 KiB Q
    static constexpr float TH = 8.f;
};

template <bool F16>
__global__ __launch_bounds__(256, 1) void fa_fwd_v3_kernel(FwdArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
    using C = FwdV3;
    constexpr int D = C::D;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int seg = blockIdx.y, hq = blockIdx.x;
    const int q0s = a.cu_q[seg], k0s = a.cu_k[seg];
    const int Lq = a.cu_q[seg + 1] - q0s, Lk = a.cu_k[seg + 1] - k0s;
    const int ntiles_q = (Lq + C::BM - 1) / C::BM;
    const int qt = a.causal ? (int)gridDim.z - 1 - (int)blockIdx.z : (int)blockIdx.z;
    if (qt >= ntiles_q) return;
    const int hk = hq / (a.Hq / a.Hkv);
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5,
              lq = lane & 31;
    const int off = Lk - Lq;
    const int qwg0 = qt * C::BM, qw0 = qwg0 + 64 * wave;
    const int qlast = min(qwg0 + C::BM - 1, Lq - 1);
    const int khi = a.causal ? min(Lk, qlast + off + 1) : Lk;  // workgroup key range [0, khi)
    // this wave's key range (its rows qw0 .. qw0 + 63); a wave with no valid row computes nothing
    const int khw = qw0 >= Lq ? 0 : (a.causal ? min(Lk, min(qw0 + 63, Lq - 1) + off + 1) : Lk);
    // tiles [0, kclean) need no mask for either block: every key < Lk and (causal) <= the wave's first row + off
    const int kclean = a.causal ? min(Lk, qw0 + off + 1) : Lk;

    int rowoff[C::NKS];  // K row fragment: row lq, cols 16 ks + 8 h
#pragma unroll
    for (int ks = 0; ks < C::NKS; ++ks) rowoff[ks] = lds_off<D>(lq, 16 * ks + 8 * h);
    int troff[C::NT][2];  // V^T fragment (ds_read_b64_tr_b16): rows 4h + i/4 (+8), cols 32t + 16g + 4(i&3)
    {
        const int g = (lane >> 4) & 1, i = lane & 15;
#pragma unroll
        for (int t = 0; t < C::NT; ++t) {
            troff[t][0] = lds_off<D>(4 * h + (i >> 2), 32 * t + 16 * g + 4 * (i & 3));
            troff[t][1] = lds_off<D>(4 * h + (i >> 2) + 8, 32 * t + 16 * g + 4 * (i & 3));
        }
    }
    DmaTile<D, C::NW> tk, tv;
    tk.init(wave, lane, a.k_tok);
    tv.init(wave, lane, a.v_tok);
    const u16* kbase = a.k + (int64_t)k0s * a.k_tok + (int64_t)hk * a.k_head;
    const u16* vbase = a.v + (int64_t)k0s * a.v_tok + (int64_t)hk * a.v_head;
    const uint32_t lds0 = lds_addr(smem);

    // Q of the whole workgroup (256 rows) lives in LDS after the K/V ring (64 KiB; 160 KiB in all): in registers the two
    // blocks' fragments would take 64 VGPRs that the softmax of two blocks needs.  Row qwg0 + r sits at image row r, so
    // a fragment read is the K-row read offset (same swizzle: it depends on r & 15 only) + this wave's row base.
    {
        DmaTile<D, C::NW, C::BM> tq;
        tq.init(wave, lane, a.q_tok);
        dma_load_asm(tq, a.q + (int64_t)(q0s + qwg0) * a.q_tok + (int64_t)hq * a.q_head, a.q_tok, Lq - qwg0,
                     lds0 + C::QOFF, wave);
    }
    int qoff[C::NKS];
#pragma unroll
    for (int ks = 0; ks < C::NKS; ++ks) qoff[ks] = rowoff[ks] + 64 * wave * D * 2;
    const float c2 = a.scale_log2;

    // ---- per-block state
    f32x16 oA[C::NT], oB[C::NT], sA[2], sB[2];
#pragma unroll
    for (int t = 0; t < C::NT; ++t) { oA[t] = f32x16{}; oB[t] = f32x16{}; }
    float mA = -INFINITY, mB = -INFINITY, lA = 0.f, lB = 0.f, alA = 1.f, alB = 1.f;
    bool needA = false, needB = false;  // wave-uniform: O rescale pending before the block's next P.V
    bf16x8 pA[2][2], pB[2][2];
    float rsA[4], rsB[4];

    auto qk = [&](f32x16 (&s)[2], int qblk, const char* K) __attribute__((always_inline)) {
        const char* Q = smem + C::QOFF + 32 * qblk * D * 2;
        s[0] = f32x16{};
        s[1] = f32x16{};
#pragma unroll
        for (int ks = 0; ks < C::NKS; ++ks) {
            const bf16x8 qf = *reinterpret_cast<const bf16x8*>(Q + qoff[ks]);
#pragma unroll
            for (int b = 0; b < 2; ++b)
                s[b] = mma<F16>(*reinterpret_cast<const bf16x8*>(K + 32 * b * D * 2 + rowoff[ks]), qf, s[b]);
        }
    };
    // O += V^T P: inline-asm MFMAs with the accumulators pinned in AGPRs ("+a"): O never has to leave the accumulator
    // file, which keeps the arch VGPRs for S, Q, P and the fragments (with compiler MFMAs the allocator shuffles 2 x 64
    // O registers through v_accvgpr copies and spills).  The asm is invisible to the hazard recognizer: P is written by
    // VALU (v_cvt_pk) and read as SrcB, which needs 2 wait states, so the first MFMA of every P register carries
    // s_nop 1 -- "first" in program order, which asm volatile pins (non-volatile asm MFMAs of different accumulators
    // were reordered so that a t > 0 MFMA read a fresh P without the pad: rare wrong outputs); readers of O (rescale,
    // epilogue) sit behind o_fence.
    auto pv = [&](f32x16 (&o)[C::NT], const bf16x8 (&p)[2][2], const char* V) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < C::NT; ++t)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    const int kb = (32 * b + 16 * ss) * D * 2;
                    const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(V + kb + troff[t][0]));
                    const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(V + kb + troff[t][1]));
                    const bf16x8 vf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
                    if (t == 0) {
                        if constexpr (F16) asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(o[t]) : "v"(vf), "v"(p[b][ss]));
                        else asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(o[t]) : "v"(vf), "v"(p[b][ss]));
                    } else {
                        if constexpr (F16) asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(o[t]) : "v"(vf), "v"(p[b][ss]));
                        else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(o[t]) : "v"(vf), "v"(p[b][ss]));
                    }
                }
    };
    // MFMA -> VALU / v_accvgpr_read of the accumulators needs up to 18 wait states (16-pass MFMA); the asm takes every O
    // register as an operand, so no read of O can be scheduled above it and no MFMA writing O below it
    auto o_fence = [&](f32x16 (&o)[C::NT]) __attribute__((always_inline)) {
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" : "+a"(o[0]), "+a"(o[1]), "+a"(o[2]), "+a"(o[3]));
    };
    // row max + lazy-rescale decision (applied to O before the block's next P.V, to l now)
    auto smax = [&](f32x16 (&s)[2], float& m, float& l, float& al, bool& need) __attribute__((always_inline)) {
        const float m0 = vmax16(s[0]), m1 = vmax16(s[1]);
        const float mrow = max_xchg32(vmax3(m0, m1, m1)) * c2;
        const bool up = __builtin_amdgcn_ballot_w64(mrow > m + C::TH) != 0;
        const float mnew = up ? fmaxf(m, mrow) : m;
        al = (!up || mnew == -INFINITY) ? 1.f : fast_exp2(m - mnew);
        l *= al;
        m = mnew;
        need = up;  // never pending twice: the block's rescale runs before its next max phase
    };
    // exps of elements [lo, lo + 16) of the 32 this lane holds (s[lo/16]), row sum into rs
    auto sexp = [&](f32x16 (&s)[2], float m, float (&rs)[4], int half) __attribute__((always_inline)) {
        const float nm = m == -INFINITY ? 0.f : -m;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const float p = fast_exp2(__builtin_fmaf(s[half][j], c2, nm));
            s[half][j] = p;
            if (half == 0) rs[j & 3] = (j < 4) ? p : rs[j & 3] + p;
            else rs[j & 3] += p;
        }
    };
    auto sfin = [&](f32x16 (&s)[2], float& l, float (&rs)[4], bf16x8 (&p)[2][2]) __attribute__((always_inline)) {
        l += sum_xchg32((rs[0] + rs[1]) + (rs[2] + rs[3]));
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) p[b][ss] = pack_acc_t<F16>(s[b], ss);
    };
    auto rescale = [&](f32x16 (&o)[C::NT], float al) __attribute__((always_inline)) {
        mask_fence();
        o_fence(o);
#pragma unroll
        for (int t = 0; t < C::NT; ++t)
#pragma unroll
            for (int j = 0; j < 16; ++j) o[t][j] *= al;
        // v_accvgpr_write -> MFMA SrcC: covered by the same kind of fence before the next P.V
        o_fence(o);
    };
    // serial step of one block over a tile that needs a mask (row r0 + lq)
    auto masked = [&](f32x16 (&s)[2], f32x16 (&o)[C::NT], int qblk, float& m, float& l,
                      bf16x8 (&p)[2][2], const char* K, int kt, int r0) __attribute__((always_inline)) {
        qk(s, qblk, K);
        mask_fence();
        const int myq = r0 + lq;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int base = kt + 32 * b + 4 * h;
            int hi = Lk - 1 - base;
            if (a.causal) hi = min(hi, myq + off - base);
#pragma unroll
            for (int j = 0; j < 16; ++j) s[b][j] = crow(j) <= hi ? s[b][j] : -INFINITY;
        }
        float al;
        bool need = false;
        smax(s, m, l, al, need);
        if (need) rescale(o, al);
        float rs[4];
        sexp(s, m, rs, 0);
        sexp(s, m, rs, 1);
        sfin(s, l, rs, p);
        pv(o, p, K + C::TILE);
    };

    bool pend = false;  // block B's softmax tail + P.V of the previous tile still to run (wave-uniform)
    // finish block B's pending tile with V in `Vp` (out of the pipeline: masked / skipped tile or the end)
    auto drainB = [&](const char* Vp) __attribute__((always_inline)) {
        sexp(sB, mB, rsB, 1);
        sfin(sB, lB, rsB, pB);
        if (needB) { rescale(oB, alB); needB = false; }
        pv(oB, pB, Vp);
        pend = false;
    };

    const int ntiles = (khi + C::KT - 1) / C::KT;
    // K/V tile t into ring slot `cs` (asm LDS-DMA: waited for by the s_waitcnt vmcnt(0) in front of the next tile's
    // barrier, a whole tile later)
    auto issue = [&](int t, int cs) __attribute__((always_inline)) {
        const int kt = t * C::KT;
        dma_load_asm(tk, kbase + (int64_t)kt * a.k_tok, a.k_tok, Lk - kt, lds0 + cs * C::SLOT, wave);
        dma_load_asm(tv, vbase + (int64_t)kt * a.v_tok, a.v_tok, Lk - kt, lds0 + cs * C::SLOT + C::TILE, wave);
    };
    auto tile_barrier = [&]() __attribute__((always_inline)) { dma_barrier(); };
    if (ntiles > 0) issue(0, 0);

    // one pipelined tile (no mask for either block).  PEND: block B's tile t-1 is still in flight (the steady state);
    // a compile-time flag, so no branch splits a phase's MFMAs from the filler work scheduled beside them
    auto pipe = [&](auto pendc, const char* K, const char* Vprev) __attribute__((always_inline)) {
        constexpr bool PEND = decltype(pendc)::value;
        // phase 1: S_A(t) || block B of tile t-1: second half of the exps, row sum, bf16 pack
        qk(sA, 0, K);
        if constexpr (PEND) {
            sexp(sB, mB, rsB, 1);
            sfin(sB, lB, rsB, pB);
            if (needB) { rescale(oB, alB); needB = false; }
            // phase 2: O_B += V(t-1) P_B || block A: row max, rescale decision, first half of the exps
            pv(oB, pB, Vprev);
        }
        smax(sA, mA, lA, alA, needA);
        sexp(sA, mA, rsA, 0);
        // phase 3: S_B(t) || block A: second half
        qk(sB, 1, K);
        sexp(sA, mA, rsA, 1);
        sfin(sA, lA, rsA, pA);
        if (needA) { rescale(oA, alA); needA = false; }
        // phase 4: O_A += V(t) P_A || block B: row max, rescale decision, first half of the exps
        pv(oA, pA, K + C::TILE);
        smax(sB, mB, lB, alB, needB);
        sexp(sB, mB, rsB, 0);
        // keep block B's first-half exps in this phase: without a use here hipcc sinks them below the next tile's
        // barrier into phase 1, which then carries twice its share of VALU beside the same 16 MFMAs
        asm volatile("" : "+v"(sB[0]), "+v"(rsB[0]), "+v"(rsB[1]), "+v"(rsB[2]), "+v"(rsB[3]));
        pend = true;
    };

    // main part: tiles [0, nmain) need no mask for ANY wave (causal: every key <= the workgroup's first row + off), so
    // every wave runs the same straight-line pipelined code (a control-flow join in the loop would make the register
    // allocator shuffle the 128 O accumulators between AGPR homes).  Slots rotate 0, 1, 2: loop unrolled x3.
    const int nmain = max(0, min(a.causal ? (qwg0 + off + 1) / C::KT : ntiles, Lk / C::KT));
    auto head = [&](auto cslot, int t) __attribute__((always_inline)) {
        constexpr int CS = decltype(cslot)::value;
        tile_barrier();  // tile t landed (every wave waited for its own pieces); slot of tile t-2 is free
        if (t + 1 < ntiles) issue(t + 1, (CS + 1) % 3);
    };
    auto mtile = [&](auto cslot, auto pendc, int t) __attribute__((always_inline)) {
        constexpr int CS = decltype(cslot)::value;
        head(cslot, t);
        pipe(pendc, smem + CS * C::SLOT, smem + ((CS + 2) % 3) * C::SLOT + C::TILE);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    int t = 0;
    if (nmain > 0) {
        mtile(I0{}, std::false_type{}, 0);
        t = 1;
        for (; t + 3 <= nmain; t += 3) {
            mtile(I1{}, std::true_type{}, t);
            mtile(I2{}, std::true_type{}, t + 1);
            mtile(I0{}, std::true_type{}, t + 2);
        }
        if (t < nmain) { mtile(I1{}, std::true_type{}, t); ++t; }
        if (t < nmain) { mtile(I2{}, std::true_type{}, t); ++t; }
        drainB(smem + ((nmain - 1) % 3) * C::SLOT + C::TILE);
    }
    // tail: the causal diagonal block / a ragged last key tile, per wave: skip the tiles past its last row, run the
    // others as serial masked steps (runtime slot addresses: a few tiles per workgroup)
    for (; t < ntiles; ++t) {
        const int cs = t % 3;
        tile_barrier();
        if (t + 1 < ntiles) issue(t + 1, (cs + 1) % 3);
        const int kt = t * C::KT;
        if (kt < khw) {
            const char* K = smem + cs * C::SLOT;
            masked(sA, oA, 0, mA, lA, pA, K, kt, qw0);
            masked(sB, oB, 1, mB, lB, pB, K, kt, qw0 + 32);
        }
    }

    // ---- epilogue: O = O^T / l, lse = (m + log2 l) * ln2
    auto store = [&](const f32x16 (&o)[C::NT], float m, float l, int myq) __attribute__((always_inline)) {
        if (myq >= Lq) return;
        const float inv = l > 0.f ? 1.f / l : 0.f;
        u16* op = a.o + (int64_t)(q0s + myq) * a.o_tok + (int64_t)hq * a.o_head;
#pragma unroll
        for (int t2 = 0; t2 < C::NT; ++t2)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                u16x4 w;
#pragma unroll
                for (int j = 0; j < 4; ++j) w[j] = f2t<F16>(o[t2][4 * g + j] * inv);
                *reinterpret_cast<u16x4*>(op + 32 * t2 + 8 * g + 4 * h) = w;
            }
        if (h == 0)
            a.lse[(int64_t)hq * a.lse_stride + q0s + myq] = l > 0.f ? (m + __log2f(l)) * 0.69314718055994530942f : INFINITY;
    };
    o_fence(oA);
    o_fence(oB);
    store(oA, mA, lA, qw0 + lq);
    store(oB, mB, lB, qw0 + 32 + lq);
#endif
}

// v3 only with SCALING_AMD_FA_FWD_V3=1 (measured slower than v2 so far); read once
static bool fwd_v3_enabled() {
    static const int on = [] {
        const char* e = getenv("SCALING_AMD_FA_FWD_V3");
        return e == nullptr ? 0 : atoi(e);
    }();
    return on != 0;
}

template <bool F16, bool DROP>
static void launch_fwd(const FwdArgs& a, int D, int max_q, hipStream_t st) {
    if (D == 128 && !DROP && a.window < 0 && max_q >= 512 && fwd_v3_enabled()) {
        dim3 grid(a.Hq, a.nseg, (max_q + FwdV3::BM - 1) / FwdV3::BM), block(256);
        hipLaunchKernelGGL((fa_fwd_v3_kernel<F16>), grid, block, FwdV3::LDS, st, a);
        return;
    }
    if (D == 128 || D == 64) {
        dim3 grid(a.Hq, a.nseg, (max_q + FwdV2<128>::BM - 1) / FwdV2<128>::BM), block(256);
        if (D == 128) hipLaunchKernelGGL((fa_fwd_v2_kernel<128, F16, DROP>), grid, block, 4 * FwdV2<128>::TILE, st, a);
        else hipLaunchKernelGGL((fa_fwd_v2_kernel<64, F16, DROP>), grid, block, 4 * FwdV2<64>::TILE, st, a);
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
