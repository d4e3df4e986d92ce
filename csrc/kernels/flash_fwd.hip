// Flash-attention forward, gfx950.  Workgroup = 4 waves x 32 query rows (BM = 128) of one
// (segment, q-head); K/V tiles of 64 keys double-buffered in LDS (register-staged: issue the next
// tile's global loads before the MFMA phase, write them to LDS after it — T14).  Per wave:
//   S^T = K Q^T   (query on the lane; 2 x 32x32 accumulators per 64 keys)
//   online softmax in base 2, lane-local row statistics (+1 exchange with lane^32)
//   O^T += V^T P^T (P^T accumulators reused as B operands; V^T via ds_read_b64_tr_b16)
// GQA is native (kv head = q head / group); varlen via cu_seqlens; causal (bottom-right aligned,
// flash-attn convention) and sliding window.
#include <cstdlib>

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
// v2 (D = 64, 128): 8 waves x 32 query rows (BM = 256) share each K/V tile; one workgroup per CU,
// two waves per SIMD.  VALU per MFMA is the limiter of the v1 loop (rocprof: 10.9 VALU/MFMA), so:
//  * every LDS address is a per-lane register computed once (swizzle folded in) + a compile-time
//    immediate: the K/V loop is unrolled x2 so both buffer bases are constants;
//  * row max on raw scores with v_max3 (no canonicalising max), scale folded into one FMA;
//  * lazy rescale: the running max only moves when a row max exceeds it by > 8 (log2 units), and
//    the O / l rescale is skipped by a wave-uniform test otherwise (P <= 2^8 stays exact in fp32,
//    representable in bf16);
//  * lane^32 exchanges through v_permlane32_swap;
//  * masking only on boundary tiles, as 1-2 compares against per-lane bounds.
template <int D, int NW_ = 8>
struct FwdV2 {
    static constexpr int NW = NW_, BM = 32 * NW, KT = 64, TILE = KT * D * 2, NKS = D / 16, NT = D / 32;
    static constexpr float TH = 8.f;
};

// NW = 8: one 512-thread workgroup per CU; NW = 4: two independent 256-thread workgroups per CU (their phases
// drift apart, so one workgroup's softmax can overlap the other's MFMAs on a SIMD)
// ADMA: the per-tile LDS-DMA as inline asm retired by an explicit vmcnt(0) before the barrier (with compiler-visible
// LDS-DMA hipcc waits for the NEXT tile's DMA in front of this tile's transposed V reads)
// RA: explicit LDS read-ahead (K fragments RA_K MFMAs ahead in S = K Q^T, V^T fragments RA_V ahead in O += V^T P^T),
// pinned by sched barriers: hipcc otherwise sinks every read right in front of the MFMA that consumes it
template <int D, bool F16, bool DROP, int NW = 8, bool ADMA = false, bool RA = false>
__global__ __launch_bounds__(64 * NW, 8 / NW) void fa_fwd_v2_kernel(FwdArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)  // the host pass only needs the signature for the launch stub
    using C = FwdV2<D, NW>;
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
        if constexpr (ADMA) {                                                                           \
            dma_tile_asm(tk, kbase + (int64_t)(KT) * a.k_tok, a.k_tok, Lk - (KT), (BUFP), wave_u);           \
            dma_tile_asm(tv, vbase + (int64_t)(KT) * a.v_tok, a.v_tok, Lk - (KT), (BUFP) + C::TILE, wave_u); \
        } else {                                                                                        \
            dma_load(tk, kbase + (int64_t)(KT) * a.k_tok, a.k_tok, Lk - (KT), (BUFP), wave_u);               \
            dma_load(tv, vbase + (int64_t)(KT) * a.v_tok, a.v_tok, Lk - (KT), (BUFP) + C::TILE, wave_u);     \
        }                                                                                               \
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
        if constexpr (RA) {
            constexpr int NF = 2 * C::NKS, PK = 4;  // fragment f = (ks = f / 2, b = f % 2)
            bf16x8 kb[PK];
#pragma unroll
            for (int f = 0; f < PK; ++f) kb[f] = *reinterpret_cast<const bf16x8*>(K + 32 * (f & 1) * D * 2 + rowoff[f >> 1]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                s[f & 1] = mma<F16>(kb[f % PK], qf[f >> 1], s[f & 1]);
                if (f + PK < NF) {
                    const int g = f + PK;
                    kb[f % PK] = *reinterpret_cast<const bf16x8*>(K + 32 * (g & 1) * D * 2 + rowoff[g >> 1]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
#pragma unroll
            for (int ks = 0; ks < C::NKS; ++ks)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    s[b] = mma<F16>(*reinterpret_cast<const bf16x8*>(K + 32 * b * D * 2 + rowoff[ks]), qf[ks], s[b]);
            // keep the K fragment reads one or two MFMAs ahead instead of hoisting all of them
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
        float mx = vmax3(s[0][0], s[0][1], s[0][2]);
#pragma unroll
        for (int j = 3; j < 15; j += 2) mx = vmax3(mx, s[0][j], s[0][j + 1]);
        mx = vmax3(mx, s[0][15], s[1][0]);
#pragma unroll
        for (int j = 1; j < 15; j += 2) mx = vmax3(mx, s[1][j], s[1][j + 1]);
        mx = vmax3(mx, s[1][15], s[1][15]);
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
        float rs = 0.f;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const float p = fast_exp2(__builtin_fmaf(s[b][j], c2, nm));
                s[b][j] = p;
                rs += p;
            }
        l += sum_xchg32(rs);
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
        if constexpr (RA) {
            // step i = (t, b, ss) in the original order; V^T fragments PV steps ahead
            constexpr int NS = 4 * C::NT, PV = 3;
            auto vfrag = [&](int i) -> bf16x8 {
                const int t = i / 4, b = (i / 2) & 1, ss = i & 1;
                const int kb = (32 * b + 16 * ss) * D * 2;
                const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(V + kb + troff[t][0]));
                const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(V + kb + troff[t][1]));
                return __builtin_bit_cast(bf16x8, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7));
            };
            bf16x8 vb[PV];
#pragma unroll
            for (int i = 0; i < PV; ++i) vb[i] = vfrag(i);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                const int t = i / 4, b = (i / 2) & 1, ss = i & 1;
                o[t] = mma<F16>(vb[i % PV], pf[b][ss], o[t]);
                if (i + PV < NS) vb[i % PV] = vfrag(i + PV);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
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
    if constexpr (ADMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // pairs of tiles (buffer 0 then 1) so every LDS address is register + immediate; odd tail peeled
    const int ntiles = khi > klo ? (khi - klo + C::KT - 1) / C::KT : 0;
    int kt = klo;
    for (int pr = 0; pr < ntiles / 2; ++pr, kt += 2 * C::KT) {
        SA_FWD_ISSUE(kt + C::KT, buf1);
        tile(buf0, kt);
        if constexpr (ADMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (kt + 2 * C::KT < khi) SA_FWD_ISSUE(kt + 2 * C::KT, buf0);
        tile(buf1, kt + C::KT);
        if constexpr (ADMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
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
// Ping-pong forward (D = 128, no dropout): 8 waves x 32 query rows (BM = 256), two groups of four (waves 0-3 = A,
// 4-7 = B; wave w and w + 4 share a SIMD).  Per key tile j a wave runs two phases:
//   X(j): O += V_{j-1}^T P_{j-1} and S_j = K_j Q^T  (32 MFMAs, LDS reads only)
//   Y(j): online softmax of S_j -> P_j, lazy O / l rescale (VALU only)
// and the groups are one phase apart (A: X Y X Y ..., B: Y X Y X ...), one barrier per phase, so on every SIMD one
// wave's MFMAs run beside its partner's softmax instead of both waves doing the same kind of work at once (the v2
// kernel's barrier per tile keeps the partners in lockstep: MFMA util 0.49 at VALU/MFMA 6.3).
// K / V tiles by LDS-DMA: K_j and V_{j-1} are issued in phase 2j-2 and retired at the end of phase 2j-1 (two
// buffers each; K_j is read in phases 2j (A) and 2j+1 (B), V_{j-1} in the same phases).
template <int D, bool F16>
__global__ __launch_bounds__(512, 1) void fa_fwd_pp_kernel(FwdArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
    using C = FwdV2<D, 8>;
    extern __shared__ __attribute__((aligned(16))) char smem[];  // K0 K1 V0 V1
    const int seg = blockIdx.y, hq = blockIdx.x;
    const int q0s = a.cu_q[seg], k0s = a.cu_k[seg];
    const int Lq = a.cu_q[seg + 1] - q0s, Lk = a.cu_k[seg + 1] - k0s;
    const int ntiles_q = (Lq + C::BM - 1) / C::BM;
    const int qt = a.causal ? (int)gridDim.z - 1 - (int)blockIdx.z : (int)blockIdx.z;
    if (qt >= ntiles_q) return;
    const int hk = hq / (a.Hq / a.Hkv);
    const int win = hq < a.local_heads ? a.window : -1;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5,
              lq = lane & 31;
    const int grp = wave >> 2;
    const int off = Lk - Lq;
    const int qwg0 = qt * C::BM, qw0 = qwg0 + 32 * wave, myq = qw0 + lq;
    const int qlast = min(qwg0 + C::BM - 1, Lq - 1);
    int khi = Lk;
    if (a.causal) khi = min(Lk, qlast + off + 1);
    else if (win >= 0) khi = min(Lk, qlast + off + win + 1);
    int klo = 0;
    if (win >= 0) klo = max(0, qwg0 + off - win);
    klo = (klo / C::KT) * C::KT;
    const int ntiles = khi > klo ? (khi - klo + C::KT - 1) / C::KT : 0;

    int rowoff[C::NKS];
#pragma unroll
    for (int ks = 0; ks < C::NKS; ++ks) rowoff[ks] = lds_off<D>(lq, 16 * ks + 8 * h);
    int troff[C::NT][2];
    {
        const int g = (lane >> 4) & 1, i = lane & 15;
#pragma unroll
        for (int t = 0; t < C::NT; ++t) {
            troff[t][0] = lds_off<D>(4 * h + (i >> 2), 32 * t + 16 * g + 4 * (i & 3));
            troff[t][1] = lds_off<D>(4 * h + (i >> 2) + 8, 32 * t + 16 * g + 4 * (i & 3));
        }
    }
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    DmaTile<D, 8> tk, tv;
    tk.init(wave_u, lane, a.k_tok);
    tv.init(wave_u, lane, a.v_tok);
    const u16* kbase = a.k + (int64_t)k0s * a.k_tok + (int64_t)hk * a.k_head;
    const u16* vbase = a.v + (int64_t)k0s * a.v_tok + (int64_t)hk * a.v_head;
    char* kbuf0 = smem;
    char* vbuf0 = smem + 2 * C::TILE;

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
    f32x16 s[2] = {f32x16{}, f32x16{}};
    bf16x8 pf[2][2];
    float m = -INFINITY, l = 0.f;
    const float c2 = a.scale_log2;

    // X(j) part 1: O += V^T P with P = pf (tile j-1), V image at V
    auto pv = [&](const char* V) {
#pragma unroll
        for (int t = 0; t < C::NT; ++t)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    const int kb = (32 * b + 16 * ss) * D * 2;
                    const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(V + kb + troff[t][0]));
                    const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(V + kb + troff[t][1]));
                    o[t] = mma<F16>(__builtin_bit_cast(bf16x8, __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7)),
                                    pf[b][ss], o[t]);
                }
#pragma unroll
        for (int i = 0; i < 4 * C::NT; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
        }
    };
    // X(j) part 2: S = K Q^T, K image at K; the first NPRE K fragments were read ahead (kpre, during the
    // preceding softmax phase) so the MFMAs start without waiting for LDS
    constexpr int NPRE = 4;
    bf16x8 kpre[NPRE];
    auto prefetch_k = [&](const char* K) {
#pragma unroll
        for (int f = 0; f < NPRE; ++f)
            kpre[f] = *reinterpret_cast<const bf16x8*>(K + 32 * (f & 1) * D * 2 + rowoff[f >> 1]);
    };
    auto qk = [&](const char* K) {
        s[0] = f32x16{};
        s[1] = f32x16{};
#pragma unroll
        for (int ks = 0; ks < C::NKS; ++ks)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const int f = 2 * ks + b;
                const bf16x8 kf = f < NPRE ? kpre[f < NPRE ? f : 0]
                                           : *reinterpret_cast<const bf16x8*>(K + 32 * b * D * 2 + rowoff[ks]);
                s[b] = mma<F16>(kf, qf[ks], s[b]);
            }
#pragma unroll
        for (int i = 0; i < 2 * C::NKS - NPRE; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 2);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 2);
        }
    };
    // Y(j): softmax of s (keys kt ..) -> pf
    auto softmax = [&](int kt) {
        const bool need_mask = (kt + C::KT > Lk) || (a.causal && kt + C::KT - 1 > qw0 + off) ||
                               (win >= 0 && (kt < qw0 + 31 + off - win ||
                                                  (!a.causal && kt + C::KT - 1 > qw0 + off + win)));
        if (need_mask) {
            mask_fence();
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const int base = kt + 32 * b + 4 * h;
                int hi = Lk - 1 - base;
                if (a.causal) hi = min(hi, myq + off - base);
                else if (win >= 0) hi = min(hi, myq + off + win - base);
                const int lo = win >= 0 ? myq + off - win - base : -1;
#pragma unroll
                for (int j = 0; j < 16; ++j) s[b][j] = (crow(j) <= hi && crow(j) >= lo) ? s[b][j] : -INFINITY;
            }
        }
        float mx = vmax3(s[0][0], s[0][1], s[0][2]);
#pragma unroll
        for (int j = 3; j < 15; j += 2) mx = vmax3(mx, s[0][j], s[0][j + 1]);
        mx = vmax3(mx, s[0][15], s[1][0]);
#pragma unroll
        for (int j = 1; j < 15; j += 2) mx = vmax3(mx, s[1][j], s[1][j + 1]);
        mx = vmax3(mx, s[1][15], s[1][15]);
        const float mrow = max_xchg32(mx) * c2;
        if (__builtin_amdgcn_ballot_w64(mrow > m + C::TH) != 0) {
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
        float rs = 0.f;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const float p = fast_exp2(__builtin_fmaf(s[b][j], c2, nm));
                s[b][j] = p;
                rs += p;
            }
        l += sum_xchg32(rs);
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) pf[b][ss] = pack_acc_t<F16>(s[b], ss);
    };

    if (ntiles > 0) dma_tile_asm(tk, kbase + (int64_t)klo * a.k_tok, a.k_tok, Lk - klo, kbuf0, wave_u);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // X(j): S_j = K_j Q^T (after the last tile it reads a stale K buffer into s, which no softmax consumes), then
    // O += V_{j-1}^T P_{j-1} (not at j = 0: the V buffer is not loaded yet and may hold NaN patterns)
    auto xphase = [&](int j) {
        qk(kbuf0 + (j & 1) * C::TILE);
        if (j > 0) pv(vbuf0 + ((j + 1) & 1) * C::TILE);
    };
    auto issue = [&](int j) {  // K_j and V_{j-1} into the buffers their predecessors released
        if (j < ntiles)
            dma_tile_asm(tk, kbase + (int64_t)(klo + j * C::KT) * a.k_tok, a.k_tok, Lk - klo - j * C::KT,
                         kbuf0 + (j & 1) * C::TILE, wave_u);
        if (j - 1 < ntiles)
            dma_tile_asm(tv, vbase + (int64_t)(klo + (j - 1) * C::KT) * a.v_tok, a.v_tok, Lk - klo - (j - 1) * C::KT,
                         vbuf0 + ((j - 1) & 1) * C::TILE, wave_u);
    };
    // phases 2i (A: X(i), B: Y(i-1)) and 2i+1 (A: Y(i), B: X(i)), i = 0 .. ntiles.  K_{i+1} and V_i are issued at
    // the start of phase 2i and retired at its end, so both are readable from phase 2i+1 on: each wave reads the first
    // K fragments of its next X phase during the softmax phase before it.
    prefetch_k(kbuf0);
    if (grp == 0) {
        for (int i = 0; i <= ntiles; ++i) {
            issue(i + 1);
            xphase(i);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (i < ntiles) softmax(klo + i * C::KT);
            prefetch_k(kbuf0 + ((i + 1) & 1) * C::TILE);
            __syncthreads();
        }
    } else {
        for (int i = 0; i <= ntiles; ++i) {
            issue(i + 1);
            if (i >= 1) softmax(klo + (i - 1) * C::KT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            xphase(i);
            __syncthreads();
            prefetch_k(kbuf0 + ((i + 1) & 1) * C::TILE);
        }
    }
    if (myq < Lq) {
        const float inv = l > 0.f ? 1.f / l : 0.f;
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
    static const bool pp = [] {
        const char* e = getenv("SCALING_AMD_FA_FWD_PP");  // ping-pong forward (D = 128, no dropout)
        return e && atoi(e) == 1;
    }();
    if (pp && D == 128 && !DROP) {
        dim3 grid(a.Hq, a.nseg, (max_q + FwdV2<128>::BM - 1) / FwdV2<128>::BM), block(512);
        hipLaunchKernelGGL((fa_fwd_pp_kernel<128, F16>), grid, block, 4 * FwdV2<128>::TILE, st, a);
        return;
    }
    if (D == 128 || D == 64) {
        static const int nw = [] {
            const char* e = getenv("SCALING_AMD_FA_FWD_WAVES");  // 4 (default, measured faster) or 8
            return e && atoi(e) == 8 ? 8 : 4;
        }();
        static const bool adma = [] {
            const char* e = getenv("SCALING_AMD_FA_FWD_ADMA");
            return e && atoi(e) == 1;
        }();
        if (nw == 4) {
            dim3 grid(a.Hq, a.nseg, (max_q + FwdV2<128, 4>::BM - 1) / FwdV2<128, 4>::BM), block(256);
            static const bool ra = [] {
                const char* e = getenv("SCALING_AMD_FA_FWD_RA");
                return e && atoi(e) == 1;
            }();
            if (D == 128 && ra)
                hipLaunchKernelGGL((fa_fwd_v2_kernel<128, F16, DROP, 4, false, true>), grid, block, 4 * FwdV2<128>::TILE, st, a);
            else if (D == 128 && adma)
                hipLaunchKernelGGL((fa_fwd_v2_kernel<128, F16, DROP, 4, true>), grid, block, 4 * FwdV2<128>::TILE, st, a);
            else if (D == 128) hipLaunchKernelGGL((fa_fwd_v2_kernel<128, F16, DROP, 4>), grid, block, 4 * FwdV2<128>::TILE, st, a);
            else hipLaunchKernelGGL((fa_fwd_v2_kernel<64, F16, DROP, 4>), grid, block, 4 * FwdV2<64>::TILE, st, a);
            return;
        }
        dim3 grid(a.Hq, a.nseg, (max_q + FwdV2<128>::BM - 1) / FwdV2<128>::BM), block(64 * FwdV2<128>::NW);
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
