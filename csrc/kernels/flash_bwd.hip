// Flash-attention backward, gfx950, deterministic (no float atomics):
//   fa_bwd_dot : delta[q] = rowsum(dO * O)
//   fa_bwd_dkdv: workgroup = 4 waves x 32 keys (128 keys) of one (segment, kv-head); sweeps every
//                q-head of the GQA group x 64-query tiles.  Key on the lane:
//                  S = Q K^T, dP = dO V^T  (C col = key)  -> P, dS lane-local per key
//                  dV^T += dO^T P, dK^T += Q^T dS      (P/dS accumulators are the B operands,
//                                                        dO^T / Q^T via ds_read_b64_tr_b16)
//   fa_bwd_dq  : workgroup = 4 waves x 32 queries of one (segment, q-head); sweeps key tiles:
//                  S^T = K Q^T, dP^T = V dO^T (query on the lane), dQ^T += K^T dS^T.
// dK/dV and dQ are each owned by exactly one workgroup, so results are bitwise reproducible.
#include "flash_attn.h"
#include "launch.h"

using namespace sa;
using namespace sa::fa;

template <int D, typename E>
__global__ __launch_bounds__(256) void fa_bwd_dot_kernel(const E* __restrict__ o, int64_t o_tok, int64_t o_head,
                                                         const E* __restrict__ dO, int64_t d_tok, int64_t d_head,
                                                         float* __restrict__ delta, const float* __restrict__ lse,
                                                         float* __restrict__ lse2, int64_t T, int H) {
    constexpr int LPR = D / 8;  // lanes per row
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t row = gid / LPR;
    const int c = (int)(gid % LPR);
    float s = 0.f;
    const bool ok = row < T * H;
    int64_t t = 0;
    int hh = 0;
    if (ok) {
        t = row / H;
        hh = (int)(row % H);
        float a[8], b[8];
        V8<E>::ld(o + t * o_tok + hh * o_head + 8 * c, a);
        V8<E>::ld(dO + t * d_tok + hh * d_head + 8 * c, b);
#pragma unroll
        for (int j = 0; j < 8; ++j) s += a[j] * b[j];
    }
#pragma unroll
    for (int w = LPR / 2; w > 0; w >>= 1) s += __shfl_xor(s, w, 64);
    if (ok && c == 0) {
        delta[(int64_t)hh * T + t] = s;
        lse2[(int64_t)hh * T + t] = lse[(int64_t)hh * T + t] * 1.4426950408889634f;
    }
}

// Stores one lane's gradient row (NT x 16 accumulators: element 4g + j of acc[t] is dim 32t + 8g + 4h + j) scaled by
// `scale`, with the inverse RoPE of the row's token folded in when a.rcos is set -- the arithmetic of the stand-alone
// rope kernel on the rounded gradient (round, rotate with rot_pair and sign -1, round), so the fold is bit-identical
// to flash backward + rope(..., inverse).  NeoX (full rotation, rrd == D: the binding checks) pairs dims d, d + D/2 =
// accumulators t and t + NT/2 of the same lane; interleaved pairs are elements (2p, 2p+1) of one 4-element group.
// Only wave-uniform branches, and the row's cos / sin loads are issued together before the first use (a branch per
// group exposed one global-load latency per group: +2.8 ms/step of dQ epilogue, profiles/rocprof_7b_r4j_step.md).
template <int D, bool F16>
__device__ __forceinline__ void store_grad_row(const BwdArgs& a, const f32x16 (&acc)[D / 32], float scale, int64_t tok,
                                               int h, u16* dst) {
    constexpr int NT = D / 32;
    auto rd = [&](int t, int g, float (&x)[4]) {
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = t2f<F16>(f2t<F16>(acc[t][4 * g + j] * scale));
    };
    auto st = [&](int t, int g, const float (&x)[4]) {
        u16x4 w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = f2t<F16>(x[j]);
        *reinterpret_cast<u16x4*>(dst + 32 * t + 8 * g + 4 * h) = w;
    };
    if (a.rcos == nullptr) {  // wave-uniform branches only; the table loads of a rotating row are all issued up front
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                float x[4];
                rd(t, g, x);
                st(t, g, x);
            }
        return;
    }
    const int64_t ps = a.rpos ? a.rpos[tok] : (tok % a.rseq);
    const float* cb = a.rcos + ps * (a.rrd / 2);
    const float* sb = a.rsin + ps * (a.rrd / 2);
    if constexpr (NT < 2) return;  // D = 32: never folded (fa_bwd binding)
    if (!a.ril) {  // NeoX, rrd == D: dims d (acc t < NT/2) and d + D/2 (acc t + NT/2) share cos / sin [d]
        constexpr int NH = NT / 2 > 0 ? NT / 2 : 1;
        f32x4 cv[NH][4], sv[NH][4];
#pragma unroll
        for (int t = 0; t < NT / 2; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                cv[t][g] = *reinterpret_cast<const f32x4*>(cb + 32 * t + 8 * g + 4 * h);
                sv[t][g] = *reinterpret_cast<const f32x4*>(sb + 32 * t + 8 * g + 4 * h);
            }
#pragma unroll
        for (int t = 0; t < NT / 2; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                float x[4], y[4];
                rd(t, g, x);
                rd(t + NT / 2, g, y);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float o0, o1;
                    rot_pair(x[j], y[j], cv[t][g][j], -sv[t][g][j], o0, o1);
                    x[j] = o0;
                    y[j] = o1;
                }
                st(t, g, x);
                st(t + NT / 2, g, y);
            }
        return;
    }
    // interleaved: elements (2p, 2p+1) of a 4-element group are pair p = d/2 of dims below rrd; cos / sin pairs of
    // dims past rrd are read clamped and the rotation is discarded by a select
    const int hr = a.rrd / 2 - 2;
    float2 cv[NT][4], sv[NT][4];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int p = min((32 * t + 8 * g + 4 * h) / 2, hr);
            cv[t][g] = *reinterpret_cast<const float2*>(cb + p);
            sv[t][g] = *reinterpret_cast<const float2*>(sb + p);
        }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const bool rot = 32 * t + 8 * g + 4 * h < a.rrd;
            float x[4];
            rd(t, g, x);
            float o[4];
            rot_pair(x[0], x[1], cv[t][g].x, -sv[t][g].x, o[0], o[1]);
            rot_pair(x[2], x[3], cv[t][g].y, -sv[t][g].y, o[2], o[3]);
#pragma unroll
            for (int j = 0; j < 4; ++j) x[j] = rot ? o[j] : x[j];
            st(t, g, x);
        }
}

// dK / dV: workgroup = 4 waves x 32 keys of one (segment, kv head); the key is on the MFMA lane.  Each
// wave keeps its 32 K rows as register-resident B-operand fragments and reads its V rows from the
// workgroup's V image (LDS, loaded once); it sweeps the GQA (sub)group's q heads x 32-query tiles.  Q, dO,
// lse2 (= lse * log2 e) and delta arrive by LDS-DMA into a double buffer.  LDS = V image + 2 x 32-query
// buffers (65 KiB at D = 128), so two workgroups (2 waves / SIMD) share a CU.  Per 32-query tile:
//   S = Q K^T, dP = dO V^T (row reads), p = exp2(S c - lse2), dS = p (dP - delta),
//   dV^T += dO^T P, dK^T += Q^T dS (transposed reads; P / dS accumulators are the B operands).
// Query rows past the segment arrive as zeros (Q = dO = 0, lse2 = delta = 0) and contribute nothing.
// Variants measured against this one and dropped (one wave per SIMD with explicit read-ahead, inline-asm LDS-DMA,
// paired software-pipelined query tiles): profiles/attn_bwd_variants_ab_r3.log, attn_bwd_pair_ab_r3.log; their code is
// in git history before commit "Delete losing attention variants".
template <int D, bool F16, bool DROP>
__global__ __launch_bounds__(256, 2) void fa_bwd_dkdv_kernel(BwdArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)  // the host pass only needs the signature for the launch stub
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int QT = 32, TILE = QT * D * 2, BUF = 2 * TILE + 512, VIMG = 128 * D * 2, NKS = D / 16, NT = D / 32;
    // grid (Hkv * hsplit, nseg, key blocks): key block slowest so causal work is issued heaviest-first (a segment-major
    // order, the forward's choice, measured 7 % slower here: profiles/attn_segmajor_ab_r5.log)
    const int seg = blockIdx.y, hk = blockIdx.x / a.hsplit, sub = blockIdx.x % a.hsplit;
    const int q0s = a.cu_q[seg], k0s = a.cu_k[seg];
    const int Lq = a.cu_q[seg + 1] - q0s, Lk = a.cu_k[seg + 1] - k0s;
    const int kwg0 = blockIdx.z * 128;
    if (kwg0 >= Lk) return;
    const int grp = a.Hq / a.Hkv / a.hsplit;  // q heads swept by this workgroup: hk * Hq/Hkv + sub * grp + [0, grp)
    const int h0 = hk * (a.Hq / a.Hkv) + sub * grp;
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, lk = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int off = Lk - Lq;
    const int kw0 = kwg0 + 32 * wave, mykey = kw0 + lk;
    const int klast = min(kwg0 + 127, Lk - 1);
    // the swept q heads h0 .. h0+grp-1 may mix windowed and global heads: the q range is their union
    const int wun = (a.window >= 0 && h0 + grp <= a.local_heads) ? a.window : -1;
    int qlo = 0, qhi = Lq;
    if (a.causal) qlo = max(0, kwg0 - off);
    if (wun >= 0) {
        qhi = min(Lq, klast - off + wun + 1);
        if (!a.causal) qlo = max(0, kwg0 - off - wun);
    }
    qlo = (qlo / QT) * QT;
    const int ntq = qhi > qlo ? (qhi - qlo + QT - 1) / QT : 0;
    const int nwork = ntq * grp;

    char* vimg = smem;  // V rows [kwg0, kwg0 + 128)
    {
        DmaTile<D, 4> dv_;
        dv_.init(wave, lane, a.v_tok);
        const u16* vb = a.v + (int64_t)(k0s + kwg0) * a.v_tok + (int64_t)hk * a.v_head;
        dma_load(dv_, vb, a.v_tok, Lk - kwg0, vimg, wave);
        dma_load(dv_, vb + 64 * a.v_tok, a.v_tok, Lk - kwg0 - 64, vimg + 64 * D * 2, wave);
    }
    const char* vw_img = vimg + 32 * wave * D * 2;
    bf16x8 kf[NKS];  // lane: key kw0 + (lane & 31), dims 16 ks + 8 h .. + 7
    {
        const u16* kp = a.k + (int64_t)(k0s + min(mykey, Lk - 1)) * a.k_tok + (int64_t)hk * a.k_head;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) kf[ks] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u16x8*>(kp + 16 * ks + 8 * h));
        // consume K here: hipcc retires the loads before the tile loop (inside it its vmcnt would also wait for
        // the asm LDS-DMA in flight)
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) asm volatile("" ::"v"(kf[ks]));
    }
    LdsOffsets<D> lo;
    lo.init(lane);
    DmaTile<D, 4, QT> tq, td;
    tq.init(wave, lane, a.q_tok);
    td.init(wave, lane, a.do_tok);
    // work item (q head h0 + gi, query tile qlo + QT qi), qi fastest; the issue and compute cursors advance
    // incrementally (no runtime divisions in the loop)
    auto issue = [&](int gi, int qi, char* buf) {
        const int qt = qlo + qi * QT, hq = h0 + gi;
        dma_load(tq, a.q + (int64_t)(q0s + qt) * a.q_tok + (int64_t)hq * a.q_head, a.q_tok, Lq - qt, buf, wave);
        dma_load(td, a.dO + (int64_t)(q0s + qt) * a.do_tok + (int64_t)hq * a.do_head, a.do_tok, Lq - qt, buf + TILE, wave);
        if (wave == 0) {  // QT lse2 then QT delta (lanes past QT read out of range -> zeros into the pad)
            const int64_t ix = (int64_t)hq * a.lse_stride + q0s + qt;
            const uint32_t nb = (uint32_t)max(min(QT, Lq - qt), 0) * 4u;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(uniform_rsrc(a.lse2 + ix, nb), (lds_void*)(buf + 2 * TILE), 4, 4 * lane, 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(uniform_rsrc(a.delta + ix, nb), (lds_void*)(buf + 2 * TILE + 256), 4, 4 * lane, 0, 0, 0);
        }
    };
    f32x16 dk[NT], dv[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) { dk[t] = f32x16{}; dv[t] = f32x16{}; }
    const float c2 = a.scale_log2;

    auto tile = [&](const char* Q, int gi, int qi) {
        const char* DO = Q + TILE;
        const float* LS = reinterpret_cast<const float*>(Q + 2 * TILE);
        const float* DL = LS + 64;
        const int qt = qlo + qi * QT;
        const int win = (h0 + gi) < a.local_heads ? a.window : -1;
        uint32_t hs = 0;
        if constexpr (DROP) hs = drop_head(a.seed, h0 + gi);
        const bool need_mask = (a.causal && kw0 + 31 > qt + off) ||
                               (win >= 0 && (kw0 < qt + QT - 1 + off - win || (!a.causal && kw0 + 31 > qt + off + win)));
        f32x16 s = f32x16{}, dp = f32x16{};
        {
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                s = mma<F16>(rd_row<D>(Q, 0, lo.row(ks)), kf[ks], s);
                dp = mma<F16>(rd_row<D>(DO, 0, lo.row(ks)), rd_row<D>(vw_img, 0, lo.row(ks)), dp);
            }
            // Q / dO / V row fragments one k-step (3 reads) ahead of their MFMAs (two spill at 256 VGPRs; the one-per-MFMA
            // form left every MFMA behind an lgkmcnt(0): 1.5 % slower backward, profiles/attn_sched_ab_r4.log)
            __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#pragma unroll
            for (int i = 0; i < NKS - 1; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        }
        // query of register j: qt + 4h + crow(j)
        int mlo = -1 << 30, mhi = 1 << 30;
        if (need_mask) {
            const int rel = mykey - off - qt - 4 * h;
            if (a.causal) mlo = rel;                  // key <= q + off
            if (win >= 0) {
                mhi = rel + win;                 // key >= q + off - window
                if (!a.causal) mlo = rel - win;  // key <= q + off + window
            }
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const f32x4 l4 = *reinterpret_cast<const f32x4*>(LS + 8 * g + 4 * h);
#pragma unroll
            for (int j = 0; j < 4; ++j) s[4 * g + j] = fast_exp2(__builtin_fmaf(s[4 * g + j], c2, -l4[j]));
        }
        if (need_mask) {  // boundary tiles only: a real (wave-uniform) branch, not per-element selects every tile
            mask_fence();
#pragma unroll
            for (int r = 0; r < 16; ++r) s[r] = (crow(r) >= mlo && crow(r) <= mhi) ? s[r] : 0.f;
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const f32x4 d4 = *reinterpret_cast<const f32x4*>(DL + 8 * g + 4 * h);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int r = 4 * g + j;
                const float p = s[r];
                if constexpr (DROP) {  // dV sees the dropped P; dS = P (Z dP / (1-p) - delta)
                    const bool keep = drop_keep(drop_row(hs, q0s + qt + 4 * h + crow(r)), k0s + mykey, a.drop_thr);
                    s[r] = keep ? p * a.rp_drop : 0.f;
                    dp[r] = p * ((keep ? dp[r] * a.rp_drop : 0.f) - d4[j]);
                } else {
                    s[r] = p;
                    dp[r] = p * (dp[r] - d4[j]);
                }
            }
        }
        {
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                const bf16x8 pb = pack_acc_t<F16>(s, ss), db = pack_acc_t<F16>(dp, ss);
                const int kb = 16 * ss * D * 2;
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    dv[t] = mma<F16>(rd_tr<D>(DO, kb, lo, t), pb, dv[t]);
                    dk[t] = mma<F16>(rd_tr<D>(Q, kb, lo, t), db, dk[t]);
                }
            }
            // transposed dO / Q fragments one MFMA ahead (two spill at 256 VGPRs)
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
#pragma unroll
            for (int i = 0; i < 4 * NT - 1; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
        }
    };

    char* buf0 = smem + VIMG;
    char* buf1 = buf0 + BUF;
    int ig = 0, iq = 0, cg = 0, cq = 0;  // next item to issue / to compute
    auto adv = [&](int& g, int& q) {
        if (++q == ntq) {
            q = 0;
            ++g;
        }
    };
    if (nwork > 0) {
        issue(ig, iq, buf0);
        adv(ig, iq);
    }
    dma_barrier();
    int w = 0;
    for (; w + 1 < nwork; w += 2) {
        issue(ig, iq, buf1);
        adv(ig, iq);
        tile(buf0, cg, cq);
        adv(cg, cq);
        dma_barrier();  // every wave's pieces of the next work item landed (see dma_barrier)
        if (w + 2 < nwork) {
            issue(ig, iq, buf0);
            adv(ig, iq);
        }
        tile(buf1, cg, cq);
        adv(cg, cq);
        dma_barrier();
    }
    if (w < nwork) tile(buf0, cg, cq);

    if (mykey < Lk) {
        if (a.hsplit > 1) {  // fp32 partials, summed by fa_bwd_reduce_kernel
            const int64_t pix = (((int64_t)sub * a.Tk + k0s + mykey) * a.Hkv + hk) * D;
            float* kp = a.dk_part + pix;
            float* vp = a.dv_part + pix;
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    f32x4 wk, wv;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        wk[j] = dk[t][4 * g + j] * a.scale;
                        wv[j] = dv[t][4 * g + j];
                    }
                    *reinterpret_cast<f32x4*>(kp + 32 * t + 8 * g + 4 * h) = wk;
                    *reinterpret_cast<f32x4*>(vp + 32 * t + 8 * g + 4 * h) = wv;
                }
        } else {
            u16* vp = a.dv + (int64_t)(k0s + mykey) * a.dv_tok + (int64_t)hk * a.dv_head;
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    u16x4 wv;
#pragma unroll
                    for (int j = 0; j < 4; ++j) wv[j] = f2t<F16>(dv[t][4 * g + j]);
                    *reinterpret_cast<u16x4*>(vp + 32 * t + 8 * g + 4 * h) = wv;
                }
            store_grad_row<D, F16>(a, dk, a.scale, k0s + mykey, h,
                                   a.dk + (int64_t)(k0s + mykey) * a.dk_tok + (int64_t)hk * a.dk_head);
        }
    }
#endif
}

// dQ: workgroup = 4 waves x 32 queries of one (segment, q head); query on the lane (Q, dO rows are
// register-resident B operands), K / V tiles of 64 keys double-buffered in LDS by LDS-DMA.  Per 32-key block:
//   S^T = K Q^T, dP^T = V dO^T, p = exp2(S c - lse2), dS = p (dP - delta), dQ^T += K^T dS^T.
template <int D, bool F16, bool DROP>
__global__ __launch_bounds__(256, 2) void fa_bwd_dq_kernel(BwdArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)  // the host pass only needs the signature for the launch stub
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int TILE = 64 * D * 2, NKS = D / 16, NT = D / 32;
    const int seg = attn_seg(), hq = xcd_head(blockIdx.x, a.Hq);  // see attn_grid
    const int q0s = a.cu_q[seg], k0s = a.cu_k[seg];
    const int Lq = a.cu_q[seg + 1] - q0s, Lk = a.cu_k[seg + 1] - k0s;
    const int ntiles_q = (Lq + 127) / 128;
    const int qt = attn_qtile(a.causal);
    if (qt >= ntiles_q) return;
    const int hk = hq / (a.Hq / a.Hkv);
    const int win = hq < a.local_heads ? a.window : -1;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5,
              lq = lane & 31;
    const int wave_u = wave;  // wave-uniform: qw0 and the mask test below are scalar
    const int off = Lk - Lq;
    const int qwg0 = qt * 128, qw0 = qwg0 + wave * 32, myq = qw0 + lq;
    const int qlast = min(qwg0 + 127, Lq - 1);
    int khi = Lk;
    if (a.causal) khi = min(Lk, qlast + off + 1);
    else if (win >= 0) khi = min(Lk, qlast + off + win + 1);
    int klo = 0;
    if (win >= 0) klo = max(0, qwg0 + off - win);
    klo = (klo / 64) * 64;

    bf16x8 qf[NKS], df[NKS];
    {
        const int qrow = q0s + min(myq, Lq - 1);
        const u16* qp = a.q + (int64_t)qrow * a.q_tok + (int64_t)hq * a.q_head;
        const u16* dp = a.dO + (int64_t)qrow * a.do_tok + (int64_t)hq * a.do_head;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            qf[ks] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u16x8*>(qp + 16 * ks + 8 * h));
            df[ks] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u16x8*>(dp + 16 * ks + 8 * h));
        }
    }
    const float nl2 = myq < Lq ? -a.lse[(int64_t)hq * a.lse_stride + q0s + myq] * 1.4426950408889634f : -INFINITY;
    const float dlt = myq < Lq ? a.delta[(int64_t)hq * a.lse_stride + q0s + myq] : 0.f;
    // consume the register-resident operands here (their loads retire before the loop, see fa_bwd_dkdv_kernel)
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) asm volatile("" ::"v"(qf[ks]), "v"(df[ks]));
    asm volatile("" ::"v"(nl2), "v"(dlt));
    uint32_t drow = 0;
    if constexpr (DROP) drow = drop_row(drop_head(a.seed, hq), q0s + myq);
    LdsOffsets<D> lo;
    lo.init(lane);
    DmaTile<D, 4> tk, tv;
    tk.init(wave_u, lane, a.k_tok);
    tv.init(wave_u, lane, a.v_tok);
    const u16* kbase = a.k + (int64_t)k0s * a.k_tok + (int64_t)hk * a.k_head;
    const u16* vbase = a.v + (int64_t)k0s * a.v_tok + (int64_t)hk * a.v_head;
    // (DMA issued through the free function dma_load: a direct DmaTile::load call in this kernel makes
    //  hipcc's host pass treat the kernel as undefined and drop its launch stub)
#define SA_DQ_ISSUE(KT, BUFP)                                                                          \
    do {                                                                                               \
        const int kp_ = (KT);                                                                          \
        dma_load(tk, kbase + (int64_t)kp_ * a.k_tok, a.k_tok, Lk - kp_, (BUFP), wave_u);                 \
        dma_load(tv, vbase + (int64_t)kp_ * a.v_tok, a.v_tok, Lk - kp_, (BUFP) + TILE, wave_u);          \
    } while (0)
    f32x16 dq[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) dq[t] = f32x16{};
    const float c2 = a.scale_log2;

    auto tile = [&](const char* K, int kt) {
        const char* V = K + TILE;
        const bool need_mask = (kt + 64 > Lk) || (a.causal && kt + 63 > qw0 + off) ||
                               (win >= 0 && (kt < qw0 + 31 + off - win || (!a.causal && kt + 63 > qw0 + off + win)));
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            f32x16 s = f32x16{}, dp = f32x16{};
            {
#pragma unroll
                for (int ks = 0; ks < NKS; ++ks) {
                    s = mma<F16>(rd_row<D>(K, 32 * b * D * 2, lo.row(ks)), qf[ks], s);
                    dp = mma<F16>(rd_row<D>(V, 32 * b * D * 2, lo.row(ks)), df[ks], dp);
                }
            }
            // key of register j: kt + 32b + 4h + crow(j)
#pragma unroll
            for (int r = 0; r < 16; ++r) s[r] = fast_exp2(__builtin_fmaf(s[r], c2, nl2));
            if (need_mask) {  // boundary tiles only: a real (wave-uniform) branch, not per-element selects
                mask_fence();
                const int base = kt + 32 * b + 4 * h;
                int hi = Lk - 1 - base, low = -1 << 30;
                if (a.causal) hi = min(hi, myq + off - base);
                else if (win >= 0) hi = min(hi, myq + off + win - base);
                if (win >= 0) low = myq + off - win - base;
#pragma unroll
                for (int r = 0; r < 16; ++r) s[r] = (crow(r) <= hi && crow(r) >= low) ? s[r] : 0.f;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float p = s[r];
                if constexpr (DROP) {
                    const bool keep = drop_keep(drow, k0s + kt + 32 * b + 4 * h + crow(r), a.drop_thr);
                    dp[r] = p * ((keep ? dp[r] * a.rp_drop : 0.f) - dlt);
                } else {
                    dp[r] = p * (dp[r] - dlt);
                }
            }
            {
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    const bf16x8 db = pack_acc_t<F16>(dp, ss);
                    const int kb = (32 * b + 16 * ss) * D * 2;
#pragma unroll
                    for (int t = 0; t < NT; ++t) dq[t] = mma<F16>(rd_tr<D>(K, kb, lo, t), db, dq[t]);
                }
            }
        }
    };

    char* buf0 = smem;
    char* buf1 = smem + 2 * TILE;
    if (klo < khi) SA_DQ_ISSUE(klo, buf0);
    dma_barrier();
    const int ntiles = khi > klo ? (khi - klo + 63) / 64 : 0;
    int kt = klo;
    for (int pr = 0; pr < ntiles / 2; ++pr, kt += 128) {
        SA_DQ_ISSUE(kt + 64, buf1);
        tile(buf0, kt);
        dma_barrier();  // every wave's pieces of tile kt + 64 landed (see dma_barrier)
        if (kt + 128 < khi) SA_DQ_ISSUE(kt + 128, buf0);
        tile(buf1, kt + 64);
        dma_barrier();
    }
    if (ntiles & 1) tile(buf0, kt);
#undef SA_DQ_ISSUE
    if (myq < Lq)
        store_grad_row<D, F16>(a, dq, a.scale, q0s + myq, h,
                               a.dq + (int64_t)(q0s + myq) * a.dq_tok + (int64_t)hq * a.dq_head);
#endif
}

// dK/dV = sum of the hsplit fp32 partials (fixed order: deterministic), cast into the strided outputs.
template <int D, bool F16>
__global__ __launch_bounds__(256) void fa_bwd_reduce_kernel(BwdArgs a) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per = (int64_t)a.Tk * a.Hkv * (D / 8);
    if (gid >= per) return;
    const int c = (int)(gid % (D / 8));
    const int64_t th = gid / (D / 8);
    const int hk = (int)(th % a.Hkv);
    const int64_t tok = th / a.Hkv;
    const int64_t pstride = (int64_t)a.Tk * a.Hkv * D;
    float sk[8] = {}, sv[8] = {};
    for (int s = 0; s < a.hsplit; ++s) {
        const float* kp = a.dk_part + s * pstride + th * D + 8 * c;
        const float* vp = a.dv_part + s * pstride + th * D + 8 * c;
        float x[8], y[8];
        V8<float>::ld(kp, x);
        V8<float>::ld(vp, y);
#pragma unroll
        for (int j = 0; j < 8; ++j) { sk[j] += x[j]; sv[j] += y[j]; }
    }
    u16x8 wk, wv;
#pragma unroll
    for (int j = 0; j < 8; ++j) { wk[j] = fa::f2t<F16>(sk[j]); wv[j] = fa::f2t<F16>(sv[j]); }
    *reinterpret_cast<u16x8*>(a.dk + tok * a.dk_tok + (int64_t)hk * a.dk_head + 8 * c) = wk;
    *reinterpret_cast<u16x8*>(a.dv + tok * a.dv_tok + (int64_t)hk * a.dv_head + 8 * c) = wv;
}

template <bool F16, bool DROP>
static void launch_bwd_main(const BwdArgs& a, int D, int max_q, int max_k, hipStream_t st) {
    {
        dim3 grid(a.Hkv * a.hsplit, a.nseg, (max_k + 127) / 128);
        const size_t lds = 128 * D * 2 + 2 * (2 * 32 * D * 2 + 512);
        if (D == 128) hipLaunchKernelGGL((fa_bwd_dkdv_kernel<128, F16, DROP>), grid, 256, lds, st, a);
        else if (D == 64) hipLaunchKernelGGL((fa_bwd_dkdv_kernel<64, F16, DROP>), grid, 256, lds, st, a);
        else hipLaunchKernelGGL((fa_bwd_dkdv_kernel<32, F16, DROP>), grid, 256, lds, st, a);
    }
    {
        dim3 grid = attn_grid(a.Hq, a.nseg, (max_q + 127) / 128);
        const size_t lds = 4 * 64 * D * 2;
        if (D == 128) hipLaunchKernelGGL((fa_bwd_dq_kernel<128, F16, DROP>), grid, 256, lds, st, a);
        else if (D == 64) hipLaunchKernelGGL((fa_bwd_dq_kernel<64, F16, DROP>), grid, 256, lds, st, a);
        else hipLaunchKernelGGL((fa_bwd_dq_kernel<32, F16, DROP>), grid, 256, lds, st, a);
    }
    if (a.hsplit > 1) {
        const int64_t threads = (int64_t)a.Tk * a.Hkv * (D / 8);
        const int grid = (int)((threads + 255) / 256);
        if (D == 128) hipLaunchKernelGGL((fa_bwd_reduce_kernel<128, F16>), grid, 256, 0, st, a);
        else if (D == 64) hipLaunchKernelGGL((fa_bwd_reduce_kernel<64, F16>), grid, 256, 0, st, a);
        else hipLaunchKernelGGL((fa_bwd_reduce_kernel<32, F16>), grid, 256, 0, st, a);
    }
}

template <int D, typename T>
static void launch_bwd_dot(const BwdArgs& a, const uint16_t* o, int64_t o_tok, int64_t o_head, int64_t Tq, hipStream_t st) {
    const int64_t threads = Tq * a.Hq * (D / 8);
    const int grid = (int)((threads + 255) / 256);
    hipLaunchKernelGGL((fa_bwd_dot_kernel<D, T>), grid, 256, 0, st, (const T*)o, o_tok, o_head, (const T*)a.dO, a.do_tok,
                       a.do_head, a.delta, a.lse, a.lse2, Tq, a.Hq);
}

template <int D>
static void launch_bwd(const BwdArgs& a, const uint16_t* o, int64_t o_tok, int64_t o_head, int64_t Tq, int max_q,
                       int max_k, bool f16, hipStream_t st) {
    const bool drop = a.p_drop > 0.f;
    if (f16) {
        launch_bwd_dot<D, _Float16>(a, o, o_tok, o_head, Tq, st);
        if (drop) launch_bwd_main<true, true>(a, D, max_q, max_k, st);
        else launch_bwd_main<true, false>(a, D, max_q, max_k, st);
    } else {
        launch_bwd_dot<D, u16>(a, o, o_tok, o_head, Tq, st);
        if (drop) launch_bwd_main<false, true>(a, D, max_q, max_k, st);
        else launch_bwd_main<false, false>(a, D, max_q, max_k, st);
    }
}

namespace sa_launch {
void fa_bwd(const BwdArgs& a, const uint16_t* o, int64_t o_tok, int64_t o_head, int64_t Tq, int D, int max_q, int max_k,
            bool f16, hipStream_t st) {
    if (D == 128) launch_bwd<128>(a, o, o_tok, o_head, Tq, max_q, max_k, f16, st);
    else if (D == 64) launch_bwd<64>(a, o, o_tok, o_head, Tq, max_q, max_k, f16, st);
    else launch_bwd<32>(a, o, o_tok, o_head, Tq, max_q, max_k, f16, st);
}
}  // namespace sa_launch
