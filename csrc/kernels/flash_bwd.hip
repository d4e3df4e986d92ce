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

template <int D>
__global__ __launch_bounds__(256) void fa_bwd_dot_kernel(const u16* __restrict__ o, int64_t o_tok, int64_t o_head,
                                                         const u16* __restrict__ dO, int64_t d_tok, int64_t d_head,
                                                         float* __restrict__ delta, int64_t T, int H) {
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
        V8<u16>::ld(o + t * o_tok + hh * o_head + 8 * c, a);
        V8<u16>::ld(dO + t * d_tok + hh * d_head + 8 * c, b);
#pragma unroll
        for (int j = 0; j < 8; ++j) s += a[j] * b[j];
    }
#pragma unroll
    for (int w = LPR / 2; w > 0; w >>= 1) s += __shfl_xor(s, w, 64);
    if (ok && c == 0) delta[(int64_t)hh * T + t] = s;
}

template <int D>
__global__ __launch_bounds__(256, 1) void fa_bwd_dkdv_kernel(BwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int TILE = 64 * D * 2;
    // layout: K image [128][D] | V image [128][D] | 2 x (Q tile | dO tile) | 2 x (lse[64] | delta[64])
    char* kimg = smem;
    char* vimg = smem + 2 * TILE;
    char* qbuf = smem + 4 * TILE;  // buffer b: Q at qbuf + 2*b*TILE, dO at +TILE
    float* stat = reinterpret_cast<float*>(smem + 8 * TILE);  // buffer b: lse at stat + 128*b, delta +64

    const int seg = blockIdx.z, hk = blockIdx.y;
    const int q0s = a.cu_q[seg], k0s = a.cu_k[seg];
    const int Lq = a.cu_q[seg + 1] - q0s, Lk = a.cu_k[seg + 1] - k0s;
    const int kwg0 = blockIdx.x * 128;
    if (kwg0 >= Lk) return;
    const int grp = a.Hq / a.Hkv;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, lk = lane & 31;
    const int off = Lk - Lq;
    const int mykey_rel = wave * 32 + lk;  // row in K/V image
    const int mykey = kwg0 + mykey_rel;

    // query range touching these keys
    const int klast = min(kwg0 + 127, Lk - 1);
    int qlo = 0, qhi = Lq;
    if (a.causal) qlo = max(0, kwg0 - off);
    if (a.window >= 0) {
        qhi = min(Lq, klast - off + a.window + 1);
        if (!a.causal) qlo = max(0, kwg0 - off - a.window);
    }
    qlo = (qlo / 64) * 64;
    const int ntq = qhi > qlo ? (qhi - qlo + 63) / 64 : 0;
    const int nwork = ntq * grp;

    {  // K/V images for the workgroup's 128 keys
        Stage<D> st;
        const u16* kb = a.k + (int64_t)(k0s + kwg0) * a.k_tok + (int64_t)hk * a.k_head;
        const u16* vb = a.v + (int64_t)(k0s + kwg0) * a.v_tok + (int64_t)hk * a.v_head;
        st.load(kb, a.k_tok, min(64, Lk - kwg0));
        st.store(kimg);
        st.load(kb + 64 * a.k_tok, a.k_tok, max(0, min(64, Lk - kwg0 - 64)));
        st.store(kimg + TILE);
        st.load(vb, a.v_tok, min(64, Lk - kwg0));
        st.store(vimg);
        st.load(vb + 64 * a.v_tok, a.v_tok, max(0, min(64, Lk - kwg0 - 64)));
        st.store(vimg + TILE);
    }
    f32x16 dk[D / 32], dv[D / 32];
#pragma unroll
    for (int t = 0; t < D / 32; ++t) { dk[t] = f32x16{}; dv[t] = f32x16{}; }

    Stage<D> sq, sd;
    float st_l = 0.f, st_d = 0.f;
    auto issue = [&](int w) {
        const int gi = w / ntq, qt = qlo + (w % ntq) * 64;
        const int hq = hk * grp + gi;
        const int valid = min(64, Lq - qt);
        sq.load(a.q + (int64_t)(q0s + qt) * a.q_tok + (int64_t)hq * a.q_head, a.q_tok, valid);
        sd.load(a.dO + (int64_t)(q0s + qt) * a.do_tok + (int64_t)hq * a.do_head, a.do_tok, valid);
        if (threadIdx.x < 64) {
            const int r = threadIdx.x;
            const bool ok = r < valid;
            st_l = ok ? a.lse[(int64_t)hq * a.lse_stride + q0s + qt + r] * 1.4426950408889634f : INFINITY;
            st_d = ok ? a.delta[(int64_t)hq * a.lse_stride + q0s + qt + r] : 0.f;
        }
    };
    auto commit = [&](int b) {
        sq.store(qbuf + 2 * b * TILE);
        sd.store(qbuf + (2 * b + 1) * TILE);
        if (threadIdx.x < 64) {
            stat[128 * b + threadIdx.x] = st_l;
            stat[128 * b + 64 + threadIdx.x] = st_d;
        }
    };
    if (nwork > 0) {
        issue(0);
        commit(0);
    }
    __syncthreads();
    int cur = 0;
    for (int w = 0; w < nwork; ++w) {
        const bool has_next = w + 1 < nwork;
        if (has_next) issue(w + 1);
        const int qt = qlo + (w % ntq) * 64;
        const char* Q = qbuf + 2 * cur * TILE;
        const char* DO = Q + TILE;
        const float* LS = stat + 128 * cur;
        const float* DL = LS + 64;
        // ---- S = Q K^T, dP = dO V^T  (2 query blocks of 32)
        f32x16 s[2] = {f32x16{}, f32x16{}}, dp[2] = {f32x16{}, f32x16{}};
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) {
            const bf16x8 kf = ld_row<D>(kimg, mykey_rel, 16 * ks + 8 * h);
            const bf16x8 vf = ld_row<D>(vimg, mykey_rel, 16 * ks + 8 * h);
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                s[b] = mfma(ld_row<D>(Q, 32 * b + lk, 16 * ks + 8 * h), kf, s[b]);
                dp[b] = mfma(ld_row<D>(DO, 32 * b + lk, 16 * ks + 8 * h), vf, dp[b]);
            }
        }
        const bool need_mask = (kwg0 + 128 > Lk) || (qt + 64 > Lq) || (a.causal && qt < kwg0 + 127 - off) ||
                               (a.window >= 0);
#pragma unroll
        for (int b = 0; b < 2; ++b) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x4 l4 = *reinterpret_cast<const f32x4*>(LS + 32 * b + 8 * g + 4 * h);
                const f32x4 d4 = *reinterpret_cast<const f32x4*>(DL + 32 * b + 8 * g + 4 * h);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int r = 4 * g + j;
                    float p = fast_exp2(s[b][r] * a.scale_log2 - l4[j]);
                    if (need_mask) {
                        const int q = qt + 32 * b + 8 * g + 4 * h + j;
                        bool ok = mykey < Lk && q < Lq;
                        if (a.causal) ok = ok && mykey <= q + off;
                        if (a.window >= 0) ok = ok && mykey >= q + off - a.window && (a.causal || mykey <= q + off + a.window);
                        p = ok ? p : 0.f;
                    }
                    s[b][r] = p;
                    dp[b][r] = p * (dp[b][r] - d4[j]);
                }
            }
        }
        // ---- dV^T += dO^T P ; dK^T += Q^T dS
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                const bf16x8 pb = pack_acc(s[b], ss);
                const bf16x8 db = pack_acc(dp[b], ss);
#pragma unroll
                for (int t = 0; t < D / 32; ++t) {
                    dv[t] = mfma(ld_tr<D>(DO, 32 * b + 16 * ss, 32 * t), pb, dv[t]);
                    dk[t] = mfma(ld_tr<D>(Q, 32 * b + 16 * ss, 32 * t), db, dk[t]);
                }
            }
        if (has_next) commit(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
    if (mykey < Lk) {
        u16* kp = a.dk + (int64_t)(k0s + mykey) * a.dk_tok + (int64_t)hk * a.dk_head;
        u16* vp = a.dv + (int64_t)(k0s + mykey) * a.dv_tok + (int64_t)hk * a.dv_head;
#pragma unroll
        for (int t = 0; t < D / 32; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                u16x4 wk, wv;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    wk[j] = f2bf(dk[t][4 * g + j] * a.scale);
                    wv[j] = f2bf(dv[t][4 * g + j]);
                }
                *reinterpret_cast<u16x4*>(kp + 32 * t + 8 * g + 4 * h) = wk;
                *reinterpret_cast<u16x4*>(vp + 32 * t + 8 * g + 4 * h) = wv;
            }
    }
}

template <int D>
__global__ __launch_bounds__(256, 1) void fa_bwd_dq_kernel(BwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int TILE = 64 * D * 2;
    const int seg = blockIdx.z, hq = blockIdx.y;
    const int q0s = a.cu_q[seg], k0s = a.cu_k[seg];
    const int Lq = a.cu_q[seg + 1] - q0s, Lk = a.cu_k[seg + 1] - k0s;
    const int ntiles_q = (Lq + 127) / 128;
    const int qt = a.causal ? (int)gridDim.x - 1 - (int)blockIdx.x : (int)blockIdx.x;
    if (qt >= ntiles_q) return;
    const int hk = hq / (a.Hq / a.Hkv);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, lq = lane & 31;
    const int off = Lk - Lq;
    const int qwg0 = qt * 128, qw0 = qwg0 + wave * 32, myq = qw0 + lq;
    const int qlast = min(qwg0 + 127, Lq - 1);
    int khi = Lk;
    if (a.causal) khi = min(Lk, qlast + off + 1);
    else if (a.window >= 0) khi = min(Lk, qlast + off + a.window + 1);
    int klo = 0;
    if (a.window >= 0) klo = max(0, qwg0 + off - a.window);
    klo = (klo / 64) * 64;

    bf16x8 qf[D / 16], df[D / 16];
    const int qrow = q0s + min(myq, Lq - 1);
    {
        const u16* qp = a.q + (int64_t)qrow * a.q_tok + (int64_t)hq * a.q_head;
        const u16* dp = a.dO + (int64_t)qrow * a.do_tok + (int64_t)hq * a.do_head;
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) {
            qf[ks] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u16x8*>(qp + 16 * ks + 8 * h));
            df[ks] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u16x8*>(dp + 16 * ks + 8 * h));
        }
    }
    const float lse2 = myq < Lq ? a.lse[(int64_t)hq * a.lse_stride + q0s + myq] * 1.4426950408889634f : INFINITY;
    const float dlt = myq < Lq ? a.delta[(int64_t)hq * a.lse_stride + q0s + myq] : 0.f;
    f32x16 dq[D / 32];
#pragma unroll
    for (int t = 0; t < D / 32; ++t) dq[t] = f32x16{};

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
        f32x16 s[2] = {f32x16{}, f32x16{}}, dp[2] = {f32x16{}, f32x16{}};
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                s[b] = mfma(ld_row<D>(K, 32 * b + lq, 16 * ks + 8 * h), qf[ks], s[b]);
                dp[b] = mfma(ld_row<D>(V, 32 * b + lq, 16 * ks + 8 * h), df[ks], dp[b]);
            }
        const bool need_mask = (kt + 64 > Lk) || (a.causal && kt + 63 > qw0 + off) || (a.window >= 0);
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float p = fast_exp2(s[b][r] * a.scale_log2 - lse2);
                if (need_mask) {
                    const int key = kt + 32 * b + (r & 3) + 8 * (r >> 2) + 4 * h;
                    bool ok = key < Lk && myq < Lq;
                    if (a.causal) ok = ok && key <= myq + off;
                    if (a.window >= 0) ok = ok && key >= myq + off - a.window && (a.causal || key <= myq + off + a.window);
                    p = ok ? p : 0.f;
                }
                dp[b][r] = p * (dp[b][r] - dlt);
            }
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                const bf16x8 db = pack_acc(dp[b], ss);
#pragma unroll
                for (int t = 0; t < D / 32; ++t) dq[t] = mfma(ld_tr<D>(K, 32 * b + 16 * ss, 32 * t), db, dq[t]);
            }
        if (has_next) {
            sk.store(smem + 2 * (cur ^ 1) * TILE);
            sv.store(smem + (2 * (cur ^ 1) + 1) * TILE);
        }
        __syncthreads();
        cur ^= 1;
    }
    if (myq < Lq) {
        u16* qp = a.dq + (int64_t)(q0s + myq) * a.dq_tok + (int64_t)hq * a.dq_head;
#pragma unroll
        for (int t = 0; t < D / 32; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                u16x4 w;
#pragma unroll
                for (int j = 0; j < 4; ++j) w[j] = f2bf(dq[t][4 * g + j] * a.scale);
                *reinterpret_cast<u16x4*>(qp + 32 * t + 8 * g + 4 * h) = w;
            }
    }
}

namespace sa_launch {
void fa_bwd(const BwdArgs& a, const uint16_t* o, int64_t o_tok, int64_t o_head, int64_t Tq, int D, int max_q, int max_k,
            hipStream_t st) {
    {
        const int64_t threads = Tq * a.Hq * (D / 8);
        const int grid = (int)((threads + 255) / 256);
        if (D == 128) hipLaunchKernelGGL(fa_bwd_dot_kernel<128>, grid, 256, 0, st, o, o_tok, o_head, a.dO, a.do_tok, a.do_head, a.delta, Tq, a.Hq);
        else if (D == 64) hipLaunchKernelGGL(fa_bwd_dot_kernel<64>, grid, 256, 0, st, o, o_tok, o_head, a.dO, a.do_tok, a.do_head, a.delta, Tq, a.Hq);
        else hipLaunchKernelGGL(fa_bwd_dot_kernel<32>, grid, 256, 0, st, o, o_tok, o_head, a.dO, a.do_tok, a.do_head, a.delta, Tq, a.Hq);
    }
    {
        dim3 grid((max_k + 127) / 128, a.Hkv, a.nseg);
        const size_t lds = 8 * 64 * D * 2 + 2 * 128 * sizeof(float);
        if (D == 128) hipLaunchKernelGGL(fa_bwd_dkdv_kernel<128>, grid, 256, lds, st, a);
        else if (D == 64) hipLaunchKernelGGL(fa_bwd_dkdv_kernel<64>, grid, 256, lds, st, a);
        else hipLaunchKernelGGL(fa_bwd_dkdv_kernel<32>, grid, 256, lds, st, a);
    }
    {
        dim3 grid((max_q + 127) / 128, a.Hq, a.nseg);
        const size_t lds = 4 * 64 * D * 2;
        if (D == 128) hipLaunchKernelGGL(fa_bwd_dq_kernel<128>, grid, 256, lds, st, a);
        else if (D == 64) hipLaunchKernelGGL(fa_bwd_dq_kernel<64>, grid, 256, lds, st, a);
        else hipLaunchKernelGGL(fa_bwd_dq_kernel<32>, grid, 256, lds, st, a);
    }
}
}  // namespace sa_launch
