// Flash-decoding for short query segments (token-by-token generation, speculative / chunked steps) on gfx950.
// The prefill kernels tile 256 query rows per workgroup and walk all keys serially: for one query per segment
// that is 1/256 useful rows and one workgroup per q head.  Here:
//  * GQA packing: the Lq queries of all Hq/Hkv q heads sharing a KV head form the 32 MFMA rows of ONE wave
//    (packed row r -> head r / Lq, query r % Lq), so each K/V row is read once per KV head, not per q head;
//  * split-K: the key range is cut into splits across workgroups (grid split x kv head x segment) so a
//    single decode step fills the chip; each split writes an unnormalised (O, max, sum) partial in fp32 and
//    fa_decode_combine merges them (and writes lse, so the result is interchangeable with the prefill path).
//    (Merging in the last-arriving split instead -- arrival counter, agent-scope acquire/release -- measured
//    45 vs 9.8 + 6.6 us on the 7B decode step: the release writes back L2 in every split);
//  * per split, 32-key tiles: S^T = K Q^T with K fragments loaded straight from global memory (16 B per lane,
//    contiguous rows), online softmax in base 2 with lane-local row statistics (+1 lane^32 exchange), and
//    O^T += V^T P^T with V^T read transposed (ds_read_b64_tr_b16) from a swizzled LDS image of the V tile.
// Causal masking is bottom-right aligned (key <= q + Lk - Lq), sliding windows per head (local_heads) as in
// the prefill kernels.  Rows / keys past their ranges contribute nothing.
#include <algorithm>

#include "flash_attn.h"
#include "launch.h"

using namespace sa;
using namespace sa::fa;

namespace {

// out[token][hq][d] = sum_s 2^(m_s - M) O_s[d] / sum_s 2^(m_s - M) l_s ; lse = (M + log2 L) ln 2 (written for d == 0)
template <int D, bool F16>
__device__ __forceinline__ void merge_dim(const DecArgs& a, int64_t tok, int hq, int d) {
    float M = -INFINITY, L = 0.f, O = 0.f;
    constexpr int R = 16;  // up to R splits: every partial load issued before the first use (one round trip)
    if (a.nsplit <= R) {
        float ms[R], ls[R], os[R];
#pragma unroll
        for (int s = 0; s < R; ++s) {
            const int64_t row = (s * a.Tq + tok) * a.Hq + hq;
            const bool on = s < a.nsplit;
            ms[s] = on ? a.part_ml[2 * row] : -INFINITY;
            ls[s] = on ? a.part_ml[2 * row + 1] : 0.f;
            os[s] = on ? a.part_o[row * D + d] : 0.f;
        }
#pragma unroll
        for (int s = 0; s < R; ++s) M = fmaxf(M, ms[s]);
        if (M != -INFINITY) {
#pragma unroll
            for (int s = 0; s < R; ++s) {
                const float w = ms[s] == -INFINITY ? 0.f : fast_exp2(ms[s] - M);
                L += w * ls[s];
                O += w * os[s];
            }
        }
    } else {
        for (int s = 0; s < a.nsplit; ++s) M = fmaxf(M, a.part_ml[2 * ((s * a.Tq + tok) * a.Hq + hq)]);
        if (M != -INFINITY) {
            for (int s = 0; s < a.nsplit; ++s) {
                const int64_t row = (s * a.Tq + tok) * a.Hq + hq;
                const float ms = a.part_ml[2 * row];
                if (ms == -INFINITY) continue;
                const float w = fast_exp2(ms - M);
                L += w * a.part_ml[2 * row + 1];
                O += w * a.part_o[row * D + d];
            }
        }
    }
    const float out = L > 0.f ? O / L : 0.f;
    a.o[tok * a.o_tok + (int64_t)hq * a.o_head + d] = f2t<F16>(out);
    if (d == 0) a.lse[(int64_t)hq * a.lse_stride + tok] = L > 0.f ? (M + __log2f(L)) * 0.69314718055994530942f : INFINITY;
}

template <int D, bool F16>
__global__ __launch_bounds__(64) void fa_decode_kernel(DecArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
    __shared__ __attribute__((aligned(16))) char vimg[32 * D * 2];
    constexpr int NKS = D / 16, NT = D / 32;
    const int split = blockIdx.x, hk = blockIdx.y, seg = blockIdx.z;
    const int q0s = a.cu_q[seg], k0s = a.cu_k[seg];
    const int Lq = a.cu_q[seg + 1] - q0s, Lk = a.cu_k[seg + 1] - k0s;
    const int grp = a.Hq / a.Hkv;
    const int lane = threadIdx.x, h = lane >> 5, r = lane & 31;
    const int off = Lk - Lq;
    const int g = Lq > 0 ? r / Lq : 0, qi = Lq > 0 ? r % Lq : 0;
    const bool valid = Lq > 0 && r < Lq * grp;
    const int hq = hk * grp + min(g, grp - 1);
    const int win = hq < a.local_heads ? a.window : -1;
    const int k_begin = split * a.split_keys;
    int k_end = min(Lk, k_begin + a.split_keys);
    if (a.causal) k_end = min(k_end, Lq + off);  // beyond the last query's causal bound nothing is visible
    const float c2 = a.scale_log2;

    bf16x8 qf[NKS];
    {
        const u16* qp = a.q + (int64_t)(q0s + (valid ? qi : 0)) * a.q_tok + (int64_t)hq * a.q_head;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const u16x8 v = valid ? *reinterpret_cast<const u16x8*>(qp + 16 * ks + 8 * h) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            qf[ks] = __builtin_bit_cast(bf16x8, v);
        }
    }
    f32x16 o[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) o[t] = f32x16{};
    float m = -INFINITY, l = 0.f;
    const u16* kb = a.k + (int64_t)k0s * a.k_tok + (int64_t)hk * a.k_head;
    const u16* vb = a.v + (int64_t)k0s * a.v_tok + (int64_t)hk * a.v_head;

    for (int kt = k_begin; kt < k_end; kt += 32) {
        // K rows (A operand: key kt + r, dims 16 ks + 8 h) and the V tile are all issued before anything waits on
        // them: one memory round trip per tile instead of V, then K
        const bool krow = kt + r < k_end;
        const u16* kp = kb + (int64_t)(krow ? kt + r : kt) * a.k_tok;
        u16x8 kv[NKS];
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
            kv[ks] = krow ? *reinterpret_cast<const u16x8*>(kp + 16 * ks + 8 * h) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        // V tile [32][D] -> swizzled LDS image (rows past k_end as zeros)
        constexpr int PASSES = 32 * D / 8 / 64;
        u16x8 vv[PASSES];
#pragma unroll
        for (int p = 0; p < PASSES; ++p) {
            const int id = lane + 64 * p, row = id / (D / 8), c = id % (D / 8);
            vv[p] = kt + row < k_end ? *reinterpret_cast<const u16x8*>(vb + (int64_t)(kt + row) * a.v_tok + c * 8)
                                     : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
        // S^T = K Q^T
        f32x16 s = f32x16{};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) s = mma<F16>(__builtin_bit_cast(bf16x8, kv[ks]), qf[ks], s);
#pragma unroll
        for (int p = 0; p < PASSES; ++p) {
            const int id = lane + 64 * p, row = id / (D / 8), c = id % (D / 8);
            *reinterpret_cast<u16x8*>(vimg + row * D * 2 + 16 * swz<D>(row, c)) = vv[p];
        }
        // scale + mask; key of register j: kt + crow(j) + 4h
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int key = kt + crow(j) + 4 * h;
            bool ok = valid && key < k_end;
            if (a.causal) ok = ok && key <= qi + off;
            if (win >= 0) ok = ok && key >= qi + off - win && (a.causal || key <= qi + off + win);
            const float x = ok ? s[j] * c2 : -INFINITY;
            s[j] = x;
            mx = fmaxf(mx, x);
        }
        mx = max_xchg32(mx);
        const float mnew = fmaxf(m, mx);
        const float msafe = mnew == -INFINITY ? 0.f : mnew;
        const float alpha = fast_exp2(m - msafe);
        float rs = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const float p = fast_exp2(s[j] - msafe);
            s[j] = p;
            rs += p;
        }
        l = l * alpha + sum_xchg32(rs);
        m = mnew;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int j = 0; j < 16; ++j) o[t][j] *= alpha;
        __syncthreads();  // V image complete
        const bf16x8 p0 = pack_acc_t<F16>(s, 0), p1 = pack_acc_t<F16>(s, 1);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            o[t] = mma<F16>(ld_tr<D>(vimg, 0, 32 * t), p0, o[t]);
            o[t] = mma<F16>(ld_tr<D>(vimg, 16, 32 * t), p1, o[t]);
        }
        __syncthreads();  // before the next tile overwrites the image
    }
    if (valid) {
        const int64_t row = ((int64_t)split * a.Tq + q0s + qi) * a.Hq + hq;
        float* po = a.part_o + row * D;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int j = 0; j < 16; ++j) po[32 * t + crow(j) + 4 * h] = o[t][j];
        if (h == 0) {
            a.part_ml[2 * row] = m;
            a.part_ml[2 * row + 1] = l;
        }
    }
#endif
}

template <int D, bool F16>
__global__ __launch_bounds__(D) void fa_decode_combine_kernel(DecArgs a) {
    merge_dim<D, F16>(a, blockIdx.x, blockIdx.y, threadIdx.x);
}

template <int D, bool F16>
void launch(const DecArgs& a, int nseg, hipStream_t st) {
    hipLaunchKernelGGL((fa_decode_kernel<D, F16>), dim3(a.nsplit, a.Hkv, nseg), dim3(64), 0, st, a);
    hipLaunchKernelGGL((fa_decode_combine_kernel<D, F16>), dim3((unsigned)a.Tq, a.Hq), dim3(D), 0, st, a);
}

}  // namespace

namespace sa_launch {
// splits so that split x kv head x segment workgroups fill the chip; split length a multiple of the 32-key tile
void fa_decode_plan(int64_t max_k, int Hkv, int nseg, int& split_keys, int& nsplit) {
    const int64_t want = std::max<int64_t>(1, (1024 + (int64_t)Hkv * nseg - 1) / ((int64_t)Hkv * nseg));
    const int64_t tiles = std::max<int64_t>(1, (max_k + 31) / 32);
    // one 32-key tile per split while that still leaves <= `want` splits: a decode step is a latency chain of
    // (load K/V tile -> MFMA -> softmax -> MFMA) per tile, so short contexts want the tiles side by side
    const int64_t per = std::max<int64_t>(1, (tiles + want - 1) / want);
    split_keys = (int)(per * 32);
    nsplit = (int)std::max<int64_t>(1, (max_k + split_keys - 1) / split_keys);
}
void fa_decode(const DecArgs& a, int D, bool f16, hipStream_t st) {
    const int nseg = a.nseg;
    if (f16) {
        if (D == 128) launch<128, true>(a, nseg, st);
        else if (D == 64) launch<64, true>(a, nseg, st);
        else launch<32, true>(a, nseg, st);
    } else {
        if (D == 128) launch<128, false>(a, nseg, st);
        else if (D == 64) launch<64, false>(a, nseg, st);
        else launch<32, false>(a, nseg, st);
    }
}
}  // namespace sa_launch
