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

template <int D>
__global__ __launch_bounds__(256, 2) void fa_fwd_kernel(FwdArgs a) {
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
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, lq = lane & 31;
    const int off = Lk - Lq;  // bottom-right causal alignment
    const int qwg0 = qt * 128;
    const int qw0 = qwg0 + wave * 32;
    const int myq = qw0 + lq;

    // key range for the workgroup
    const int qlast = min(qwg0 + 127, Lq - 1);
    int khi = Lk;
    if (a.causal) khi = min(Lk, qlast + off + 1);
    else if (a.window >= 0) khi = min(Lk, qlast + off + a.window + 1);
    int klo = 0;
    if (a.window >= 0) klo = max(0, qwg0 + off - a.window);
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
            for (int b = 0; b < 2; ++b) s[b] = mfma(ld_row<D>(K, 32 * b + lq, 16 * ks + 8 * h), qf[ks], s[b]);
        }
        // ---- scale + mask (mask only on boundary tiles; wave-uniform decision)
        const bool need_mask = (kt + 64 > Lk) || (a.causal && kt + 63 > qw0 + off) ||
                               (a.window >= 0 && (kt < qw0 + 31 + off - a.window || (!a.causal && kt + 63 > qw0 + off + a.window)));
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
                    if (a.window >= 0) ok = ok && key >= myq + off - a.window && (a.causal || key <= myq + off + a.window);
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
#pragma unroll
        for (int t = 0; t < D / 32; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
        // ---- O^T += V^T P^T
        bf16x8 pf[2][2];
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) pf[b][ss] = pack_acc(s[b], ss);
#pragma unroll
        for (int t = 0; t < D / 32; ++t)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) o[t] = mfma(ld_tr<D>(V, 32 * b + 16 * ss, 32 * t), pf[b][ss], o[t]);
        if (has_next) {
            sk.store(smem + 2 * (cur ^ 1) * TILE);
            sv.store(smem + (2 * (cur ^ 1) + 1) * TILE);
        }
        __syncthreads();
        cur ^= 1;
    }
    // ---- epilogue: O = O^T / l, lse = (m + log2 l) * ln2
    if (myq < Lq) {
        const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
        u16* op = a.o + (int64_t)(q0s + myq) * a.o_tok + (int64_t)hq * a.o_head;
#pragma unroll
        for (int t = 0; t < D / 32; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                u16x4 w;
#pragma unroll
                for (int j = 0; j < 4; ++j) w[j] = f2bf(o[t][4 * g + j] * inv);
                *reinterpret_cast<u16x4*>(op + 32 * t + 8 * g + 4 * h) = w;
            }
        if (h == 0) a.lse[(int64_t)hq * a.lse_stride + q0s + myq] = lsum > 0.f ? (m + __log2f(lsum)) * 0.69314718055994530942f : INFINITY;
    }
}

namespace sa_launch {
void fa_fwd(const FwdArgs& a, int D, int max_q, hipStream_t st) {
    dim3 grid((max_q + 127) / 128, a.Hq, a.nseg), block(256);
    const size_t lds = 4 * 64 * D * 2;
    if (D == 128) hipLaunchKernelGGL(fa_fwd_kernel<128>, grid, block, lds, st, a);
    else if (D == 64) hipLaunchKernelGGL(fa_fwd_kernel<64>, grid, block, lds, st, a);
    else hipLaunchKernelGGL(fa_fwd_kernel<32>, grid, block, lds, st, a);
}
}  // namespace sa_launch
