// Host-side launcher declarations shared between the HIP kernel TUs and the torch bindings.
// Kernels take raw pointers + a hipStream_t; bindings.cpp owns all tensor/dtype checking.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

enum SaDType { DT_F32 = 0, DT_BF16 = 1, DT_F16 = 2 };

namespace sa_launch {
// norm.hip
void norm_fwd(int dtype, bool layer, const void* x, const void* w, const void* b, void* y, float* mean, float* rstd,
              int64_t rows, int H, float eps, hipStream_t st, const void* res = nullptr, void* sum_out = nullptr);
int norm_bwd_waves(int64_t rows, int H);
int64_t norm_bwd_scratch(int64_t rows, int H, bool layer);
void norm_bwd(int dtype, bool layer, const void* dy, const void* x, const void* w, const float* mean,
              const float* rstd, void* dx, void* dw, void* db, float* part, int64_t rows, int H, hipStream_t st,
              const void* dadd = nullptr);
}  // namespace sa_launch

namespace sa_launch {
// swiglu_rope.hip
void swiglu_fwd(int dtype, const void* a, const void* b, int64_t lda, void* out, int64_t rows, int F, hipStream_t st);
void swiglu_bwd(int dtype, const void* dy, const void* a, const void* b, int64_t lda, void* da, void* db, int64_t ldd,
                int64_t rows, int F, hipStream_t st);
void rope(int dtype, bool interleaved, const void* x, int64_t x_tok, int64_t x_head, void* out, int64_t o_tok,
          int64_t o_head, const float* cosb, const float* sinb, const int64_t* pos, int64_t T_, int nh, int hd, int rd,
          int seq_len, float sign, hipStream_t st);
// graph decode: RoPE(q) -> q_out, RoPE(k) -> K cache row *pos, v -> V cache row *pos (one token); false = unsupported
// lim = min(cache rows, rotary table rows); a position outside [0, lim) writes nothing but zeros into q and sets *err
bool rope_kv_append(int dtype, bool interleaved, const void* x, void* q_out, void* kc, void* vc, const int64_t* pos,
                    const float* cosb, const float* sinb, int nq, int nkv, int hd, int rd, int64_t lim, int* err,
                    hipStream_t st);
}  // namespace sa_launch

namespace sa_launch {
// xent_embed_optim.hip
void xent_stats(int dtype, const void* logits, const int64_t* tgt, int64_t rows, int V, int64_t v0, float* m, float* s,
                float* t, int64_t* amax, hipStream_t st);
void xent_bwd(int dtype, const void* logits, const int64_t* tgt, const float* lse, const float* gscale, void* dlogits,
              int64_t rows, int V, int64_t v0, hipStream_t st);
void embed_fwd(int dtype, const int64_t* ids, const void* W, void* out, int64_t ntok, int H, int64_t v0, int64_t Vp,
               hipStream_t st);
void embed_bwd(int dtype, const void* dy, const int64_t* order, const int64_t* sid, int64_t ntok, void* dW, int H,
               int64_t v0, int64_t Vp, hipStream_t st);
void adamw(int gdtype, int pdtype, float* p, const void* g, float* m, float* v, void* pout, int64_t n, float lr,
           float b1, float b2, float eps, float wd, float bc1, float bc2_sqrt, float gscale, hipStream_t st);
int sumsq_blocks(int64_t n);
void sumsq(int dtype, const void* x, int64_t n, float scale, float* part_sq, float* part_bad, float* out_sq,
           float* out_bad, int accumulate, hipStream_t st);
void cast_scale(int sdt, int ddt, const void* x, void* y, int64_t n, float scale, hipStream_t st);
bool transpose_supported(int64_t R, int64_t C, int64_t ld_in);
void transpose_u16(const void* in, int64_t ld_in, void* out, int64_t R, int64_t C, hipStream_t st);
}  // namespace sa_launch

namespace sa_launch {
// gemm.hip: C[M, N] (+)= A^T B, A [K, M] / B [K, N] row-major (k-major operands), bf16 (weight gradient)
bool gemm_tn_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc);
int64_t gemm_tn_plan(int64_t M, int64_t N, int64_t K, int slots, int& full_blocks, int& split);
void gemm_tn(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int64_t N,
             int64_t K, bool beta, hipStream_t st, int full_blocks = -1, int split = 1, float* ws = nullptr);
}  // namespace sa_launch

// flash attention (bf16, head dim 32/64/128)
struct FwdArgs {
    const uint16_t* q; const uint16_t* k; const uint16_t* v; uint16_t* o; float* lse;
    int64_t q_tok, q_head, k_tok, k_head, v_tok, v_head, o_tok, o_head, lse_stride;
    const int* cu_q; const int* cu_k;
    int nseg, Hq, Hkv, causal, window;
    int local_heads;  // q heads [0, local_heads) use `window`, the rest attend globally (mixed local/global)
    float scale_log2;
    // attention-probability dropout (p_drop > 0): keep iff mix(seed, q head, q token, k token) >= drop_thr
    float p_drop, rp_drop;  // rp_drop = 1 / (1 - p_drop)
    uint32_t seed, drop_thr;
};
namespace sa_launch {
void fa_fwd(const FwdArgs& a, int D, int max_q, bool f16, hipStream_t st);
}

// flash-decoding (short query segments, GQA rows packed into one wave, split-K + combine)
struct DecArgs {
    const uint16_t* q; const uint16_t* k; const uint16_t* v;
    int64_t q_tok, q_head, k_tok, k_head, v_tok, v_head;
    const int* cu_q; const int* cu_k;
    int nseg, Hq, Hkv, causal, window, local_heads;
    float scale_log2;
    int split_keys, nsplit;
    int64_t Tq;
    float* part_o;   // [nsplit][Tq][Hq][D]
    float* part_ml;  // [nsplit][Tq][Hq][2] running max (log2 units) and sum
    uint16_t* o; int64_t o_tok, o_head;
    float* lse; int64_t lse_stride;
};
namespace sa_launch {
void fa_decode_plan(int64_t max_k, int Hkv, int nseg, int& split_keys, int& nsplit);
void fa_decode(const DecArgs& a, int D, bool f16, hipStream_t st);
}

struct BwdArgs {
    const uint16_t* q; const uint16_t* k; const uint16_t* v; const uint16_t* dO;
    const float* lse; float* delta; float* lse2;
    uint16_t* dq; uint16_t* dk; uint16_t* dv;
    int64_t q_tok, q_head, k_tok, k_head, v_tok, v_head, do_tok, do_head;
    int64_t dq_tok, dq_head, dk_tok, dk_head, dv_tok, dv_head, lse_stride;
    const int* cu_q; const int* cu_k;
    int nseg, Hq, Hkv, causal, window;
    int local_heads;
    float scale, scale_log2;
    float p_drop, rp_drop;
    uint32_t seed, drop_thr;
    // dK/dV GQA head split: hsplit workgroups per (kv head, key block) each sweep grp/hsplit q heads and
    // (hsplit > 1) write fp32 partials [hsplit][Tk][Hkv][D] that fa_bwd_reduce sums (causal load balance)
    int hsplit, Tk;
    float* dk_part;
    float* dv_part;
    // inverse RoPE folded into the dQ / dK epilogues (rcos == nullptr: none): tables [max_pos][rrd / 2], positions
    // rpos[token] or token % rseq, rotary dims rrd (NeoX pairs (i, i + rrd/2) need rrd % 64 == 0), interleaved pairs
    const float* rcos; const float* rsin; const int64_t* rpos;
    int rrd, rseq, ril;
};
namespace sa_launch {
void fa_bwd(const BwdArgs& a, const uint16_t* o, int64_t o_tok, int64_t o_head, int64_t Tq, int D, int max_q, int max_k,
            bool f16, hipStream_t st);
}

namespace sa_launch {
// elementwise.hip: masked softmax, activations, dropout(+residual)
void masked_softmax_fwd(int dtype, const void* x, const void* mask, void* y, int64_t rows, int N, int H, int Sq, int64_t mb,
                        int64_t mh, int64_t mq, float scale, float fill, bool round, hipStream_t st);
void masked_softmax_bwd(int dtype, const void* dy, const void* y, const void* mask, void* dx, int64_t rows, int N, int H,
                        int Sq, int64_t mb, int64_t mh, int64_t mq, float scale, hipStream_t st);
void act_fwd(int dtype, const void* x, void* y, int64_t n, int kind, hipStream_t st);
void act_bwd(int dtype, const void* dy, const void* x, void* dx, int64_t n, int kind, hipStream_t st);
void dropout(int dtype, const void* x, const void* res, void* out, int64_t n, uint32_t seed, uint32_t thr, float rp,
             hipStream_t st);
}  // namespace sa_launch

namespace sa_launch {
// debug: a one-wave busy-wait of `us` microseconds on stream st (elementwise.hip)
void spin(int64_t us, hipStream_t st);
void xgmi_emulate(const void* src, int64_t src_bytes, void* scratch, int64_t scratch_bytes, int64_t bytes, double us,
                  int nwg, hipStream_t st);
// one-shot all-reduce over IPC-mapped peer buffers (oneshot_allreduce.hip)
void oneshot_allreduce(int dtype, char* const* bases, int world, int rank, int64_t slot_off, int64_t flag_off,
                       uint32_t epoch, bool signal, void* out, int64_t n, int* err, int64_t max_spins,
                       hipStream_t st);
}

// gemv.hip epi 3: interleaved RoPE of q / k and the K/V cache append at the device-side position
struct GemvRope {
    const float* cosb; const float* sinb; const int64_t* pos;
    void* q_out; void* kc; void* vc;
    int nq, nkv, hd, rd;
    int64_t lim; int* err;  // position bound (min(cache rows, rotary table rows)); out of range: no write, *err = 1
};
namespace sa_launch {
// gemv.hip: y[M, N] = x[M, K] W[N, K]^T (+ b) for M <= 4 (decode-time linear layers), bf16 / fp16, K % 8 == 0
void gemv(int dtype, int M, const void* x, int64_t ldx, const void* W, int64_t ldw, const void* b, void* y, int64_t ldy,
          int N, int K, hipStream_t st, int epi = 0, const void* res = nullptr, int64_t ldr = 0,
          const void* norm_w = nullptr, const void* norm_add = nullptr, void* norm_sum = nullptr, float eps = 0.f,
          const struct GemvRope* rope = nullptr);
}  // namespace sa_launch
