// torch bindings for the scaling_amd HIP kernels (module scaling_amd._C).
// All tensor/dtype/shape validation lives here; kernels see raw pointers and the current HIP stream.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>

#include <atomic>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>
#include "kernels/launch.h"

void register_rehearsal(pybind11::module& m);  // rehearsal.cpp: asynchronous rehearsal worker
void register_blaslt(pybind11::module& m);     // blaslt.cpp: small GEMMs through cached hipBLASLt plans

namespace {

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

int dt(const at::Tensor& t) {
    switch (t.scalar_type()) {
        case at::kFloat: return DT_F32;
        case at::kBFloat16: return DT_BF16;
        case at::kHalf: return DT_F16;
        default: TORCH_CHECK(false, "scaling_amd: unsupported dtype ", t.scalar_type());
    }
    return -1;
}

void check_cuda(const at::Tensor& t, const char* name) {
    TORCH_CHECK(t.is_cuda(), "scaling_amd: ", name, " must be a GPU tensor");
    TORCH_CHECK(t.is_contiguous(), "scaling_amd: ", name, " must be contiguous");
}

// ------------------------------------------------------------------ norms
// res given: normalises s = x + res and also returns s (fused residual add)
std::vector<at::Tensor> norm_fwd(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& b,
                                 double eps, bool layer, const c10::optional<at::Tensor>& res) {
    check_cuda(x, "x");
    check_cuda(w, "weight");
    const int64_t H = x.size(-1);
    TORCH_CHECK(H % 8 == 0, "norm: hidden size must be a multiple of 8");
    TORCH_CHECK(w.numel() == H && w.scalar_type() == x.scalar_type(), "norm: weight shape/dtype mismatch");
    const int64_t rows = x.numel() / H;
    const at::DeviceGuard g(x.device());
    auto y = at::empty_like(x);
    auto opts = x.options().dtype(at::kFloat);
    auto rstd = at::empty({rows}, opts);
    auto mean = layer ? at::empty({rows}, opts) : at::empty({0}, opts);
    const void* bp = nullptr;
    if (layer) {
        TORCH_CHECK(b.has_value(), "layernorm needs a bias");
        check_cuda(*b, "bias");
        bp = b->data_ptr();
    }
    at::Tensor sum = at::empty({0}, x.options());
    const void* rp = nullptr;
    if (res.has_value()) {
        check_cuda(*res, "residual");
        TORCH_CHECK(res->sizes() == x.sizes() && res->scalar_type() == x.scalar_type(), "norm: residual mismatch");
        sum = at::empty_like(x);
        rp = res->data_ptr();
    }
    sa_launch::norm_fwd(dt(x), layer, x.data_ptr(), w.data_ptr(), bp, y.data_ptr(),
                        layer ? mean.data_ptr<float>() : nullptr, rstd.data_ptr<float>(), rows, (int)H, (float)eps,
                        cur_stream(), rp, rp ? sum.data_ptr() : nullptr);
    return {y, mean, rstd, sum};
}

// dadd given: dx = norm_bwd(dy) + dadd (fused residual-gradient add)
std::vector<at::Tensor> norm_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w,
                                 const at::Tensor& mean, const at::Tensor& rstd, bool layer,
                                 const c10::optional<at::Tensor>& dadd) {
    check_cuda(dy, "dy");
    check_cuda(x, "x");
    const int64_t H = x.size(-1);
    const int64_t rows = x.numel() / H;
    const at::DeviceGuard g(x.device());
    auto dx = at::empty_like(x);
    auto dw = at::empty_like(w);
    auto db = layer ? at::empty_like(w) : at::empty({0}, w.options());
    auto part = at::empty({sa_launch::norm_bwd_scratch(rows, (int)H, layer)}, x.options().dtype(at::kFloat));
    const void* ap = nullptr;
    if (dadd.has_value()) {
        check_cuda(*dadd, "dadd");
        TORCH_CHECK(dadd->is_contiguous() && dadd->numel() == x.numel() && dadd->scalar_type() == x.scalar_type(),
                    "norm_bwd: dadd mismatch");
        ap = dadd->data_ptr();
    }
    sa_launch::norm_bwd(dt(x), layer, dy.data_ptr(), x.data_ptr(), w.data_ptr(),
                        layer ? mean.data_ptr<float>() : nullptr, rstd.data_ptr<float>(), dx.data_ptr(),
                        dw.data_ptr(), layer ? db.data_ptr() : nullptr, part.data_ptr<float>(), rows, (int)H,
                        cur_stream(), ap);
    return {dx, dw, db};
}

// ------------------------------------------------------------------ swiglu
// z: [..., 2F] (a | b halves) or separate a/b with equal row stride
at::Tensor swiglu_fwd(const at::Tensor& a, const at::Tensor& b) {
    TORCH_CHECK(a.is_cuda() && b.is_cuda(), "swiglu: GPU tensors required");
    TORCH_CHECK(a.sizes() == b.sizes() && a.stride(-1) == 1 && b.stride(-1) == 1 && a.stride(-2) == b.stride(-2),
                "swiglu: a/b must share shape and row stride");
    const int64_t F = a.size(-1);
    TORCH_CHECK(F % 8 == 0, "swiglu: feature size must be a multiple of 8");
    const int64_t rows = a.numel() / F;
    const at::DeviceGuard g(a.device());
    auto out = at::empty(a.sizes(), a.options());
    sa_launch::swiglu_fwd(dt(a), a.data_ptr(), b.data_ptr(), a.stride(-2), out.data_ptr(), rows, (int)F, cur_stream());
    return out;
}
std::vector<at::Tensor> swiglu_bwd(const at::Tensor& dy, const at::Tensor& a, const at::Tensor& b, bool fused_out) {
    const int64_t F = a.size(-1);
    const int64_t rows = a.numel() / F;
    const at::DeviceGuard g(a.device());
    auto dyc = dy.contiguous();
    if (fused_out) {
        auto sizes = a.sizes().vec();
        sizes.back() = 2 * F;
        auto dz = at::empty(sizes, a.options());
        sa_launch::swiglu_bwd(dt(a), dyc.data_ptr(), a.data_ptr(), b.data_ptr(), a.stride(-2), dz.data_ptr(),
                              (char*)dz.data_ptr() + F * dz.element_size(), 2 * F, rows, (int)F, cur_stream());
        return {dz};
    }
    auto da = at::empty(a.sizes(), a.options());
    auto db = at::empty(a.sizes(), a.options());
    sa_launch::swiglu_bwd(dt(a), dyc.data_ptr(), a.data_ptr(), b.data_ptr(), a.stride(-2), da.data_ptr(), db.data_ptr(),
                          F, rows, (int)F, cur_stream());
    return {da, db};
}

// ------------------------------------------------------------------ rope
// x: [T, nh, hd] (any token/head stride, unit element stride) -> out (given: same shape, any strides, may be x
// itself for an in-place rotation; else a new contiguous [T, nh, hd])
at::Tensor rope(const at::Tensor& x, const at::Tensor& cosb, const at::Tensor& sinb, const c10::optional<at::Tensor>& pos,
                int64_t rot_dim, int64_t seq_len, bool interleaved, bool inverse, const c10::optional<at::Tensor>& out_) {
    TORCH_CHECK(x.is_cuda() && x.dim() == 3 && x.stride(2) == 1, "rope: x must be [T, nh, hd] with unit last stride");
    TORCH_CHECK(cosb.scalar_type() == at::kFloat && cosb.is_contiguous() && sinb.is_contiguous(), "rope: fp32 tables");
    const int64_t T = x.size(0), nh = x.size(1), hd = x.size(2);
    TORCH_CHECK(rot_dim % 2 == 0 && rot_dim <= hd && cosb.size(-1) == rot_dim / 2, "rope: bad rotary dims");
    const at::DeviceGuard g(x.device());
    at::Tensor out;
    if (out_.has_value()) {
        out = *out_;
        TORCH_CHECK(out.sizes() == x.sizes() && out.stride(2) == 1 && out.scalar_type() == x.scalar_type(),
                    "rope: out must match x with unit last stride");
        TORCH_CHECK(out.data_ptr() == x.data_ptr() ? out.strides() == x.strides() : true,
                    "rope: in-place output must have the input's strides");
    } else {
        out = at::empty({T, nh, hd}, x.options());
    }
    const int64_t* pp = nullptr;
    at::Tensor pc;
    if (pos.has_value()) {
        pc = pos->to(at::kLong).contiguous();
        TORCH_CHECK(pc.numel() == T, "rope: position ids must have one entry per token");
        pp = pc.data_ptr<int64_t>();
    }
    sa_launch::rope(dt(x), interleaved, x.data_ptr(), x.stride(0), x.stride(1), out.data_ptr(), out.stride(0),
                    out.stride(1), cosb.data_ptr<float>(), sinb.data_ptr<float>(), pp, T, (int)nh, (int)hd,
                    (int)rot_dim, (int)seq_len, inverse ? -1.f : 1.f, cur_stream());
    return out;
}

// graph decode: q = RoPE(q heads) (returned), K cache[pos] = RoPE(k heads), V cache[pos] = v heads, one launch;
// qkv: the projection row [1, nq + 2 nkv, hd] (contiguous), caches [cap, nkv, hd] (contiguous), pos [1] int64
static bool err_word(const at::Tensor& e) {
    return e.is_cuda() && e.scalar_type() == at::kInt && e.numel() >= 1;
}
c10::optional<at::Tensor> rope_kv_append(const at::Tensor& qkv, const at::Tensor& cosb, const at::Tensor& sinb,
                                         const at::Tensor& pos, int64_t nq, int64_t nkv, int64_t rot_dim, bool interleaved,
                                         at::Tensor kc, at::Tensor vc, at::Tensor err) {
    TORCH_CHECK(err_word(err), "rope_kv_append: err must be an int32 GPU tensor");
    check_cuda(qkv, "qkv");
    const int64_t hd = qkv.size(-1);
    if (!(qkv.is_contiguous() && qkv.numel() == (nq + 2 * nkv) * hd && kc.is_contiguous() && vc.is_contiguous() &&
          kc.dim() == 3 && kc.size(1) == nkv && kc.size(2) == hd && vc.sizes() == kc.sizes() &&
          kc.scalar_type() == qkv.scalar_type() && vc.scalar_type() == qkv.scalar_type() && pos.is_cuda() &&
          pos.scalar_type() == at::kLong && pos.numel() == 1 && cosb.scalar_type() == at::kFloat &&
          cosb.is_contiguous() && sinb.is_contiguous() && cosb.size(-1) == rot_dim / 2 &&
          (uintptr_t)qkv.data_ptr() % 16 == 0 && (uintptr_t)kc.data_ptr() % 16 == 0 && (uintptr_t)vc.data_ptr() % 16 == 0))
        return c10::nullopt;
    const at::DeviceGuard g(qkv.device());
    auto q = at::empty({1, nq, hd}, qkv.options());
    if (!sa_launch::rope_kv_append(dt(qkv), interleaved, qkv.data_ptr(), q.data_ptr(), kc.data_ptr(), vc.data_ptr(),
                                   pos.data_ptr<int64_t>(), cosb.data_ptr<float>(), sinb.data_ptr<float>(), (int)nq,
                                   (int)nkv, (int)hd, (int)rot_dim, std::min<int64_t>(kc.size(0), cosb.size(0)),
                                   err.data_ptr<int>(), cur_stream()))
        return c10::nullopt;
    return q;
}

// ------------------------------------------------------------------ cross entropy
std::vector<at::Tensor> xent_stats(const at::Tensor& logits, const at::Tensor& target, int64_t v0) {
    check_cuda(logits, "logits");
    const int64_t V = logits.size(-1), rows = logits.numel() / V;
    const at::DeviceGuard g(logits.device());
    auto t = target.to(at::kLong).contiguous();
    auto fo = logits.options().dtype(at::kFloat);
    auto m = at::empty({rows}, fo), s = at::empty({rows}, fo), tl = at::empty({rows}, fo);
    auto am = at::empty({rows}, logits.options().dtype(at::kLong));
    sa_launch::xent_stats(dt(logits), logits.data_ptr(), t.data_ptr<int64_t>(), rows, (int)V, v0, m.data_ptr<float>(),
                          s.data_ptr<float>(), tl.data_ptr<float>(), am.data_ptr<int64_t>(), cur_stream());
    return {m, s, tl, am};
}
at::Tensor xent_bwd(const at::Tensor& logits, const at::Tensor& target, const at::Tensor& lse, const at::Tensor& gscale,
                    int64_t v0, bool inplace) {
    check_cuda(logits, "logits");
    const int64_t V = logits.size(-1), rows = logits.numel() / V;
    const at::DeviceGuard g(logits.device());
    auto t = target.to(at::kLong).contiguous();
    auto out = inplace ? logits : at::empty_like(logits);
    sa_launch::xent_bwd(dt(logits), logits.data_ptr(), t.data_ptr<int64_t>(), lse.data_ptr<float>(),
                        gscale.data_ptr<float>(), out.data_ptr(), rows, (int)V, v0, cur_stream());
    return out;
}

// ------------------------------------------------------------------ embedding
at::Tensor embed_fwd(const at::Tensor& ids, const at::Tensor& W, int64_t v0) {
    check_cuda(W, "weight");
    const int64_t H = W.size(1);
    TORCH_CHECK(H % 8 == 0, "embedding: hidden size must be a multiple of 8");
    const at::DeviceGuard g(W.device());
    auto idc = ids.to(at::kLong).contiguous();
    auto sizes = idc.sizes().vec();
    sizes.push_back(H);
    auto out = at::empty(sizes, W.options());
    sa_launch::embed_fwd(dt(W), idc.data_ptr<int64_t>(), W.data_ptr(), out.data_ptr(), idc.numel(), (int)H, v0,
                         W.size(0), cur_stream());
    return out;
}
at::Tensor embed_bwd(const at::Tensor& dy, const at::Tensor& ids, int64_t num_rows, int64_t v0) {
    const int64_t H = dy.size(-1);
    const at::DeviceGuard g(dy.device());
    auto idc = ids.to(at::kLong).reshape({-1});
    auto sorted = at::sort(idc, /*stable=*/true, /*dim=*/0, /*descending=*/false);
    auto sid = std::get<0>(sorted).contiguous();
    auto order = std::get<1>(sorted).contiguous();
    auto dW = at::zeros({num_rows, H}, dy.options());
    auto dyc = dy.contiguous();
    sa_launch::embed_bwd(dt(dyc), dyc.data_ptr(), order.data_ptr<int64_t>(), sid.data_ptr<int64_t>(), sid.numel(),
                         dW.data_ptr(), (int)H, v0, num_rows, cur_stream());
    return dW;
}

// ------------------------------------------------------------------ optimizer
void adamw_(at::Tensor p, const at::Tensor& grad, at::Tensor m, at::Tensor v, c10::optional<at::Tensor> pout, double lr,
            double b1, double b2, double eps, double wd, int64_t step, double gscale) {
    TORCH_CHECK(p.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat,
                "adamw: fp32 master/state");
    TORCH_CHECK(p.is_contiguous() && grad.is_contiguous() && m.is_contiguous() && v.is_contiguous(), "adamw: contiguous");
    TORCH_CHECK(p.numel() == grad.numel() && p.numel() == m.numel() && p.numel() == v.numel(), "adamw: sizes");
    const at::DeviceGuard g(p.device());
    void* po = nullptr;
    int pdt = DT_F32;
    if (pout.has_value() && pout->defined()) {
        TORCH_CHECK(pout->numel() == p.numel() && pout->is_contiguous(), "adamw: param out");
        po = pout->data_ptr();
        pdt = dt(*pout);
    }
    const double bc1 = 1.0 - std::pow(b1, (double)step);
    const double bc2 = 1.0 - std::pow(b2, (double)step);
    sa_launch::adamw(dt(grad), pdt, p.data_ptr<float>(), grad.data_ptr(), m.data_ptr<float>(), v.data_ptr<float>(), po,
                     p.numel(), (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (float)bc1,
                     (float)std::sqrt(bc2), (float)gscale, cur_stream());
}
// accumulates (sum of squares, count of non-finite) of x*scale into out[0], out[1] (fp32, on device)
void sumsq_(const at::Tensor& x, at::Tensor out, double scale, bool accumulate) {
    TORCH_CHECK(x.is_contiguous() && out.scalar_type() == at::kFloat && out.numel() >= 2, "sumsq: bad args");
    const at::DeviceGuard g(x.device());
    const int nb = sa_launch::sumsq_blocks(x.numel());
    auto part = at::empty({2 * nb}, out.options());
    float* o = out.data_ptr<float>();
    sa_launch::sumsq(dt(x), x.data_ptr(), x.numel(), (float)scale, part.data_ptr<float>(), part.data_ptr<float>() + nb,
                     o, o + 1, accumulate ? 1 : 0, cur_stream());
}
void cast_scale_(const at::Tensor& x, at::Tensor y, double scale) {
    TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && x.numel() == y.numel(), "cast_scale: bad args");
    const at::DeviceGuard g(x.device());
    sa_launch::cast_scale(dt(x), dt(y), x.data_ptr(), y.data_ptr(), x.numel(), (float)scale, cur_stream());
}

// ------------------------------------------------------------------ one-shot all-reduce (IPC peer buffers)
// registered buffer: [slot 0 | slot 1 | flag row]; returns (device address, IPC handle bytes)
py::tuple ar_alloc(int64_t nbytes, int64_t device) {
    TORCH_CHECK(nbytes > 0, "ar_alloc: size");
    TORCH_CHECK(hipSetDevice((int)device) == hipSuccess, "ar_alloc: hipSetDevice");
    void* p = nullptr;
    TORCH_CHECK(hipMalloc(&p, (size_t)nbytes) == hipSuccess, "ar_alloc: hipMalloc failed");
    TORCH_CHECK(hipMemset(p, 0, (size_t)nbytes) == hipSuccess, "ar_alloc: hipMemset failed");
    hipIpcMemHandle_t h;
    TORCH_CHECK(hipIpcGetMemHandle(&h, p) == hipSuccess, "ar_alloc: hipIpcGetMemHandle failed");
    return py::make_tuple((int64_t)reinterpret_cast<uintptr_t>(p), py::bytes(reinterpret_cast<const char*>(&h), sizeof(h)));
}
int64_t ar_open(const std::string& handle, int64_t device) {
    TORCH_CHECK(handle.size() == sizeof(hipIpcMemHandle_t), "ar_open: bad handle size");
    TORCH_CHECK(hipSetDevice((int)device) == hipSuccess, "ar_open: hipSetDevice");
    hipIpcMemHandle_t h;
    memcpy(&h, handle.data(), sizeof(h));
    void* p = nullptr;
    TORCH_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) == hipSuccess, "ar_open: hipIpcOpenMemHandle failed");
    return (int64_t)reinterpret_cast<uintptr_t>(p);
}
void ar_close(int64_t ptr) { (void)hipIpcCloseMemHandle(reinterpret_cast<void*>((uintptr_t)ptr)); }
void ar_free(int64_t ptr) { (void)hipFree(reinterpret_cast<void*>((uintptr_t)ptr)); }
// x (+)= sum over ranks, in place; x is first copied into this rank's slot `slot_off`
void ar_allreduce(at::Tensor x, const std::vector<int64_t>& bases, int64_t rank, int64_t slot_off, int64_t flag_off,
                  int64_t epoch, bool signal, at::Tensor err, int64_t max_spins) {
    check_cuda(x, "x");
    TORCH_CHECK(x.is_contiguous(), "ar_allreduce: contiguous input");
    TORCH_CHECK(bases.size() >= 1 && bases.size() <= 8 && rank >= 0 && rank < (int64_t)bases.size(), "ar_allreduce: ranks");
    const int vec = x.scalar_type() == at::kFloat ? 4 : 8;
    TORCH_CHECK(x.numel() % vec == 0, "ar_allreduce: numel must be a multiple of the vector width");
    TORCH_CHECK(err.is_cuda() && err.scalar_type() == at::kInt, "ar_allreduce: err must be a cuda int32 tensor");
    const at::DeviceGuard g(x.device());
    char* own = reinterpret_cast<char*>((uintptr_t)bases[rank]) + slot_off;
    TORCH_CHECK(hipMemcpyAsync(own, x.data_ptr(), x.nbytes(), hipMemcpyDeviceToDevice, cur_stream()) == hipSuccess,
                "ar_allreduce: slot copy");
    std::vector<char*> b(bases.size());
    for (size_t i = 0; i < bases.size(); ++i) b[i] = reinterpret_cast<char*>((uintptr_t)bases[i]);
    sa_launch::oneshot_allreduce(dt(x), b.data(), (int)bases.size(), (int)rank, slot_off, flag_off, (uint32_t)epoch,
                                 signal, x.data_ptr(), x.numel(), err.data_ptr<int>(), max_spins, cur_stream());
}

// ------------------------------------------------------------------ transpose (dgrad weight cache)
// out = x^T for a 2-D bf16 / fp16 matrix with unit inner stride (R, C multiples of 64); returns false if the
// operands are not supported so the caller can fall back
bool transpose_ok(const at::Tensor& x) {
    return x.is_cuda() && x.dim() == 2 && x.element_size() == 2 && x.stride(1) == 1 &&
           (uintptr_t)x.data_ptr() % 16 == 0 && sa_launch::transpose_supported(x.size(0), x.size(1), x.stride(0));
}
at::Tensor transpose2d(const at::Tensor& x) {
    TORCH_CHECK(transpose_ok(x), "transpose2d: 2-byte 2-D cuda tensor, unit inner stride, dims multiple of 64");
    const at::DeviceGuard g(x.device());
    auto out = at::empty({x.size(1), x.size(0)}, x.options());
    sa_launch::transpose_u16(x.data_ptr(), x.stride(0), out.data_ptr(), x.size(0), x.size(1), cur_stream());
    return out;
}

// ------------------------------------------------------------------ GEMV (decode-time linear layers)
// y[M, N] = x[M, K] W[N, K]^T (+ b), M <= 4, bf16 / fp16, unit inner strides, 16-B aligned rows
bool gemv_ok(const at::Tensor& x, const at::Tensor& W) {
    if (!(x.is_cuda() && W.is_cuda() && x.dim() == 2 && W.dim() == 2)) return false;
    if (x.scalar_type() != W.scalar_type() || (x.scalar_type() != at::kBFloat16 && x.scalar_type() != at::kHalf))
        return false;
    if (x.size(0) < 1 || x.size(0) > 4 || x.size(1) != W.size(1) || x.size(1) % 8 != 0 || W.size(0) < 1) return false;
    if (x.stride(1) != 1 || W.stride(1) != 1 || (x.size(0) > 1 && x.stride(0) % 8 != 0) || W.stride(0) % 8 != 0)
        return false;
    return (uintptr_t)x.data_ptr() % 16 == 0 && (uintptr_t)W.data_ptr() % 16 == 0;
}
at::Tensor gemv(const at::Tensor& x, const at::Tensor& W, c10::optional<at::Tensor> bias) {
    TORCH_CHECK(gemv_ok(x, W), "gemv: unsupported operands (x [M<=4, K], W [N, K], bf16/fp16, K % 8 == 0, aligned)");
    const at::DeviceGuard g(x.device());
    const int64_t M = x.size(0), N = W.size(0), K = W.size(1);
    const void* bp = nullptr;
    at::Tensor bc;
    if (bias.has_value() && bias->defined()) {
        TORCH_CHECK(bias->numel() == N && bias->scalar_type() == W.scalar_type(), "gemv: bias");
        bc = bias->contiguous();
        bp = bc.data_ptr();
    }
    auto y = at::empty({M, N}, x.options());
    sa_launch::gemv(dt(x), (int)M, x.data_ptr(), x.stride(0), W.data_ptr(), W.stride(0), bp, y.data_ptr(), N, (int)N,
                    (int)K, cur_stream());
    return y;
}
// decode epilogues: y = rnd(x W^T) + res  (res [M, N]) ...
at::Tensor gemv_residual(const at::Tensor& x, const at::Tensor& W, const at::Tensor& res) {
    TORCH_CHECK(gemv_ok(x, W), "gemv_residual: unsupported operands");
    const int64_t M = x.size(0), N = W.size(0), K = W.size(1);
    TORCH_CHECK(res.is_cuda() && res.dim() == 2 && res.size(0) == M && res.size(1) == N && res.stride(1) == 1 &&
                    res.scalar_type() == x.scalar_type(), "gemv_residual: res must be [M, N] of the input dtype");
    const at::DeviceGuard g(x.device());
    auto y = at::empty({M, N}, x.options());
    sa_launch::gemv(dt(x), (int)M, x.data_ptr(), x.stride(0), W.data_ptr(), W.stride(0), nullptr, y.data_ptr(), N, (int)N,
                    (int)K, cur_stream(), 1, res.data_ptr(), res.stride(0));
    return y;
}
// ... and SwiGLU over W = [gate; up] ([2F, K]): y[:, n] = silu(x W_gate^T)[n] * (x W_up^T)[n], rounded as gemv + swiglu
at::Tensor gemv_swiglu(const at::Tensor& x, const at::Tensor& W) {
    TORCH_CHECK(gemv_ok(x, W) && W.size(0) % 2 == 0, "gemv_swiglu: unsupported operands");
    const int64_t M = x.size(0), F = W.size(0) / 2, K = W.size(1);
    const at::DeviceGuard g(x.device());
    auto y = at::empty({M, F}, x.options());
    sa_launch::gemv(dt(x), (int)M, x.data_ptr(), x.stride(0), W.data_ptr(), W.stride(0), nullptr, y.data_ptr(), F, (int)F,
                    (int)K, cur_stream(), 2, nullptr, 0);
    return y;
}
// ... with the RMSNorm in front fused into the same pass: s = x (+ add); y = gemv(rms_norm(s, gamma, eps), W) with
// epi 0 (plain) or 2 (SwiGLU over [gate; up]), the normalised row kept in fp32; returns (s, y), s written by the
// kernel when add is given
bool gemv_norm_ok(const at::Tensor& x, const at::Tensor& W, const at::Tensor& gamma) {
    if (!gemv_ok(x, W) || !x.is_contiguous()) return false;
    if (!(gamma.is_cuda() && gamma.dim() == 1 && gamma.numel() == x.size(1) && gamma.is_contiguous() &&
          gamma.scalar_type() == x.scalar_type() && (uintptr_t)gamma.data_ptr() % 16 == 0))
        return false;
    return true;
}
std::vector<at::Tensor> gemv_norm(const at::Tensor& x, c10::optional<at::Tensor> add, const at::Tensor& gamma,
                                  double eps, const at::Tensor& W, int64_t epi) {
    TORCH_CHECK(gemv_norm_ok(x, W, gamma) && (epi == 0 || (epi == 2 && W.size(0) % 2 == 0)),
                "gemv_norm: unsupported operands");
    const int64_t M = x.size(0), K = W.size(1), N = epi == 2 ? W.size(0) / 2 : W.size(0);
    const at::DeviceGuard g(x.device());
    at::Tensor s = x;
    const void* ap = nullptr;
    if (add.has_value() && add->defined()) {
        TORCH_CHECK(add->sizes() == x.sizes() && add->is_contiguous() && add->scalar_type() == x.scalar_type() &&
                        (uintptr_t)add->data_ptr() % 16 == 0, "gemv_norm: add must be a contiguous, aligned [M, K]");
        s = at::empty_like(x);
        ap = add->data_ptr();
    }
    auto y = at::empty({M, N}, x.options());
    sa_launch::gemv(dt(x), (int)M, x.data_ptr(), x.stride(0), W.data_ptr(), W.stride(0), nullptr, y.data_ptr(), N, (int)N,
                    (int)K, cur_stream(), (int)epi, nullptr, 0, gamma.data_ptr(), ap, ap ? s.data_ptr() : nullptr,
                    (float)eps);
    return {s, y};
}
// graph-decode q/k/v step in ONE launch: q = RoPE(rms_norm(x) Wq^T) is returned, RoPE(rms_norm(x) Wk^T) and
// rms_norm(x) Wv^T are written into the K / V cache rows at the device-side position pos (interleaved rotary pairs,
// rotary dims rd of hd; x one token).  None when the operands do not fit (the caller runs gemv_norm + rope_kv_append).
c10::optional<at::Tensor> gemv_norm_rope(const at::Tensor& x, const at::Tensor& gamma, double eps, const at::Tensor& W,
                                         const at::Tensor& cosb, const at::Tensor& sinb, const at::Tensor& pos,
                                         int64_t nq, int64_t nkv, int64_t rd, at::Tensor kc, at::Tensor vc,
                                         at::Tensor err) {
    TORCH_CHECK(err_word(err), "gemv_norm_rope: err must be an int32 GPU tensor");
    if (!gemv_norm_ok(x, W, gamma) || x.size(0) != 1) return c10::nullopt;
    if (!(kc.is_cuda() && kc.dim() == 3 && kc.is_contiguous() && vc.is_contiguous() && vc.sizes() == kc.sizes() &&
          kc.size(1) == nkv && kc.scalar_type() == x.scalar_type() && vc.scalar_type() == x.scalar_type()))
        return c10::nullopt;
    const int64_t hd = kc.size(2);
    if (hd % 2 || rd % 2 || rd > hd || W.size(0) != (nq + 2 * nkv) * hd) return c10::nullopt;
    if (!(pos.is_cuda() && pos.scalar_type() == at::kLong && pos.numel() == 1 && cosb.scalar_type() == at::kFloat &&
          sinb.scalar_type() == at::kFloat && cosb.is_contiguous() && sinb.is_contiguous() && cosb.size(-1) == rd / 2 &&
          sinb.sizes() == cosb.sizes()))
        return c10::nullopt;
    const at::DeviceGuard g(x.device());
    auto q = at::empty({1, nq, hd}, x.options());
    GemvRope r{cosb.data_ptr<float>(), sinb.data_ptr<float>(), pos.data_ptr<int64_t>(), q.data_ptr(), kc.data_ptr(),
               vc.data_ptr(), (int)nq, (int)nkv, (int)hd, (int)rd, std::min<int64_t>(kc.size(0), cosb.size(0)),
               err.data_ptr<int>()};
    sa_launch::gemv(dt(x), 1, x.data_ptr(), x.stride(0), W.data_ptr(), W.stride(0), nullptr, nullptr, 0,
                    (int)W.size(0), (int)W.size(1), cur_stream(), 3, nullptr, 0, gamma.data_ptr(), nullptr, nullptr,
                    (float)eps, &r);
    return q;
}

// ------------------------------------------------------------------ GEMM (weight gradient)
// C[M, N] = A^T B (+ C if accumulate); A: [K, M], B: [K, N], C: [M, N], bf16, unit inner strides.
bool gemm_tn_ok(const at::Tensor& A, const at::Tensor& B, const at::Tensor& C) {
    if (!(A.is_cuda() && B.is_cuda() && C.is_cuda() && A.dim() == 2 && B.dim() == 2 && C.dim() == 2)) return false;
    if (A.scalar_type() != at::kBFloat16 || B.scalar_type() != at::kBFloat16 || C.scalar_type() != at::kBFloat16)
        return false;
    if (A.stride(1) != 1 || B.stride(1) != 1 || C.stride(1) != 1 || A.size(0) != B.size(0) || C.size(0) != A.size(1) ||
        C.size(1) != B.size(1))
        return false;
    for (const at::Tensor* t : {&A, &B}) if ((uintptr_t)t->data_ptr() % 16 != 0) return false;
    if ((uintptr_t)C.data_ptr() % 8 != 0) return false;  // C tiles are written with 8-byte (4 x bf16) stores
    return sa_launch::gemm_tn_supported(A.size(1), B.size(1), A.size(0), A.stride(0), B.stride(0), C.stride(0));
}
void gemm_tn(const at::Tensor& A, const at::Tensor& B, const at::Tensor& C, bool accumulate) {
    TORCH_CHECK(gemm_tn_ok(A, B, C), "gemm_tn: unsupported operands (bf16 2-D, M/N multiples of 16, K of 128)");
    const at::DeviceGuard g(A.device());
    static int slots = -1;  // one 256x256 tile per CU
    if (slots < 0) {
        hipDeviceProp_t prop;
        slots = hipGetDeviceProperties(&prop, A.device().index()) == hipSuccess ? prop.multiProcessorCount : 0;
    }
    int full_blocks = -1, split = 1;
    const int64_t ws_floats = sa_launch::gemm_tn_plan(A.size(1), B.size(1), A.size(0), slots, full_blocks, split);
    at::Tensor ws;
    if (ws_floats > 0) ws = at::empty({ws_floats}, A.options().dtype(at::kFloat));
    sa_launch::gemm_tn(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), C.data_ptr(), C.stride(0), A.size(1),
                       B.size(1), A.size(0), accumulate, cur_stream(), full_blocks, split,
                       ws_floats > 0 ? ws.data_ptr<float>() : nullptr);
}

// ------------------------------------------------------------------ flash attention
void check_qkv(const at::Tensor& t, const char* n) {
    TORCH_CHECK(t.is_cuda() && t.dim() == 3 && t.stride(2) == 1, "flash_attn: ", n, " must be [T, heads, D] with unit last stride");
    TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf, "flash_attn: ", n, " must be bfloat16 or float16");
    TORCH_CHECK(t.stride(1) % 8 == 0 && t.stride(0) % 8 == 0, "flash_attn: ", n, " strides must be multiples of 8");
}
// dropout keep threshold on the 32-bit mix: P(keep) = 1 - p
uint32_t drop_threshold(double p) {
    const double t = p * 4294967296.0;
    return t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
}
std::vector<at::Tensor> fa_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, const at::Tensor& cu_q,
                               const at::Tensor& cu_k, int64_t max_q, double scale, bool causal, int64_t window,
                               double p_drop, int64_t seed, int64_t local_heads, int64_t max_k) {
    check_qkv(q, "q"); check_qkv(k, "k"); check_qkv(v, "v");
    TORCH_CHECK(k.scalar_type() == q.scalar_type() && v.scalar_type() == q.scalar_type(), "flash_attn: q/k/v dtypes differ");
    TORCH_CHECK(p_drop >= 0.0 && p_drop < 1.0, "flash_attn: dropout probability must be in [0, 1)");
    const int64_t D = q.size(2);
    TORCH_CHECK(D == 32 || D == 64 || D == 128, "flash_attn: head dim must be 32, 64 or 128");
    TORCH_CHECK(k.size(2) == D && v.size(2) == D && k.size(1) == v.size(1) && q.size(1) % k.size(1) == 0, "flash_attn: shapes");
    TORCH_CHECK(cu_q.scalar_type() == at::kInt && cu_k.scalar_type() == at::kInt && cu_q.numel() == cu_k.numel(), "flash_attn: cu_seqlens int32");
    const at::DeviceGuard g(q.device());
    const int64_t T = q.size(0), H = q.size(1);
    auto o = at::empty({T, H, D}, q.options());
    auto lse = at::empty({H, T}, q.options().dtype(at::kFloat));
    FwdArgs a{};
    a.q = (const uint16_t*)q.data_ptr(); a.k = (const uint16_t*)k.data_ptr(); a.v = (const uint16_t*)v.data_ptr();
    a.o = (uint16_t*)o.data_ptr(); a.lse = lse.data_ptr<float>();
    a.q_tok = q.stride(0); a.q_head = q.stride(1); a.k_tok = k.stride(0); a.k_head = k.stride(1);
    a.v_tok = v.stride(0); a.v_head = v.stride(1); a.o_tok = o.stride(0); a.o_head = o.stride(1); a.lse_stride = T;
    a.cu_q = cu_q.data_ptr<int>(); a.cu_k = cu_k.data_ptr<int>();
    a.nseg = (int)cu_q.numel() - 1; a.Hq = (int)H; a.Hkv = (int)k.size(1); a.causal = causal ? 1 : 0; a.window = (int)window;
    a.local_heads = local_heads < 0 ? (int)H : (int)local_heads;
    a.scale_log2 = (float)(scale * 1.4426950408889634);
    a.p_drop = (float)p_drop; a.rp_drop = (float)(1.0 / (1.0 - p_drop)); a.seed = (uint32_t)seed; a.drop_thr = drop_threshold(p_drop);
    const int64_t grp = H / k.size(1);
    if (T > 0 && a.nseg > 0 && p_drop == 0.0 && max_q * grp <= 32) {
        // short query segments (decode): GQA-packed rows, split-K over the keys, then a combine pass
        DecArgs d{};
        d.q = a.q; d.k = a.k; d.v = a.v;
        d.q_tok = a.q_tok; d.q_head = a.q_head; d.k_tok = a.k_tok; d.k_head = a.k_head; d.v_tok = a.v_tok; d.v_head = a.v_head;
        d.cu_q = a.cu_q; d.cu_k = a.cu_k; d.nseg = a.nseg; d.Hq = a.Hq; d.Hkv = a.Hkv; d.causal = a.causal;
        d.window = a.window; d.local_heads = a.local_heads; d.scale_log2 = a.scale_log2; d.Tq = T;
        sa_launch::fa_decode_plan(max_k > 0 ? max_k : k.size(0), a.Hkv, a.nseg, d.split_keys, d.nsplit);
        auto part_o = at::empty({(int64_t)d.nsplit, T, H, D}, q.options().dtype(at::kFloat));
        auto part_ml = at::empty({(int64_t)d.nsplit, T, H, 2}, q.options().dtype(at::kFloat));
        d.part_o = part_o.data_ptr<float>(); d.part_ml = part_ml.data_ptr<float>();
        d.o = a.o; d.o_tok = a.o_tok; d.o_head = a.o_head; d.lse = a.lse; d.lse_stride = a.lse_stride;
        sa_launch::fa_decode(d, (int)D, q.scalar_type() == at::kHalf, cur_stream());
        return {o, lse};
    }
    if (T > 0 && a.nseg > 0) sa_launch::fa_fwd(a, (int)D, (int)max_q, q.scalar_type() == at::kHalf, cur_stream());
    return {o, lse};
}
std::vector<at::Tensor> fa_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                               const at::Tensor& o, const at::Tensor& lse, const at::Tensor& cu_q, const at::Tensor& cu_k,
                               int64_t max_q, int64_t max_k, double scale, bool causal, int64_t window,
                               const c10::optional<at::Tensor>& dq_out, const c10::optional<at::Tensor>& dk_out,
                               const c10::optional<at::Tensor>& dv_out, double p_drop, int64_t seed, int64_t local_heads,
                               const c10::optional<at::Tensor>& rope_cos, const c10::optional<at::Tensor>& rope_sin,
                               const c10::optional<at::Tensor>& rope_pos, int64_t rope_dim, int64_t rope_seq,
                               bool rope_interleaved) {
    // d*_out: write the gradients into caller-provided strided views (e.g. slices of one dQKV buffer)
    // rope_*: dq / dk leave rotated back by the inverse RoPE (the forward rotated q / k): folded into the dQ / dK
    // epilogues where the layout allows it, else the stand-alone rope kernel runs on dq / dk afterwards
    check_qkv(q, "q"); check_qkv(k, "k"); check_qkv(v, "v"); check_qkv(o, "o");
    TORCH_CHECK(k.scalar_type() == q.scalar_type() && v.scalar_type() == q.scalar_type() && o.scalar_type() == q.scalar_type() &&
                dout.scalar_type() == q.scalar_type(), "fa_bwd: dtypes differ");
    auto dO = dout.contiguous();
    check_qkv(dO, "dout");
    const int64_t D = q.size(2), T = q.size(0), H = q.size(1), Tk = k.size(0), Hk = k.size(1);
    const at::DeviceGuard g(q.device());
    auto take = [](const c10::optional<at::Tensor>& t, const at::Tensor& like, const char* n) {
        if (!t.has_value()) return at::empty(like.sizes(), like.options());
        TORCH_CHECK(t->sizes() == like.sizes() && t->scalar_type() == like.scalar_type(), "fa_bwd: ", n, " shape/dtype");
        check_qkv(*t, n);
        return *t;
    };
    auto dq = take(dq_out, q, "dq_out");
    auto dk = take(dk_out, k, "dk_out");
    auto dv = take(dv_out, v, "dv_out");
    auto delta = at::empty({H, T}, q.options().dtype(at::kFloat));
    auto lse2 = at::empty({H, T}, q.options().dtype(at::kFloat));
    BwdArgs a{};
    a.q = (const uint16_t*)q.data_ptr(); a.k = (const uint16_t*)k.data_ptr(); a.v = (const uint16_t*)v.data_ptr();
    a.dO = (const uint16_t*)dO.data_ptr(); a.lse = lse.data_ptr<float>(); a.delta = delta.data_ptr<float>(); a.lse2 = lse2.data_ptr<float>();
    a.dq = (uint16_t*)dq.data_ptr(); a.dk = (uint16_t*)dk.data_ptr(); a.dv = (uint16_t*)dv.data_ptr();
    a.q_tok = q.stride(0); a.q_head = q.stride(1); a.k_tok = k.stride(0); a.k_head = k.stride(1);
    a.v_tok = v.stride(0); a.v_head = v.stride(1); a.do_tok = dO.stride(0); a.do_head = dO.stride(1);
    a.dq_tok = dq.stride(0); a.dq_head = dq.stride(1); a.dk_tok = dk.stride(0); a.dk_head = dk.stride(1);
    a.dv_tok = dv.stride(0); a.dv_head = dv.stride(1); a.lse_stride = T;
    a.cu_q = cu_q.data_ptr<int>(); a.cu_k = cu_k.data_ptr<int>();
    a.nseg = (int)cu_q.numel() - 1; a.Hq = (int)H; a.Hkv = (int)Hk; a.causal = causal ? 1 : 0; a.window = (int)window;
    a.local_heads = local_heads < 0 ? (int)H : (int)local_heads;
    a.scale = (float)scale; a.scale_log2 = (float)(scale * 1.4426950408889634);
    a.p_drop = (float)p_drop; a.rp_drop = (float)(1.0 / (1.0 - p_drop)); a.seed = (uint32_t)seed; a.drop_thr = drop_threshold(p_drop);
    // GQA head split of the dK/dV sweep: causal/windowed work is triangular, and with few (kv head, key
    // block) workgroups the heaviest one bounds the kernel; splitting the q-head group evens it out
    a.hsplit = 1; a.Tk = (int)Tk;
    const int grp = (int)(H / Hk);
    const int64_t kblocks = (max_k + 127) / 128;
    if (causal || window >= 0)
        while (a.hsplit < grp && grp % (2 * a.hsplit) == 0 && Hk * a.hsplit * a.nseg * kblocks < 1024) a.hsplit *= 2;
    at::Tensor part;
    if (a.hsplit > 1) {
        part = at::empty({2, a.hsplit, Tk, Hk, D}, q.options().dtype(at::kFloat));
        a.dk_part = part[0].data_ptr<float>();
        a.dv_part = part[1].data_ptr<float>();
    }
    const bool rope = rope_cos.has_value();
    bool fold = false;
    if (rope) {
        TORCH_CHECK(rope_sin.has_value() && rope_cos->scalar_type() == at::kFloat && rope_sin->scalar_type() == at::kFloat &&
                    rope_cos->is_contiguous() && rope_sin->is_contiguous() && rope_cos->size(-1) == rope_dim / 2 &&
                    (!rope_pos.has_value() ||
                     (rope_pos->scalar_type() == at::kLong && rope_pos->numel() == T && rope_pos->is_contiguous() &&
                      rope_pos->device() == q.device())),
                    "fa_bwd: rope tables / positions (contiguous fp32 tables, contiguous int64 positions of [T])");
        // NeoX pairs sit in one lane for a full rotation (partner accumulator t + D/64), interleaved pairs in one
        // 4-element group; with the dK head split the partials are summed in fa_bwd_reduce_kernel, which does not rotate
        fold = D >= 64 && (rope_interleaved ? rope_dim <= D && rope_dim % 8 == 0 : rope_dim == D) && a.hsplit == 1 &&
               Tk == T;
        if (fold) {
            a.rcos = rope_cos->data_ptr<float>(); a.rsin = rope_sin->data_ptr<float>();
            a.rpos = rope_pos.has_value() ? rope_pos->data_ptr<int64_t>() : nullptr;
            a.rrd = (int)rope_dim; a.rseq = (int)rope_seq; a.ril = rope_interleaved ? 1 : 0;
        }
    }
    if (T > 0 && a.nseg > 0)
        sa_launch::fa_bwd(a, (const uint16_t*)o.data_ptr(), o.stride(0), o.stride(1), T, (int)D, (int)max_q, (int)max_k,
                          q.scalar_type() == at::kHalf, cur_stream());
    if (rope && !fold) {
        const int64_t* pp = rope_pos.has_value() ? rope_pos->data_ptr<int64_t>() : nullptr;
        for (at::Tensor* t : {&dq, &dk}) {
            sa_launch::rope(dt(*t), rope_interleaved, t->data_ptr(), t->stride(0), t->stride(1), t->data_ptr(),
                            t->stride(0), t->stride(1), rope_cos->data_ptr<float>(), rope_sin->data_ptr<float>(), pp,
                            t->size(0), (int)t->size(1), (int)t->size(2), (int)rope_dim, (int)rope_seq, -1.f,
                            cur_stream());
        }
    }
    return {dq, dk, dv};
}
// ------------------------------------------------------------------ masked softmax / activations / dropout
at::Tensor aligned16(const at::Tensor& t) {
    auto c = t.contiguous();
    return (reinterpret_cast<uintptr_t>(c.data_ptr()) % 16 == 0) ? c : c.clone();
}
// mask: optional bool tensor broadcastable to x [B, H, Sq, Sk] with unit last stride
std::tuple<const void*, int64_t, int64_t, int64_t> mask_view(const c10::optional<at::Tensor>& mask, const at::Tensor& x,
                                                             at::Tensor& keep) {
    if (!mask.has_value()) return {nullptr, 0, 0, 0};
    TORCH_CHECK(mask->scalar_type() == at::kBool, "masked_softmax: mask must be bool");
    auto m = mask->to(x.device()).expand(x.sizes());
    if (m.stride(3) != 1) m = m.contiguous();
    keep = m;
    return {m.data_ptr(), m.stride(0), m.stride(1), m.stride(2)};
}
at::Tensor masked_softmax_fwd(const at::Tensor& x_, const c10::optional<at::Tensor>& mask, double scale, double fill,
                              bool round_scaled) {
    TORCH_CHECK(x_.is_cuda() && x_.dim() == 4, "masked_softmax: x must be a [B, H, Sq, Sk] GPU tensor");
    const at::DeviceGuard g(x_.device());
    auto x = aligned16(x_);
    at::Tensor keep;
    auto [mp, mb, mh, mq] = mask_view(mask, x, keep);
    auto y = at::empty_like(x);
    const int64_t N = x.size(3), rows = x.numel() / std::max<int64_t>(N, 1);
    if (rows > 0 && N > 0)
        sa_launch::masked_softmax_fwd(dt(x), x.data_ptr(), mp, y.data_ptr(), rows, (int)N, (int)x.size(1), (int)x.size(2), mb, mh,
                                      mq, (float)scale, (float)fill, round_scaled, cur_stream());
    return y;
}
at::Tensor masked_softmax_bwd(const at::Tensor& dy_, const at::Tensor& y_, const c10::optional<at::Tensor>& mask, double scale) {
    TORCH_CHECK(y_.is_cuda() && y_.dim() == 4 && dy_.sizes() == y_.sizes() && dy_.scalar_type() == y_.scalar_type(),
                "masked_softmax_bwd: shapes");
    const at::DeviceGuard g(y_.device());
    auto y = aligned16(y_);
    auto dy = aligned16(dy_);
    at::Tensor keep;
    auto [mp, mb, mh, mq] = mask_view(mask, y, keep);
    auto dx = at::empty_like(y);
    const int64_t N = y.size(3), rows = y.numel() / std::max<int64_t>(N, 1);
    if (rows > 0 && N > 0)
        sa_launch::masked_softmax_bwd(dt(y), dy.data_ptr(), y.data_ptr(), mp, dx.data_ptr(), rows, (int)N, (int)y.size(1),
                                      (int)y.size(2), mb, mh, mq, (float)scale, cur_stream());
    return dx;
}
at::Tensor act_fwd(const at::Tensor& x_, int64_t kind) {
    TORCH_CHECK(x_.is_cuda(), "activation: GPU tensor expected");
    const at::DeviceGuard g(x_.device());
    auto x = aligned16(x_);
    auto y = at::empty_like(x);
    if (x.numel() > 0) sa_launch::act_fwd(dt(x), x.data_ptr(), y.data_ptr(), x.numel(), (int)kind, cur_stream());
    return y;
}
at::Tensor act_bwd(const at::Tensor& dy_, const at::Tensor& x_, int64_t kind) {
    TORCH_CHECK(x_.is_cuda() && dy_.sizes() == x_.sizes() && dy_.scalar_type() == x_.scalar_type(), "activation_bwd: shapes");
    const at::DeviceGuard g(x_.device());
    auto x = aligned16(x_);
    auto dy = aligned16(dy_);
    auto dx = at::empty_like(x);
    if (x.numel() > 0) sa_launch::act_bwd(dt(x), dy.data_ptr(), x.data_ptr(), dx.data_ptr(), x.numel(), (int)kind, cur_stream());
    return dx;
}
// out = res + dropout(x); res optional (plain dropout).  Backward = dropout(g) with the same seed.
void spin_us(int64_t us) { sa_launch::spin(us, cur_stream()); }
// ---- stream gates (asynchronous rehearsal collectives, core/topology/gloo_gpu.py): a stream waits in the command
// processor (hipStreamWaitValue32, no CU spins) until the host writes a generation number into a flag word.
// kind 0: hipMallocSignalMemory words; kind 1: coherent pinned host memory.  Returns the base address.
// flag words in coherent, device-mapped host memory (hipMallocSignalMemory was refused on the pool's boxes)
int64_t gate_flags_alloc(int64_t n) {
    void* p = nullptr;
    const size_t bytes = (size_t)std::max<int64_t>(n, 1) * sizeof(uint32_t);
    TORCH_CHECK(hipHostMalloc(&p, bytes, hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess, "gate: pinned memory");
    std::memset(p, 0, bytes);
    return (int64_t)(uintptr_t)p;
}
void gate_flag_write(int64_t base, int64_t idx, int64_t value) {
    std::atomic_thread_fence(std::memory_order_seq_cst);  // every host write before (the results) lands first
    __atomic_store_n(reinterpret_cast<uint32_t*>((uintptr_t)base) + idx, (uint32_t)value, __ATOMIC_SEQ_CST);
}
int64_t gate_flag_read(int64_t base, int64_t idx) {
    return __atomic_load_n(reinterpret_cast<uint32_t*>((uintptr_t)base) + idx, __ATOMIC_SEQ_CST);
}
void gate_stream_wait(int64_t base, int64_t idx, int64_t value) {
    void* p = reinterpret_cast<uint32_t*>((uintptr_t)base) + idx;
    TORCH_CHECK(hipStreamWaitValue32(cur_stream(), p, (uint32_t)value, hipStreamWaitValueGte, 0xFFFFFFFFu) == hipSuccess,
                "gate: hipStreamWaitValue32 failed");
}
// per-rank proxy: a collective's local footprint (HBM bytes through nwg CUs, then held to the modelled link time)
void xgmi_emulate(const at::Tensor& src, const at::Tensor& scratch, int64_t bytes, double us, int64_t nwg) {
    TORCH_CHECK(src.is_cuda() && scratch.is_cuda() && scratch.is_contiguous(), "xgmi_emulate: GPU tensors");
    TORCH_CHECK((uintptr_t)src.data_ptr() % 16 == 0 && (uintptr_t)scratch.data_ptr() % 16 == 0, "xgmi_emulate: 16-B aligned");
    const at::DeviceGuard g(src.device());
    // the source is read as its contiguous storage span (the collective's bytes, whatever the view's strides)
    const int64_t sb = src.is_contiguous() ? src.numel() * src.element_size() : 0;
    sa_launch::xgmi_emulate(src.data_ptr(), sb, scratch.data_ptr(), scratch.numel() * scratch.element_size(),
                            sb > 0 ? bytes : 0, us, (int)nwg, cur_stream());
}

at::Tensor dropout_add(const at::Tensor& x_, const c10::optional<at::Tensor>& res_, double p, int64_t seed) {
    TORCH_CHECK(x_.is_cuda(), "dropout: GPU tensor expected");
    TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout: probability must be in [0, 1)");
    const at::DeviceGuard g(x_.device());
    auto x = aligned16(x_);
    at::Tensor res;
    if (res_.has_value()) {
        TORCH_CHECK(res_->sizes() == x.sizes() && res_->scalar_type() == x.scalar_type(), "dropout_add: residual mismatch");
        res = aligned16(*res_);
    }
    auto out = at::empty_like(x);
    if (x.numel() > 0)
        sa_launch::dropout(dt(x), x.data_ptr(), res.defined() ? res.data_ptr() : nullptr, out.data_ptr(), x.numel(),
                           (uint32_t)seed, drop_threshold(p), (float)(1.0 / (1.0 - p)), cur_stream());
    return out;
}
}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
    m.doc() = "scaling_amd CDNA4 (gfx950) HIP kernels";
    register_rehearsal(m);
    register_blaslt(m);
    m.def("norm_fwd", &norm_fwd, "RMSNorm/LayerNorm forward (optional fused residual add)", py::arg("x"), py::arg("w"), py::arg("b"), py::arg("eps"), py::arg("layer"), py::arg("res") = py::none());
    m.def("norm_bwd", &norm_bwd, "RMSNorm/LayerNorm backward (optional fused residual-gradient add)", py::arg("dy"), py::arg("x"), py::arg("w"), py::arg("mean"), py::arg("rstd"), py::arg("layer"), py::arg("dadd") = py::none());
    m.def("swiglu_fwd", &swiglu_fwd, "SwiGLU forward");
    m.def("swiglu_bwd", &swiglu_bwd, "SwiGLU backward");
    m.def("ar_alloc", &ar_alloc, "one-shot all-reduce: allocate + IPC-export a registered buffer");
    m.def("ar_open", &ar_open, "one-shot all-reduce: map a peer's registered buffer");
    m.def("ar_close", &ar_close, "unmap a peer buffer");
    m.def("ar_free", &ar_free, "free an own registered buffer");
    m.def("ar_allreduce", &ar_allreduce, "one-shot all-reduce of x over the registered buffers (in place)",
          py::arg("x"), py::arg("bases"), py::arg("rank"), py::arg("slot_off"), py::arg("flag_off"), py::arg("epoch"),
          py::arg("signal"), py::arg("err"), py::arg("max_spins") = int64_t(1) << 26);
    m.def("transpose_ok", &transpose_ok, "whether transpose2d supports this tensor");
    m.def("transpose2d", &transpose2d, "x^T (contiguous) for 2-byte 2-D matrices");
    m.def("gemv_ok", &gemv_ok, "whether gemv supports these operands");
    m.def("gemv", &gemv, "y = x W^T (+ b) for at most 4 rows of x (decode-time linear layers)", py::arg("x"), py::arg("W"), py::arg("bias") = py::none());
    m.def("gemv_residual", &gemv_residual, "y = x W^T + res for at most 4 rows (decode MLP-out + residual)");
    m.def("gemv_swiglu", &gemv_swiglu, "y = silu(x Wg^T) * (x Wu^T) for W = [Wg; Wu], at most 4 rows (decode)");
    m.def("gemv_norm_ok", &gemv_norm_ok, "whether gemv_norm supports these operands");
    m.def("gemv_norm_rope", &gemv_norm_rope, "graph decode: rms_norm + q/k/v GEMV + interleaved RoPE + K/V cache append "
          "in one launch; returns q or None");
    m.def("gemv_norm", &gemv_norm, "(s, gemv(rms_norm(s), W)) with s = x (+ add); epi 0 plain, 2 SwiGLU (decode)",
          py::arg("x"), py::arg("add"), py::arg("gamma"), py::arg("eps"), py::arg("W"), py::arg("epi") = 0);
    m.def("gemm_tn_ok", &gemm_tn_ok, "whether gemm_tn supports these operands");
    m.def("gemm_tn", &gemm_tn, "C (+)= A^T B for k-major bf16 operands (weight-gradient GEMM)");
    m.def("rope", &rope, "rotary embedding (fwd / inverse), optional strided / in-place output", py::arg("x"), py::arg("cos"), py::arg("sin"), py::arg("pos"), py::arg("rot_dim"), py::arg("seq_len"), py::arg("interleaved"), py::arg("inverse"), py::arg("out") = py::none());
    m.def("rope_kv_append", &rope_kv_append, "graph decode: RoPE q, RoPE k into the K cache row, v into the V cache row");
    m.def("xent_stats", &xent_stats, "cross-entropy row statistics");
    m.def("xent_bwd", &xent_bwd, "cross-entropy backward");
    m.def("embed_fwd", &embed_fwd, "vocab-parallel embedding forward");
    // (the GIL released: an embedding backward that waited for the device here -- its former unique / count
    // formulation -- while holding it deadlocked the asynchronous rehearsal's collectives)
    m.def("embed_bwd", &embed_bwd, "deterministic embedding backward", py::call_guard<py::gil_scoped_release>());
    m.def("adamw_", &adamw_, "fused AdamW on flat fp32 buffers");
    m.def("sumsq_", &sumsq_, "sum of squares + non-finite count");
    m.def("cast_scale_", &cast_scale_, "y = cast(x * scale)");
    m.def("masked_softmax_fwd", &masked_softmax_fwd, "softmax(masked_fill(x * scale, mask, fill)) over the last dim", py::arg("x"), py::arg("mask"), py::arg("scale"), py::arg("fill"), py::arg("round_scaled"));
    m.def("masked_softmax_bwd", &masked_softmax_bwd, "masked softmax backward", py::arg("dy"), py::arg("y"), py::arg("mask"), py::arg("scale"));
    m.def("act_fwd", &act_fwd, "activation forward (0 gelu, 1 silu, 2 gelu-tanh)");
    m.def("act_bwd", &act_bwd, "activation backward");
    m.def("spin_us", &spin_us, "debug: busy-wait kernel of ~us microseconds on the current stream");
    m.def("gate_flags_alloc", &gate_flags_alloc, "stream gates: n flag words (coherent pinned host memory)");
    m.def("gate_flag_write", &gate_flag_write, "stream gates: host store of a flag word (after a full fence)");
    m.def("gate_flag_read", &gate_flag_read, "stream gates: host load of a flag word");
    m.def("gate_stream_wait", &gate_stream_wait, "stream gates: the current stream waits until flag[idx] >= value");
    m.def("xgmi_emulate", &xgmi_emulate, "per-rank proxy: emulated collective (HBM traffic on nwg CUs, held to us)",
          py::arg("src"), py::arg("scratch"), py::arg("bytes"), py::arg("us"), py::arg("nwg") = 16);
    m.def("dropout_add", &dropout_add, "residual + dropout(x) with a hashed keep mask", py::arg("x"), py::arg("res"), py::arg("p"), py::arg("seed"));
    m.def("fa_fwd", &fa_fwd, "flash attention forward (bf16/fp16, optional attention dropout)", py::arg("q"), py::arg("k"), py::arg("v"), py::arg("cu_q"), py::arg("cu_k"), py::arg("max_q"), py::arg("scale"), py::arg("causal"), py::arg("window"), py::arg("p_drop") = 0.0, py::arg("seed") = 0, py::arg("local_heads") = -1, py::arg("max_k") = -1);
    m.def("fa_bwd", &fa_bwd, "flash attention backward (optional strided dq/dk/dv outputs)", py::arg("dout"), py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"), py::arg("lse"), py::arg("cu_q"), py::arg("cu_k"), py::arg("max_q"), py::arg("max_k"), py::arg("scale"), py::arg("causal"), py::arg("window"), py::arg("dq_out") = py::none(), py::arg("dk_out") = py::none(), py::arg("dv_out") = py::none(), py::arg("p_drop") = 0.0, py::arg("seed") = 0, py::arg("local_heads") = -1, py::arg("rope_cos") = py::none(), py::arg("rope_sin") = py::none(), py::arg("rope_pos") = py::none(), py::arg("rope_dim") = 0, py::arg("rope_seq") = 1, py::arg("rope_interleaved") = false);
}
