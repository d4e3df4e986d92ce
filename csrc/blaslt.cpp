// Small library GEMMs through hipBLASLt with a per-shape plan cache (scaling_amd/ops/gemm.py: ``linear`` / ``mm``
// for products of at most SCALING_AMD_LT_SMALL_FLOP multiply-adds).
//
// torch's hipBLASLt path builds the matmul descriptor and matrix layouts and queries the heuristic on every call:
// ~25-30 us of host time per GEMM, which a small model's host-bound step pays 30+ times (the transformer example:
// ~1 ms of a 4.3 ms step, profiles/example_host_profile_r6.txt).  Here each (shape, layout, bias) gets its descriptor,
// layouts and heuristic algorithm once; a call sets the bias pointer and launches.  Row-major products are expressed
// in hipBLASLt's column-major terms (a row-major [r, c] matrix is a column-major [c, r] one):
//   linear: Y[M,N] = X[M,K] W[N,K]^T (+ b)  ->  Y^T[N,M] = op_T(Wc[K,N]) Xc[K,M] (+ b per row of Y^T)
//   mm:     Y[M,N] = A[M,K] B[K,N]          ->  Y^T[N,M] = Bc[N,K] Ac[K,M]
// Both run on the current stream with one cached workspace per device.  The library instance is torch's own
// (libhipblaslt.so from torch/lib), so the process holds one hipBLASLt.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

namespace {

struct Plan {
    hipblasLtMatmulDesc_t desc = nullptr;
    hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
    hipblasLtMatmulAlgo_t algo{};
    bool ok = false;
};

using Key = std::tuple<int, int64_t, int64_t, int64_t, int, int, int>;  // device, M, N, K, kind, dtype, bias

struct State {
    std::mutex m;
    std::map<int, hipblasLtHandle_t> handles;
    std::map<int, at::Tensor> workspace;
    std::map<Key, Plan> plans;
};
State& state() {
    static State* s = new State();  // process lifetime (torch's library may unload before static destructors)
    return *s;
}
constexpr size_t kWorkspace = 32u << 20;

hipDataType lt_type(at::ScalarType t) {
    return t == at::kHalf ? HIP_R_16F : HIP_R_16BF;
}

// kind 0: linear (A = W as column-major [K,N], transposed; B = X as [K,M]); kind 1: mm (A = B_row as [N,K]; B = A_row)
Plan* plan_for(int dev, int64_t M, int64_t N, int64_t K, int kind, at::ScalarType dt, bool bias) {
    State& s = state();
    const Key key{dev, M, N, K, kind, (int)dt, bias ? 1 : 0};
    auto it = s.plans.find(key);
    if (it != s.plans.end()) return it->second.ok ? &it->second : nullptr;
    Plan& p = s.plans[key];
    auto& h = s.handles[dev];
    if (h == nullptr && hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) return nullptr;
    if (s.workspace.find(dev) == s.workspace.end())
        s.workspace[dev] = at::empty({(int64_t)kWorkspace}, at::TensorOptions().dtype(at::kByte).device(at::kCUDA, dev));
    const hipDataType t = lt_type(dt);
    if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return nullptr;
    const hipblasOperation_t ta = kind == 0 ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = HIPBLAS_OP_N;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
    if (bias) {
        const hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BIAS;
        const int32_t bt = (int32_t)t;
        hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep));
        hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
    }
    // A: kind 0 -> Wc [K, N] (ld K); kind 1 -> Bc [N, K] (ld N).  B: Xc / Ac [K, M] (ld K).  C: [N, M] (ld N)
    if (kind == 0) hipblasLtMatrixLayoutCreate(&p.la, t, K, N, K);
    else hipblasLtMatrixLayoutCreate(&p.la, t, N, K, N);
    hipblasLtMatrixLayoutCreate(&p.lb, t, K, M, K);
    hipblasLtMatrixLayoutCreate(&p.lc, t, N, M, N);
    hipblasLtMatmulPreference_t pref = nullptr;
    hipblasLtMatmulPreferenceCreate(&pref);
    const uint64_t ws = kWorkspace;
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
    hipblasLtMatmulHeuristicResult_t res[1];
    int n = 0;
    const bool found = hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.la, p.lb, p.lc, p.lc, pref, 1, res, &n) ==
                           HIPBLAS_STATUS_SUCCESS && n > 0;
    hipblasLtMatmulPreferenceDestroy(pref);
    if (!found) return nullptr;
    p.algo = res[0].algo;
    p.ok = true;
    return &p;
}

bool run(Plan* p, int dev, const void* A, const void* B, void* C, const void* bias) {
    State& s = state();
    if (bias != nullptr)
        hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias));
    const float alpha = 1.f, beta = 0.f;
    return hipblasLtMatmul(s.handles[dev], p->desc, &alpha, A, p->la, B, p->lb, &beta, C, p->lc, C, p->lc, &p->algo,
                           s.workspace[dev].data_ptr(), kWorkspace, at::hip::getCurrentHIPStream().stream()) ==
           HIPBLAS_STATUS_SUCCESS;
}

bool usable(const at::Tensor& t) {
    return t.is_cuda() && t.is_contiguous() && (t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf);
}

// y = x2 @ w^T (+ b) for 2-D x2 [M, K], w [N, K]; an undefined tensor when no plan exists (the caller falls back)
// `out` (optional): a contiguous tensor of M * N elements to write (any shape: callers pass the un-flattened one, so
// the result is not a view of a 2-D temporary)
at::Tensor lt_linear(const at::Tensor& x2, const at::Tensor& w, const c10::optional<at::Tensor>& b,
                     const c10::optional<at::Tensor>& out) {
    if (!usable(x2) || !usable(w) || x2.dim() != 2 || w.dim() != 2 || x2.size(1) != w.size(1) ||
        x2.scalar_type() != w.scalar_type())
        return at::Tensor();
    const bool has_b = b.has_value() && b->defined();
    if (has_b && (!usable(*b) || b->numel() != w.size(0) || b->scalar_type() != w.scalar_type())) return at::Tensor();
    const int64_t M = x2.size(0), K = x2.size(1), N = w.size(0);
    const int dev = x2.get_device();
    const at::DeviceGuard g(x2.device());
    std::lock_guard<std::mutex> lk(state().m);
    Plan* p = plan_for(dev, M, N, K, 0, x2.scalar_type(), has_b);
    if (p == nullptr) return at::Tensor();
    at::Tensor y = out.has_value() && out->defined() ? *out : at::empty({M, N}, x2.options());
    TORCH_CHECK(y.is_contiguous() && y.numel() == M * N && y.scalar_type() == x2.scalar_type(), "lt_linear: out");
    if (!run(p, dev, w.data_ptr(), x2.data_ptr(), y.data_ptr(), has_b ? b->data_ptr() : nullptr)) return at::Tensor();
    return y;
}

// y = a @ bm for 2-D a [M, K], bm [K, N]
at::Tensor lt_mm(const at::Tensor& a, const at::Tensor& bm, const c10::optional<at::Tensor>& out) {
    if (!usable(a) || !usable(bm) || a.dim() != 2 || bm.dim() != 2 || a.size(1) != bm.size(0) ||
        a.scalar_type() != bm.scalar_type())
        return at::Tensor();
    const int64_t M = a.size(0), K = a.size(1), N = bm.size(1);
    const int dev = a.get_device();
    const at::DeviceGuard g(a.device());
    std::lock_guard<std::mutex> lk(state().m);
    Plan* p = plan_for(dev, M, N, K, 1, a.scalar_type(), false);
    if (p == nullptr) return at::Tensor();
    at::Tensor y = out.has_value() && out->defined() ? *out : at::empty({M, N}, a.options());
    TORCH_CHECK(y.is_contiguous() && y.numel() == M * N && y.scalar_type() == a.scalar_type(), "lt_mm: out");
    if (!run(p, dev, bm.data_ptr(), a.data_ptr(), y.data_ptr(), nullptr)) return at::Tensor();
    return y;
}

}  // namespace

void register_blaslt(pybind11::module& m) {
    m.def("lt_linear", &lt_linear, "small GEMM x @ w^T (+ b) through a cached hipBLASLt plan (undefined: no plan)",
          pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("b") = pybind11::none(),
          pybind11::arg("out") = pybind11::none());
    m.def("lt_mm", &lt_mm, "small GEMM a @ b through a cached hipBLASLt plan (undefined: no plan)", pybind11::arg("a"),
          pybind11::arg("b"), pybind11::arg("out") = pybind11::none());
}
