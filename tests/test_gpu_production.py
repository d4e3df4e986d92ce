"""HIP kernels at the production shapes of the Llama-2-7B benchmark, against fp32 PyTorch references
(reference tolerances: tests/core/test_nn/test_flash_attention.py, test_backwards_compatibility.py).

* flash attention fwd+bwd: 2 x 4096 tokens, 32 query / 8 KV heads, head dim 128, causal, bf16
  (reference in fp32, one KV-head group at a time to bound memory);
* weight-gradient GEMM dW += dY^T X at 11008 x 4096 over 8192 tokens, accumulating into bf16;
* fused vocab cross-entropy at 8192 x 32000;
* one 7B-dimension TransformerLayer (h 4096, 32/8 heads, SwiGLU 11008, RMSNorm, RoPE) forward+backward
  on the HIP path in bf16 against the same layer on the CPU fp32 path.
"""
from __future__ import annotations

import math

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from scaling_amd.ops import attention, gemm, xent  # noqa: E402

DEV = "cuda"


def _rel(a: torch.Tensor, b: torch.Tensor) -> float:
    return float((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-12))


def test_flash_attention_7b_shape():
    torch.manual_seed(0)
    S, B, Hq, Hk, D = 4096, 2, 32, 8, 128
    T = S * B
    cu = torch.tensor([0, S, 2 * S], device=DEV, dtype=torch.int32)
    q = torch.randn(T, Hq, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(T, Hk, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(T, Hk, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    scale = 1 / math.sqrt(D)
    o = attention.flash_attention(q, k, v, cu, cu, S, S, scale, True, None)
    g = torch.randn_like(o)
    o.backward(g)
    grp = Hq // Hk
    worst = {"o": 0.0, "dq": 0.0, "dk": 0.0, "dv": 0.0}
    for j in range(Hk):
        hs = slice(grp * j, grp * (j + 1))
        qr = q.detach()[:, hs].float().requires_grad_(True)
        kr = k.detach()[:, j : j + 1].float().requires_grad_(True)
        vr = v.detach()[:, j : j + 1].float().requires_grad_(True)
        orf = attention.attention_reference(qr, kr, vr, cu, cu, scale, True, -1)
        orf.backward(g[:, hs].float())
        worst["o"] = max(worst["o"], _rel(o[:, hs], orf))
        worst["dq"] = max(worst["dq"], _rel(q.grad[:, hs], qr.grad))
        worst["dk"] = max(worst["dk"], _rel(k.grad[:, j : j + 1], kr.grad))
        worst["dv"] = max(worst["dv"], _rel(v.grad[:, j : j + 1], vr.grad))
        del qr, kr, vr, orf
    assert all(e < 2e-2 for e in worst.values()), worst


@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("T,N,K", [(8192, 11008, 4096), (16384, 6144, 4096), (16384, 22016, 4096)])
def test_wgrad_gemm_7b_shapes(accumulate, T, N, K):
    """MLP-out, QKV and gate/up weight gradients at 8k / 16k tokens; the last two have a ragged last round
    of 256x256 tiles that runs as split-K slices plus a combine pass."""
    torch.manual_seed(0)
    dy = torch.randn(T, N, device=DEV, dtype=torch.bfloat16)
    x = torch.randn(T, K, device=DEV, dtype=torch.bfloat16)
    out = (0.5 * torch.randn(N, K, device=DEV)).to(torch.bfloat16)
    base = out.float().clone()
    assert gemm.ext().gemm_tn_ok(dy, x, out)  # the hand-written kernel, not a fallback
    gemm.wgrad(dy, x, out, accumulate=accumulate)
    ref = dy.float().t() @ x.float()
    if accumulate:
        ref += base
    assert _rel(out, ref) < 1e-2


def test_cross_entropy_7b_shape():
    torch.manual_seed(0)
    N, V = 8192, 32000
    logits = (3 * torch.randn(N, V, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    tgt = torch.randint(0, V, (N,), device=DEV)
    loss, am = xent.vocab_parallel_cross_entropy(logits, tgt)
    lr = logits.detach().float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(lr, tgt, reduction="none")
    torch.testing.assert_close(loss, ref, atol=1e-3, rtol=1e-4)
    assert torch.equal(am, lr.argmax(-1))
    loss.mean().backward()
    ref.mean().backward()
    assert _rel(logits.grad, lr.grad) < 1e-2


def _arch(precision: str, kernel: str):
    from scaling_amd.models import llama_architecture
    from scaling_amd.transformer.context.config import TransformerArchitectureConfig

    a = llama_architecture("llama2_7b", sequence_length=1024, precision=precision, num_layers=1)
    a["masked_softmax"] = {"kernel": kernel}
    return TransformerArchitectureConfig.from_dict(a)


def test_transformer_layer_7b_dims_gpu_vs_cpu_fp32():
    from unittest import mock

    from scaling_amd.transformer.model.layers import TransformerLayer
    from scaling_amd.transformer.model.layers.base import TransformerLayerIO

    torch.manual_seed(0)
    gpu = TransformerLayer(_arch("bfloat16", "flash_attention"), layer_index=0).to(DEV)
    with mock.patch("torch.cuda.is_available", return_value=False):  # build the fp32 twin natively on the CPU
        cpu = TransformerLayer(_arch("float32", "torch"), layer_index=0)
    assert all(p.device.type == "cpu" for p in cpu.parameters())
    sd = {k: v.detach().float().cpu() for k, v in gpu.state_dict().items()}
    res = cpu.load_state_dict(sd, strict=False)
    assert not res.unexpected_keys and not [k for k in res.missing_keys if not k.endswith(("cos_table", "sin_table"))]
    with torch.no_grad():  # non-trivial norm weights
        for (n, p), (_, pc) in zip(gpu.named_parameters(), cpu.named_parameters()):
            if "norm" in n:
                p.copy_(1 + 0.1 * torch.randn_like(p))
                pc.copy_(p.float().cpu())
    S, H = 1024, 4096
    x = torch.randn(1, S, H)
    pos = torch.arange(S).unsqueeze(0)
    cu = torch.tensor([0, S], dtype=torch.int32)

    def run(layer, dev, dtype):
        xi = x.to(dev, dtype).requires_grad_(True)
        io = TransformerLayerIO(activations=xi, position_ids=pos.to(dev), cumulative_seq_lengths=cu.to(dev),
                                cumulative_seq_lengths_padded=cu.to(dev))
        y = layer(io).hidden()  # with the MLP residual add the layer may hand to the next one
        g = torch.linspace(-1, 1, y.numel(), device=dev).reshape(y.shape).to(dtype)
        y.backward(g)
        return y, xi.grad, {n: p.grad for n, p in layer.named_parameters()}

    yg, dxg, pg = run(gpu, DEV, torch.bfloat16)
    yc, dxc, pc = run(cpu, "cpu", torch.float32)
    errs = {"y": _rel(yg.cpu(), yc), "dx": _rel(dxg.cpu(), dxc)}
    for n in pc:
        errs[n] = _rel(pg[n].cpu(), pc[n])
    assert all(e < 2e-2 for e in errs.values()), errs
