"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op (GPU only)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from scaling_amd.ops import attention, embedding, norm, optim, rope, swiglu, xent  # noqa: E402
from scaling_amd.ops._ext import ext  # noqa: E402

DEV = "cuda"


def test_extension_is_native():
    assert ext().__file__.endswith(".so")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("H", [256, 4096, 1000 - 1000 % 8])
def test_rms_norm(dtype, H):
    torch.manual_seed(0)
    x = torch.randn(37, 5, H, device=DEV, dtype=dtype, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=DEV, dtype=dtype)).requires_grad_(True)
    y = norm.rms_norm(x, w, 1e-5)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    yr = norm.rms_norm_reference(xr, wr, 1e-5)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=tol * 2, rtol=tol * 2)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=tol * 20, rtol=tol * 2)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_layer_norm(dtype):
    torch.manual_seed(0)
    H = 768
    x = torch.randn(64, 3, H, device=DEV, dtype=dtype, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=DEV, dtype=dtype)).requires_grad_(True)
    b = (0.1 * torch.randn(H, device=DEV, dtype=dtype)).requires_grad_(True)
    y = norm.layer_norm(x, w, b, 1e-5)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xr, (H,), wr, br, 1e-5)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=tol * 2, rtol=tol * 2)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=tol * 20, rtol=tol * 2)
    torch.testing.assert_close(b.grad.float(), br.grad, atol=tol * 20, rtol=tol * 2)


@pytest.mark.parametrize("layer", [False, True])
@pytest.mark.parametrize("dtype,rows", [(torch.bfloat16, 8192), (torch.float32, 300)])
def test_add_norm_fused(layer, dtype, rows):
    """s = x + r; y = norm(s): both outputs feed the loss so the fused residual-gradient add is exercised."""
    torch.manual_seed(1)
    H = 4096 if rows > 1000 else 512
    x = torch.randn(rows, H, device=DEV, dtype=dtype, requires_grad=True)
    r = torch.randn(rows, H, device=DEV, dtype=dtype, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=DEV, dtype=dtype)).requires_grad_(True)
    b = (0.1 * torch.randn(H, device=DEV, dtype=dtype)).requires_grad_(True)
    if layer:
        s, y = norm.add_layer_norm(x, r, w, b, 1e-5)
    else:
        s, y = norm.add_rms_norm(x, r, w, 1e-5)
    xr, rr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, r, w, b))
    sr = (xr + rr).to(dtype).float()  # the unfused path rounds the add to the activation dtype
    sr = xr + rr + (sr - (xr + rr)).detach()
    yr = (torch.nn.functional.layer_norm(sr, (H,), wr, br, 1e-5) if layer else norm.rms_norm_reference(sr, wr, 1e-5))
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    torch.testing.assert_close(s.float(), sr, atol=0, rtol=0)
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    gs, gy = torch.randn_like(s), torch.randn_like(y)
    torch.autograd.backward([s, y], [gs, gy])
    torch.autograd.backward([sr, yr], [gs.float(), gy.float()])
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=tol * 3, rtol=tol * 2)
    torch.testing.assert_close(r.grad.float(), rr.grad, atol=tol * 3, rtol=tol * 2)
    wt = tol * (50 if rows > 1000 else 20)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=wt, rtol=tol * 2)
    if layer:
        torch.testing.assert_close(b.grad.float(), br.grad, atol=wt, rtol=tol * 2)
    # dgamma reduction is deterministic (fixed-order two-level column sum)
    dw0 = w.grad.clone()
    w.grad = None
    s, y = norm.add_layer_norm(x, r, w, b, 1e-5) if layer else norm.add_rms_norm(x, r, w, 1e-5)
    torch.autograd.backward([s, y], [gs, gy])
    assert torch.equal(dw0, w.grad)


def test_norm_passthrough_and_layer_fusion():
    """res=None: s aliases x and the gradient through s is added in the norm backward; the transformer layer's
    fused residual path matches its unfused attention_block/mlp_block composition."""
    torch.manual_seed(2)
    H = 1024
    x0 = torch.randn(64, H, device=DEV, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=DEV)).requires_grad_(True)
    x = x0 * 1.5
    s, y = norm.add_rms_norm(x, None, w, 1e-5)
    ((s * s).sum() + (y * y.flip(0)).sum()).backward()
    xr = (x0.detach() * 1.5).requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    yr = norm.rms_norm_reference(xr, wr, 1e-5)
    ((xr * xr).sum() + (yr * yr.flip(0)).sum()).backward()
    torch.testing.assert_close(x0.grad, xr.grad * 1.5, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(w.grad, wr.grad, atol=1e-3, rtol=1e-4)

    from scaling_amd.models import llama_architecture
    from scaling_amd.transformer.context.config import TransformerArchitectureConfig
    from scaling_amd.transformer.model.layers.base import TransformerLayerIO
    from scaling_amd.transformer.model.layers.layer import TransformerLayer

    arch = TransformerArchitectureConfig.from_dict(llama_architecture("llama_tiny", sequence_length=128))
    layer = TransformerLayer(arch, layer_index=0).to(DEV)
    seqs, T = 2, 128
    a = torch.randn(seqs, T, arch.hidden_size, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    cu = torch.arange(0, (seqs + 1) * T, T, device=DEV, dtype=torch.int32)
    pos = torch.arange(T, device=DEV).repeat(seqs, 1)
    out = layer(TransformerLayerIO(activations=a, position_ids=pos, cumulative_seq_lengths_padded=cu,
                                   cumulative_seq_lengths=cu)).hidden()
    g = torch.randn_like(out)
    out.backward(g)
    ga, gw = a.grad.clone(), [p.grad.clone() for p in layer.parameters()]
    a.grad = None
    layer.zero_grad()
    ref = layer.mlp_block(layer.attention_block(a, cu, pos))
    ref.backward(g)
    torch.testing.assert_close(out.float(), ref.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(ga.float(), a.grad.float(), atol=5e-2, rtol=5e-2)
    for p1, p2 in zip(gw, layer.parameters()):
        torch.testing.assert_close(p1.float(), p2.grad.float(), atol=5e-1, rtol=5e-2)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_swiglu_fused(dtype):
    torch.manual_seed(0)
    z = torch.randn(33, 7, 2 * 344, device=DEV, dtype=dtype, requires_grad=True)
    y = swiglu.swiglu_fused(z)
    zr = z.detach().float().requires_grad_(True)
    yr = swiglu.swiglu_reference(zr[..., :344], zr[..., 344:])
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g.float())
    torch.testing.assert_close(z.grad.float(), zr.grad, atol=tol * 2, rtol=tol * 2)


@pytest.mark.parametrize("interleaved", [False, True])
@pytest.mark.parametrize("rot_frac", [1.0, 0.5, 0.3125])  # 0.3125 -> rd 20: scalar fallback kernel
def test_rope(interleaved, rot_frac):
    torch.manual_seed(0)
    T, nh, hd = 96, 6, 64
    rd = int(hd * rot_frac)
    qkv = torch.randn(T, nh, 3 * hd, device=DEV, dtype=torch.bfloat16)
    x = qkv[:, :, hd : 2 * hd].detach().requires_grad_(True)  # strided view
    cos, sin = rope.rope_tables(rd, 128, 10000, interleaved, torch.bfloat16, DEV)
    pos = torch.randint(0, 128, (T,), device=DEV)
    y = rope.apply_rope(x, cos, sin, pos, rd, 48, interleaved)
    xr = x.detach().float().requires_grad_(True)
    yr = rope.rope_reference(xr, cos, sin, pos, rd, 48, interleaved)
    torch.testing.assert_close(y.float(), yr, atol=2e-2, rtol=2e-2)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=3e-2, rtol=3e-2)
    # no position ids -> position = t % seq_len
    y2 = rope.apply_rope(x.detach(), cos, sin, None, rd, 48, interleaved)
    y2r = rope.rope_reference(x.detach().float(), cos, sin, None, rd, 48, interleaved)
    torch.testing.assert_close(y2.float(), y2r, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("interleaved", [False, True])
def test_rope_strided_and_inplace_out(interleaved):
    torch.manual_seed(0)
    T, nh, hd = 80, 4, 128
    cos, sin = rope.rope_tables(hd, 256, 10000, interleaved, torch.bfloat16, DEV)
    pos = torch.randint(0, 256, (T,), device=DEV)
    x = torch.randn(T, nh, hd, device=DEV, dtype=torch.bfloat16)
    ref = ext().rope(x, cos, sin, pos, hd, 64, interleaved, False)
    buf = torch.zeros(T, 2 * nh * hd, device=DEV, dtype=torch.bfloat16)
    out = buf[:, nh * hd:].view(T, nh, hd)
    ext().rope(x, cos, sin, pos, hd, 64, interleaved, False, out)
    assert torch.equal(out, ref) and torch.count_nonzero(buf[:, : nh * hd]) == 0
    ext().rope(out, cos, sin, pos, hd, 64, interleaved, True, out)  # in place inverse
    torch.testing.assert_close(out.float(), x.float(), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("qkv_in_one", [False, True])
def test_rope_flash_attention_fused(qkv_in_one):
    """Fused rope+attention node == rope then flash attention, including the gradient of the QKV buffer."""
    torch.manual_seed(3)
    seqs, S, nq, nkv, hd = 2, 256, 8, 2, 128
    if qkv_in_one:
        nkv = nq
    T = seqs * S
    base = torch.randn(T, (nq + 2 * nkv) * hd, device=DEV, dtype=torch.bfloat16, requires_grad=True)

    def views(b):
        if qkv_in_one:
            qkv = b.view(T, nq, 3 * hd)
            return qkv[..., :hd], qkv[..., hd:2 * hd], qkv[..., 2 * hd:]
        return (b[:, : nq * hd].view(T, nq, hd), b[:, nq * hd:(nq + nkv) * hd].view(T, nkv, hd),
                b[:, (nq + nkv) * hd:].view(T, nkv, hd))

    cos, sin = rope.rope_tables(hd, S, 10000, False, torch.bfloat16, DEV)
    pos = torch.arange(S, device=DEV).repeat(seqs)
    cu = torch.arange(0, T + 1, S, device=DEV, dtype=torch.int32)
    scale = hd ** -0.5
    q, k, v = views(base)
    o = attention.rope_flash_attention(base, q, k, v, cos, sin, pos, hd, S, False, cu, S, scale, True)
    assert o is not None
    g = torch.randn_like(o)
    o.backward(g)
    gf = base.grad.clone()
    base.grad = None
    q, k, v = views(base)
    qr = rope.apply_rope(q, cos, sin, pos, hd, S, False)
    kr = rope.apply_rope(k, cos, sin, pos, hd, S, False)
    o2 = attention.flash_attention(qr, kr, v, cu, max_seqlen_q=S, softmax_scale=scale, causal=True)
    o2.backward(g)
    assert torch.equal(o, o2)
    torch.testing.assert_close(gf.float(), base.grad.float(), atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("hd,rd,il,nq,nkv,S", [(128, 128, False, 8, 8, 256), (128, 64, False, 8, 8, 256),
                                               (128, 128, True, 8, 8, 256), (64, 64, False, 4, 4, 192),
                                               (128, 32, False, 8, 8, 256), (128, 128, False, 16, 2, 128)])
def test_flash_bwd_rope_fold_bit_exact(hd, rd, il, nq, nkv, S):
    """Inverse RoPE folded into the dQ / dK epilogues == flash backward then the stand-alone inverse rope, bit for
    bit (NeoX full / partial, interleaved, head_dim 64; rot_dim 32 and the GQA head-split backward take the
    unfolded path inside the binding)."""
    torch.manual_seed(11)
    T = 2 * S
    q, k, v, do = (torch.randn(T, h, hd, device=DEV, dtype=torch.bfloat16) for h in (nq, nkv, nkv, nq))
    cu = torch.arange(0, T + 1, S, device=DEV, dtype=torch.int32)
    cos, sin = rope.rope_tables(rd, S, 10000, il, torch.bfloat16, DEV)
    pos = torch.arange(S, device=DEV).repeat(2)
    o, lse = ext().fa_fwd(q, k, v, cu, cu, S, hd ** -0.5, True, -1)
    args = (do, q, k, v, o, lse, cu, cu, S, S, hd ** -0.5, True, -1)
    dq, dk, dv = ext().fa_bwd(*args)
    ext().rope(dq, cos, sin, pos, rd, S, il, True, dq)
    ext().rope(dk, cos, sin, pos, rd, S, il, True, dk)
    for p in (pos, None):
        fq, fk, fv = ext().fa_bwd(*args, None, None, None, 0.0, 0, -1, cos, sin, p, rd, S, il)
        assert torch.equal(fq, dq) and torch.equal(fk, dk) and torch.equal(fv, dv)


@pytest.mark.parametrize("V,offset", [(1000, 0), (32000, 0), (50257, 0), (1001, 0), (32000, 3)])
def test_cross_entropy(V, offset):
    """Odd vocab sizes (rows not 16-B aligned) and a misaligned base take the scalar row path."""
    torch.manual_seed(0)
    N = 67
    base = torch.empty(N * V + offset, device=DEV, dtype=torch.bfloat16)
    logits = base[offset:].view(N, V)
    logits.copy_(3 * torch.randn(N, V, device=DEV))
    logits = logits.detach().requires_grad_(True)
    tgt = torch.randint(0, V, (N,), device=DEV)
    loss, am = xent.vocab_parallel_cross_entropy(logits, tgt)
    lr = logits.detach().float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(lr, tgt, reduction="none")
    torch.testing.assert_close(loss, ref, atol=1e-4, rtol=1e-4)
    assert torch.equal(am, lr.argmax(-1))
    w = torch.rand(N, device=DEV)
    (loss * w).sum().backward()
    (ref * w).sum().backward()
    torch.testing.assert_close(logits.grad.float(), lr.grad, atol=2e-3, rtol=2e-2)


def test_embedding():
    torch.manual_seed(0)
    Vp, H = 500, 256
    W = torch.randn(Vp, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    ids = torch.randint(0, 1000, (4, 33), device=DEV)
    out = embedding.vocab_embedding(ids, W, 250, 750)
    Wr = W.detach().float().requires_grad_(True)
    ref = embedding.vocab_embedding_reference(ids, Wr, 250, 750)
    torch.testing.assert_close(out.float(), ref)
    g = torch.randn_like(out)
    out.backward(g)
    ref.backward(g.float())
    torch.testing.assert_close(W.grad.float(), Wr.grad, atol=5e-2, rtol=2e-2)
    # determinism
    W.grad = None
    embedding.vocab_embedding(ids, W, 250, 750).backward(g)
    g1 = W.grad.clone()
    W.grad = None
    embedding.vocab_embedding(ids, W, 250, 750).backward(g)
    assert torch.equal(g1, W.grad)


def test_embedding_backward_long_runs():
    """Embedding backward with long runs of one id (every token one of 9 ids, some outside the shard): the run
    boundaries are found on the device (no host count of distinct ids), each id's row summed in token order."""
    torch.manual_seed(1)
    Vp, H = 8, 512
    W = torch.randn(Vp, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    ids = torch.randint(0, 9, (6, 257), device=DEV) + 2  # ids 2..10; shard [4, 12) holds 4..10, ids 2 / 3 skipped
    out = embedding.vocab_embedding(ids, W, 4, 12)
    g = torch.randn_like(out)
    out.backward(g)
    flat, gi = g.reshape(-1, H).float(), ids.reshape(-1)
    ref = torch.zeros(Vp, H, device=DEV)
    for r in range(Vp):
        sel = gi == r + 4
        if sel.any():
            ref[r] = flat[sel].sum(0)
    torch.testing.assert_close(W.grad.float(), ref, atol=0.1, rtol=2e-2)


def test_adamw_matches_torch():
    torch.manual_seed(0)
    n = 10007
    p0 = torch.randn(n, device=DEV)
    ref = torch.nn.Parameter(p0.clone())
    opt = torch.optim.AdamW([ref], lr=1e-3, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    p, m, v = p0.clone(), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    pout = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    for step in range(1, 6):
        g = torch.randn(n, device=DEV)
        ref.grad = g.clone()
        opt.step()
        optim.adamw_step_(p, g, m, v, lr=1e-3, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.1, step=step,
                          param_out=pout)
    torch.testing.assert_close(p, ref.detach(), atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(pout.float(), ref.detach(), atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("offset", [1, 2, 3])
def test_adamw_unaligned_views(offset):
    """Buckets at element offsets that are not 16-B aligned (e.g. dp=3 chunks) use the scalar path."""
    torch.manual_seed(0)
    n = 4099
    bufs = [torch.randn(n + offset, device=DEV) for _ in range(3)]
    p, m, v = (b[offset:] for b in bufs)
    m.zero_()
    v.zero_()
    ref = torch.nn.Parameter(p.clone())
    opt = torch.optim.AdamW([ref], lr=1e-3, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    for step in range(1, 4):
        g = torch.randn(n, device=DEV)
        ref.grad = g.clone()
        opt.step()
        optim.adamw_step_(p, g, m, v, lr=1e-3, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.1, step=step)
    torch.testing.assert_close(p, ref.detach(), atol=1e-6, rtol=1e-5)


def test_sumsq():
    x = torch.randn(123457, device=DEV, dtype=torch.bfloat16)
    out = torch.zeros(2, device=DEV)
    optim.sumsq_nonfinite_(x, out, scale=0.5, accumulate=False)
    ref = ((x.float() * 0.5) ** 2).sum()
    torch.testing.assert_close(out[0], ref, rtol=1e-4, atol=1e-3)
    assert out[1].item() == 0
    x[5] = float("inf")
    optim.sumsq_nonfinite_(x, out, accumulate=True)
    assert out[1].item() == 1


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("offset", [0, 1, 3, 7, 8])
def test_sumsq_cast_unaligned(dtype, offset):
    # views at element offsets that are not 16-B aligned exercise the scalar head / vector body split
    base = torch.randn(1_000_003 + offset, device=DEV, dtype=dtype)
    x = base[offset:]
    out = torch.zeros(2, device=DEV)
    optim.sumsq_nonfinite_(x, out, scale=2.0, accumulate=False)
    ref = ((x.double() * 2.0) ** 2).sum().float()
    torch.testing.assert_close(out[0], ref, rtol=1e-4, atol=1e-2)
    x[offset + 11] = float("nan")
    x[-1] = float("inf")
    optim.sumsq_nonfinite_(x, out, accumulate=False)
    assert out[1].item() == 2
    y = torch.empty(x.numel() + 3, device=DEV, dtype=torch.float32)[3:]
    optim.cast_scale_(x, y, 0.5)
    torch.testing.assert_close(y, x.float() * 0.5, equal_nan=True)


def _attn_case(lens, Hq, Hk, D, causal, window=-1, dtype=torch.bfloat16, seed=0, p_drop=0.0, local_heads=None):
    torch.manual_seed(seed)
    T = sum(lens)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), device=DEV, dtype=torch.int32)
    qkv = torch.randn(T, Hq + 2 * Hk, D, device=DEV, dtype=dtype)
    q = qkv[:, :Hq].detach().requires_grad_(True)
    k = qkv[:, Hq : Hq + Hk].detach().requires_grad_(True)
    v = qkv[:, Hq + Hk :].detach().requires_grad_(True)
    scale = 1 / math.sqrt(D)
    if p_drop > 0:
        dseed = 12345 + seed
        o = attention._FlashAttn.apply(q, k, v, cu, cu, max(lens), max(lens), scale, causal, window, p_drop, dseed,
                                       -1 if local_heads is None else local_heads)
    else:
        dseed = None
        o = attention.flash_attention(q, k, v, cu, cu, max(lens), max(lens), scale, causal, None if window < 0 else window,
                                      local_heads=local_heads)
    assert o.dtype == dtype
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    orf = attention.attention_reference(qr, kr, vr, cu, cu, scale, causal, window, dropout_p=p_drop, training=p_drop > 0,
                                        dropout_seed_value=dseed, local_heads=local_heads)
    torch.testing.assert_close(o.float(), orf, atol=2e-2, rtol=2e-2)
    g = torch.randn_like(o)
    o.backward(g)
    orf.backward(g.float())
    for a, b in ((q, qr), (k, kr), (v, vr)):
        err = (a.grad.float() - b.grad).abs().max().item()
        scl = b.grad.abs().max().item() + 1e-6
        assert err / scl < 3e-2, (err, scl)


@pytest.mark.parametrize("lens,Hq,Hk,causal,dtype", [
    ([1024], 8, 2, True, torch.bfloat16),          # 8 q tiles, diagonal tile per wave
    ([700, 1300, 513], 4, 2, True, torch.bfloat16),  # ragged segments: partial 128-row tiles, waves with no rows
    ([640, 900], 4, 1, False, torch.bfloat16),     # non-causal: ragged last key tile through the masked tail
    ([600], 4, 2, True, torch.float16),
])
def test_flash_attention_long_ragged_shapes(lens, Hq, Hk, causal, dtype):
    """Long ragged segments at D = 128 against the fp32 reference (forward and, through its LSE, the backward)."""
    _attn_case(lens, Hq, Hk, 128, causal, dtype=dtype)


def test_flash_attention_growing_max():
    """Scores that grow along the keys make the running row max move by more than the lazy-rescale threshold in
    later tiles: the lazy O rescale (a wave-uniform branch) must match the fp32 reference."""
    torch.manual_seed(5)
    T, Hq, Hk, D = 1536, 4, 2, 128
    cu = torch.tensor([0, T], device=DEV, dtype=torch.int32)
    q = torch.randn(T, Hq, D, device=DEV, dtype=torch.bfloat16)
    grow = (1.0 + 6.0 * torch.arange(T, device=DEV, dtype=torch.float32) / T).view(T, 1, 1)
    k = (torch.randn(T, Hk, D, device=DEV) * grow).to(torch.bfloat16)
    v = torch.randn(T, Hk, D, device=DEV, dtype=torch.bfloat16)
    for causal in (True, False):
        o = attention.flash_attention(q, k, v, cu, cu, T, T, 1 / math.sqrt(D), causal)
        ref = attention.attention_reference(q.float(), k.float(), v.float(), cu, cu, 1 / math.sqrt(D), causal, -1)
        torch.testing.assert_close(o.float(), ref, atol=2e-2, rtol=2e-2)


def test_flash_attention_rejects_fp32():
    """fp32 q/k/v are refused (flash-attn's contract) instead of being computed in bf16 behind the caller's back."""
    q = torch.randn(64, 2, 64, device=DEV)
    cu = torch.tensor([0, 64], dtype=torch.int32, device=DEV)
    with pytest.raises(TypeError, match="float32"):
        attention.flash_attention(q, q, q, cu, cu, 64, 64, 0.125, True, None)


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention_basic(D, causal):
    _attn_case([256], 4, 4, D, causal)


def test_flash_attention_gqa_varlen():
    _attn_case([100, 37, 300, 1], 8, 2, 128, True)


def test_flash_attention_window():
    _attn_case([333, 129], 4, 4, 64, True, window=50)


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("local_heads", [1, 3, 6])
def test_flash_attention_mixed_local_global_heads(causal, local_heads):
    """One launch with a per-head window: q heads [0, local_heads) windowed, the rest global; GQA groups
    that mix both kinds (8 q / 2 kv heads) exercise the union q range of the dK/dV sweep."""
    _attn_case([300, 77], 8, 2, 128, causal, window=40, local_heads=local_heads)


def test_flash_attention_mixed_heads_dropout():
    _attn_case([190, 66], 8, 2, 64, True, window=30, p_drop=0.2, local_heads=3)


def test_flash_attention_d32_noncausal_odd():
    _attn_case([65, 7], 2, 1, 32, False)


@pytest.mark.parametrize("D", [32, 64, 128])
def test_flash_attention_fp16(D):
    _attn_case([200, 56], 4, 2, D, True, dtype=torch.float16)


@pytest.mark.parametrize("D,dtype", [(128, torch.bfloat16), (64, torch.float16), (32, torch.bfloat16)])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention_dropout_matches_masked_reference(D, dtype, causal):
    """Fused dropout: fwd + bwd equal the dense reference under the identical (hash) keep mask."""
    _attn_case([190, 66], 4, 2, D, causal, dtype=dtype, p_drop=0.25)


def test_flash_attention_dropout_rate_and_seed():
    T, H, D = 1024, 4, 64
    cu = torch.tensor([0, T], device=DEV, dtype=torch.int32)
    keep = attention.dropout_keep_mask(7, torch.arange(H), torch.arange(T), torch.arange(T), 0.1)
    assert abs(keep.float().mean().item() - 0.9) < 0.005
    q, k = (torch.randn(T, H, D, device=DEV, dtype=torch.bfloat16) for _ in range(2))
    v = torch.ones(T, H, D, device=DEV, dtype=torch.bfloat16)
    # with V = 1 the output row sum of the (rescaled) dropped probabilities has mean ~1
    o1 = attention._FlashAttn.apply(q, k, v, cu, cu, T, T, 0.125, False, -1, 0.1, 1)
    o2 = attention._FlashAttn.apply(q, k, v, cu, cu, T, T, 0.125, False, -1, 0.1, 1)
    o3 = attention._FlashAttn.apply(q, k, v, cu, cu, T, T, 0.125, False, -1, 0.1, 2)
    assert torch.equal(o1, o2) and not torch.equal(o1, o3)
    assert abs(o1.float().mean().item() - 1.0) < 0.02


def test_rope_flash_attention_dropout_consistent():
    """The fused RoPE+attention node with dropout equals rope -> flash attention with the same seed."""
    from scaling_amd.core.nn.rotary import RotaryEmbedding
    from scaling_amd.core.nn.rotary_config import RotaryConfig

    torch.manual_seed(3)
    T, Hq, Hk, D = 256, 4, 2, 64
    re = RotaryEmbedding(RotaryConfig(dimensions=D, max_seq_length=T), device=torch.device(DEV))
    base = torch.randn(T, (Hq + 2 * Hk) * D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    cu = torch.tensor([0, T], device=DEV, dtype=torch.int32)

    def split(b):
        return (b[:, : Hq * D].view(T, Hq, D), b[:, Hq * D : (Hq + Hk) * D].view(T, Hk, D), b[:, (Hq + Hk) * D :].view(T, Hk, D))

    gen = torch.cuda.default_generators[torch.cuda.current_device()]
    st = gen.get_state()
    o1 = attention.rope_flash_attention(base, *split(base), re.cos_table, re.sin_table, None, D, T, False, cu, T, 0.125,
                                        True, None, dropout_p=0.2)
    gen.set_state(st)
    b2 = base.detach().clone().requires_grad_(True)
    q2, k2, v2 = split(b2)
    q2 = re.apply_tokens(q2, None, T)
    k2 = re.apply_tokens(k2, None, T)
    o2 = attention.flash_attention(q2, k2, v2, cu, cu, T, T, 0.125, True, None, dropout_p=0.2, training=True)
    torch.testing.assert_close(o1.float(), o2.float(), atol=2e-2, rtol=2e-2)
    g = torch.randn_like(o1)
    o1.backward(g)
    o2.backward(g)
    torch.testing.assert_close(base.grad.float(), b2.grad.float(), atol=5e-2, rtol=5e-2)


def test_flash_attention_deterministic():
    torch.manual_seed(1)
    T, H, D = 512, 4, 128
    q, k, v = (torch.randn(T, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    cu = torch.tensor([0, T], device=DEV, dtype=torch.int32)
    g = torch.randn(T, H, D, device=DEV, dtype=torch.bfloat16)
    grads = []
    for _ in range(2):
        for t in (q, k, v):
            t.grad = None
        attention.flash_attention(q, k, v, cu, cu, T, T, None, True).backward(g)
        grads.append([t.grad.clone() for t in (q, k, v)])
    for a, b in zip(*grads):
        assert torch.equal(a, b)


@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (512, 768, 384), (1024, 512, 1024), (1280, 512, 640)])
def test_gemm_tn(M, N, K, accumulate):
    """Weight-gradient GEMM C (+)= A^T B (four-slot ring kernel) against an fp32 reference, incl. a strided (sliced)
    A; 1280 x 512 = 10 tiles exercises the split-K tail on a 256-CU part only when the grid is ragged, the K = 640
    case an odd number of 128-deep pairs per split; K not a multiple of 128 is rejected (hipBLASLt fallback)."""
    torch.manual_seed(5)
    A_full = torch.randn(K, M + 64, device=DEV, dtype=torch.bfloat16)
    A = A_full[:, 64:]  # row stride M + 64, 128-B aligned start
    B = torch.randn(K, N, device=DEV, dtype=torch.bfloat16)
    C0 = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    C = C0.clone()
    assert ext().gemm_tn_ok(A, B, C)
    ext().gemm_tn(A, B, C, accumulate)
    ref = A.float().t() @ B.float() + (C0.float() if accumulate else 0)
    torch.testing.assert_close(C.float(), ref, atol=0.05 * math.sqrt(K / 64), rtol=1e-2)
    assert not ext().gemm_tn_ok(A[:, :200], B, C[:200])
    assert not ext().gemm_tn_ok(A[:64], B[:64], C)


@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("M,N,K", [(5504, 4096, 512), (4096, 5504, 256), (16000, 1024, 256), (2752, 512, 384),
                                   (272, 144, 128)])
def test_gemm_tn_ragged(M, N, K, accumulate):
    """The weight-gradient GEMM at the tensor-parallel per-rank shapes whose M / N are not multiples of 256 (TP2: MLP
    down projection [4096, 5504], LM head [16000, 4096]; TP4: [2752, .]): edge tiles load past the last row / column
    and store only the 16 x 16 blocks inside C.  C is surrounded by sentinel memory that must stay untouched."""
    torch.manual_seed(11)
    A = torch.randn(K, M, device=DEV, dtype=torch.bfloat16)
    B = torch.randn(K, N, device=DEV, dtype=torch.bfloat16)
    pad = 4096
    Cbuf = torch.full((M * N + 2 * pad,), 7.0, device=DEV, dtype=torch.bfloat16)
    C = Cbuf[pad : pad + M * N].view(M, N)
    C0 = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    C.copy_(C0)
    assert ext().gemm_tn_ok(A, B, C)
    ext().gemm_tn(A, B, C, accumulate)
    ref = A.float().t() @ B.float() + (C0.float() if accumulate else 0)
    torch.testing.assert_close(C.float(), ref, atol=0.05 * math.sqrt(K / 64), rtol=1e-2)
    assert bool((Cbuf[:pad] == 7.0).all()) and bool((Cbuf[pad + M * N :] == 7.0).all())
    # the framework entry point takes the HIP kernel for these shapes (no hipBLASLt fallback)
    from scaling_amd.ops import gemm as gemm_ops

    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    gemm_ops.wgrad(A, B, out)
    torch.testing.assert_close(out.float(), A.float().t() @ B.float(), atol=0.05 * math.sqrt(K / 64), rtol=1e-2)


# ---------------------------------------------------------------- masked softmax / activations / dropout
from scaling_amd.ops import elementwise  # noqa: E402


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("seq_len", [128, 200, 1024])
@pytest.mark.parametrize("scale", [1.0, 0.5])
@pytest.mark.parametrize("fp32", [False, True])
def test_masked_softmax_matches_torch(dtype, seq_len, scale, fp32):
    """Reference tolerance (tests/core/test_nn/test_masked_softmax.py:53): mean |delta| < 4e-6."""
    from scaling_amd.core.nn.attention import cumulative_seq_lengths_to_dense_attention_mask

    torch.manual_seed(42)
    x = torch.randn(2, 4, seq_len, seq_len, device=DEV, dtype=dtype)
    cu = torch.tensor([0, seq_len // 3, seq_len, 2 * seq_len], device=DEV)
    mask = cumulative_seq_lengths_to_dense_attention_mask(cu, seq_len, causal=True)
    y = elementwise.masked_softmax(x, mask, scale, fp32)
    ref = elementwise.masked_softmax_reference(x, mask, scale, fp32)
    assert y.dtype == ref.dtype == dtype
    assert (y.float() - ref.float()).abs().mean().item() < 4e-6
    xg = x.detach().float().requires_grad_(True)
    xh = x.detach().clone().requires_grad_(True)
    g = torch.randn_like(x)
    elementwise.masked_softmax(xh, mask, scale, fp32).backward(g)
    elementwise.masked_softmax_reference(xg, mask, scale, True).backward(g.float())
    torch.testing.assert_close(xh.grad.float(), xg.grad, atol=2e-2 if dtype != torch.float32 else 1e-5, rtol=2e-2)


def test_masked_softmax_fully_masked_rows_uniform():
    x = torch.randn(1, 2, 8, 24, device=DEV, dtype=torch.bfloat16)
    mask = torch.ones(1, 1, 8, 24, dtype=torch.bool, device=DEV)
    y = elementwise.masked_softmax(x, mask, 1.0, False)
    torch.testing.assert_close(y.float(), torch.full_like(y.float(), 1 / 24), atol=1e-3, rtol=0)


@pytest.mark.parametrize("kind", ["gelu", "silu", "gelu_tanh"])
@pytest.mark.parametrize("dtype,n", [(torch.bfloat16, 4096 * 3 + 5), (torch.float32, 1000), (torch.float16, 64)])
def test_activation(kind, dtype, n):
    torch.manual_seed(0)
    x = (torch.randn(n, device=DEV, dtype=dtype) * 3).requires_grad_(True)
    xr = x.detach().double().requires_grad_(True)
    y = elementwise.activation(x, kind)
    f = {"gelu": lambda t: torch.nn.functional.gelu(t), "silu": torch.nn.functional.silu,
         "gelu_tanh": lambda t: torch.nn.functional.gelu(t, approximate="tanh")}[kind]
    yr = f(xr)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    torch.testing.assert_close(y.double(), yr, atol=tol, rtol=tol)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g.double())
    torch.testing.assert_close(x.grad.double(), xr.grad, atol=tol * 3, rtol=tol * 3)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("with_res", [True, False])
def test_dropout_add(dtype, with_res):
    torch.manual_seed(0)
    n = 1 << 20
    x = torch.randn(n + 3, device=DEV, dtype=dtype)[3:].requires_grad_(True)  # unaligned view
    res = torch.randn(n, device=DEV, dtype=dtype).requires_grad_(True) if with_res else None
    out = elementwise._DropoutAdd.apply(x, res, 0.3, 99)
    plain = elementwise._DropoutAdd.apply(x.detach(), None, 0.3, 99)  # same seed -> same mask
    kept = plain != 0
    assert abs(kept.float().mean().item() - 0.7) < 0.005
    torch.testing.assert_close(plain.float(), torch.where(kept, x.detach().float() / 0.7, 0.0), atol=1e-2, rtol=1e-2)
    if with_res:
        torch.testing.assert_close(out.float(), res.detach().float() + plain.float(), atol=3e-2, rtol=1e-2)
    out2 = elementwise._DropoutAdd.apply(x, res, 0.3, 99)
    assert torch.equal(out, out2)
    g = torch.randn_like(out)
    out.backward(g)
    torch.testing.assert_close(x.grad.float(), torch.where(kept, g / 0.7, 0.0).float(), atol=1e-2, rtol=1e-2)
    if with_res:
        assert torch.equal(res.grad, g)


@pytest.mark.parametrize("R,C,ld", [(64, 64, 64), (4096, 6144, 6144), (11008, 4096, 4096), (128, 192, 256)])
def test_transpose2d(R, C, ld):
    from scaling_amd.ops.gemm import transpose2d

    base = torch.randn(R, ld, device=DEV, dtype=torch.bfloat16)
    x = base[:, :C]
    assert ext().transpose_ok(x)
    assert torch.equal(transpose2d(x), x.t().contiguous())


def test_linear_dgrad_with_transposed_weight_cache():
    """dX through the cached W^T (forward-layout GEMM) equals dX = dY W; the cache follows weight updates."""
    from scaling_amd.core.nn.linear import main_grad as mg

    torch.manual_seed(0)
    w = [torch.randn(n, 1024, device=DEV, dtype=torch.bfloat16, requires_grad=True) for n in (1024, 256, 256)]
    x = torch.randn(2, 512, 1024, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(2, 512, 1536, device=DEV, dtype=torch.bfloat16)
    mg.invalidate_transposed_weights()
    mg.multi_linear(x, w).backward(g)
    assert getattr(w[0], "_sa_wt_cache", None) is not None  # the cached path ran
    ref = g.float() @ torch.cat(w, 0).detach().float()
    torch.testing.assert_close(x.grad.float(), ref, atol=0.5, rtol=2e-2)
    with torch.no_grad():
        w[1].mul_(-1.0)
    mg.invalidate_transposed_weights()
    x.grad = None
    mg.multi_linear(x, w).backward(g)
    ref2 = g.float() @ torch.cat(w, 0).detach().float()
    torch.testing.assert_close(x.grad.float(), ref2, atol=0.5, rtol=2e-2)


@pytest.mark.parametrize("Lq,Lks,Hq,Hk,D,causal,window,local_heads,dtype", [
    (1, [4096], 32, 8, 128, True, -1, None, torch.bfloat16),       # 7B cached decode step
    (1, [17, 1000, 3], 8, 8, 64, True, -1, None, torch.bfloat16),  # MHA, ragged caches, one segment per sequence
    (4, [333, 64], 16, 2, 128, True, -1, None, torch.float16),    # 4-token chunk x 8 q heads = 32 packed rows
    (2, [700], 8, 2, 128, True, 50, 3, torch.bfloat16),           # mixed local/global heads
    (3, [130, 90], 4, 4, 32, False, -1, None, torch.bfloat16),    # non-causal, D 32
])
def test_flash_decoding(Lq, Lks, Hq, Hk, D, causal, window, local_heads, dtype):
    """Short query segments take the split-K flash-decoding kernels (GQA rows packed, combine pass); output and
    lse against the fp32 reference."""
    torch.manual_seed(0)
    n = len(Lks)
    cu_q = torch.arange(0, (n + 1) * Lq, Lq, device=DEV, dtype=torch.int32)
    cu_k = torch.tensor([0] + list(torch.tensor(Lks).cumsum(0)), device=DEV, dtype=torch.int32)
    q = torch.randn(n * Lq, Hq, D, device=DEV, dtype=dtype)
    k = torch.randn(sum(Lks), Hk, D, device=DEV, dtype=dtype)
    v = torch.randn(sum(Lks), Hk, D, device=DEV, dtype=dtype)
    scale = 1 / math.sqrt(D)
    with torch.no_grad():
        o = attention.flash_attention(q, k, v, cu_q, cu_k, Lq, max(Lks), scale, causal, None if window < 0 else window,
                                      local_heads=local_heads)
        o2, lse = ext().fa_fwd(q, k, v, cu_q, cu_k, Lq, scale, causal, window, 0.0, 0,
                               -1 if local_heads is None else local_heads, max(Lks))
    ref = attention.attention_reference(q.float(), k.float(), v.float(), cu_q, cu_k, scale, causal, window,
                                        local_heads=local_heads)
    torch.testing.assert_close(o.float(), ref, atol=2e-2, rtol=2e-2)
    assert torch.equal(o, o2)
    # lse of the first segment's rows against log-sum-exp of the reference scores
    qq, kk = q[:Lq].float(), k[: Lks[0]].float().repeat_interleave(Hq // Hk, 1)
    s = torch.einsum("qhd,khd->hqk", qq, kk) * scale
    qpos = torch.arange(Lq, device=DEV)[:, None] + Lks[0] - Lq
    kpos = torch.arange(Lks[0], device=DEV)[None, :]
    ok = torch.ones(Lq, Lks[0], dtype=torch.bool, device=DEV)
    if causal:
        ok &= kpos <= qpos
    okw = ok & (kpos >= qpos - window) & ((kpos <= qpos + window) if not causal else ok) if window >= 0 else ok
    nl = Hq if local_heads is None else local_heads
    mask = torch.stack([okw if h < nl else ok for h in range(Hq)])
    lse_ref = torch.logsumexp(s.masked_fill(~mask, float("-inf")), -1)
    torch.testing.assert_close(lse[:, :Lq], lse_ref, atol=2e-2, rtol=1e-3)


def test_flash_decoding_forward_with_prefill_backward():
    """Tiny training segments (max_q x group <= 32) run the decode forward and the regular backward kernels."""
    _attn_case([7, 5], 4, 1, 64, True)
    _attn_case([8], 4, 4, 128, False)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(1, 4096, 4096), (1, 22016, 4096), (1, 4096, 11008), (2, 1003, 200), (3, 77, 64),
                                   (4, 32000, 4096), (1, 5, 8)])
@pytest.mark.parametrize("bias", [False, True])
def test_gemv(dtype, M, N, K, bias):
    """Decode-time linear layer y = x W^T (+ b) for <= 4 rows against an fp32 reference, through ops.gemm.linear
    (which must route these shapes to the GEMV kernel)."""
    from scaling_amd.ops import gemm

    torch.manual_seed(0)
    x = torch.randn(M, K, device=DEV, dtype=dtype)
    w = torch.randn(N, K, device=DEV, dtype=dtype) / math.sqrt(K)
    b = torch.randn(N, device=DEV, dtype=dtype) if bias else None
    assert ext().gemv_ok(x, w)
    y = gemm.linear(x.view(M, 1, K), w, b).view(M, N)
    ref = x.float() @ w.float().t() + (b.float() if bias else 0.0)
    torch.testing.assert_close(y.float(), ref, atol=2e-2, rtol=2e-2)
    # the same through a row-strided view of a wider weight (fused q/k/v / gate-up buffers)
    wide = torch.randn(N, K + 64, device=DEV, dtype=dtype) / math.sqrt(K)
    wv = wide[:, 32 : 32 + K]
    torch.testing.assert_close(ext().gemv(x, wv).float(), x.float() @ wv.float().t(), atol=2e-2, rtol=2e-2)


def test_gemv_rejects_unsupported():
    x = torch.randn(5, 64, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(32, 64, device=DEV, dtype=torch.bfloat16)
    assert not ext().gemv_ok(x, w)  # more than 4 rows: hipBLASLt
    assert not ext().gemv_ok(x[:1, :60], w[:, :60])  # K % 8
    assert not ext().gemv_ok(x[:1].float(), w.float())  # fp32


@pytest.mark.parametrize("layer", [False, True])
@pytest.mark.parametrize("rows", [1, 2, 3, 4])
@pytest.mark.parametrize("H", [4096, 2048, 8192, 520])
def test_norm_decode_rows_kernel(layer, rows, H):
    """Decode-sized rows (<= 4) run the early-weight-load row kernel: same outputs as the fp32 reference (plain and
    residual-fused), bit-identical to the many-row kernel, and rstd / mean saved for the backward."""
    torch.manual_seed(3)
    dtype = torch.bfloat16
    x = torch.randn(rows, H, device=DEV, dtype=dtype, requires_grad=True)
    r = torch.randn(rows, H, device=DEV, dtype=dtype)
    w = (1 + 0.1 * torch.randn(H, device=DEV, dtype=dtype))
    b = 0.1 * torch.randn(H, device=DEV, dtype=dtype)
    tol = 2e-2
    y = norm.layer_norm(x, w, b, 1e-5) if layer else norm.rms_norm(x, w, 1e-5)
    xr, wr, br = x.detach().float(), w.float(), b.float()
    yr = torch.nn.functional.layer_norm(xr, (H,), wr, br, 1e-5) if layer else norm.rms_norm_reference(xr, wr, 1e-5)
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    s, y2 = norm.add_layer_norm(x, r, w, b, 1e-5) if layer else norm.add_rms_norm(x, r, w, 1e-5)
    sr = (x.detach() + r).float()
    torch.testing.assert_close(s.float(), sr, atol=0, rtol=0)
    yr2 = torch.nn.functional.layer_norm(sr, (H,), wr, br, 1e-5) if layer else norm.rms_norm_reference(sr, wr, 1e-5)
    torch.testing.assert_close(y2.float(), yr2, atol=tol, rtol=tol)
    # bit-identical to the many-row kernel (same per-lane summation order): rows of a 5-row call
    x5 = torch.cat([x.detach(), torch.randn(1, H, device=DEV, dtype=dtype)])
    r5 = torch.cat([r, torch.randn(1, H, device=DEV, dtype=dtype)])
    y5 = norm.layer_norm(x5, w, b, 1e-5) if layer else norm.rms_norm(x5, w, 1e-5)
    assert torch.equal(y5[:rows], y.detach())
    s5, y25 = norm.add_layer_norm(x5, r5, w, b, 1e-5) if layer else norm.add_rms_norm(x5, r5, w, 1e-5)
    assert torch.equal(y25[:rows], y2.detach()) and torch.equal(s5[:rows], s.detach())
    g = torch.randn_like(y)
    (gx,) = torch.autograd.grad(y, x, g)  # the backward reads the rstd / mean the row kernel stored
    xr2 = x.detach().float().requires_grad_(True)
    yr3 = (torch.nn.functional.layer_norm(xr2, (H,), wr, br, 1e-5) if layer
           else norm.rms_norm_reference(xr2, wr, 1e-5))
    (gr,) = torch.autograd.grad(yr3, xr2, g.float())
    torch.testing.assert_close(gx.float(), gr, atol=4e-2, rtol=4e-2)


@pytest.mark.parametrize("rows", [1, 2, 4])
def test_small_linear_keeps_autograd(rows):
    """ops.gemm.linear sends <= 4 rows to the (autograd-free) GEMV kernel only when no graph is needed: a tied-head
    style call on a tiny training micro-batch must still produce gradients for the input and the weight."""
    from scaling_amd.ops import gemm

    torch.manual_seed(0)
    w = torch.randn(256, 128, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    x = torch.randn(rows, 128, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = gemm.linear(x, w)
    assert y.grad_fn is not None
    y.float().sum().backward()
    wr = w.detach().float().requires_grad_(True)
    xr = x.detach().float().requires_grad_(True)
    torch.nn.functional.linear(xr, wr).sum().backward()
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=0.3, rtol=2e-2)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=0.1, rtol=2e-2)
    with torch.no_grad():  # inference keeps the GEMV path
        torch.testing.assert_close(gemm.linear(x, w).float(), xr.detach() @ wr.detach().t(), atol=0.3, rtol=2e-2)


@pytest.mark.parametrize("rows", [1, 2, 3, 4])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_gemv_epilogues_bit_identical(rows, dtype):
    """Decode GEMV epilogues: gate/up GEMV + SwiGLU and down GEMV + residual add in one launch each, bit-identical
    to the unfused GEMV / SwiGLU kernel / torch add sequence (so cached decoding rounds like the eager path)."""
    from scaling_amd.ops import swiglu

    torch.manual_seed(rows)
    F, K = 1376, 512
    x = torch.randn(rows, K, device=DEV, dtype=dtype)
    w = torch.randn(2 * F, K, device=DEV, dtype=dtype) / 16
    wo = torch.randn(K, F, device=DEV, dtype=dtype) / 16
    res = torch.randn(rows, K, device=DEV, dtype=dtype)
    h_ref = swiglu.swiglu_fused(ext().gemv(x, w, None))
    h = ext().gemv_swiglu(x, w)
    assert torch.equal(h, h_ref)
    ref = res + ext().gemv(h_ref, wo, None)
    assert torch.equal(ext().gemv_residual(h, wo, res), ref)
    # against fp32 math
    hf = torch.nn.functional.silu(x.float() @ w[:F].float().t()) * (x.float() @ w[F:].float().t())
    torch.testing.assert_close(h.float(), hf, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("rows", [1, 2, 4])
@pytest.mark.parametrize("K", [4096, 520, 8192])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_gemv_norm_fused(rows, K, dtype):
    """Decode GEMV with the RMSNorm (and its residual add) folded into the pass over the weights: the residual sum s
    is bit-identical to add_rms_norm's, y matches fp32 math of norm + GEMV (plain / SwiGLU epilogues) and stays
    within bf16 rounding of the unfused norm + GEMV kernels."""
    from scaling_amd.ops import norm as norm_ops

    torch.manual_seed(rows + K)
    N, F = 264, 136
    x = torch.randn(rows, K, device=DEV, dtype=dtype)
    add = torch.randn(rows, K, device=DEV, dtype=dtype)
    g = 1 + 0.1 * torch.randn(K, device=DEV, dtype=dtype)
    w = torch.randn(N, K, device=DEV, dtype=dtype) / math.sqrt(K)
    w2 = torch.randn(2 * F, K, device=DEV, dtype=dtype) / math.sqrt(K)
    assert ext().gemv_norm_ok(x, w, g)

    def rms(t):
        t = t.float()
        return t * torch.rsqrt(t.pow(2).mean(-1, keepdim=True) + 1e-5) * g.float()

    s, y = ext().gemv_norm(x, None, g, 1e-5, w, 0)
    assert s.data_ptr() == x.data_ptr()
    torch.testing.assert_close(y.float(), rms(x) @ w.float().t(), atol=2e-2, rtol=2e-2)
    _, xn = norm_ops.add_rms_norm(x, None, g, 1e-5)
    torch.testing.assert_close(y, ext().gemv(xn, w, None), atol=3e-2, rtol=3e-2)
    s_ref, xn2 = norm_ops.add_rms_norm(add, x, g, 1e-5)  # the layer's order: residual + attention output
    s, y2 = ext().gemv_norm(x, add, g, 1e-5, w2, 2)
    assert torch.equal(s, s_ref)
    nf = rms(s_ref)
    hf = torch.nn.functional.silu(nf @ w2[:F].float().t()) * (nf @ w2[F:].float().t())
    torch.testing.assert_close(y2.float(), hf, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(y2, ext().gemv_swiglu(xn2, w2), atol=3e-2, rtol=3e-2)
    # deterministic: the same call twice is bit-identical (eager and graph decoding run the same kernel)
    assert torch.equal(ext().gemv_norm(x, add, g, 1e-5, w2, 2)[1], y2)


@pytest.mark.parametrize("rot_frac", [1.0, 0.5])
def test_gemv_norm_rope_matches_unfused(rot_frac):
    """Graph-decode q/k/v step in one launch (norm + GEMV + interleaved RoPE + K/V cache append at the device position)
    against gemv_norm followed by rope_kv_append."""
    torch.manual_seed(5)
    nq, nkv, hd, K, cap = 8, 2, 128, 1024, 64
    rd = int(hd * rot_frac)
    half = rd // 2
    inv = 1.0 / (10000 ** (torch.arange(0, half, device=DEV, dtype=torch.float32) / half))
    ang = torch.arange(cap, device=DEV, dtype=torch.float32)[:, None] * inv[None]
    cos, sin = ang.cos().contiguous(), ang.sin().contiguous()
    x = torch.randn(1, K, device=DEV, dtype=torch.bfloat16)
    g = 1 + 0.1 * torch.randn(K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn((nq + 2 * nkv) * hd, K, device=DEV, dtype=torch.bfloat16) / math.sqrt(K)
    pos = torch.tensor([29], device=DEV, dtype=torch.long)
    kc = torch.randn(cap, nkv, hd, device=DEV, dtype=torch.bfloat16)
    vc = torch.randn(cap, nkv, hd, device=DEV, dtype=torch.bfloat16)
    kc_ref, vc_ref = kc.clone(), vc.clone()
    _, base = ext().gemv_norm(x, None, g, 1e-5, w, 0)
    err = torch.zeros(1, device=DEV, dtype=torch.int32)
    q_ref = ext().rope_kv_append(base.view(1, nq + 2 * nkv, hd), cos, sin, pos, nq, nkv, rd, True, kc_ref, vc_ref, err)
    q = ext().gemv_norm_rope(x, g, 1e-5, w, cos, sin, pos, nq, nkv, rd, kc, vc, err)
    assert q is not None and q_ref is not None
    torch.testing.assert_close(q, q_ref, atol=1e-2, rtol=1e-2)
    torch.testing.assert_close(kc, kc_ref, atol=1e-2, rtol=1e-2)
    assert torch.equal(vc, vc_ref)
    other = torch.ones(cap, dtype=torch.bool, device=DEV)
    other[29] = False
    assert torch.equal(kc[other], kc_ref[other])  # only the position's row was written
    assert int(err.item()) == 0
    assert ext().gemv_norm_rope(torch.randn(2, K, device=DEV, dtype=torch.bfloat16), g, 1e-5, w, cos, sin, pos, nq,
                                nkv, rd, kc, vc, err) is None  # one token only
    # a position past the cache: nothing written, q zeroed, the error word set (no silent out-of-bounds write)
    kc0, vc0 = kc.clone(), vc.clone()
    q = ext().gemv_norm_rope(x, g, 1e-5, w, cos, sin, torch.tensor([cap], device=DEV), nq, nkv, rd, kc, vc, err)
    assert int(err.item()) == 1 and torch.equal(kc, kc0) and torch.equal(vc, vc0) and not q.any()


def test_decode_layer_norm_gemv_matches_unfused():
    """The decode MLP block with the post-attention RMSNorm folded into the gate/up GEMV matches the unfused
    add_rms_norm + GEMV-epilogue path within bf16 rounding, and writes the same residual stream."""
    from scaling_amd.core.nn.mlp import ParallelSwiGLUMLP
    from scaling_amd.core.nn.norm import RMSNorm, LayerNormConfig

    torch.manual_seed(0)
    H = 1024
    mlp = ParallelSwiGLUMLP(H, 2.6875, bias=False, device=DEV, dtype=torch.bfloat16).requires_grad_(False)
    norm = RMSNorm(H, DEV, LayerNormConfig(), dtype=torch.bfloat16).requires_grad_(False)
    norm.weight.copy_(1 + 0.1 * torch.randn(H, device=DEV))
    resid = torch.randn(1, 1, H, device=DEV, dtype=torch.bfloat16)
    h = torch.randn(1, 1, H, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        out = mlp.decode_forward_norm(h, resid, norm)
        assert out is not None
        s, normed = norm.forward_add(resid, h)
        ref = mlp.decode_forward_residual(normed, s)
    torch.testing.assert_close(out.float(), ref.float(), atol=5e-2, rtol=2e-2)


@pytest.mark.parametrize("interleaved", [False, True])
@pytest.mark.parametrize("rot_frac", [1.0, 0.5])
def test_rope_kv_append_bit_identical(interleaved, rot_frac):
    """Graph-decode step kernel: RoPE(q), RoPE(k) into the K cache row at the device position, v into the V cache
    row -- one launch, bit-identical to rope() twice + two index_copy_."""
    torch.manual_seed(3)
    nq, nkv, hd, cap = 8, 2, 128, 64
    rd = int(hd * rot_frac)
    half = rd // 2
    inv = 1.0 / (10000 ** (torch.arange(0, half, device=DEV, dtype=torch.float32) / half))
    ang = torch.arange(cap, device=DEV, dtype=torch.float32)[:, None] * inv[None]
    cos, sin = ang.cos().contiguous(), ang.sin().contiguous()
    qkv = torch.randn(1, nq + 2 * nkv, hd, device=DEV, dtype=torch.bfloat16)
    pos = torch.tensor([37], device=DEV, dtype=torch.long)
    kc = torch.randn(cap, nkv, hd, device=DEV, dtype=torch.bfloat16)
    vc = torch.randn(cap, nkv, hd, device=DEV, dtype=torch.bfloat16)
    kc_ref, vc_ref = kc.clone(), vc.clone()
    q_ref = ext().rope(qkv[:, :nq], cos, sin, pos, rd, 1, interleaved, False)
    k_ref = ext().rope(qkv[:, nq:nq + nkv], cos, sin, pos, rd, 1, interleaved, False)
    kc_ref.index_copy_(0, pos, k_ref)
    vc_ref.index_copy_(0, pos, qkv[:, nq + nkv:])
    err = torch.zeros(1, device=DEV, dtype=torch.int32)
    q = ext().rope_kv_append(qkv, cos, sin, pos, nq, nkv, rd, interleaved, kc, vc, err)
    assert q is not None
    assert torch.equal(q, q_ref) and torch.equal(kc, kc_ref) and torch.equal(vc, vc_ref) and int(err.item()) == 0
    # positions outside [0, cap): no cache row written, q zeroed, the error word set
    for bad in (cap, cap + 5, -1):
        err.zero_()
        q = ext().rope_kv_append(qkv, cos, sin, torch.tensor([bad], device=DEV), nq, nkv, rd, interleaved, kc, vc, err)
        assert int(err.item()) == 1 and not q.any() and torch.equal(kc, kc_ref) and torch.equal(vc, vc_ref)


@pytest.mark.parametrize("T,H,F", [(512, 256, 512), (1024, 512, 768)])
def test_swiglu_mlp_matches_fp32_reference(T, H, F):
    """ParallelSwiGLUMLP on the GPU path (fused gate/up GEMM, HIP SwiGLU kernels, HIP weight-gradient GEMM): output,
    input gradient and weight gradients against an fp32 PyTorch reference of the same MLP."""
    from scaling_amd.core.nn.mlp import ParallelSwiGLUMLP

    torch.manual_seed(3)
    mlp = ParallelSwiGLUMLP(H, F / H, bias=False, device=torch.device(DEV), dtype=torch.bfloat16)
    x = torch.randn(2, T // 2, H, device=DEV, dtype=torch.bfloat16)
    dy = torch.randn(2, T // 2, H, device=DEV, dtype=torch.bfloat16)
    xi = x.clone().requires_grad_(True)
    y = mlp(xi)
    y.backward(dy)
    got = [y.float(), xi.grad.float()] + [p.grad.float() for p in (mlp.dense_in.weight, mlp.siglu_weight.weight,
                                                                     mlp.dense_out.weight)]
    xf = x.float().reshape(-1, H).requires_grad_(True)
    wg, wu, wd = (p.detach().float().requires_grad_(True) for p in (mlp.dense_in.weight, mlp.siglu_weight.weight,
                                                                   mlp.dense_out.weight))
    yf = (torch.nn.functional.silu(xf @ wg.t()) * (xf @ wu.t())) @ wd.t()
    yf.backward(dy.float().reshape(-1, H))
    for a, r in zip(got, [yf, xf.grad, wg.grad, wu.grad, wd.grad]):
        assert (a.reshape(r.shape) - r).abs().max().item() < 0.03 * r.abs().max().item()


def test_xgmi_emulate_moves_bytes_and_holds_time():
    """The per-rank proxy's emulated collective (ext().xgmi_emulate): the send volume is streamed from the source into
    the scratch ring (wrapping both), and the kernel holds its CUs until the modelled time has passed."""
    import time

    src = torch.randn(1 << 16, device=DEV)  # 256 KiB
    scratch = torch.zeros(1 << 15, device=DEV)  # 128 KiB ring
    ext().xgmi_emulate(src, scratch, src.numel() * 4, 0.0, 4)  # bytes only
    torch.cuda.synchronize()
    # the second half of the source wrapped onto the first: the ring holds src[32768:]
    assert torch.equal(scratch, src[1 << 15:])
    t0 = time.perf_counter()
    for _ in range(5):
        ext().xgmi_emulate(src, scratch, 1024, 2000.0, 4)  # 2 ms each
    torch.cuda.synchronize()
    assert time.perf_counter() - t0 >= 0.0095


def test_stream_gate_holds_until_host_flag():
    """The asynchronous rehearsal's stream gate (``ext().gate_stream_wait``: hipStreamWaitValue32 on a flag word in
    coherent pinned host memory): work queued behind the gate runs only after the host writes the flag, and a later
    gate on the same word at the next generation releases at once when the flag is written first."""
    import threading
    import time

    x = torch.zeros(1, device="cuda")
    s = torch.cuda.Stream()
    base = ext().gate_flags_alloc(4)
    ev = torch.cuda.Event()
    with torch.cuda.stream(s):
        x.fill_(1)
        ext().gate_stream_wait(base, 0, 1)
        x.add_(1)
        ev.record(s)
    t0 = time.time()
    threading.Timer(0.3, lambda: ext().gate_flag_write(base, 0, 1)).start()
    time.sleep(0.1)
    assert not ev.query()  # held by the gate
    s.synchronize()
    assert time.time() - t0 >= 0.29 and x.item() == 2.0
    ext().gate_flag_write(base, 0, 2)
    with torch.cuda.stream(s):
        ext().gate_stream_wait(base, 0, 2)
        x.add_(1)
    s.synchronize()
    assert x.item() == 3.0 and ext().gate_flag_read(base, 0) == 2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_small_gemm_plans_match_torch(dtype):
    """Small GEMMs through cached hipBLASLt plans (``ext().lt_linear`` / ``lt_mm``, ``ops/gemm.py``): x @ w^T (+ b) and
    a @ b against an fp32 reference, ragged shapes included; a second call with the same shape reuses the plan and
    gives the same bits."""
    from scaling_amd.ops import gemm

    torch.manual_seed(0)
    for M, N, K in ((128, 768, 256), (130, 1000, 256), (64, 128000, 256), (7, 96, 40)):
        x = torch.randn(M, K, device=DEV, dtype=dtype)
        w = torch.randn(N, K, device=DEV, dtype=dtype) * 0.05
        b = torch.randn(N, device=DEV, dtype=dtype)
        y = ext().lt_linear(x, w, b)
        assert y is not None and y.shape == (M, N)
        ref = x.float() @ w.float().t() + b.float()
        torch.testing.assert_close(y.float(), ref, atol=2e-2, rtol=2e-2)
        y2 = ext().lt_linear(x, w, None)
        torch.testing.assert_close(y2.float(), x.float() @ w.float().t(), atol=2e-2, rtol=2e-2)
        assert torch.equal(ext().lt_linear(x, w, b), y)
        g = torch.randn(M, N, device=DEV, dtype=dtype) * 0.1
        d = ext().lt_mm(g, w)
        torch.testing.assert_close(d.float(), g.float() @ w.float(), atol=3e-2, rtol=2e-2)
        # the ops-level entry points take the plan path for these sizes
        torch.testing.assert_close(gemm.mm(g, w).float(), d.float(), atol=0, rtol=0)
        torch.testing.assert_close(gemm.linear(x, w, b).float(), y.float(), atol=0, rtol=0)
