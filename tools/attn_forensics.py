"""Race-check forensics for the fused RoPE + flash-attention backward, outside the production autograd node.

Loaded into bench.py ranks with ``SCALING_AMD_DEBUG_HOOKS=tools/attn_forensics.py`` (``tools/race_trace.py`` passes it
through); wraps ``ops.attention._RopeFlashAttn.bwd_into``:

* ``ATTN_FORENSICS_SYNC=1``   device synchronisation right before and after every attention backward (nothing else
  of the process may run beside it);
* ``ATTN_FORENSICS_TWICE=1``  the same backward two more times into fresh buffers, with the differences recorded
  through ``core/utils/grad_probe.record_values("rope_flash.twice_mismatch", ...)``:
  [total, dq, dk, dv, first 4 flat indices, row length, third == first, third == second, distinct rows, max |diff|,
  up to 16 distinct columns (-1 padded), first 4 differing values of the first run, then of the second];
  with ``ATTN_FORENSICS_OUT=<prefix>`` each rank also writes ``<prefix>.rank<r>.json`` at exit: backwards checked,
  backwards with any difference, differing elements, largest difference (the rate a candidate fix must bring to 0);
* ``ATTN_FORENSICS_NOROPE=1`` every checked computation (the production one too) runs WITHOUT the inverse RoPE of
  dq / dk (plain attention backward; training numbers are then wrong, the comparison is not): tells whether a
  difference comes from the rotation pass or from the attention kernels.
"""
from __future__ import annotations

import atexit
import json
import os

import torch

from scaling_amd.core.utils import grad_probe
from scaling_amd.ops import attention

_SYNC = os.environ.get("ATTN_FORENSICS_SYNC") == "1"
_TWICE = os.environ.get("ATTN_FORENSICS_TWICE") == "1"
_NOROPE = os.environ.get("ATTN_FORENSICS_NOROPE") == "1"
_orig_rope = attention._RopeFlashAttn.bwd_into


def _orig(saved, cfg, do, dq, dk, dv) -> None:
    if not _NOROPE:
        return _orig_rope(saved, cfg, do, dq, dk, dv)
    from scaling_amd.ops._ext import ext

    base, q, k, o, lse, cu_q, cu_k, cos, sin, pos = saved
    specs, rot_dim, seq_len, interleaved, max_q, max_k, scale, causal, window, p_drop, seed, local_heads = cfg
    v = attention._view(base, specs[2])
    ext().fa_bwd(do, q, k, v, o, lse, cu_q, cu_k, max_q, max_k, scale, causal, window, dq, dk, dv, p_drop, seed,
                 local_heads)
_OUT = os.environ.get("ATTN_FORENSICS_OUT")
_stats: list = []  # per checked backward: the mismatch record (device tensors; read once, at exit)


def _summary() -> None:
    if not _OUT or not _stats:
        return
    allr = torch.stack([r[:13] for r in _stats]).cpu()  # total, dq, dk, dv, 4 indices, row length, d3==d1, d3==d2, rows, max
    rows, mx, third_first, third_second = allr[:, 0], allr[:, 12], allr[:, 9], allr[:, 10]
    diff = rows > 0
    rank = os.environ.get("RANK", "0")
    with open(f"{_OUT}.rank{rank}.json", "w") as f:
        json.dump({"backwards": len(_stats), "with_difference": int((rows > 0).sum()), "elements": float(rows.sum()),
                   "max_abs_diff": float(mx.max()),
                   "differing_with_third_equal_first": int((diff & (third_first > 0)).sum()),
                   "differing_with_third_equal_second": int((diff & (third_second > 0)).sum()),
                   "elements_dq_dk_dv": [float(allr[:, i].sum()) for i in (1, 2, 3)],
                   "differing_backward_index": [int(i) for i in torch.nonzero(diff).reshape(-1).tolist()],
                   "distinct_rows": [int(v) for v in allr[diff, 11].tolist()],
                   "first_differing_token": [int(v) for v in (allr[diff, 4] // allr[diff, 8]).tolist()]}, f)


atexit.register(_summary)


def _mismatch(dbase: torch.Tensor, d2: torch.Tensor, d3: torch.Tensor, views1, views2) -> torch.Tensor:
    f64 = dict(device=dbase.device, dtype=torch.float64)
    ne = d2 != dbase
    first = torch.full((4,), -1.0, **f64)
    nz = torch.nonzero(ne.reshape(-1))[:4].reshape(-1).double()
    first[:nz.numel()] = nz
    counts = torch.stack([(a != b).sum() for a, b in zip(views2, views1)]).double()
    rows_ne, cols_ne = ne.reshape(ne.shape[0], -1).any(1), ne.reshape(ne.shape[0], -1).any(0)
    cols = torch.full((16,), -1.0, **f64)
    cz = torch.nonzero(cols_ne).reshape(-1)[:16].double()
    cols[:cz.numel()] = cz
    extra = torch.stack([torch.equal(d3, dbase) * torch.ones((), **f64), torch.equal(d3, d2) * torch.ones((), **f64),
                         rows_ne.sum().double(), (d2.float() - dbase.float()).abs().max().double()])
    vals = torch.zeros(8, **f64)
    ix = first[:nz.numel()].long()
    vals[:nz.numel()] = dbase.reshape(-1)[ix].double()
    vals[4:4 + nz.numel()] = d2.reshape(-1)[ix].double()
    return torch.cat([ne.sum().double().reshape(1), counts, first, torch.tensor([float(dbase.shape[-1])], **f64), extra,
                      cols, vals])


def bwd_into(saved, cfg, do, dq, dk, dv) -> None:
    if _SYNC and do.is_cuda:
        torch.cuda.synchronize(do.device)
    _orig(saved, cfg, do, dq, dk, dv)
    if _SYNC and do.is_cuda:
        torch.cuda.synchronize(do.device)
    if not _TWICE:
        return
    base = saved[0]
    specs = cfg[0]
    dbase = dq.as_strided(base.shape, base.stride(), dq.storage_offset() - specs[0][2])
    outs = []
    for _ in range(2):
        d = torch.empty_like(base)
        views = [attention._view(d, sp) for sp in specs]
        _orig(saved, cfg, do, *views)
        outs.append((d, views))
    (d2, v2), (d3, _) = outs
    rec = _mismatch(dbase, d2, d3, (dq, dk, dv), v2)
    grad_probe.record_values("rope_flash.twice_mismatch", rec)
    if _OUT:
        _stats.append(rec)


attention._RopeFlashAttn.bwd_into = staticmethod(bwd_into)
