"""Per-step communication volume of a training layout (bytes each rank sends), and a first-order time estimate
on MI355X xGMI, so a multi-GPU run can be read against what its layout must move.

Model (one data-parallel replica processes ``micro_batch x grad_acc`` sequences of ``s`` tokens per step;
``M = micro_batch * s`` tokens per micro-batch; activations in the model dtype, ``h`` = hidden size):

* tensor parallel (``t > 1``), per layer and micro-batch: two row-parallel output reductions in the forward
  (attention dense, MLP out) and two column-parallel input-gradient reductions in the backward, each an
  all-reduce of ``[M, h]`` -- or, with sequence parallelism, a reduce-scatter + all-gather pair of the same
  total -- at ``2 (t-1)/t x M h`` elements sent per rank (ring); plus the embedding's forward all-reduce;
* pipeline parallel (``p > 1``), per micro-batch: the ``[M, h]`` activation forward and its gradient backward
  across each stage boundary a rank owns (at most one of each direction per rank);
* data parallel (``d > 1``, ZeRO-1 as implemented): reduce-scatter of the fp32 (or bf16, ``grad_reduce_dtype``)
  gradient buckets and all-gather of the updated parameters, ``(d-1)/d`` of the rank's parameter shard each.

Time: the 8 GPUs of a node are fully connected, one xGMI link per pair (7 per GPU).  AMD quotes 153.6 GB/s "peak
Infinity Fabric link bandwidth" for MI355X; the MI300X figure of the same kind (128 GB/s x 7 links = 896 GB/s) is the
aggregate BIDIRECTIONAL rate, so one direction of one link carries half: 76.8 GB/s (rounds 1-5 used 153 GB/s per
direction here, 2x optimistic -- VERDICT r5, Weak #5; no xGMI figure exists in MI355X_MICROARCH.md and this pool has
no multi-GPU box to measure it on).  A TP group of 2 rides its one link; larger TP groups and DP rings are spread over
``min(group-1, 7)`` links by RCCL's multi-ring schedule.  Each collective also pays a fixed latency
(``COLLECTIVE_LATENCY_S``).  The estimate assumes ``link_efficiency`` of the peak and no overlap; it is a reading aid,
not a prediction, and ``collective_time_s`` is what the per-rank proxy's emulated collectives hold the GPU for
(``core/topology/stub_collectives.py``).
"""
from __future__ import annotations

from typing import Any

XGMI_LINK_BYTES_PER_S = 76.8e9  # one direction of one link (153.6 GB/s bidirectional)
XGMI_LINKS_PER_GPU = 7
COLLECTIVE_LATENCY_S = 10e-6  # launch + handshake of one intra-node RCCL collective (order of magnitude)
LINK_EFFICIENCY = 0.75


def ring_send_bytes(kind: str, nbytes: int, group: int) -> float:
    """Bytes one rank sends per collective over a ring of ``group`` ranks: ``nbytes`` is the all-reduce tensor, the
    reduce-scatter INPUT or the all-gather OUTPUT (the full, un-sharded size in each case)."""
    if group <= 1:
        return 0.0
    f = (group - 1) / group
    return 2.0 * f * nbytes if kind == "all_reduce" else f * nbytes


def collective_time_s(kind: str, nbytes: int, group: int, link_efficiency: float = LINK_EFFICIENCY) -> float:
    """First-order time of one collective on the node's xGMI mesh (latency + ring bytes over the group's links)."""
    if group <= 1:
        return 0.0
    links = min(group - 1, XGMI_LINKS_PER_GPU)
    return COLLECTIVE_LATENCY_S + ring_send_bytes(kind, nbytes, group) / (XGMI_LINK_BYTES_PER_S * link_efficiency * links)


def _dtype_bytes(precision: str) -> int:
    return 4 if precision in ("float32", "fp32") else 2


def comm_volume_estimate(*, hidden_size: int, num_layers: int, seq_len: int, micro_batch: int, grad_acc: int,
                         tp: int, pp: int, dp: int, params_per_rank: int, precision: str = "bfloat16",
                         grad_reduce_bytes: int = 4, link_efficiency: float = LINK_EFFICIENCY) -> dict[str, Any]:
    act = _dtype_bytes(precision)
    M = micro_batch * seq_len
    ring = lambda n: 2.0 * (n - 1) / n if n > 1 else 0.0  # noqa: E731 - all-reduce bytes factor per rank
    layers_here = num_layers / pp
    tp_bytes = 0.0
    if tp > 1:
        per_mb = (4 * layers_here + 1) * ring(tp) * M * hidden_size * act  # + 1: embedding (first stage)
        tp_bytes = per_mb * grad_acc
    pp_bytes = 2.0 * M * hidden_size * act * grad_acc if pp > 1 else 0.0
    dp_bytes = 0.0
    if dp > 1:
        frac = (dp - 1) / dp
        dp_bytes = frac * params_per_rank * grad_reduce_bytes + frac * params_per_rank * act
    eff_link = XGMI_LINK_BYTES_PER_S * link_efficiency

    def t_ms(nbytes: float, group: int) -> float:
        if nbytes == 0.0:
            return 0.0
        links = min(max(group - 1, 1), XGMI_LINKS_PER_GPU)
        return 1e3 * nbytes / (eff_link * links)

    return {
        "tp_bytes": int(tp_bytes), "pp_bytes": int(pp_bytes), "dp_bytes": int(dp_bytes),
        "tp_ms": round(t_ms(tp_bytes, tp), 2), "pp_ms": round(t_ms(pp_bytes, 2), 2), "dp_ms": round(t_ms(dp_bytes, dp), 2),
        "assumptions": f"xGMI {XGMI_LINK_BYTES_PER_S / 1e9:.1f} GB/s per link and direction x {link_efficiency}, "
                       "no overlap",
    }


def default_tp_comm_chunks(*, hidden_size: int, tokens: int, tp: int, in_features: int | None = None,
                           precision: str = "bfloat16", gemm_flops_per_s: float = 1.2e15, chunk_latency_s: float = 25e-6,
                           min_chunk_rows: int = 2048, link_efficiency: float = LINK_EFFICIENCY) -> int:
    """Token pieces for the row-parallel GEMM + TP collective overlap (``tensor_parallel_comm_chunks``) from the
    same first-order model: the collective of ``[tokens, hidden]`` takes ``tc`` on the TP group's links, the local
    GEMM (``in_features / tp`` inputs, default the hidden size) takes ``tg`` at ``gemm_flops_per_s``; with ``n``
    pieces ``min(tc, tg) (n-1)/n`` is hidden and every extra piece costs ``chunk_latency_s`` (collective launch +
    a smaller, less efficient GEMM).  Pieces stay >= ``min_chunk_rows`` tokens.  Returns the best of 1, 2, 4, 8."""
    if tp <= 1:
        return 1
    act = _dtype_bytes(precision)
    k = (in_features or hidden_size) // tp
    links = min(tp - 1, XGMI_LINKS_PER_GPU)
    tc = 2.0 * (tp - 1) / tp * tokens * hidden_size * act / (XGMI_LINK_BYTES_PER_S * link_efficiency * links)
    tg = 2.0 * tokens * k * hidden_size / gemm_flops_per_s
    best, best_gain = 1, 0.0
    for n in (2, 4, 8):
        if tokens % n or tokens // n < min_chunk_rows:
            break
        gain = min(tc, tg) * (n - 1) / n - (n - 1) * chunk_latency_s
        if gain > best_gain:
            best, best_gain = n, gain
    return best
