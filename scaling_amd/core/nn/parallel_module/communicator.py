"""Pipeline p2p of arbitrary pytrees (tensors + picklable python objects).

Parity: reference ``parallel_module/communicator.py:193-512`` (activations forward, gradients of the
``requires_grad`` leaves backward, meta handshake, python objects travel with the meta).  MI355X-first
design: no private pytree internals; a fixed 1-int64 header per message says whether the pickled
meta changed since the last message on this edge (meta re-sent only then); all tensor payloads of
a message go out as one ``batch_isend_irecv`` group (one RCCL group call over the xGMI link).
"""
from __future__ import annotations

import pickle
from typing import Any, NamedTuple, Optional

import torch
import torch.distributed as dist


class GradientPack(NamedTuple):
    tensors: list[torch.Tensor]
    grad_tensors: list[torch.Tensor]


class CommunicationMetaBase(NamedTuple):
    shape: tuple
    dtype: torch.dtype
    requires_grad: bool


def _flatten(obj: Any, tensors: list[torch.Tensor]) -> Any:
    if torch.is_tensor(obj):
        tensors.append(obj)
        return ("T", len(tensors) - 1, tuple(obj.shape), obj.dtype, bool(obj.requires_grad))
    if isinstance(obj, tuple) and not hasattr(obj, "_fields"):
        return ("U", [_flatten(o, tensors) for o in obj])
    if isinstance(obj, list):
        return ("L", [_flatten(o, tensors) for o in obj])
    if isinstance(obj, dict):
        return ("D", [(k, _flatten(v, tensors)) for k, v in obj.items()])
    return ("O", obj)


def _unflatten(spec: Any, tensors: list[torch.Tensor]) -> Any:
    kind = spec[0]
    if kind == "T":
        return tensors[spec[1]]
    if kind == "U":
        return tuple(_unflatten(s, tensors) for s in spec[1])
    if kind == "L":
        return [_unflatten(s, tensors) for s in spec[1]]
    if kind == "D":
        return {k: _unflatten(s, tensors) for k, s in spec[1]}
    return spec[1]


def _tensor_metas(spec: Any, out: list) -> list:
    kind = spec[0]
    if kind == "T":
        out.append(CommunicationMetaBase(spec[2], spec[3], spec[4]))
    elif kind in ("U", "L"):
        for s in spec[1]:
            _tensor_metas(s, out)
    elif kind == "D":
        for _, s in spec[1]:
            _tensor_metas(s, out)
    return out


def _p2p(ops: list) -> None:
    if not ops:
        return
    for req in dist.batch_isend_irecv(ops):
        req.wait()


class PipeCommunicator:
    def __init__(self, local_device: torch.device, recv_grads: bool, recv_data: bool,
                 use_continuous_recommunication: bool = False) -> None:
        self.local_device = local_device
        self.recv_grads = recv_grads
        self.recv_data_flag = recv_data
        self.use_continuous_recommunication = use_continuous_recommunication
        self._sent_meta: dict[int, bytes] = {}
        self._recv_spec: dict[int, Any] = {}

    def reset_communication_meta(self) -> None:
        self._sent_meta.clear()
        self._recv_spec.clear()

    # ------------------------------------------------------------------ data
    def send_data(self, data: Any, target_global_rank: int) -> None:
        tensors: list[torch.Tensor] = []
        spec = _flatten(data, tensors)
        meta = pickle.dumps(spec)
        changed = self.use_continuous_recommunication or self._sent_meta.get(target_global_rank) != meta
        header = torch.tensor([len(meta) if changed else 0], dtype=torch.int64, device=self.local_device)
        dist.send(header, target_global_rank)
        if changed:
            dist.send(torch.frombuffer(bytearray(meta), dtype=torch.uint8).to(self.local_device), target_global_rank)
            self._sent_meta[target_global_rank] = meta
        _p2p([dist.P2POp(dist.isend, t.detach().contiguous(), target_global_rank) for t in tensors])

    def recv_data(self, origin_global_rank: int) -> Any:
        header = torch.empty(1, dtype=torch.int64, device=self.local_device)
        dist.recv(header, origin_global_rank)
        n = int(header.item())
        if n > 0:
            buf = torch.empty(n, dtype=torch.uint8, device=self.local_device)
            dist.recv(buf, origin_global_rank)
            self._recv_spec[origin_global_rank] = pickle.loads(buf.cpu().numpy().tobytes())  # own-process protocol
        spec = self._recv_spec[origin_global_rank]
        metas = _tensor_metas(spec, [])
        tensors = [torch.empty(m.shape, dtype=m.dtype, device=self.local_device) for m in metas]
        _p2p([dist.P2POp(dist.irecv, t, origin_global_rank) for t in tensors])
        for t, m in zip(tensors, metas):
            if m.requires_grad and t.is_floating_point():
                t.requires_grad_(True)
        return _unflatten(spec, tensors)

    # ------------------------------------------------------------------ gradients
    def send_gradients(self, data: Any, target_global_rank: int) -> None:
        tensors: list[torch.Tensor] = []
        _flatten(data, tensors)
        grads = []
        for t in tensors:
            if t.requires_grad:
                grads.append(t.grad if t.grad is not None else torch.zeros_like(t))
        _p2p([dist.P2POp(dist.isend, g.contiguous(), target_global_rank) for g in grads])

    def recv_gradients(self, data: Any, origin_global_rank: int) -> GradientPack:
        tensors: list[torch.Tensor] = []
        _flatten(data, tensors)
        outs = [t for t in tensors if t.requires_grad]
        grads = [torch.empty_like(t) for t in outs]
        _p2p([dist.P2POp(dist.irecv, g, origin_global_rank) for g in grads])
        return GradientPack(tensors=outs, grad_tensors=grads)


class ModelParallelCommunicator:
    """Broadcast a pytree from mp-rank 0 to the TP group (reference ``communicator.py:513-759``)."""

    def __init__(self, topology: Any) -> None:
        self.topology = topology

    def sync_data(self, data: Optional[Any]) -> Any:
        topo = self.topology
        if topo.config.model_parallel_size == 1:
            return data
        src = dist.get_global_rank(topo.model_parallel_group, 0)
        objs = [None]
        tensors: list[torch.Tensor] = []
        if topo.model_parallel_rank == 0:
            objs = [_flatten(data, tensors)]
        dist.broadcast_object_list(objs, src=src, group=topo.model_parallel_group, device=topo.device)
        spec = objs[0]
        metas = _tensor_metas(spec, [])
        if topo.model_parallel_rank != 0:
            tensors = [torch.empty(m.shape, dtype=m.dtype, device=topo.device) for m in metas]
        else:
            tensors = [t.detach().to(topo.device).contiguous() for t in tensors]
        for t in tensors:
            dist.broadcast(t, src=src, group=topo.model_parallel_group)
        return _unflatten(spec, tensors)
