"""Pipeline p2p of arbitrary pytrees (tensors + picklable python objects).

Parity: reference ``parallel_module/communicator.py:193-512`` — activations go forward, gradients
of the ``requires_grad`` leaves go backward, the communication meta (tree structure, shapes, dtypes,
``requires_grad``) is exchanged on the first message after ``reset_communication_meta`` and assumed
constant afterwards; with ``use_continuous_recommunication`` every message carries a same/changed
flag and the meta is re-sent only when it changed; python objects travel as a pickled, padded byte
blob whose capacity is part of the meta (a larger object grows it and re-sends the meta).

MI355X-first protocol (the reference sends a blocking message per tensor):
* the steady state (fixed meta) sends NO metadata at all and never reads device memory on the
  host: all tensor payloads of a message go out as ONE ``batch_isend_irecv`` group (one RCCL group
  call over the xGMI link to the neighbouring stage);
* sends are asynchronous: their work handles are parked (tensors kept alive) and retired by
  ``wait_pending_sends`` at the step end or when the queue grows, so the next forward/backward's
  kernels are never ordered behind an outgoing transfer.  On RCCL ``Work.wait`` only makes the
  current stream wait for the transfer, it does not block the host;
* gradient receive buffers are allocated once per meta and reused (the backward consuming one is
  enqueued before the next receive is issued, and RCCL orders its stream after the compute stream);
  activation receives take fresh blocks from the caching allocator because the pipeline keeps
  several in flight for their backward;
* python objects are exchanged with the meta; in fixed-meta mode they must stay equal (like the
  reference's shape assert), in continuous mode they ride in the per-message control blob;
* metadata and control blobs use the same batched, non-blocking sends as the payloads (no blocking
  ``dist.send`` while batched sends are in flight): one ordered p2p stream per peer.
"""
from __future__ import annotations

import pickle
import struct
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


class _Meta(NamedTuple):
    structure: Any  # nested ("T", i) / ("O", j) / ("U"|"L", [...]) / ("D", [(k, ...)])
    tensors: tuple  # CommunicationMetaBase per tensor leaf
    object_capacity: int  # bytes reserved for the pickled object blob in continuous mode


def _flatten(obj: Any, tensors: list[torch.Tensor], objects: list[Any]) -> Any:
    if torch.is_tensor(obj):
        tensors.append(obj)
        return ("T", len(tensors) - 1)
    if isinstance(obj, tuple) and not hasattr(obj, "_fields"):
        return ("U", [_flatten(o, tensors, objects) for o in obj])
    if isinstance(obj, list):
        return ("L", [_flatten(o, tensors, objects) for o in obj])
    if isinstance(obj, dict):
        return ("D", [(k, _flatten(v, tensors, objects)) for k, v in obj.items()])
    objects.append(obj)
    return ("O", len(objects) - 1)


def _unflatten(spec: Any, tensors: list[Any], objects: list[Any]) -> Any:
    kind = spec[0]
    if kind == "T":
        return tensors[spec[1]]
    if kind == "O":
        return objects[spec[1]]
    if kind == "U":
        return tuple(_unflatten(s, tensors, objects) for s in spec[1])
    if kind == "L":
        return [_unflatten(s, tensors, objects) for s in spec[1]]
    return {k: _unflatten(s, tensors, objects) for k, s in spec[1]}


def _tensor_meta(t: torch.Tensor) -> CommunicationMetaBase:
    return CommunicationMetaBase(tuple(t.shape), t.dtype, bool(t.requires_grad))


def dump_objects(objects: list[Any], capacity: Optional[int] = None) -> bytes:
    """8-byte little-endian length + pickle, zero-padded to ``capacity`` (if it fits)."""
    body = pickle.dumps(objects)
    out = struct.pack("<Q", len(body)) + body
    if capacity is not None and len(out) <= capacity:
        out += bytes(capacity - len(out))
    return out


def load_objects(blob: bytes) -> list[Any]:
    (n,) = struct.unpack("<Q", blob[:8])
    return pickle.loads(blob[8 : 8 + n])  # peer rank of the same job (own protocol)


def _bytes_tensor(b: bytes, device: torch.device) -> torch.Tensor:
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).to(device)


class _HostStagedWork:
    """p2p of GPU tensors over gloo (the 1-GPU rehearsal mode, ``TopologyConfig.gloo_on_gpu``): gloo moves raw
    pointers without ordering against the producing HIP stream, so payloads travel through host copies (the
    D2H copy of a send is stream-ordered and synchronous; a receive lands in host memory and is copied to the
    device on the current stream once the transfer finished).  RCCL needs none of this: its p2p is
    stream-ordered."""

    def __init__(self, works: list[Any], copies: list[tuple[torch.Tensor, torch.Tensor]]) -> None:
        self.works = works
        self.copies = copies

    def wait(self) -> bool:
        for w in self.works:
            w.wait()
        for dev_t, host_t in self.copies:
            dev_t.copy_(host_t)
        self.works, self.copies = [], []
        return True


class PipeCommunicator:
    max_pending_sends = 8

    def __init__(self, local_device: torch.device, recv_grads: bool, recv_data: bool = True,
                 use_continuous_recommunication: bool = False) -> None:
        self.local_device = local_device
        self.recv_grads = recv_grads
        self.recv_data_flag = recv_data
        self.use_continuous_recommunication = use_continuous_recommunication
        self._meta: Optional[_Meta] = None
        self._objects: list[Any] = []
        self._object_blob: bytes = b""
        self._grad_buffers: Optional[list[Optional[torch.Tensor]]] = None
        self._pending: list[tuple[list[Any], list[torch.Tensor]]] = []

    # ------------------------------------------------------------------ meta
    def reset_communication_meta(self, use_continuous_recommunication: Optional[bool] = None) -> None:
        self._meta = None
        self._objects = []
        self._object_blob = b""
        self._grad_buffers = None
        if use_continuous_recommunication is not None:
            self.use_continuous_recommunication = use_continuous_recommunication

    @property
    def communication_meta(self) -> Optional[_Meta]:
        return self._meta

    def _set_meta(self, meta: _Meta, objects: list[Any]) -> None:
        self._meta = meta
        self._objects = objects
        self._grad_buffers = None

    @property
    def _host_staged(self) -> bool:
        # (the asynchronous rehearsal routes GPU p2p through its own stream-ordered staging: core/topology/gloo_gpu.py)
        from ...topology import gloo_gpu

        return (self.local_device.type == "cuda" and dist.get_backend() == "gloo"
                and not (gloo_gpu.installed() and gloo_gpu.async_mode()))

    @property
    def _wire_device(self) -> torch.device:
        """Device of the (rare) metadata messages: host memory when gloo carries them."""
        return torch.device("cpu") if self._host_staged else self.local_device

    # Every message of the protocol -- metadata, continuous-recommunication control blobs and payloads -- goes
    # through batch_isend_irecv: there is no blocking dist.send/recv interleaved with in-flight batched sends, so
    # on RCCL all traffic to a peer is one ordered stream of grouped p2p calls on the communicator.
    def _send_wire(self, tensors: list[torch.Tensor], dst: int) -> None:
        self._park(self._issue([dist.P2POp(dist.isend, t, dst) for t in tensors]), tensors)

    def _recv_wire(self, t: torch.Tensor, src: int) -> torch.Tensor:
        for w in self._issue([dist.P2POp(dist.irecv, t, src)]):
            w.wait()
        return t

    def _send_bytes(self, b: bytes, dst: int) -> None:
        hdr = torch.tensor([len(b)], dtype=torch.int64, device=self._wire_device)
        self._send_wire([hdr, _bytes_tensor(b, self._wire_device)], dst)

    def _recv_bytes(self, src: int) -> bytes:
        n = self._recv_wire(torch.empty(1, dtype=torch.int64, device=self._wire_device), src)
        buf = self._recv_wire(torch.empty(int(n.item()), dtype=torch.uint8, device=self._wire_device), src)
        return buf.cpu().numpy().tobytes()

    def send_meta(self, data: Any, target_global_rank: int) -> tuple[list[torch.Tensor], bool]:
        """Meta part of a send; returns (tensor leaves, whether the meta was (re-)sent)."""
        tensors: list[torch.Tensor] = []
        objects: list[Any] = []
        structure = _flatten(data, tensors, objects)
        tmetas = tuple(_tensor_meta(t) for t in tensors)
        blob = dump_objects(objects) if objects else b""
        blob_len = len(blob)
        if self._meta is None:
            changed = True
        else:
            same = (structure == self._meta.structure and tmetas == self._meta.tensors
                    and blob_len <= self._meta.object_capacity)
            if self.use_continuous_recommunication:
                ctrl = bytes([1 if same else 0])
                if same and self._meta.object_capacity:
                    ctrl += dump_objects(objects, self._meta.object_capacity)
                else:
                    ctrl += bytes(self._meta.object_capacity)
                self._send_wire([_bytes_tensor(ctrl, self._wire_device)], target_global_rank)
                changed = not same
            else:
                if not same or blob != self._object_blob:
                    raise AssertionError(
                        "Try to communicate data with a different structure/shape/dtype (or python objects) than "
                        "saved in the meta. Try to reset the 'communication_meta' or use continuous recommunication."
                    )
                changed = False
        if changed:
            cap = max(2 * blob_len, 256) if objects else 0
            meta = _Meta(structure, tmetas, cap)
            self._send_bytes(pickle.dumps((meta, objects)), target_global_rank)
            self._set_meta(meta, objects)
            self._object_blob = blob
        return tensors, changed

    def recv_meta(self, origin_global_rank: int) -> bool:
        """Meta part of a receive; returns whether a new meta arrived."""
        if self._meta is not None:
            if not self.use_continuous_recommunication:
                return False
            ctrl = self._recv_wire(torch.empty(1 + self._meta.object_capacity, dtype=torch.uint8,
                                               device=self._wire_device), origin_global_rank)
            cb = ctrl.cpu().numpy().tobytes()
            if cb[0] == 1:
                if self._meta.object_capacity:
                    self._objects = load_objects(cb[1:])
                return False
        meta, objects = pickle.loads(self._recv_bytes(origin_global_rank))  # own protocol, same job
        self._set_meta(meta, objects)
        return True

    # ------------------------------------------------------------------ p2p
    def _issue(self, ops: list) -> list[Any]:
        if not ops:
            return []
        if self._host_staged:
            host_ops, copies = [], []
            for op in ops:
                if op.op == dist.isend:
                    h = op.tensor.to("cpu")
                else:
                    h = torch.empty(op.tensor.shape, dtype=op.tensor.dtype)
                    copies.append((op.tensor, h))
                host_ops.append(dist.P2POp(op.op, h, op.peer, op.group, op.tag))
            return [_HostStagedWork(dist.batch_isend_irecv(host_ops), copies)]
        return dist.batch_isend_irecv(ops)

    def wait_pending_sends(self) -> None:
        pending, self._pending = self._pending, []
        for works, _tensors in pending:
            for w in works:
                w.wait()

    def _park(self, works: list[Any], tensors: list[torch.Tensor]) -> None:
        if works:
            self._pending.append((works, tensors))
        if len(self._pending) > self.max_pending_sends:
            works0, _ = self._pending.pop(0)
            for w in works0:
                w.wait()

    # ------------------------------------------------------------------ data
    def send_data(self, data: Any, target_global_rank: int) -> None:
        tensors, _ = self.send_meta(data, target_global_rank)
        payload = [t.detach().contiguous() for t in tensors]
        self._park(self._issue([dist.P2POp(dist.isend, t, target_global_rank) for t in payload]), payload)

    def recv_data(self, origin_global_rank: int) -> Any:
        self.recv_meta(origin_global_rank)
        assert self._meta is not None
        tensors = [torch.empty(m.shape, dtype=m.dtype, device=self.local_device) for m in self._meta.tensors]
        for w in self._issue([dist.P2POp(dist.irecv, t, origin_global_rank) for t in tensors]):
            w.wait()
        for t, m in zip(tensors, self._meta.tensors):
            if m.requires_grad and t.is_floating_point():
                t.requires_grad_(True)
        return _unflatten(self._meta.structure, tensors, self._objects)

    # ------------------------------------------------------------------ gradients
    def send_gradients(self, data: Any, target_global_rank: int) -> None:
        tensors: list[torch.Tensor] = []
        _flatten(data, tensors, [])
        grads = [(t.grad if t.grad is not None else torch.zeros_like(t)).contiguous() for t in tensors if t.requires_grad]
        self._park(self._issue([dist.P2POp(dist.isend, g, target_global_rank) for g in grads]), grads)

    def recv_gradients(self, data: Any, origin_global_rank: int) -> GradientPack:
        tensors: list[torch.Tensor] = []
        _flatten(data, tensors, [])
        outs = [t for t in tensors if t.requires_grad]
        shapes = [(tuple(t.shape), t.dtype) for t in outs]
        bufs = self._grad_buffers
        if bufs is None or [(tuple(b.shape), b.dtype) for b in bufs] != shapes:
            bufs = [torch.empty(s, dtype=d, device=self.local_device) for s, d in shapes]
            self._grad_buffers = bufs
        for w in self._issue([dist.P2POp(dist.irecv, g, origin_global_rank) for g in bufs]):
            w.wait()
        return GradientPack(tensors=outs, grad_tensors=list(bufs))


class ModelParallelCommunicator:
    """Broadcast a pytree from mp-rank 0 to the TP group (reference ``communicator.py:513-759``)."""

    def __init__(self, topology: Any) -> None:
        self.topology = topology

    def sync_data(self, data: Optional[Any]) -> Any:
        topo = self.topology
        if topo.config.model_parallel_size == 1:
            return data
        src = dist.get_global_rank(topo.model_parallel_group, 0)
        objs: list[Any] = [None]
        tensors: list[torch.Tensor] = []
        objects: list[Any] = []
        if topo.model_parallel_rank == 0:
            spec = _flatten(data, tensors, objects)
            objs = [(spec, tuple(_tensor_meta(t) for t in tensors), objects)]
        dist.broadcast_object_list(objs, src=src, group=topo.model_parallel_group, device=topo.device)
        spec, metas, objects = objs[0]
        if topo.model_parallel_rank != 0:
            tensors = [torch.empty(m.shape, dtype=m.dtype, device=topo.device) for m in metas]
        else:
            tensors = [t.detach().to(topo.device).contiguous() for t in tensors]
        for t in tensors:
            dist.broadcast(t, src=src, group=topo.model_parallel_group)
        return _unflatten(spec, tensors, objects)
