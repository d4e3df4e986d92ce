"""Stream-ordered collectives for the 1-GPU rehearsal mode (``TopologyConfig.gloo_on_gpu``).

In the rehearsal several ranks share one MI355X and gloo stands in for RCCL.  gloo is not a HIP-stream-aware
backend: handed GPU tensors, it moves their bytes from its own worker threads, not in the order of the issuing HIP
stream, so whether a collective sees its input before or after the producing kernel -- and whether the next kernel
sees its output -- depends on timing.  That made the race check (``tests/test_gpu_rehearsal.py``) disagree on cold
runs even with every side stream folded onto the compute stream (``profiles/race_bisect_r4.log``: the first run on a
fresh box differs, the warm reruns agree, independent of which side stream is folded).

``install()`` wraps the ``torch.distributed`` collectives this framework calls so that GPU tensors travel through
host copies, gloo runs on host tensors and sums over 3+ ranks are done in rank order (``_ordered_sum``: gloo's own
order follows message arrival).  Two modes:

* synchronous (default): the device-to-host copy of every input is ordered after the current stream's work and waited
  for, gloo runs, the results are copied back on the current stream; ``async_op=True`` calls complete before
  returning.  Stream order is RCCL's, but the collective has READ its input and its result is on the way before the
  call returns -- so a tensor freed or reused too early, or a consumer stream that does not wait for the
  communication stream, stays invisible.
* asynchronous (``SCALING_AMD_REHEARSAL_ASYNC=1``): RCCL's lifetimes.  The call only ENQUEUES, on the
  current stream (``async_op=True``: on a side stream that first waits for the current one, the work handle's ``wait``
  makes the waiting stream wait for it, and the handle keeps the tensors alive, as ProcessGroupNCCL does): the input's
  device-to-host copy into pinned memory, a stream gate (``hipStreamWaitValue32`` on a flag word: the stream holds in
  the command processor, no CU spins), and the host-to-device copy of the result.  One worker thread per process runs
  every gloo call in program order (also the CPU-tensor and object collectives, so both ranks issue gloo work in the same
  order): it waits until the stream has copied the input out, runs gloo on the host copies, writes the result, and
  opens the gate.  So the input is read when the STREAM gets there, long after the call returned, and the output lands
  when the peers are done -- a missing ``record_stream`` / early free / missing stream wait in this framework changes
  the result, which the race check's multi- vs single-stream comparison then shows.  Pipeline p2p goes the same way
  (``_async_batch_p2p``): a send's payload is copied out when the stream gets there and the worker posts the gloo
  send behind that copy without waiting for it; a receive lands through a gate.

Only the rehearsal installs this; with RCCL (``nccl``) or CPU gloo nothing is wrapped.
"""
from __future__ import annotations

import functools
import os
import threading
from typing import Any, Callable, Optional

import torch
import torch.distributed as dist

_installed = False
_orig: dict[str, Callable[..., Any]] = {}
_ASYNC = os.environ.get("SCALING_AMD_REHEARSAL_ASYNC", "0") == "1"
_TRACE = os.environ.get("SCALING_AMD_REHEARSAL_TRACE", "0") == "1"  # debug: every enqueue / gate step to stderr


def _trace(msg: str) -> None:
    if _TRACE:
        import sys

        print(f"[gloo_gpu r{os.environ.get('RANK', '?')} {threading.current_thread().name}] {msg}", file=sys.stderr,
              flush=True)


class _Done:
    """Work handle of a collective that already completed (stream-ordered)."""

    def wait(self, timeout: Any = None) -> bool:
        return True

    def is_completed(self) -> bool:
        return True


def _cuda(t: Any) -> bool:
    return isinstance(t, torch.Tensor) and t.is_cuda


def _host(t: torch.Tensor) -> torch.Tensor:
    return t.detach().to("cpu").contiguous()  # ordered after the current stream's writes of t, synchronous


def _ordered_sum(h: torch.Tensor, group: Any) -> Optional[torch.Tensor]:
    """SUM over ``group`` of the host tensor ``h`` in rank order (None for groups of <= 2 ranks, where gloo's own sum
    is already order-independent).  gloo reduces larger groups in message-arrival order, so fp32 sums of 3+ ranks
    differ from run to run (``profiles/race_repeat_dp4_r4.log``: DP4 runs disagree with every stream folded and any
    GEMM backend); gathering every rank's tensor and adding in rank order makes the result a pure function of the
    inputs, as RCCL's fixed ring order is."""
    n = dist.get_world_size(group)
    if n <= 2:
        return None
    flat = h.contiguous().reshape(-1)
    parts = torch.empty(n * flat.numel(), dtype=h.dtype)
    _orig["all_gather_into_tensor"](parts, flat, group=group)
    parts = parts.view(n, -1)
    out = parts[0].clone()
    for i in range(1, n):
        out += parts[i]
    return out.view(h.shape)


def _is_sum(op: Any) -> bool:
    return op is None or op == dist.ReduceOp.SUM


def _op(op: Any) -> Any:
    return op if op is not None else dist.ReduceOp.SUM


# ------------------------------------------------------------------------------------------ host-side algorithms
# Each takes host copies of the GPU inputs and returns the host result to copy into the GPU output (both modes).
def _h_all_reduce(h: torch.Tensor, op: Any, group: Any) -> torch.Tensor:
    red = _ordered_sum(h, group) if _is_sum(op) else None
    if red is None:
        _orig["all_reduce"](h, _op(op), group)
        red = h
    return red


def _h_reduce_scatter(hi: torch.Tensor, out_shape: torch.Size, out_dtype: torch.dtype, op: Any, group: Any) -> torch.Tensor:
    red = _ordered_sum(hi, group) if _is_sum(op) else None
    if red is None:
        ho = torch.empty(out_shape, dtype=out_dtype)
        _orig["reduce_scatter_tensor"](ho, hi, _op(op), group)
        return ho
    r, n = dist.get_rank(group), int(torch.Size(out_shape).numel())
    return red.reshape(-1)[r * n:(r + 1) * n].reshape(out_shape)


# ------------------------------------------------------------------------------------------ asynchronous mode
# The worker that runs every gloo call of the rank in program order is C++ (csrc/rehearsal.cpp): a Python thread
# needs the GIL between its steps, and a main thread blocked in a GIL-holding call on a tensor behind a gate (a
# .tolist()) deadlocked the rank (profiles/race_forensics_r6.md).
class _Gates:
    """A ring of flag words; each use of a word waits for the next generation number."""

    def __init__(self, n: int = 1 << 14) -> None:
        from ...ops._ext import ext

        self.base = ext().gate_flags_alloc(n)  # coherent pinned host memory
        self.n, self.i = n, 0
        self.gen = [0] * n

    def take(self) -> tuple[int, int]:
        i = self.i % self.n
        self.i += 1
        self.gen[i] += 1
        return i, self.gen[i]


class _AsyncWork:
    """Handle of an ``async_op=True`` collective: ``wait`` makes the current stream wait for its side stream."""

    def __init__(self, ev: Any, keep: tuple) -> None:
        self.ev, self.keep = ev, keep

    def wait(self, timeout: Any = None) -> bool:
        torch.cuda.current_stream().wait_event(self.ev)
        return True

    def is_completed(self) -> bool:
        return bool(self.ev.query())


_state: dict[str, Any] = {}
_KIND = {"all_reduce": 0, "broadcast": 1, "reduce_scatter": 2, "all_gather": 3}


def _op_code(op: Any) -> int:
    if op is None or op == dist.ReduceOp.SUM:
        return 0
    if op == dist.ReduceOp.MAX:
        return 1
    if op == dist.ReduceOp.MIN:
        return 2
    if op == dist.ReduceOp.PRODUCT:
        return 3
    raise ValueError(f"asynchronous rehearsal: unsupported reduce op {op}")


def _pg(group: Any) -> Any:
    return group if group is not None else dist.distributed_c10d._get_default_group()


def _side_stream(dev: torch.device) -> Any:
    key = ("side", dev.index)
    if key not in _state:
        _state[key] = torch.cuda.Stream(device=dev)
    return _state[key]


def _retire_pinned() -> None:
    """Drops the staging buffers / events whose host-to-device copy has completed."""
    live = _state.setdefault("pinned", [])
    live[:] = [item for item in live if not item[0].query()]


def _enqueue(kind: str, gpu_in: torch.Tensor, gpu_out: torch.Tensor, group: Any, op: Any, async_op: bool,
             root: int = 0) -> Any:
    """RCCL-like collective: input copy-out, gate and result copy-in enqueued on the stream; gloo in the worker."""
    from ...ops._ext import ext

    ext().rw_check()
    if "gates" not in _state:
        _state["gates"] = _Gates()
    gates = _state["gates"]
    _retire_pinned()
    cur = torch.cuda.current_stream(gpu_out.device)
    st = _side_stream(gpu_out.device) if async_op else cur
    if async_op:
        st.wait_stream(cur)
    in_place = gpu_in.data_ptr() == gpu_out.data_ptr() and gpu_in.shape == gpu_out.shape
    h_in = torch.empty(gpu_in.shape, dtype=gpu_in.dtype, pin_memory=True)
    h_out = h_in if in_place else torch.empty(gpu_out.shape, dtype=gpu_out.dtype, pin_memory=True)
    idx, gen = gates.take()
    with torch.cuda.stream(st):
        h_in.copy_(gpu_in, non_blocking=True)  # read when the stream gets here
        e_in = torch.cuda.Event()
        e_in.record(st)
        ext().gate_stream_wait(gates.base, idx, gen)
        gpu_out.copy_(h_out, non_blocking=True)  # written once the peers are done
        e_out = torch.cuda.Event()
        e_out.record(st)
    _state.setdefault("pinned", []).append((e_out, e_in, h_in, h_out))
    _trace(f"#{gates.i} {kind} {tuple(gpu_in.shape)} {gpu_in.dtype} async_op={async_op} stream {st.stream_id} "
           f"gate {idx}/{gen}")
    ext().rw_collective(_KIND[kind], _pg(group), h_in, h_out, _op_code(op), root, e_in.cuda_event, gates.base, idx, gen)
    if async_op:
        gpu_in.record_stream(st)
        gpu_out.record_stream(st)
        return _AsyncWork(e_out, (gpu_in, gpu_out))
    return None


def _host_call(fn: Callable[[], Any]) -> Any:
    """A gloo call on host tensors / objects: in asynchronous mode in its program-order turn among the worker's jobs."""
    if not (_ASYNC and _installed):
        return fn()
    from ...ops._ext import ext

    ticket = ext().rw_host_begin()
    try:
        return fn()
    finally:
        ext().rw_host_end(ticket)


# ------------------------------------------------------------------------------------------ wrappers
def _wrap_all_reduce(orig: Callable[..., Any]) -> Callable[..., Any]:
    @functools.wraps(orig)
    def fn(tensor: torch.Tensor, op: Any = None, group: Any = None, async_op: bool = False) -> Any:
        if not _cuda(tensor):
            return _host_call(lambda: orig(tensor, _op(op), group, async_op))
        if _ASYNC and tensor.is_contiguous():
            return _enqueue("all_reduce", tensor, tensor, group, op, async_op)
        h = _host(tensor)
        tensor.copy_(_host_call(lambda: _h_all_reduce(h, op, group)))
        return _Done() if async_op else None

    return fn


def _wrap_broadcast(orig: Callable[..., Any]) -> Callable[..., Any]:
    @functools.wraps(orig)
    def fn(tensor: torch.Tensor, *args: Any, async_op: bool = False, **kwargs: Any) -> Any:
        if not _cuda(tensor):
            return _host_call(lambda: orig(tensor, *args, async_op=async_op, **kwargs))

        def host(h: torch.Tensor) -> torch.Tensor:
            orig(h, *args, **kwargs)
            return h

        if _ASYNC and tensor.is_contiguous():
            src = args[0] if args else kwargs.get("src", 0)
            group = args[1] if len(args) > 1 else kwargs.get("group")
            root = dist.get_group_rank(group, src) if group is not None else src
            return _enqueue("broadcast", tensor, tensor, group, None, async_op, root=root)
        h = _host(tensor)
        tensor.copy_(_host_call(lambda: host(h)))
        return _Done() if async_op else None

    return fn


def _wrap_reduce_scatter(orig: Callable[..., Any]) -> Callable[..., Any]:
    @functools.wraps(orig)
    def fn(output: torch.Tensor, input: torch.Tensor, op: Any = None, group: Any = None,
           async_op: bool = False) -> Any:
        if not (_cuda(output) or _cuda(input)):
            return _host_call(lambda: orig(output, input, _op(op), group, async_op))
        host = lambda h: _h_reduce_scatter(h, output.shape, output.dtype, op, group)  # noqa: E731
        if _ASYNC and _cuda(output) and _cuda(input) and input.is_contiguous() and output.is_contiguous():
            return _enqueue("reduce_scatter", input, output, group, op, async_op)
        h = _host(input)
        output.copy_(_host_call(lambda: host(h)))
        return _Done() if async_op else None

    return fn


def _wrap_all_gather_into(orig: Callable[..., Any]) -> Callable[..., Any]:
    @functools.wraps(orig)
    def fn(output: torch.Tensor, input: torch.Tensor, *args: Any, async_op: bool = False, **kwargs: Any) -> Any:
        if not (_cuda(output) or _cuda(input)):
            return _host_call(lambda: orig(output, input, *args, async_op=async_op, **kwargs))

        def host(h: torch.Tensor) -> torch.Tensor:
            ho = torch.empty(output.shape, dtype=output.dtype)
            orig(ho, h, *args, **kwargs)
            return ho

        if _ASYNC and _cuda(output) and _cuda(input) and input.is_contiguous() and output.is_contiguous():
            group = args[0] if args else kwargs.get("group")
            return _enqueue("all_gather", input, output, group, None, async_op)
        h = _host(input)
        output.copy_(_host_call(lambda: host(h)))
        return _Done() if async_op else None

    return fn


def _wrap_all_gather(orig: Callable[..., Any]) -> Callable[..., Any]:
    """all_gather(tensor_list, tensor, ...): always through the synchronous path (used outside the step)."""

    @functools.wraps(orig)
    def fn(tensor_list: list[torch.Tensor], tensor: torch.Tensor, *args: Any, async_op: bool = False,
           **kwargs: Any) -> Any:
        if not (_cuda(tensor) or any(_cuda(t) for t in tensor_list)):
            return _host_call(lambda: orig(tensor_list, tensor, *args, async_op=async_op, **kwargs))
        h = _host(tensor)
        hl = [torch.empty(t.shape, dtype=t.dtype) for t in tensor_list]
        _host_call(lambda: orig(hl, h, *args, **kwargs))
        for t, x in zip(tensor_list, hl):
            t.copy_(x)
        return _Done() if async_op else None

    return fn


def _wrap_host_only(orig: Callable[..., Any]) -> Callable[..., Any]:
    """Object collectives / barrier: routed through the worker in asynchronous mode (global gloo order)."""

    @functools.wraps(orig)
    def fn(*args: Any, **kwargs: Any) -> Any:
        return _host_call(lambda: orig(*args, **kwargs))

    return fn


class _AsyncSendWork:
    """Handle of a queued send batch: ``wait`` returns once gloo completed the sends, in program order among the
    worker's jobs (a host turn); the payload copies stay alive until then."""

    def __init__(self, send_id: int, keep: tuple) -> None:
        self.send_id, self.keep = send_id, keep

    def wait(self, timeout: Any = None) -> bool:
        if self.keep is not None:
            from ...ops._ext import ext

            _host_call(lambda: ext().rw_send_wait(self.send_id))
            self.keep = None
        return True

    def is_completed(self) -> bool:
        return self.keep is None


def _async_batch_p2p(ops: list) -> list:
    """``batch_isend_irecv`` with RCCL's lifetimes: each send's payload is copied out when the current stream gets
    there and the worker posts the gloo sends behind that copy; receives land through a stream gate.  One handle for
    the sends, one for the receives (``wait``: the current stream waits for the received data)."""
    from ...ops._ext import ext

    ext().rw_check()
    if "gates" not in _state:
        _state["gates"] = _Gates()
    _retire_pinned()
    works: list = []
    dev = ops[0].tensor.device
    cur = torch.cuda.current_stream(dev)

    def peer(op: Any) -> int:
        return dist.get_group_rank(op.group, op.peer) if op.group is not None else op.peer

    for kind in ("send", "recv"):
        sel = [op for op in ops if (op.op is dist.isend) == (kind == "send")]
        if not sel:
            continue
        groups = {id(op.group) for op in sel}
        assert len(groups) == 1, "asynchronous rehearsal: one process group per p2p batch"
        pg = _pg(sel[0].group)
        hs = [torch.empty(op.tensor.shape, dtype=op.tensor.dtype, pin_memory=True) for op in sel]
        peers, tags = [peer(op) for op in sel], [int(op.tag or 0) for op in sel]
        if kind == "send":
            with torch.cuda.stream(cur):
                for h, op in zip(hs, sel):
                    h.copy_(op.tensor, non_blocking=True)  # read when the stream gets here
                e_in = torch.cuda.Event()
                e_in.record(cur)
            sid = _state.get("send_id", 0)
            _state["send_id"] = sid + 1
            _trace(f"send batch {sid}: {[tuple(op.tensor.shape) for op in sel]} -> {peers}")
            ext().rw_p2p_send(pg, hs, peers, tags, e_in.cuda_event, sid)
            works.append(_AsyncSendWork(sid, (hs, e_in, [op.tensor for op in sel])))
        else:
            gates = _state["gates"]
            idx, gen = gates.take()
            with torch.cuda.stream(cur):
                ext().gate_stream_wait(gates.base, idx, gen)
                for h, op in zip(hs, sel):
                    op.tensor.copy_(h, non_blocking=True)  # written once the peers' data arrived
                e_out = torch.cuda.Event()
                e_out.record(cur)
            _state.setdefault("pinned", []).append((e_out, None, hs, None))
            _trace(f"recv batch gate {idx}/{gen}: {[tuple(op.tensor.shape) for op in sel]} <- {peers}")
            ext().rw_p2p_recv(pg, hs, peers, tags, gates.base, idx, gen)
            works.append(_AsyncWork(e_out, tuple(op.tensor for op in sel)))
    return works


def install() -> None:
    """Routes GPU tensors of the wrapped collectives through host copies (idempotent)."""
    global _installed
    if _installed:
        return
    _installed = True
    for name in ("all_reduce", "broadcast", "reduce_scatter_tensor", "all_gather_into_tensor", "all_gather"):
        _orig[name] = getattr(dist, name)
    dist.all_reduce = _wrap_all_reduce(dist.all_reduce)
    dist.broadcast = _wrap_broadcast(dist.broadcast)
    dist.reduce_scatter_tensor = _wrap_reduce_scatter(dist.reduce_scatter_tensor)
    dist.all_gather_into_tensor = _wrap_all_gather_into(dist.all_gather_into_tensor)
    dist.all_gather = _wrap_all_gather(dist.all_gather)
    if _ASYNC:
        for name in ("barrier", "gather_object", "broadcast_object_list", "all_gather_object"):
            _orig[name] = getattr(dist, name)
            setattr(dist, name, _wrap_host_only(getattr(dist, name)))
        _orig["destroy_process_group"] = dist.destroy_process_group

        def destroy(*a: Any, **k: Any) -> Any:
            from ...ops._ext import ext

            ext().rw_drain()
            ext().rw_check()
            return _orig["destroy_process_group"](*a, **k)

        dist.destroy_process_group = destroy
        dist.batch_isend_irecv = _async_batch_p2p


def installed() -> bool:
    return _installed


def async_mode() -> bool:
    return _ASYNC
