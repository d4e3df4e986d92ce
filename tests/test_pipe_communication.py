"""PipeCommunicator on 2 gloo ranks (reference ``tests/core/test_nn/test_pipe_communication.py``).

Covers arbitrary pytrees (nested containers, non-float tensors, python objects, numpy arrays) in
fixed-meta and continuous-recommunication mode, the meta (re-)send decisions under changing shapes
and object sizes, gradient round trips, and the steady-state protocol: after the first message no
metadata travels and nothing is read back to the host.
"""
from __future__ import annotations

import random
import string

import numpy as np
import pytest
import torch

from tests.dist_utils import make_topology, run_distributed


class DummySettings:
    def __init__(self, name: str, some_int_list: list):
        self.name = name
        self.some_int_list = some_int_list

    def __eq__(self, other: object) -> bool:
        return isinstance(other, DummySettings) and (self.name, self.some_int_list) == (other.name, other.some_int_list)


def _dummy(i: int):
    return [
        torch.tensor([[1.0]]),
        ((torch.tensor([[1.0]]),),),
        {"data": torch.tensor([[1.0]])},
        {"data": torch.tensor([[1.0]]), "more_data": torch.tensor([[2.0]])},
        (torch.tensor([[1.0]]), torch.tensor([[1.0]]), torch.tensor([[42]])),
        {"data": torch.tensor([[1.0]]), "more_data_non_fp": torch.tensor([[42]])},
        {"a": [torch.zeros(5, 33, 7), torch.ones(55, 55, 55, 1)], "b": torch.zeros(1),
         "c": {"d": torch.zeros(5, 5), "e": torch.arange(115.0)}, "d": [True, "THIS IS A TEXT"],
         "settings": DummySettings(name="THIS IS AN AMAZING NAME", some_int_list=[0, -55, 5, 5, 66])},
        [False, "TRUE", {"a": torch.zeros(1), "b": torch.ones(1)}, np.zeros((2, 2, 5))],
    ][i]


def _same(a, b) -> bool:
    if torch.is_tensor(a):
        return torch.is_tensor(b) and a.dtype == b.dtype and torch.equal(a.detach(), b.detach())
    if isinstance(a, np.ndarray):
        return isinstance(b, np.ndarray) and np.array_equal(a, b)
    if isinstance(a, (list, tuple)):
        return type(a) is type(b) and len(a) == len(b) and all(_same(x, y) for x, y in zip(a, b))
    if isinstance(a, dict):
        return a.keys() == b.keys() and all(_same(a[k], b[k]) for k in a)
    return a == b


def _any_case(idx: int, continuous: bool):
    import torch.distributed as dist

    from scaling_amd.core.nn.parallel_module.communicator import PipeCommunicator

    make_topology(pipe_parallel_size=2)
    rank = dist.get_rank()
    data = _dummy(idx)
    com = PipeCommunicator(torch.device("cpu"), recv_grads=False, recv_data=rank == 1,
                           use_continuous_recommunication=continuous)
    com.reset_communication_meta()
    for _ in range(3):
        if rank == 0:
            com.send_data(data, 1)
        else:
            assert _same(data, com.recv_data(0))
    com.wait_pending_sends()
    return True


@pytest.mark.parametrize("continuous", [False, True])
@pytest.mark.parametrize("idx", range(8))
def test_any_communication(idx, continuous):
    assert all(run_distributed(_any_case, 2, idx=idx, continuous=continuous).values())


def _random_payload(extra: bool):
    a = torch.rand(5, 3, 3)
    b = torch.rand(1, dtype=torch.bfloat16)
    c = torch.rand(7, 7, dtype=torch.bfloat16)
    d = "".join(random.choice(string.ascii_letters) for _ in range(random.randint(12, 16)))
    e = DummySettings(name=d, some_int_list=[random.randint(-50, 50) for _ in range(random.randint(12, 16))])
    out = [a, (b, c), d, e]
    if extra:
        out.append("FFFGGG")
    return out


def _const_case():
    """Continuous mode: varying python object values within capacity never re-send the meta; a new
    leaf does (once), then the new meta holds again.  Every received payload equals what was sent."""
    import torch.distributed as dist

    from scaling_amd.core.nn.parallel_module.communicator import PipeCommunicator

    make_topology(pipe_parallel_size=2)
    rank = dist.get_rank()
    com = PipeCommunicator(torch.device("cpu"), recv_grads=False, recv_data=rank == 1, use_continuous_recommunication=True)
    random.seed(1234)  # both ranks draw the same payloads
    torch.manual_seed(1234)
    resent = []
    for i in range(12):
        payload = _random_payload(extra=i >= 6)
        if rank == 0:
            tensors, changed = com.send_meta(payload, 1)
            ops = [dist.P2POp(dist.isend, t.contiguous(), 1) for t in tensors]
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            resent.append(changed)
        else:
            resent.append(com.recv_meta(0))
            meta = com.communication_meta
            ts = [torch.empty(m.shape, dtype=m.dtype) for m in meta.tensors]
            for w in dist.batch_isend_irecv([dist.P2POp(dist.irecv, t, 0) for t in ts]):
                w.wait()
            from scaling_amd.core.nn.parallel_module.communicator import _unflatten

            got = _unflatten(meta.structure, ts, com._objects)
            assert _same(payload, got)
    expect = [True] + [False] * 5 + [True] + [False] * 5
    assert resent == expect, resent
    return True


def test_const_communication():
    assert all(run_distributed(_const_case, 2).values())


def _shape_change_case():
    """Fixed-meta mode rejects a new shape until reset; continuous mode follows shape changes
    (variable sequence length) with one meta re-send per change."""
    import torch.distributed as dist

    from scaling_amd.core.nn.parallel_module.communicator import PipeCommunicator

    make_topology(pipe_parallel_size=2)
    rank = dist.get_rank()
    fixed = PipeCommunicator(torch.device("cpu"), recv_grads=True, recv_data=True)
    if rank == 0:
        fixed.send_data((torch.ones(2, 4), ["x"]), 1)
        with pytest.raises(AssertionError, match="reset the 'communication_meta'"):
            fixed.send_data((torch.ones(3, 4), ["x"]), 1)
        with pytest.raises(AssertionError):
            fixed.send_data((torch.ones(2, 4), ["y"]), 1)  # objects must stay equal in fixed mode
        fixed.reset_communication_meta()
        fixed.send_data((torch.ones(3, 4), ["x"]), 1)
    else:
        assert fixed.recv_data(0)[0].shape == (2, 4)
        fixed.reset_communication_meta()
        assert fixed.recv_data(0)[0].shape == (3, 4)
    fixed.wait_pending_sends()

    cont = PipeCommunicator(torch.device("cpu"), recv_grads=True, recv_data=True, use_continuous_recommunication=True)
    lens = [4, 4, 7, 7, 7, 2, 9, 9]
    changes = []
    for s in lens:
        if rank == 0:
            x = torch.arange(s * 3, dtype=torch.float32).view(s, 3)
            tensors, changed = cont.send_meta((x, {"seq": s}), 1)
            for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, t, 1) for t in tensors]):
                w.wait()
            changes.append(changed)
        else:
            changes.append(cont.recv_meta(0))
            m = cont.communication_meta
            ts = [torch.empty(t.shape, dtype=t.dtype) for t in m.tensors]
            for w in dist.batch_isend_irecv([dist.P2POp(dist.irecv, t, 0) for t in ts]):
                w.wait()
            assert ts[0].shape == (s, 3) and torch.equal(ts[0].view(-1), torch.arange(s * 3, dtype=torch.float32))
    assert changes == [True, False, True, False, False, True, True, False], changes
    # send_data/recv_data themselves on the continuous communicator
    for s in lens:
        if rank == 0:
            cont.send_data((torch.full((s, 2), float(s)), {"seq": s}), 1)
        else:
            x, d = cont.recv_data(0)
            assert x.shape == (s, 2) and float(x[0, 0]) == s and d == {"seq": s}
    cont.wait_pending_sends()
    return True


def test_shape_change_and_continuous_recommunication():
    assert all(run_distributed(_shape_change_case, 2).values())


def _steady_state_case():
    """After the first message: no blocking send/recv (metadata) and no host read-back of device
    memory on either side; gradients flow back through the reused receive buffer."""
    import torch.distributed as dist

    from scaling_amd.core.nn.parallel_module.communicator import PipeCommunicator

    make_topology(pipe_parallel_size=2)
    rank = dist.get_rank()
    com = PipeCommunicator(torch.device("cpu"), recv_grads=True, recv_data=True)
    counts = {"send": 0, "recv": 0, "item": 0}
    real_send, real_recv, real_item = dist.send, dist.recv, torch.Tensor.item

    def c_send(*a, **k):
        counts["send"] += 1
        return real_send(*a, **k)

    def c_recv(*a, **k):
        counts["recv"] += 1
        return real_recv(*a, **k)

    def c_item(self):
        counts["item"] += 1
        return real_item(self)

    grad_bufs = []
    for step in range(4):
        if step == 1:
            dist.send, dist.recv, torch.Tensor.item = c_send, c_recv, c_item
        if rank == 0:
            x = torch.full((2, 3), float(step), requires_grad=True)
            com.send_data((x, torch.arange(4), ["names"]), 1)
            g = com.recv_gradients((x, torch.arange(4), ["names"]), 1)
            assert torch.equal(g.grad_tensors[0], torch.full((2, 3), 2.0 * step)) and g.tensors[0] is x
            grad_bufs.append(g.grad_tensors[0].data_ptr())
        else:
            t = com.recv_data(0)
            assert torch.equal(t[0], torch.full((2, 3), float(step))) and torch.equal(t[1], torch.arange(4))
            assert t[2] == ["names"] and t[0].requires_grad and not t[1].requires_grad
            y = t[0]
            y.grad = 2 * y.detach()
            com.send_gradients(t, 0)
    com.wait_pending_sends()
    dist.send, dist.recv, torch.Tensor.item = real_send, real_recv, real_item
    assert counts == {"send": 0, "recv": 0, "item": 0}, counts
    if rank == 0:
        assert len(set(grad_bufs)) == 1  # gradient receive buffer allocated once per meta
    return True


def test_steady_state_has_no_metadata_traffic():
    assert all(run_distributed(_steady_state_case, 2).values())


def test_object_blob_roundtrip():
    from scaling_amd.core.nn.parallel_module.communicator import dump_objects, load_objects

    a = dump_objects(["HHISDFUGS"])
    b = dump_objects(["HHISDFUGS_x"], capacity=len(a) + 16)
    assert len(b) == len(a) + 16
    assert load_objects(a) == ["HHISDFUGS"] and load_objects(b) == ["HHISDFUGS_x"]
