"""Pipeline/tensor/data-parallel training engine (instruction interpreter).

Parity: reference ``ParallelModule`` (``parallel_module/parallel_module.py:89-747``): same constructor,
``train_step``/``evaluation_step``/``run_instructions``, instruction semantics, loss transfer from
the last to the first stage, tied-grad reduction, activation checkpointing modes,
``named_parameters_with_meta``/``get_params_count``/``broadcast_model``, ``TrainStepOutput``.

MI355X-first: the optimizer's data-parallel gradient buckets are armed right before the last
micro-batch's backward so their reduce-scatter overlaps with backward compute on a side stream;
the step timer uses HIP events; p2p goes through the batched ``PipeCommunicator``.
"""
from __future__ import annotations

import time
from typing import Any, Callable, Generic, NamedTuple, Optional, Union

import torch
import torch.distributed as dist

from ....parallel import custom_allreduce
from ...data import BaseLayerIO
from ...optimizer.allreduce import allreduce_tensor_in_float32
from ...optimizer.base import BaseOptimizer
from ...profiler import Profiler, ProfilerConfig
from ...topology import Topology
from ...topology.topology_config import ActivationCheckpointingType
from ..linear.main_grad import invalidate_transposed_weights
from ..parameter_meta import CoreParameterMeta
from ..pipeline_schedule import PipelineScheduleInference, PipelineScheduleTrain
from ..pipeline_schedule.instructions import (
    InstructionBackwardPass,
    InstructionBase,
    InstructionForwardPass,
    InstructionLoadMicroBatch,
    InstructionLoss,
    InstructionOptimizerStep,
    InstructionRecvActivation,
    InstructionRecvGrad,
    InstructionReduceTiedGrads,
    InstructionSendActivation,
    InstructionSendGrad,
    InstructionStoreMicroBatch,
)
from .activation_checkpointing import checkpoint_with_rng
from .base_layer import BaseDatasetBatchGeneric, BaseLossInputGeneric
from .buffers import Buffers, BufferType
from .communicator import PipeCommunicator
from .layer_spec import LayerSpec
from .partitioned_module import PipePartitionedModule


def get_timer_args(instruction: InstructionBase) -> tuple[str, Optional[int], Optional[int]]:
    name = instruction.__class__.__name__
    name = name[len("Instruction"):] if name.startswith("Instruction") else name
    mb, buf = instruction.micro_batch_id, instruction.buffer_id
    if isinstance(instruction, (InstructionReduceTiedGrads, InstructionOptimizerStep)):
        mb = buf = -1
    return name, mb, buf


class TrainStepOutput(NamedTuple):
    loss: Optional[float]
    metrics: Optional[dict[str, Union[int, float]]]
    global_grad_norm: Optional[float]
    global_grad_norm_clipped: Optional[float]
    learning_rates: Optional[dict[str, float]]
    overflow: Optional[bool]
    no_overflow_steps: Optional[int]
    current_loss_scale: Optional[float]
    step_duration: float
    debug_dict: Optional[dict[str, float]]


class EvaluationStepOutput(NamedTuple):
    loss: Optional[float]
    metrics: Optional[dict[str, Union[int, float]]]
    step_duration: float


def _to_python(x: Any) -> Any:
    if torch.is_tensor(x):
        return x.tolist()
    if isinstance(x, dict):
        return {k: _to_python(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_python(v) for v in x)
    return x


def _loss_and_metrics_to_python(loss: torch.Tensor, metrics: Any) -> tuple[float, Any]:
    """The step's loss and its scalar metrics read back in ONE device-to-host copy (one sync instead of one per value);
    non-scalar or non-tensor metrics go through ``_to_python``."""
    if isinstance(metrics, dict):
        keys = [k for k, v in metrics.items() if torch.is_tensor(v) and v.numel() == 1 and v.device == loss.device]
        if keys:
            vals = torch.stack([loss.detach().reshape(()).double()] +
                               [metrics[k].detach().reshape(()).double() for k in keys]).tolist()
            out = {k: (vals[1 + keys.index(k)] if k in keys else _to_python(v)) for k, v in metrics.items()}
            return float(vals[0]), out
    return float(loss.detach().cpu().item()), _to_python(metrics)


class _StepTimer:
    """Step duration from HIP events on the compute stream (no device-wide synchronize).

    A device-wide sync at the step boundary would also wait for the ZeRO parameter all-gathers the
    optimizer leaves in flight on its comm stream, which are meant to overlap the next forward.
    The end event is waited on alone; the step's loss read-back has already drained the compute
    stream, so this costs nothing extra."""

    def __init__(self, device: Optional[torch.device] = None) -> None:
        self.device = device
        self.t0 = 0.0
        self.t1 = 0.0
        self._ev0: Optional[Any] = None
        self._ev1: Optional[Any] = None

    def _gpu(self) -> bool:
        return self.device is not None and self.device.type == "cuda"

    def start(self) -> None:
        self.t0 = time.perf_counter()
        if self._gpu():
            self._ev0 = torch.cuda.Event(enable_timing=True)
            self._ev0.record(torch.cuda.current_stream(self.device))

    def stop(self) -> None:
        if self._gpu():
            self._ev1 = torch.cuda.Event(enable_timing=True)
            self._ev1.record(torch.cuda.current_stream(self.device))
            self._ev1.synchronize()
        self.t1 = time.perf_counter()

    def duration(self) -> float:
        if self._ev0 is not None and self._ev1 is not None:
            # wall time covers the host-side start latency before the first kernel too
            return max(self.t1 - self.t0, self._ev0.elapsed_time(self._ev1) / 1000.0)
        return self.t1 - self.t0


class ParallelModule(PipePartitionedModule, Generic[BaseLossInputGeneric, BaseDatasetBatchGeneric]):
    def __init__(self, layer_specs: list[LayerSpec], topology: Topology, profiler_config: ProfilerConfig = ProfilerConfig(),
                 use_continuous_recommunication: bool = False):
        super().__init__(layer_specs=layer_specs, topology=topology)
        self.train_schedule = PipelineScheduleTrain(topology=topology)
        self.train_instructions = self.train_schedule.instructions()
        self.train_required_buffer_count = self.train_schedule.required_buffer_count()
        self.evaluation_schedule = PipelineScheduleInference(topology=topology)
        self.evaluation_instructions = self.evaluation_schedule.instructions()
        self.evaluation_required_buffer_count = self.evaluation_schedule.required_buffer_count()
        self.pipe_buffer = Buffers()
        dev = topology.device
        self.communicator_in = PipeCommunicator(dev, recv_grads=False, recv_data=True,
                                                use_continuous_recommunication=use_continuous_recommunication)
        self.communicator_out = PipeCommunicator(dev, recv_grads=True, recv_data=False,
                                                 use_continuous_recommunication=use_continuous_recommunication)
        self.communicator_loss_in: Optional[PipeCommunicator] = None
        self.communicator_loss_out: Optional[PipeCommunicator] = None
        if topology.config.pipe_parallel_size > 1:
            if topology.is_first_pipe_parallel_rank:
                # loss + metrics may hold python values that change every step: continuous mode
                self.communicator_loss_in = PipeCommunicator(dev, recv_grads=False, recv_data=True,
                                                             use_continuous_recommunication=True)
            if topology.is_last_pipe_parallel_rank:
                self.communicator_loss_out = PipeCommunicator(dev, recv_grads=False, recv_data=False,
                                                              use_continuous_recommunication=True)
        self.profiler = Profiler(config=profiler_config, topology=topology)
        self._param_sync_optimizer: Optional[BaseOptimizer] = None
        self.step_timer = _StepTimer(dev)
        self.broadcast_model()

    # ------------------------------------------------------------------ parameters
    def named_parameters_with_meta(self) -> list[tuple[str, torch.Tensor, CoreParameterMeta]]:
        out = []
        start = self._pipe_partition_coordinates[0].start
        for i, layer in enumerate(self._layers):
            dups = self.tied_layer_index.layer_index_to_tied_local_duplicate_parameter_names(start + i)
            for name, p in layer.named_parameters():
                if name in dups:
                    continue
                out.append((name, p, p.core_parameter_meta))
        return out

    def broadcast_model(self) -> None:
        invalidate_transposed_weights()
        topo = self.topology
        if topo is None or not topo.is_distributed_initialized:
            return
        with torch.no_grad():
            for p in self._layers.parameters():
                if p.core_parameter_meta.is_model_parallel_duplicate and topo.config.model_parallel_size > 1:
                    dist.broadcast(p.data, dist.get_global_rank(topo.model_parallel_group, 0), group=topo.model_parallel_group)
                if topo.config.data_parallel_size > 1:
                    dist.broadcast(p.data, dist.get_global_rank(topo.data_parallel_group, 0), group=topo.data_parallel_group)
            for p, pg, ranks in self.tied_layer_index.local_parameters_and_process_groups():
                if len(ranks) > 1:
                    dist.broadcast(p.data, dist.get_global_rank(pg, 0), group=pg)

    def get_params_count(self) -> tuple[int, int]:
        params = unique = 0
        topo = self.topology
        if topo.data_parallel_rank == 0:
            start = self._pipe_partition_coordinates[0].start
            for i, layer in enumerate(self._layers):
                tied_dup = self.tied_layer_index.layer_index_is_tied_global_duplicate(start + i)
                for p in layer.parameters():
                    params += p.numel()
                    mp_dup = topo.model_parallel_rank != 0 and p.core_parameter_meta.is_model_parallel_duplicate
                    if not (tied_dup or mp_dup):
                        unique += p.numel()
        t = torch.tensor([params, unique], dtype=torch.long, device=topo.device)
        if dist.is_initialized():
            dist.all_reduce(t)
        return int(t[0].item()), int(t[1].item())

    # ------------------------------------------------------------------ forward
    def _param_sync(self, layer: Any) -> None:
        """Waits for the ZeRO all-gather of this layer's parameters (issued asynchronously by the optimizer)."""
        if self._param_sync_optimizer is not None:
            self._param_sync_optimizer.wait_param_sync(layer)

    def _forward_tuple_input(self, *args: Any) -> Any:
        x = self._layers[0].tuple_to_input(tuple(args))
        for layer in self._layers:
            self._param_sync(layer)
            x = layer(x)
        return x

    def forward(self, x: BaseLayerIO) -> BaseLayerIO:
        ac = self.topology.config.activation_checkpointing_type
        if self.training and ac == ActivationCheckpointingType.EVERY_PIPE_STAGE:
            return checkpoint_with_rng(self._forward_tuple_input, self.topology, True, *self._layers[0].input_to_tuple(x))
        if self.training and ac in (ActivationCheckpointingType.EVERY_LAYER,
                                    ActivationCheckpointingType.EVERY_LAYER_KEEP_ATTENTION,
                                    ActivationCheckpointingType.EVERY_LAYER_SAVE_MATMULS):
            gemms = ac == ActivationCheckpointingType.EVERY_LAYER_SAVE_MATMULS
            keep = gemms or ac == ActivationCheckpointingType.EVERY_LAYER_KEEP_ATTENTION
            for layer in self._layers:
                self._param_sync(layer)
                x = checkpoint_with_rng(layer._forward_tuple_input, self.topology, True, *layer.input_to_tuple(x),
                                        keep_attention=keep, keep_gemms=gemms)
            return x
        for layer in self._layers:
            self._param_sync(layer)
            x = layer(x)
        return x

    # ------------------------------------------------------------------ loss
    def get_loss(self, metrics_aggregation_fn: Optional[Callable]) -> tuple[Optional[float], Optional[dict[str, float]]]:
        topo = self.topology
        data = None
        if topo.is_last_pipe_parallel_rank:
            assert self.pipe_buffer.accum_loss is not None
            loss = self.pipe_buffer.accum_loss / topo.config.gradient_accumulation_steps
            mlist = list(self.pipe_buffer.dump(BufferType.METRICS).values())
            metrics = metrics_aggregation_fn(topo, mlist) if (mlist and metrics_aggregation_fn is not None) else None
            if topo.config.data_parallel_size > 1:
                dist.all_reduce(loss, group=topo.data_parallel_group)
                loss = loss / topo.config.data_parallel_size
            data = (loss, metrics)
        if topo.config.pipe_parallel_size > 1:
            if topo.is_first_pipe_parallel_rank:
                assert self.communicator_loss_in is not None
                loss, metrics = self.communicator_loss_in.recv_data(topo.get_global_rank(pipe_parallel_rank=topo.config.pipe_parallel_size - 1))
                return float(loss.cpu().item()), _to_python(metrics)
            if topo.is_last_pipe_parallel_rank:
                assert self.communicator_loss_out is not None
                self.communicator_loss_out.send_data(data, topo.get_global_rank(pipe_parallel_rank=0))
            return None, None
        assert data is not None
        return _loss_and_metrics_to_python(data[0], data[1])

    # ------------------------------------------------------------------ steps
    def train_step(self, dataloader: Any, optimizer: BaseOptimizer, sync_batch_to_model_parallel: Callable,
                   loss_function: Callable, metrics_aggregation_fn: Optional[Callable]) -> TrainStepOutput:
        if not torch.is_grad_enabled():
            raise RuntimeError("train_step() requires gradients enabled. Use evaluation_step() instead.")
        self.step_timer.start()
        if not self._layers.training:  # (the recursive mode switch costs ~0.3 ms of host time per step; skip when set)
            self._layers.train()
        self.pipe_buffer.reset()
        self.profiler.step()
        invalidate_transposed_weights()  # weights may have been changed in place since the last step
        if self._param_sync_optimizer is not optimizer:
            optimizer.attach_param_sync(self._layers)
            self._param_sync_optimizer = optimizer
        last_mb = self.topology.config.gradient_accumulation_steps - 1
        opt_out = None
        for ins in self.train_instructions:
            name, mb, buf = get_timer_args(ins)
            with self.profiler.time(name, mb, buf):
                if isinstance(ins, InstructionLoadMicroBatch):
                    self._execute_load_micro_batch(dataloader, ins.buffer_id, sync_batch_to_model_parallel)
                elif isinstance(ins, InstructionForwardPass):
                    self._execute_forward_pass(ins.buffer_id, ins.buffer_id)
                elif isinstance(ins, InstructionLoss):
                    self._execute_loss_fn(ins.buffer_id, ins.buffer_id, bool(ins.is_first_pass), loss_function)
                elif isinstance(ins, InstructionBackwardPass):
                    if ins.micro_batch_id == last_mb:
                        optimizer.prepare_grad_sync()
                    self._execute_backward_pass(ins.buffer_id, optimizer)
                elif isinstance(ins, InstructionSendActivation):
                    self._execute_send_activations(ins.buffer_id)
                elif isinstance(ins, InstructionRecvActivation):
                    self._execute_receive_activations(ins.buffer_id)
                elif isinstance(ins, InstructionSendGrad):
                    self._execute_send_gradients(ins.buffer_id)
                elif isinstance(ins, InstructionRecvGrad):
                    self._execute_receive_gradients(ins.buffer_id)
                elif isinstance(ins, InstructionReduceTiedGrads):
                    self._execute_reduce_tied_grads()
                elif isinstance(ins, InstructionOptimizerStep):
                    opt_out = optimizer.step()
                else:
                    raise NotImplementedError(f"Instruction '{ins.__class__.__name__}' not implemented")
        loss, metrics = self.get_loss(metrics_aggregation_fn)
        self.wait_pending_sends()
        self.profiler.flush()
        self.step_timer.stop()
        assert opt_out is not None
        return TrainStepOutput(loss=loss, metrics=metrics, step_duration=self.step_timer.duration(), **opt_out._asdict())

    def evaluation_step(self, dataloader: Any, sync_batch_to_model_parallel: Callable, loss_function: Callable,
                        metrics_aggregation_fn: Optional[Callable]) -> EvaluationStepOutput:
        self.step_timer.start()
        self._layers.eval()
        self.pipe_buffer.reset()
        self.profiler.step()
        if self._param_sync_optimizer is not None:
            self._param_sync_optimizer.wait_param_sync()
        for ins in self.evaluation_instructions:
            name, mb, buf = get_timer_args(ins)
            with self.profiler.time(name, mb, buf):
                if isinstance(ins, InstructionLoadMicroBatch):
                    self._execute_load_micro_batch(dataloader, ins.buffer_id, sync_batch_to_model_parallel)
                elif isinstance(ins, InstructionForwardPass):
                    with torch.no_grad():
                        self._execute_forward_pass(ins.buffer_id, ins.buffer_id)
                elif isinstance(ins, InstructionLoss):
                    with torch.no_grad():
                        self._execute_loss_fn(ins.buffer_id, ins.buffer_id, True, loss_function)
                elif isinstance(ins, InstructionSendActivation):
                    self._execute_send_activations(ins.buffer_id)
                elif isinstance(ins, InstructionRecvActivation):
                    self._execute_receive_activations(ins.buffer_id)
                else:
                    raise NotImplementedError(f"Instruction '{ins.__class__.__name__}' not implemented")
        loss, metrics = self.get_loss(metrics_aggregation_fn)
        self.wait_pending_sends()
        custom_allreduce.raise_on_errors()  # forward-only: no optimizer step reads the one-shot error words
        self.profiler.flush()
        self.step_timer.stop()
        self._layers.train()
        return EvaluationStepOutput(loss=loss, metrics=metrics, step_duration=self.step_timer.duration())

    def run_instructions(self, instructions: list[InstructionBase], sync_batch_to_model_parallel: Callable,
                         collect_outputs_from_model_parallel: Callable, batch: Any = None) -> Any:
        if self._param_sync_optimizer is not None:
            self._param_sync_optimizer.wait_param_sync()
        ins = None
        for ins in instructions:
            if isinstance(ins, InstructionStoreMicroBatch):
                self._execute_store_micro_batch(batch, ins.buffer_id, sync_batch_to_model_parallel)
            elif isinstance(ins, InstructionForwardPass):
                self._execute_forward_pass(ins.buffer_id, ins.buffer_id, take_input=True)
            elif isinstance(ins, InstructionSendActivation):
                self._execute_send_activations(ins.buffer_id)
            elif isinstance(ins, InstructionRecvActivation):
                self._execute_receive_activations(ins.buffer_id)
            else:
                raise NotImplementedError(f"Instruction '{ins.__class__.__name__}' not implemented for run_instructions.")
        self.wait_pending_sends()
        custom_allreduce.raise_on_errors()
        topo = self.topology
        if batch is not None and topo.config.pipe_parallel_size == 1 and ins is not None:
            out = self.pipe_buffer.take(BufferType.PIPELINE_STAGE_OUTPUT, ins.buffer_id)
            return collect_outputs_from_model_parallel(topo, out)
        if (topo.config.pipe_parallel_size > 1 and topo.pipe_parallel_rank == 0 and instructions
                and isinstance(instructions[-1], InstructionRecvActivation)):
            out = self.pipe_buffer.take(BufferType.PIPELINE_STAGE_INPUT, instructions[-1].buffer_id)
            return collect_outputs_from_model_parallel(topo, out)
        return None

    # ------------------------------------------------------------------ instruction bodies
    def _execute_store_micro_batch(self, batch: Any, buffer_id: int, sync: Callable) -> None:
        self.pipe_buffer.write(BufferType.PIPELINE_STAGE_INPUT, buffer_id, sync(self.topology, batch))

    def _execute_load_micro_batch(self, dataloader: Any, io_buffer_id: int, sync: Callable) -> None:
        batch = next(dataloader) if self.topology.is_io_rank else None
        batch = sync(self.topology, batch)
        if self.topology.is_first_pipe_parallel_rank:
            self.pipe_buffer.write(BufferType.PIPELINE_STAGE_INPUT, io_buffer_id, batch.only_inputs())
        if self.topology.is_last_pipe_parallel_rank:
            self.pipe_buffer.write(BufferType.TARGET, io_buffer_id, batch.only_targets())

    def _execute_forward_pass(self, io_buffer_id: int, buffer_id: int, take_input: bool = False) -> None:
        get = self.pipe_buffer.take if take_input else self.pipe_buffer.get
        x = get(BufferType.PIPELINE_STAGE_INPUT, io_buffer_id)
        self.pipe_buffer.write(BufferType.PIPELINE_STAGE_OUTPUT, buffer_id, self(x))

    def _execute_loss_fn(self, buffer_id: int, io_buffer_id: int, is_first_pass: bool, loss_function: Callable) -> None:
        out = self.pipe_buffer.get(BufferType.PIPELINE_STAGE_OUTPUT, buffer_id)
        target = (self.pipe_buffer.get if is_first_pass else self.pipe_buffer.take)(BufferType.TARGET, io_buffer_id)
        res = loss_function(out, target)
        if isinstance(res, tuple):
            loss, metrics = res
            self.pipe_buffer.write(BufferType.METRICS, buffer_id, metrics)
        else:
            loss = res
        assert torch.is_tensor(loss) and list(loss.size()) == [], f"The loss needs to be a scalar, got {loss.shape}"
        self.pipe_buffer.add_loss(loss)
        self.pipe_buffer.write(BufferType.LOSS, buffer_id, loss)
        # outputs are only needed for the backward graph from here on
        self.pipe_buffer.write(BufferType.PIPELINE_STAGE_OUTPUT, buffer_id, None)

    def _execute_backward_pass(self, buffer_id: int, optimizer: BaseOptimizer) -> None:
        optimizer.wait_grad_zeroing()  # an overlapped optimizer step zeroes the gradient buffers on its stream
        if self.topology.is_last_pipe_parallel_rank:
            optimizer.backward(self.pipe_buffer.take(BufferType.LOSS, buffer_id))
        else:
            g = self.pipe_buffer.take(BufferType.GRAD, buffer_id)
            torch.autograd.backward(tensors=g.tensors, grad_tensors=g.grad_tensors)

    def _execute_send_activations(self, buffer_id: int) -> None:
        out = self.pipe_buffer.get(BufferType.PIPELINE_STAGE_OUTPUT, buffer_id)
        nxt = self.topology.next_pipe_parallel_rank
        self.communicator_out.send_data(self._layers[-1].output_to_tuple(out),
                                        self.topology.get_global_rank(pipe_parallel_rank=0 if nxt is None else nxt))

    def _execute_receive_activations(self, buffer_id: int) -> None:
        prv = self.topology.previous_pipe_parallel_rank
        if prv is None:
            prv = self.topology.config.pipe_parallel_size - 1
        tup = self.communicator_in.recv_data(self.topology.get_global_rank(pipe_parallel_rank=prv))
        layer0 = self._layers[0]
        x = layer0.tuple_to_last_stage_activation(tup) if self.topology.is_first_pipe_parallel_rank else layer0.tuple_to_input(tup)
        self.pipe_buffer.write(BufferType.PIPELINE_STAGE_INPUT, buffer_id, x)

    def _execute_send_gradients(self, buffer_id: int) -> None:
        x = self.pipe_buffer.take(BufferType.PIPELINE_STAGE_INPUT, buffer_id)
        self.communicator_in.send_gradients(self._layers[0].input_to_tuple(x),
                                            self.topology.get_global_rank(pipe_parallel_rank=self.topology.previous_pipe_parallel_rank))

    def _execute_receive_gradients(self, buffer_id: int) -> None:
        out = self.pipe_buffer.take(BufferType.PIPELINE_STAGE_OUTPUT, buffer_id)
        g = self.communicator_out.recv_gradients(self._layers[-1].output_to_tuple(out),
                                                 self.topology.get_global_rank(pipe_parallel_rank=self.topology.next_pipe_parallel_rank))
        self.pipe_buffer.write(BufferType.GRAD, buffer_id, g)

    def _execute_reduce_tied_grads(self) -> None:
        for p, pg, ranks in self.tied_layer_index.local_parameters_and_process_groups():
            if len(ranks) > 1 and p.grad is not None:
                allreduce_tensor_in_float32(p.grad, process_group=pg)
        if self.topology.config.model_parallel_size > 1:
            for layer in self._layers:
                for p in layer.parameters():
                    if p.core_parameter_meta.tied_grad_on_model_parallel and p.grad is not None:
                        allreduce_tensor_in_float32(p.grad, process_group=self.topology.model_parallel_group)

    def _communicators(self) -> list[PipeCommunicator]:
        return [c for c in (self.communicator_in, self.communicator_out, self.communicator_loss_in,
                            self.communicator_loss_out) if c is not None]

    def wait_pending_sends(self) -> None:
        """Retires the asynchronous pipeline sends of this step (their buffers may be freed after)."""
        for c in self._communicators():
            c.wait_pending_sends()

    def reset_activation_shape(self) -> None:
        self.communicator_in.reset_communication_meta()
        self.communicator_out.reset_communication_meta()
        for c in (self.communicator_loss_in, self.communicator_loss_out):
            if c is not None:
                c.reset_communication_meta()
