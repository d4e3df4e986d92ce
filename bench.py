"""Headline benchmark: whole-node training tokens/s of the Llama-2-7B shape in bf16 (BASELINE.json).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Each step is a full training step of the framework (``TransformerParallelModule.train_step``): all
micro-batches forward+backward through the HIP kernels, DP gradient reduce-scatter overlapped with the
last backward, grad-norm clipping and the fused ZeRO-1 AdamW update + parameter all-gather.  Data is
synthetic token ids of the benchmark shape, weights are random-init.  Per-GPU work is fixed (weak
scaling): every data-parallel rank processes ``micro_batch * grad_acc`` sequences per step.

Rank 0 prints one JSON line; ``value`` is the whole-job tokens/s (global tokens / max-over-ranks step time).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from typing import Any, Optional

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _args() -> argparse.Namespace:
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--model", type=str, default="llama2_7b")
    p.add_argument("--seq-len", type=int, default=4096)
    p.add_argument("--micro-batch", type=int, default=2)
    p.add_argument("--grad-acc", type=int, default=4)
    p.add_argument("--tp", type=int, default=1)
    p.add_argument("--pp", type=int, default=1)
    p.add_argument("--activation-checkpointing", type=str, default="disabled",
                   choices=["disabled", "every_layer", "every_pipe_stage"])
    p.add_argument("--sequence-parallel", action="store_true")
    p.add_argument("--zero", type=int, default=1)
    p.add_argument("--num-layers", type=int, default=None, help="debug only: marks the result as not the headline config")
    p.add_argument("--gemm-tuning", type=str, default="use", choices=["use", "tune", "off"],
                   help="hipBLASLt solution table (scaling_amd/tuning/gemm_gfx950.csv); tune = benchmark and write")
    p.add_argument("--gemm-tuning-out", type=str, default=None)
    p.add_argument("--profile-json", type=str, default=None, help="write per-step times to this file")
    return p.parse_args()


def _env_int(k: str, d: int) -> int:
    v = os.environ.get(k)
    return d if v is None else int(v)


class _SyntheticLoader:
    """Infinite iterator of fixed random token batches (generated once per slot, on host)."""

    def __init__(self, micro_batch: int, seq_len: int, vocab: int, seed: int, slots: int = 4):
        from scaling_amd.transformer.data.text_dataset_batch import TextDatasetBatchBeforeSync

        g = torch.Generator().manual_seed(seed)
        self.batches = [
            TextDatasetBatchBeforeSync(token_ids=torch.randint(1, vocab, (micro_batch, seq_len + 1), generator=g).pin_memory()
                                       if torch.cuda.is_available() else
                                       torch.randint(1, vocab, (micro_batch, seq_len + 1), generator=g))
            for _ in range(slots)
        ]
        self.i = 0

    def __iter__(self) -> "_SyntheticLoader":
        return self

    def __next__(self) -> Any:
        b = self.batches[self.i % len(self.batches)]
        self.i += 1
        return b


def main() -> None:
    a = _args()
    world = _env_int("WORLD_SIZE", 1)
    rank = _env_int("RANK", 0)
    local = _env_int("LOCAL_RANK", 0)
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}; launch N>1 with torch.distributed.run")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29611")
    assert world % (a.tp * a.pp) == 0, "world size must be divisible by tp*pp"
    dp = world // (a.tp * a.pp)

    from scaling_amd.core import Topology
    from scaling_amd.core.logging import LoggerConfig, logger
    from scaling_amd.models import llama_architecture
    from scaling_amd.transformer.context import TransformerConfig, TransformerContext
    from scaling_amd.transformer.data.text_dataset import TextDataset
    from scaling_amd.transformer.model import init_model, init_optimizer
    from scaling_amd.transformer.model.model import loss_function, metrics_aggregation_fn

    from scaling_amd.utils.gemm_tuning import enable_tuned_gemms

    gemm_mode = enable_tuned_gemms(a.gemm_tuning, a.gemm_tuning_out, rank)
    arch = llama_architecture(a.model, sequence_length=a.seq_len)
    if a.num_layers is not None:
        arch["num_layers"] = a.num_layers
    cfg_dict = {
        "topology": {
            "world_size": world, "global_rank": rank, "local_slot": local,
            "model_parallel_size": a.tp, "pipe_parallel_size": a.pp, "data_parallel_size": dp,
            "micro_batch_size": a.micro_batch, "gradient_accumulation_steps": a.grad_acc,
            "activation_checkpointing_type": a.activation_checkpointing, "sequence_parallel": a.sequence_parallel,
        },
        "optimizer": {"beta1": 0.9, "beta2": 0.95, "eps": 1e-8, "gradient_clipping": 1.0, "zero": bool(a.zero)},
        "learning_rate_scheduler": {"learning_rate": 3e-4, "learning_rate_minimum": 3e-5,
                                    "learning_rate_decay_style": "cosine", "learning_rate_warmup_steps": 2,
                                    "learning_rate_decay_iters": 1000},
        "training": {"weight_decay": 0.1},
        "trainer": {"seed": 42, "train_iterations": a.warmup + a.steps},
        "logger": {"log_level": "warning"},
        "transformer_architecture": arch,
    }
    config = TransformerConfig.from_dict(cfg_dict)
    logger.configure(LoggerConfig(log_level="warning"), name=f"RANK {rank}", global_rank=rank)
    topology = Topology(config=config.topology)
    context = TransformerContext(config=config, topology=topology)
    context.initialize(master_addr=os.environ["MASTER_ADDR"], master_port=os.environ["MASTER_PORT"], seed=42)
    model = init_model(context=context)
    optimizer = init_optimizer(context=context, model=model)
    loader = _SyntheticLoader(a.micro_batch, a.seq_len, arch["vocab_size"], seed=1234 + topology.data_parallel_rank)

    def step() -> Any:
        out = model.train_step(loader, optimizer, TextDataset.sync_batch_to_model_parallel, loss_function,
                               metrics_aggregation_fn)
        context.step()
        return out

    for _ in range(a.warmup):
        step()
    dev = topology.device
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    per_step = []
    last: Optional[Any] = None
    for _ in range(a.steps):
        s0 = time.perf_counter()
        last = step()
        per_step.append(time.perf_counter() - s0)
    dist.barrier()
    torch.cuda.synchronize()
    elapsed = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    sec = float(elapsed.item())
    gbs = config.topology.global_batch_size
    tokens = gbs * a.seq_len * a.steps
    ms = 1000.0 * sec / a.steps
    if rank == 0:
        headline = a.num_layers is None and a.model == "llama2_7b" and a.seq_len == 4096
        res = {
            "metric": "tokens/sec (whole node) Llama-2-7B-shape bf16, TP×PP×DP on 1/2/4/8 MI355X",
            "value": tokens / sec,
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random token ids, random-init weights)",
            "config": {
                "model": ("Llama-2-7B-shape (h4096 L32 heads32 kv8 GQA, SwiGLU 11008, RoPE, RMSNorm, V32000)"
                          if headline else f"{a.model} layers={arch['num_layers']} seq={a.seq_len} (NOT headline)"),
                "global_batch": gbs,
                "seq_len": a.seq_len,
                "parallelism": f"tp{a.tp}_pp{a.pp}_dp{dp}" + ("_zero1" if a.zero else "") +
                               (f"_ac-{a.activation_checkpointing}" if a.activation_checkpointing != "disabled" else "") +
                               ("_sp" if a.sequence_parallel else ""),
                "micro_batch": a.micro_batch,
                "grad_acc": a.grad_acc,
                "loss": None if last is None else last.loss,
                "mfu_palm": None,
                "gemm_tuning": gemm_mode,
            },
        }
        n_params = sum(p.numel() for p in model.parameters()) * a.tp * a.pp if a.pp == 1 else None
        if n_params:
            flops_tok = 6 * n_params + 12 * arch["num_layers"] * arch["hidden_size"] * a.seq_len
            res["config"]["mfu_palm"] = (tokens / sec) * flops_tok / (2.5166e15 * world)
        if a.profile_json:
            with open(a.profile_json, "w") as f:
                json.dump({"per_step_s": per_step, **res}, f)
        print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
