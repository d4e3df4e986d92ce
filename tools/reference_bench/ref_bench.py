"""Same-hardware baseline: the UNMODIFIED reference (``marcobellagente93/scaling``) training the headline
Llama-2-7B shape on one MI355X through PyTorch-ROCm, timed with bench.py's protocol ("Optional
same-hardware reference point").

    python tools/reference_bench/ref_bench.py --ref-src /path/to/reference/src [--steps K --warmup W
        --micro-batch B --grad-acc A --kernel torch|flash_attention]

The reference source is imported as-is from ``--ref-src`` (a scratch copy; nothing of it is vendored into this
repository).  Its optional integrations that this image does not ship (wandb, determined, torchvision,
tensorboard) are replaced by inert import stubs (``stubs.py``); none of them is on the training-step path.
Differences forced by the environment, stated in the JSON line:
  * attention ``kernel: torch`` (the reference's flash path needs the CUDA-only ``flash_attn`` package);
  * ``layernorm.optimization_type: torch`` (its only option without the CUDA extras).
Data: synthetic token ids of the benchmark shape, random-init weights — identical to bench.py.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from typing import Any

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def _args() -> argparse.Namespace:
    p = argparse.ArgumentParser()
    p.add_argument("--ref-src", required=True)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--seq-len", type=int, default=4096)
    p.add_argument("--micro-batch", type=int, default=1)
    p.add_argument("--grad-acc", type=int, default=8)
    p.add_argument("--num-layers", type=int, default=None, help="debug only (not the headline shape)")
    p.add_argument("--kernel", default="torch", choices=["torch", "flash_attention"])
    return p.parse_args()


def _arch(a: argparse.Namespace) -> dict[str, Any]:
    # the benchmark architecture in the reference's own schema (shared with bench.py's preset); values only
    sys.path.insert(0, ROOT)
    from scaling_amd.models.llama import llama_architecture

    arch = llama_architecture("llama2_7b", sequence_length=a.seq_len)
    sys.path.remove(ROOT)
    arch["layernorm"] = {"optimization_type": "torch", "layernorm_epsilon": 1e-5}
    arch["masked_softmax"] = {"kernel": a.kernel}
    if a.num_layers is not None:
        arch["num_layers"] = a.num_layers
    return arch


def main() -> None:
    a = _args()
    arch = _arch(a)
    for k in [k for k in sys.modules if k == "scaling" or k.startswith("scaling.")]:
        del sys.modules[k]
    sys.path.insert(0, os.path.abspath(a.ref_src))
    sys.path.insert(0, HERE)
    import stubs

    stubs.install()
    import torch

    import scaling  # the reference package
    from scaling.transformer.context import TransformerConfig, TransformerContext
    from scaling.transformer.data.text_dataset import TextDataset
    from scaling.transformer.data.text_dataset_batch import TextDatasetBatchBeforeSync
    from scaling.transformer.model import init_model, init_optimizer
    from scaling.transformer.model.model import loss_function, metrics_aggregation_fn
    from scaling.core import Topology

    assert os.path.abspath(a.ref_src) in os.path.abspath(scaling.__file__), scaling.__file__
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29621")
    cfg = {
        "topology": {"world_size": 1, "global_rank": 0, "local_slot": 0, "model_parallel_size": 1,
                     "pipe_parallel_size": 1, "data_parallel_size": 1, "micro_batch_size": a.micro_batch,
                     "gradient_accumulation_steps": a.grad_acc, "activation_checkpointing_type": "disabled"},
        "optimizer": {"beta1": 0.9, "beta2": 0.95, "eps": 1e-8, "gradient_clipping": 1.0, "zero": True},
        "learning_rate_scheduler": {"learning_rate": 3e-4, "learning_rate_minimum": 3e-5,
                                    "learning_rate_decay_style": "cosine", "learning_rate_warmup_steps": 2,
                                    "learning_rate_decay_iters": 1000},
        "training": {"weight_decay": 0.1},
        "trainer": {"seed": 42, "train_iterations": a.warmup + a.steps},
        "logger": {"log_level": "warning"},
        "transformer_architecture": arch,
    }
    config = TransformerConfig.from_dict(cfg)
    topology = Topology(config=config.topology)
    context = TransformerContext(config=config, topology=topology)
    context.initialize(master_addr=os.environ["MASTER_ADDR"], master_port=os.environ["MASTER_PORT"], seed=42)
    model = init_model(context=context)
    optimizer = init_optimizer(context=context, model=model)
    g = torch.Generator().manual_seed(1234)
    batches = [TextDatasetBatchBeforeSync(token_ids=torch.randint(1, arch["vocab_size"], (a.micro_batch, a.seq_len + 1),
                                                                   generator=g)) for _ in range(4)]

    class _Loader:
        i = 0

        def __iter__(self) -> "_Loader":
            return self

        def __next__(self) -> Any:
            b = batches[self.i % len(batches)]
            self.i += 1
            return b

    loader = _Loader()

    def step() -> Any:
        out = model.train_step(loader, optimizer, TextDataset.sync_batch_to_model_parallel, loss_function,
                               metrics_aggregation_fn)
        context.step()
        return out

    for i in range(a.warmup):
        step()
        print(f"warmup step {i} done", flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = None
    for i in range(a.steps):
        last = step()
        print(f"step {i} done", flush=True)
    torch.cuda.synchronize()
    sec = time.perf_counter() - t0
    gbs = a.micro_batch * a.grad_acc
    tokens = gbs * a.seq_len * a.steps
    print(json.dumps({
        "impl": "reference (unmodified marcobellagente93/scaling, PyTorch-ROCm eager)",
        "metric": "tokens/sec (whole node) Llama-2-7B-shape bf16", "value": tokens / sec, "unit": "tokens/s",
        "n_gpus": 1, "steps": a.steps, "warmup": a.warmup, "ms_per_step": 1000.0 * sec / a.steps,
        "config": {"global_batch": gbs, "seq_len": a.seq_len, "micro_batch": a.micro_batch, "grad_acc": a.grad_acc,
                   "attention_kernel": a.kernel, "layernorm": "torch", "num_layers": arch["num_layers"],
                   "loss": None if last is None else float(last.loss),
                   "peak_mem_gib": round(torch.cuda.max_memory_allocated() / 2**30, 1)},
    }), flush=True)


if __name__ == "__main__":
    main()
