"""Headline benchmark: whole-node training tokens/s of the Llama-2-7B shape in bf16 (BASELINE.json).

    python bench.py --gpus N --steps K --warmup W            # self-launches N ranks (one per GPU)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Each step is a full training step of the framework (``TransformerParallelModule.train_step``): all
micro-batches forward+backward through the HIP kernels, DP gradient reduce-scatter overlapped with the
last backward, grad-norm clipping and the fused ZeRO-1 AdamW update + parameter all-gather.  Data is
synthetic token ids of the benchmark shape, weights are random-init.  Per-GPU work is fixed (weak
scaling): every data-parallel rank processes ``micro_batch * grad_acc`` sequences per step.

Launch: without ``WORLD_SIZE`` in the environment and ``--gpus N > 1`` this process becomes a launcher
(reference ``core/runner/launch.py:73-161``): it spawns N worker processes of itself with
RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, never touches the GPU, kills the siblings as soon as one rank
fails and exits with that rank's code.

Rank 0 prints one JSON line; ``value`` is the whole-job tokens/s (global tokens / max-over-ranks time).
The line also carries what the ranks saw: the world size of the process group, every rank's step time,
and whether the parameters of all data-parallel replicas agree bit-for-bit after the last step.

``--backend gloo`` runs the same path on CPU processes (plumbing mode for the CPU test-suite);
``--backend gloo-gpu`` runs GPU ranks (several may share one GPU, which RCCL refuses) with gloo collectives
standing in for RCCL: a multi-rank rehearsal of the GPU-side paths (streams, events, kernels) on a 1-GPU box.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import time
from typing import Any, Optional

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "tokens/sec (whole node) Llama-2-7B-shape bf16, TP×PP×DP on 1/2/4/8 MI355X"
# the unmodified reference on one MI355X, same shape / batch / protocol (BASELINE.md "Measured same-hardware
# reference point", tools/reference_bench/ref_bench.py): the reference publishes no number of its own
REFERENCE_TOK_S_1GPU = 9909.0


def _args(argv: Optional[list[str]] = None) -> argparse.Namespace:
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--model", type=str, default="llama2_7b")
    p.add_argument("--seq-len", type=int, default=4096)
    # 8 sequences of 4096 tokens per GPU per step.  4 x 2 measured +2.8 % over 2 x 4 (bigger GEMMs, fewer
    # weight-gradient read-modify-writes; profiles/bench_7b_r2_microbatch_ab.log); 8 x 1 with the 32k-token
    # GEMMs in the tuned table another +0.6 % (profiles/bench_7b_r2i_mb8_ab.log, peak 230 GiB of 288 at one GPU)
    # and, with data parallelism, the gradient reduce-scatter overlaps the whole backward instead of the last
    # micro-batch's
    p.add_argument("--micro-batch", type=int, default=8)
    p.add_argument("--grad-acc", type=int, default=1)
    p.add_argument("--tp", type=int, default=1)
    p.add_argument("--pp", type=int, default=1)
    p.add_argument("--activation-checkpointing", type=str, default="disabled",
                   choices=["disabled", "every_layer", "every_layer_keep_attention", "every_layer_save_matmuls",
                            "every_pipe_stage"])
    p.add_argument("--sequence-parallel", action="store_true")
    p.add_argument("--tp-comm-chunks", type=int, default=0,
                   help="row-parallel GEMM + TP all-reduce / SP reduce-scatter in this many overlapped token pieces; "
                   "0 = chosen by comm_estimate.default_tp_comm_chunks (1 without TP)")
    p.add_argument("--zero", type=int, default=1)
    p.add_argument("--overlap-step", type=int, default=1,
                   help="run the optimizer update on a side stream, overlapped with the next forward (1) or inline (0)")
    p.add_argument("--lazy-zero", type=int, default=1,
                   help="optimizer lazy_grad_zeroing: no per-step gradient memset, first weight-gradient GEMM writes")
    p.add_argument("--lora", action="store_true",
                   help="LoRA finetune path (BASELINE #5): q/k/v/dense adapters trained, base weights frozen")
    p.add_argument("--lora-rank", type=int, default=64)
    p.add_argument("--preset", type=str, default=None, choices=sorted(PRESETS),
                   help="BASELINE.json layouts: baseline3 = TP2 x DP(N/2) ZeRO-1 + SP, baseline4 = TP2 x PP2 x DP(N/4) "
                        "1F1B + every_layer activation checkpointing + SP (baseline4_save_matmuls: the same with the "
                        "selective recompute), baseline5 = LoRA TP1 x DP(N) ZeRO-1 (overrides the layout flags it "
                        "names; see PRESETS)")
    p.add_argument("--shard-proxy", type=str, default=None, choices=["baseline3", "baseline4", "baseline4_save_matmuls"],
                   help="1-GPU per-rank proxy of an 8-GPU preset: ONE process runs rank 0's tensor-parallel shard "
                        "(TP2: 16 q / 4 kv heads, SwiGLU 5504, vocab 16000) of one pipeline stage's layers (baseline4: "
                        "16) with the preset's micro-batching, sequence parallelism and checkpointing; collectives are "
                        "stubbed (core/topology/stub_collectives.py), so the number is per-rank compute, not the "
                        "headline")
    p.add_argument("--proxy-comm", type=str, default="stub", choices=["stub", "emulate"],
                   help="--shard-proxy collectives: stub = free (per-rank compute only); emulate = each collective "
                        "streams its per-rank send volume through HBM on 16 CUs and holds them for its modelled xGMI "
                        "time (scaling_amd/core/topology/stub_collectives.py, transformer/utils/comm_estimate.py)")
    p.add_argument("--backend", type=str, default="auto", choices=["auto", "gloo", "gloo-gpu"],
                   help="gloo = CPU processes (plumbing mode, no GPU); gloo-gpu = rehearsal: GPU ranks (several "
                        "may share one GPU) with gloo collectives standing in for RCCL")
    p.add_argument("--precision", type=str, default="bfloat16", choices=["bfloat16", "float32"])
    p.add_argument("--num-layers", type=int, default=None, help="debug only: marks the result as not the headline config")
    p.add_argument("--gemm-tuning", type=str, default="use", choices=["use", "tune", "off"],
                   help="hipBLASLt solution table (scaling_amd/tuning/gemm_gfx950.csv); tune = benchmark and write")
    p.add_argument("--gemm-tuning-out", type=str, default=None)
    p.add_argument("--profile-json", type=str, default=None, help="write per-step times to this file")
    p.add_argument("--launch-timeout", type=float, default=3000.0, help="launcher: kill all ranks after this many s")
    argv = sys.argv[1:] if argv is None else argv
    return apply_example(apply_shard_proxy(apply_preset(p.parse_args(argv), argv), argv), argv)


# BASELINE.json config 2: "examples/transformer_example config.yml small GPT, TP=1 PP=1 DP=1 bf16 on one MI355X"
EXAMPLE_CONFIG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "examples", "transformer_example", "config.yml")


def example_config() -> dict[str, Any]:
    """The transformer example's config (examples/transformer_example/config.yml) as a dict."""
    from scaling_amd.transformer import TransformerConfig

    return TransformerConfig.from_yaml(EXAMPLE_CONFIG).as_dict()


def apply_example(a: argparse.Namespace, argv: Optional[list[str]] = None) -> argparse.Namespace:
    """``--model transformer_example``: the example's model, micro-batching and sequence length (explicit flags win)."""
    if a.model != "transformer_example":
        return a
    given = _explicit_flags(argv or [])
    t = example_config()["topology"]
    if "micro_batch" not in given:
        a.micro_batch = t["micro_batch_size"]
    if "grad_acc" not in given:
        a.grad_acc = t["gradient_accumulation_steps"]
    if "seq_len" not in given:
        a.seq_len = example_config()["transformer_architecture"]["sequence_length"]
    if "gemm_tuning" not in given:
        # the TunableOp table holds the 7B shapes only: for this model "use" is a per-GEMM lookup miss (~20 us of host
        # time each in a host-bound step), 4.7 vs 4.4 ms/step (profiles/bench_ab_ex_tuning_r6.log)
        a.gemm_tuning = "off"
    return a


# BASELINE.json configs 3-5 (the 8-GPU layouts; any N the layout divides).  Values override the corresponding flags.
PRESETS: dict[str, dict[str, Any]] = {
    # "Llama-2-7B-shape TP=2 PP=1 DP=4 bf16 + ZeRO-1": Megatron-SP inside the TP pair (reduce-scatter / all-gather
    # instead of all-reduce, activations sharded), row-parallel GEMMs overlapped with their collective in 4 pieces
    "baseline3": {"tp": 2, "pp": 1, "micro_batch": 8, "grad_acc": 1, "sequence_parallel": True, "tp_comm_chunks": 0,
                  "activation_checkpointing": "disabled", "lora": False, "zero": 1},
    # "TP=2 PP=2 DP=2 (full 3D parallel, 1F1B pipeline) with activation checkpointing": the reference's per-layer
    # checkpointing (every_layer).  Micro-batching 4 x 4: per-stage proxy with emulated comm, bubble applied, 2041 ms vs
    # 2058 (2 x 8) and 2080 (1 x 16) -- profiles/proxy_baseline4_mb_r6.md
    "baseline4": {"tp": 2, "pp": 2, "micro_batch": 4, "grad_acc": 4, "sequence_parallel": True, "tp_comm_chunks": 0,
                  "activation_checkpointing": "every_layer", "lora": False, "zero": 1},
    # the same layout with this framework's selective recompute (every_layer_save_matmuls keeps every GEMM output, the
    # recompute runs only the element-wise work): per-rank proxy 626 ms/step vs 807 for every_layer, 39.0 vs 30.8 GiB
    # (profiles/proxy_baseline4_ac_r5.log).  A labelled variant, not BASELINE #4's checkpointing semantics
    "baseline4_save_matmuls": {"tp": 2, "pp": 2, "micro_batch": 4, "grad_acc": 4, "sequence_parallel": True,
                               "tp_comm_chunks": 0, "activation_checkpointing": "every_layer_save_matmuls",
                               "lora": False, "zero": 1},
    # "7B + LoRA fine-tune path, TP=1 PP=1 DP=8 ZeRO-1 (PEFT adapters exercised)"
    "baseline5": {"tp": 1, "pp": 1, "micro_batch": 8, "grad_acc": 1, "sequence_parallel": False, "tp_comm_chunks": 1,
                  "activation_checkpointing": "disabled", "lora": True, "zero": 1},
}


def _explicit_flags(argv: list[str]) -> set[str]:
    """Destinations of the options given on the command line (``--micro-batch 2`` / ``--micro-batch=2``)."""
    out = set()
    for tok in argv:
        if tok.startswith("--"):
            out.add(tok[2:].split("=", 1)[0].replace("-", "_"))
    return out


def apply_shard_proxy(a: argparse.Namespace, argv: Optional[list[str]] = None) -> argparse.Namespace:
    """``--shard-proxy P``: P's layout for rank 0 of its tensor-parallel group, one pipeline stage, no data parallelism,
    in one process with the stubbed ("fake") process group.  Explicit --micro-batch / --grad-acc /
    --activation-checkpointing flags win (the A/B of checkpointing modes at the per-rank shape)."""
    if a.shard_proxy is None:
        return a
    lay = PRESETS[a.shard_proxy]
    given = _explicit_flags(argv or [])
    for k in ("micro_batch", "grad_acc", "sequence_parallel", "tp_comm_chunks", "lora", "zero",
              "activation_checkpointing"):
        if k not in given:
            setattr(a, k, lay[k])
    a.tp, a.pp = lay["tp"], 1
    if a.num_layers is None:
        from scaling_amd.models import llama_architecture

        a.num_layers = llama_architecture(a.model)["num_layers"] // lay["pp"]
    a.gpus = a.tp
    return a


def apply_preset(a: argparse.Namespace, argv: Optional[list[str]] = None) -> argparse.Namespace:
    """Overrides the layout flags of ``a`` with its ``--preset`` (if any) and checks that the GPU count fits.

    A flag given explicitly on the command line that the preset sets to a different value is an error: the run would
    otherwise report the preset's name for a layout that was not the one requested."""
    if a.preset is None:
        return a
    given = _explicit_flags(argv or [])
    clash = sorted(k for k, v in PRESETS[a.preset].items() if k in given and getattr(a, k) != v)
    if clash:
        raise SystemExit(f"bench.py: --preset {a.preset} sets " +
                         ", ".join(f"--{k.replace('_', '-')}={PRESETS[a.preset][k]}" for k in clash) +
                         "; drop the conflicting flag(s) or the preset")
    for k, v in PRESETS[a.preset].items():
        setattr(a, k, v)
    if a.gpus % (a.tp * a.pp) != 0:
        raise SystemExit(f"bench.py: --preset {a.preset} needs a multiple of {a.tp * a.pp} GPUs (got {a.gpus})")
    return a


def _env_int(k: str, d: int) -> int:
    v = os.environ.get(k)
    return d if v is None else int(v)


# ---------------------------------------------------------------------------------------------- launcher
def _free_port() -> int:
    from scaling_amd.core.utils.port import find_free_port  # outside the ephemeral range (no EADDRINUSE race)

    return find_free_port()


def _visible_devices() -> int:
    """GPU count without initialising the GPU (torch.cuda.device_count() does not; 1 when torch cannot tell)."""
    try:
        import torch

        return max(1, torch.cuda.device_count())
    except Exception:  # noqa: BLE001 - launcher on a host without torch GPU support
        return 1


def _rehearsal_slot(rank: int, world: int, ndev: Optional[int] = None) -> tuple[int, int, int]:
    """(device, index among the ranks on that device, ranks on that device) of a rehearsal rank: ranks are dealt over
    the visible devices round-robin (rank % ndev, as Topology.device places them)."""
    n = ndev or _visible_devices()
    dev = rank % n
    return dev, rank // n, len(range(dev, world, n))


def _launch(a: argparse.Namespace) -> int:
    """Spawns one worker per GPU (this file, with the rank env set); fail-fast on the first bad exit."""
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs: list[subprocess.Popen] = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if a.backend == "gloo":  # CPU ranks: do not oversubscribe the host's cores
            env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // a.gpus)))
        # optional: rehearsal ranks sharing a GPU each on a disjoint CU range, as each would own a GPU (value: the
        # device's CU count, "1" = MI355X's 256).  Rank r runs on device r % ndev (Topology.device), so the mask names
        # that device and splits its CUs among the ranks placed on it
        split = os.environ.get("SCALING_AMD_REHEARSAL_CU_SPLIT", "0") or "0"
        cus = 256 if split == "1" else int(split)
        if a.backend == "gloo-gpu" and cus and a.gpus > 1:
            dev, slot, per_dev = _rehearsal_slot(r, a.gpus)
            per = cus // per_dev
            env["HSA_CU_MASK"] = f"{dev}:{slot * per}-{(slot + 1) * per - 1}"
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))

    def _kill_all(sig: int) -> None:
        for q in procs:
            if q.poll() is None:
                try:
                    q.send_signal(sig)
                except ProcessLookupError:
                    pass

    def _on_signal(signum: int, _frame: Any) -> None:
        _kill_all(signum)

    signal.signal(signal.SIGTERM, _on_signal)
    signal.signal(signal.SIGINT, _on_signal)
    deadline = time.time() + a.launch_timeout
    rc = 0
    while True:
        codes = [q.poll() for q in procs]
        bad = [(i, c) for i, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            i, rc = bad[0]
            print(f"bench launcher: rank {i} exited with {rc}; terminating the other ranks", file=sys.stderr, flush=True)
            break
        if all(c == 0 for c in codes):
            return 0
        if time.time() > deadline:
            print("bench launcher: timeout, terminating all ranks", file=sys.stderr, flush=True)
            rc = 124
            break
        time.sleep(0.2)
    _kill_all(signal.SIGTERM)
    t_end = time.time() + 20
    while time.time() < t_end and any(q.poll() is None for q in procs):
        time.sleep(0.2)
    _kill_all(signal.SIGKILL)
    for q in procs:
        q.wait()
    return rc if rc > 0 else 1


# ---------------------------------------------------------------------------------------------- worker
class _SyntheticLoader:
    """Infinite iterator of fixed random token batches (generated once per slot, on host)."""

    def __init__(self, micro_batch: int, seq_len: int, vocab: int, seed: int, pin: bool, slots: int = 4):
        import torch

        from scaling_amd.transformer.data.text_dataset_batch import TextDatasetBatchBeforeSync

        g = torch.Generator().manual_seed(seed)
        self.batches = []
        for _ in range(slots):
            ids = torch.randint(1, vocab, (micro_batch, seq_len + 1), generator=g)
            self.batches.append(TextDatasetBatchBeforeSync(token_ids=ids.pin_memory() if pin else ids))
        self.i = 0

    def __iter__(self) -> "_SyntheticLoader":
        return self

    def __next__(self) -> Any:
        b = self.batches[self.i % len(self.batches)]
        self.i += 1
        return b


def _config_dict(a: argparse.Namespace, world: int, rank: int, local: int) -> dict[str, Any]:
    from scaling_amd.models import llama_architecture

    dp = world // (a.tp * a.pp)
    ex = example_config() if a.model == "transformer_example" else None
    if ex is not None:  # the example's architecture, optimizer and schedule as written (BASELINE #2)
        arch = dict(ex["transformer_architecture"], sequence_length=a.seq_len)
    else:
        arch = llama_architecture(a.model, sequence_length=a.seq_len, precision=a.precision)
    if a.num_layers is not None:
        arch["num_layers"] = a.num_layers
    training: dict[str, Any] = {"weight_decay": 0.1}
    if a.lora:
        arch["lora_config"] = {"name": "lora", "rank": a.lora_rank, "alpha": 16,
                               "parallel_modules": ["query", "key", "value", "dense"]}
        training.update(finetune=True, finetunable_parameters=["lora"])
    if a.tp_comm_chunks == 0:  # auto: from the first-order xGMI / GEMM time model
        from scaling_amd.transformer.utils.comm_estimate import default_tp_comm_chunks

        a.tp_comm_chunks = default_tp_comm_chunks(hidden_size=arch["hidden_size"], tokens=a.micro_batch * a.seq_len,
                                                  tp=a.tp)
    topo: dict[str, Any] = {
        "world_size": world, "global_rank": rank, "local_slot": local,
        "model_parallel_size": a.tp, "pipe_parallel_size": a.pp, "data_parallel_size": dp,
        "micro_batch_size": a.micro_batch, "gradient_accumulation_steps": a.grad_acc,
        "activation_checkpointing_type": a.activation_checkpointing, "sequence_parallel": a.sequence_parallel,
        "tensor_parallel_comm_chunks": a.tp_comm_chunks,
    }
    if a.backend in ("gloo", "gloo-gpu"):
        topo["backend"] = "gloo"
        topo["gloo_on_gpu"] = a.backend == "gloo-gpu"
    if a.shard_proxy is not None:
        topo["backend"] = "fake"
    optim = {"beta1": 0.9, "beta2": 0.95, "eps": 1e-8, "gradient_clipping": 1.0}
    lrs = {"learning_rate": 3e-4, "learning_rate_minimum": 3e-5, "learning_rate_decay_style": "cosine",
           "learning_rate_warmup_steps": 2, "learning_rate_decay_iters": 1000}
    if ex is not None:
        optim = {k: ex["optimizer"][k] for k in ("beta1", "beta2", "eps", "gradient_clipping", "allreduce_bucket_size")}
        lrs = dict(ex["learning_rate_scheduler"])
        training = dict(weight_decay=ex["training"]["weight_decay"], **{k: v for k, v in training.items()
                                                                        if k != "weight_decay"})
    return {
        "topology": topo,
        "optimizer": {**optim, "zero": bool(a.zero), "overlap_optimizer_step": bool(a.overlap_step),
                      "lazy_grad_zeroing": bool(a.lazy_zero)},
        "learning_rate_scheduler": lrs,
        "training": training,
        "trainer": {"seed": 42, "train_iterations": a.warmup + a.steps},
        "logger": {"log_level": "warning"},
        "transformer_architecture": arch,
    }


def _param_checksum(model: Any, device: Any) -> Any:
    """(sum, sum of squares, index-weighted sum) over this rank's parameters, in float64."""
    import torch

    acc = torch.zeros(3, dtype=torch.float64, device=device)
    with torch.no_grad():
        for i, p in enumerate(model.parameters()):
            x = p.detach().double()
            acc[0] += x.sum()
            acc[1] += (x * x).sum()
            acc[2] += (i + 1) * x.sum()
    return acc


def _worker(a: argparse.Namespace) -> None:
    import torch
    import torch.distributed as dist

    world = _env_int("WORLD_SIZE", 1)
    rank = _env_int("RANK", 0)
    local = _env_int("LOCAL_RANK", 0)
    if a.shard_proxy is not None:  # one process = rank 0 of the TP group (stubbed collectives)
        world, rank, local = a.gpus, 0, 0
        os.environ["SCALING_AMD_PROXY_COMM"] = a.proxy_comm
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(_free_port()) if world == 1 else "29611")
    assert world % (a.tp * a.pp) == 0, "world size must be divisible by tp*pp"
    dp = world // (a.tp * a.pp)

    from scaling_amd.core import Topology
    from scaling_amd.core.logging import LoggerConfig, logger
    from scaling_amd.transformer.context import TransformerConfig, TransformerContext
    from scaling_amd.transformer.data.text_dataset import TextDataset
    from scaling_amd.transformer.model import init_model, init_optimizer
    from scaling_amd.transformer.model.model import loss_function, metrics_aggregation_fn
    from scaling_amd.transformer.utils.comm_estimate import comm_volume_estimate
    from scaling_amd.utils.gemm_tuning import enable_tuned_gemms

    gpu = a.backend != "gloo"
    # forensics / A-B instrumentation kept outside the production code (e.g. tools/attn_forensics.py): each listed file
    # is executed once here, before the model is built, and may wrap framework functions
    for hook in filter(None, os.environ.get("SCALING_AMD_DEBUG_HOOKS", "").split(",")):
        import runpy

        runpy.run_path(hook)
    if os.environ.get("SCALING_AMD_DETERMINISTIC") == "1":  # library-side determinism (race-check forensics)
        from scaling_amd.core.utils.debug_env import DETERMINISTIC_ENV, apply

        apply(DETERMINISTIC_ENV)
        torch.use_deterministic_algorithms(True)
    gemm_mode = enable_tuned_gemms(a.gemm_tuning, a.gemm_tuning_out, rank) if gpu else "off"
    cfg_dict = _config_dict(a, world, rank, local)
    arch = cfg_dict["transformer_architecture"]
    config = TransformerConfig.from_dict(cfg_dict)
    logger.configure(LoggerConfig(log_level="warning"), name=f"RANK {rank}", global_rank=rank)
    topology = Topology(config=config.topology)
    context = TransformerContext(config=config, topology=topology)
    context.initialize(master_addr=os.environ["MASTER_ADDR"], master_port=os.environ["MASTER_PORT"], seed=42)
    dev = topology.device
    if gpu and dev.type != "cuda":
        raise SystemExit("bench.py: no GPU visible (use --backend gloo for the CPU plumbing mode)")
    if os.environ.get("BENCH_FAIL_RANK") == str(rank):  # launcher fail-fast test hook
        raise SystemExit(3)
    model = init_model(context=context)
    optimizer = init_optimizer(context=context, model=model)
    # per-rank proxy: token ids from rank 0's vocabulary shard.  The stubbed collectives cannot sum the other shard's
    # embedding rows in, so an id outside the shard would embed as a zero vector (in the real layout the TP all-reduce
    # supplies it); such rows normalise to ~0 and their gradient explodes through every norm of the backward
    vocab = arch["vocab_size"] // a.tp if a.shard_proxy else arch["vocab_size"]
    loader = _SyntheticLoader(a.micro_batch, a.seq_len, vocab, seed=1234 + topology.data_parallel_rank,
                              pin=gpu)

    def sync() -> None:
        if dev.type == "cuda":
            torch.cuda.synchronize()

    trace = os.environ.get("SCALING_AMD_BENCH_TRACE")  # race-check forensics: per-step values per rank (JSON lines)
    n_steps = [0]
    pre: list = []
    if trace:  # local gradients as the backward left them, before the optimizer step touches anything
        orig_step = optimizer.step

        def traced_step() -> Any:  # a stream-ordered snapshot (no host sync: it must not change the schedule)
            with torch.no_grad():
                pre[:] = [torch.stack([p.grad.double().sum() if p.grad is not None else p.new_zeros((), dtype=torch.float64)
                                       for p in model.parameters()])]
            return orig_step()

        optimizer.step = traced_step

    # race-check forensics: the gradient ENTERING every module's backward, in backward execution order, as stream-ordered
    # device checksums (no host sync inside the step): the first entry where two runs differ names the module whose
    # successor (in forward order) produced a different input gradient
    gtrace: list = []
    if trace and os.environ.get("SCALING_AMD_BENCH_TRACE_GRADS") == "1":
        def _grad_probe(name: str) -> Any:
            def fwd_hook(_m: Any, _inp: Any, out: Any) -> None:
                ts = [out] if torch.is_tensor(out) else [t for t in (out if isinstance(out, (tuple, list)) else [])
                                                           if torch.is_tensor(t)]
                ts += [v for v in (getattr(out, "__dict__", {}) or {}).values() if torch.is_tensor(v)]
                for i, t in enumerate(ts):
                    if t.requires_grad and t.is_floating_point():
                        t.register_hook(lambda g, n=f"{name}[{i}]": gtrace.append(
                            (n, torch.stack([g.double().sum(), (g.double() * g.double()).sum()]))))
            return fwd_hook

        for mname, mod in model.named_modules():
            if mname:
                mod.register_forward_hook(_grad_probe(mname))
        from scaling_amd.core.utils import grad_probe

        grad_probe.enable(gtrace)  # + the probes inside the layers (attention input / q,k,v / core output, layer input)

    if os.environ.get("SCALING_AMD_BENCH_NORMS") == "1":  # debug: per-module output / per-parameter gradient magnitudes
        def _norm_hook(name: str) -> Any:
            def hook(_m: Any, _inp: Any, out: Any) -> None:
                t = out if torch.is_tensor(out) else getattr(out, "activations", None)
                if torch.is_tensor(t) and t.is_floating_point() and rank == 0:
                    f = t.detach().float()
                    print(f"[norms] fwd {name}: absmax {f.abs().max().item():.4g} rms {f.pow(2).mean().sqrt().item():.4g}",
                          file=sys.stderr, flush=True)
                    if t.requires_grad:
                        t.register_hook(lambda g, n=name: print(
                            f"[norms] bwd into {n}: absmax {g.detach().float().abs().max().item():.4g}", file=sys.stderr,
                            flush=True))
                    br = getattr(out, "residual_branch", None)
                    if torch.is_tensor(br) and br.requires_grad:
                        br.register_hook(lambda g, n=name: print(
                            f"[norms] bwd into {n}.residual_branch: absmax {g.detach().float().abs().max().item():.4g}",
                            file=sys.stderr, flush=True))
            return hook

        for mname, mod in model.named_modules():
            if mname.count(".") <= 3 and mname:
                mod.register_forward_hook(_norm_hook(mname))
        orig_step2 = optimizer.step

        def norm_step() -> Any:
            if rank == 0:
                for n, p in model.named_parameters():
                    if p.grad is not None:
                        g = p.grad.detach().float()
                        print(f"[norms] grad {n}: absmax {g.abs().max().item():.4g} finite {bool(torch.isfinite(g).all())}",
                              file=sys.stderr, flush=True)
            return orig_step2()

        optimizer.step = norm_step

    def step() -> Any:
        out = model.train_step(loader, optimizer, TextDataset.sync_batch_to_model_parallel, loss_function,
                               metrics_aggregation_fn)
        context.step()
        if trace:
            optimizer.wait_param_sync()
            with torch.no_grad():
                rec = {"step": n_steps[0], "loss": out.loss, "grad_norm": out.global_grad_norm,
                       "names": [n for n, _ in model.named_parameters()] if n_steps[0] == 0 else None,
                       "params": [float(p.detach().double().sum()) for p in model.parameters()],
                       "grads": [float(g.grad_source().double().sum()) for g in optimizer.parameter_groups],
                       # local (pre-reduction) gradients: lazy zeroing leaves them in the flat buffer after the step
                       "pgrads": [float(p.grad.double().sum()) if p.grad is not None else None
                                  for p in model.parameters()],
                       "pgrads_pre": pre[0].tolist() if pre else [],
                       "gtrace": [(n, [float(x) for x in v.tolist()]) for n, v in gtrace]}
            gtrace.clear()
            with open(f"{trace}.rank{rank}.jsonl", "a") as f:
                f.write(json.dumps(rec) + "\n")
        n_steps[0] += 1
        return out

    for _ in range(a.warmup):
        step()
    dist.barrier()
    sync()
    prof_out = os.environ.get("SCALING_AMD_BENCH_CPROFILE")  # host-side profile of the timed steps only (rank 0)
    prof = None
    if prof_out and rank == 0:
        import cProfile

        prof = cProfile.Profile()
    t0 = time.perf_counter()
    per_step = []
    last: Optional[Any] = None
    if prof is not None:
        prof.enable()
    for _ in range(a.steps):
        s0 = time.perf_counter()
        last = step()
        per_step.append(time.perf_counter() - s0)
    if prof is not None:
        prof.disable()
        prof.dump_stats(prof_out)
    dist.barrier()
    sync()
    mine = time.perf_counter() - t0

    # ---- cross-rank facts: per-rank times, world size, data-parallel parameter agreement
    times = torch.zeros(world, dtype=torch.float64, device=dev)
    times[rank] = mine
    dist.all_reduce(times)
    sec = float(times.max().item())
    optimizer.wait_param_sync()
    ck = _param_checksum(model, dev)
    cks = [torch.zeros_like(ck) for _ in range(dp)]
    dist.all_gather(cks, ck, group=topology.data_parallel_group)
    dp_agree = bool(all(torch.equal(cks[0], c) for c in cks[1:]))
    agree_t = torch.tensor([1.0 if dp_agree else 0.0], device=dev)
    dist.all_reduce(agree_t, op=dist.ReduceOp.MIN)
    dp_agree = bool(agree_t.item() == 1.0)
    _, unique_params = model.get_params_count()
    local_params = sum(p.numel() for p in model.parameters() if p.requires_grad)

    gbs = config.topology.global_batch_size
    tokens = gbs * a.seq_len * a.steps
    ms = 1000.0 * sec / a.steps
    if rank == 0:
        headline = (a.num_layers is None and a.model == "llama2_7b" and a.seq_len == 4096 and a.backend == "auto"
                    and a.precision == "bfloat16" and a.shard_proxy is None)
        flops_tok = 6 * unique_params + 12 * arch["num_layers"] * arch["hidden_size"] * a.seq_len
        if a.lora:  # frozen base: no weight-gradient GEMMs for the base weights (~1/3 of the 6N)
            flops_tok = None
        parallelism = (f"tp{a.tp}_pp{a.pp}_dp{dp}" + ("_zero1" if a.zero else "") +
                       (f"_ac-{a.activation_checkpointing}" if a.activation_checkpointing != "disabled" else "") +
                       ("_sp" if a.sequence_parallel else "") + ("_lora" if a.lora else ""))
        proxy_est = None
        if a.shard_proxy is not None:
            world_note = (f"per-rank proxy of --preset {a.shard_proxy}: rank 0 of TP{a.tp}, {arch['num_layers']} layers "
                          "(one pipeline stage), collectives " +
                          ("emulated (modelled xGMI time + HBM traffic on 16 CUs)" if a.proxy_comm == "emulate"
                           else "stubbed") + "; value = ONE rank's tokens/s")
            lay = PRESETS[a.shard_proxy]
            # what 8 GPUs of the preset would reach with free communication: 8 / (tp pp) data-parallel replicas, each
            # pipeline running at the 1F1B efficiency m / (m + pp - 1) (m micro-batches)
            proxy_est = (tokens / sec) * 8 / (lay["tp"] * lay["pp"]) * a.grad_acc / (a.grad_acc + lay["pp"] - 1)
        res = {
            "metric": ("per-rank proxy tokens/s (NOT the headline): " + world_note if a.shard_proxy is not None else
                       "tokens/sec examples/transformer_example small GPT bf16 (BASELINE #2)"
                       if a.model == "transformer_example" else METRIC),
            "value": tokens / sec,
            "unit": "tokens/s",
            "n_gpus": world if a.shard_proxy is None else 1,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (tokens / sec) / (REFERENCE_TOK_S_1GPU * world) if headline and not a.lora else None,
            "baseline": ("unmodified reference on MI355X (torch attention, best micro-batch 2 x acc 4): "
                         f"{REFERENCE_TOK_S_1GPU:.0f} tok/s per GPU x n_gpus (BASELINE.md)" if headline else None),
            "dtype": "bf16" if a.precision == "bfloat16" else "fp32",
            "data": "synthetic (random token ids, random-init weights)",
            "config": {
                "model": ("Llama-2-7B-shape (h4096 L32 heads32 kv8 GQA, SwiGLU 11008, RoPE, RMSNorm, V32000)"
                          if headline else
                          "examples/transformer_example config.yml small GPT (BASELINE #2, NOT the headline): "
                          f"h{arch['hidden_size']} L{arch['num_layers']} heads{arch['num_attention_heads']} "
                          f"V{arch['vocab_size']} seq {a.seq_len}" if a.model == "transformer_example" else
                          f"{a.model} layers={arch['num_layers']} seq={a.seq_len} (NOT headline)"),
                "global_batch": gbs,
                "seq_len": a.seq_len,
                "parallelism": parallelism,
                "preset": a.preset,
                "shard_proxy": a.shard_proxy,
                "proxy_comm": a.proxy_comm if a.shard_proxy is not None else None,
                "proxy_8gpu_tokens_s_without_comm": proxy_est,
                # the effective layout (after --preset), field by field
                "tp": a.tp, "pp": a.pp, "dp": dp, "sequence_parallel": a.sequence_parallel,
                "activation_checkpointing": a.activation_checkpointing, "zero": bool(a.zero),
                "micro_batch": a.micro_batch,
                "grad_acc": a.grad_acc,
                "loss": None if last is None else last.loss,
                "mfu_palm": None if flops_tok is None or not gpu else (tokens / sec) * flops_tok / (2.5166e15 * world),
                "gemm_tuning": gemm_mode,
                "params": unique_params,
                "backend": dist.get_backend(),
                "world_size_seen": dist.get_world_size(),
                "per_rank_ms_per_step": [round(1000.0 * float(t) / a.steps, 2) for t in times.tolist()],
                "dp_param_checksum_agree": dp_agree,
                "param_checksum": [float(v) for v in ck.tolist()],
                "peak_mem_gib": round(torch.cuda.max_memory_allocated(dev) / 2**30, 1) if dev.type == "cuda" else None,
                "tp_comm_chunks": a.tp_comm_chunks,
                # what this layout must move per step and rank (first-order xGMI time, no overlap): a reading aid for
                # multi-GPU results (scaling_amd/transformer/utils/comm_estimate.py)
                "comm_estimate": comm_volume_estimate(
                    hidden_size=arch["hidden_size"], num_layers=arch["num_layers"], seq_len=a.seq_len,
                    micro_batch=a.micro_batch, grad_acc=a.grad_acc, tp=a.tp, pp=a.pp, dp=dp,
                    params_per_rank=local_params, precision=a.precision),
            },
        }
        if a.profile_json:
            with open(a.profile_json, "w") as f:
                json.dump({"per_step_s": per_step, **res}, f)
        print(json.dumps(res), flush=True)
    if gemm_mode == "tune":
        from scaling_amd.utils.gemm_tuning import write_tuning_file

        write_tuning_file()
    dist.barrier()
    dist.destroy_process_group()
    if not dp_agree:
        raise SystemExit("data-parallel replicas diverged (parameter checksums differ)")


def main() -> None:
    a = _args()
    if a.lora and a.gemm_tuning == "tune":
        # the LoRA path's GEMMs write / read column slices (ld > n): TunableOp's tuning pass mis-handles them
        # (invalid-argument errors and non-finite results measured on MI355X); tune on the full-training path
        raise SystemExit("bench.py: --gemm-tuning tune is not supported with --lora")
    if "WORLD_SIZE" not in os.environ and a.gpus > 1 and a.shard_proxy is None:
        sys.exit(_launch(a))
    _worker(a)


if __name__ == "__main__":
    main()
