"""Multi-rank rehearsal on one MI355X: bench.py's self-launched ranks share the GPU with gloo collectives
standing in for RCCL (which refuses two ranks per device).  Everything else is the production GPU path —
the comm stream of the overlapped DP reduce-scatter, the event-ordered ZeRO all-gather of the overlapped
optimizer step, lazy gradient zeroing, async TP input-gradient all-reduce, pipe p2p of GPU tensors, the HIP
kernels — at world sizes 2, 4 and 8, so stream/event ordering bugs of the multi-GPU bench surface on a 1-GPU
box.  Checks: one JSON line, every rank ran, the data-parallel replicas agree bit-for-bit, finite loss."""
from __future__ import annotations

import math

import pytest
import torch

from tests.test_bench import _json_lines, _run

pytestmark = pytest.mark.gpu

SMALL = ["--model", "llama_tiny", "--backend", "gloo-gpu", "--seq-len", "256", "--micro-batch", "2", "--steps", "3",
         "--warmup", "2"]


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
@pytest.mark.parametrize(
    "layout",
    [
        ("2", "1", "1", "1", []),                             # dp2: reduce-scatter + all-gather on the comm stream
        ("2", "2", "1", "2", ["--sequence-parallel"]),        # tp2 + SP, async input-gradient all-reduce
        ("4", "2", "2", "2", []),                             # tp2 x pp2: GPU pipe p2p
        ("4", "1", "2", "1", []),                             # pp2 x dp2, one micro-batch
        ("8", "2", "2", "2", []),                             # tp2 x pp2 x dp2
        ("8", "2", "2", "2", ["--activation-checkpointing", "every_layer"]),  # BASELINE #4 layout
        ("8", "2", "1", "1", []),                             # tp2 x dp4 (BASELINE #3 layout)
        ("4", "1", "1", "2", ["--activation-checkpointing", "every_layer"]),
        ("2", "1", "1", "2", ["--lora", "--lora-rank", "8"]),         # LoRA fast path under ZeRO dp2
        ("8", "2", "1", "1", ["--preset", "baseline3"]),              # BASELINE #3 preset: + SP, 4 comm pieces
        ("8", "2", "2", "4", ["--preset", "baseline4"]),              # BASELINE #4 preset
        ("8", "1", "1", "1", ["--preset", "baseline5", "--lora-rank", "8"]),  # BASELINE #5 preset
    ],
)
def test_bench_rehearsal_gloo_gpu(layout):
    gpus, tp, pp, acc, extra = layout
    if "--preset" in extra:  # the preset owns the layout flags (an explicit conflicting one is an error)
        small = [a for i, a in enumerate(SMALL) if a != "--micro-batch" and SMALL[i - 1] != "--micro-batch"]
        r = _run(["--gpus", gpus, *small, *extra], timeout=300)
    else:
        r = _run(["--gpus", gpus, "--tp", tp, "--pp", pp, "--grad-acc", acc, *SMALL, *extra], timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    res = lines[0]
    n = int(gpus)
    assert res["n_gpus"] == n and res["config"]["world_size_seen"] == n and res["config"]["backend"] == "gloo"
    assert len(res["config"]["per_rank_ms_per_step"]) == n
    assert res["config"]["dp_param_checksum_agree"] is True
    assert res["config"]["peak_mem_gib"] is not None  # ranks ran on the GPU
    loss = res["config"]["loss"]  # rank 0's view (None on a first pipe stage that does not see the loss)
    assert loss is None or math.isfinite(loss)
    if pp == "1":
        assert loss is not None
    assert res["vs_baseline"] is None and "NOT headline" in res["config"]["model"]


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_rehearsal_tp_loss_matches_single_rank():
    """TP2 (and TP2 + sequence parallelism) on GPU ranks trains the same model on the same data as one rank:
    after two optimizer steps the loss agrees to bf16 accuracy (the row/column splits only change the GEMM
    reduction order)."""
    base = ["--model", "llama_tiny", "--backend", "gloo-gpu", "--seq-len", "256", "--micro-batch", "2",
            "--steps", "2", "--warmup", "0"]
    losses = {}
    for tag, args in [("tp1", ["--gpus", "1"]), ("tp2", ["--gpus", "2", "--tp", "2"]),
                      ("tp2_sp", ["--gpus", "2", "--tp", "2", "--sequence-parallel"]),
                      # row-parallel GEMM + collective in 4 pieces overlapped on the TP communication stream
                      ("tp2_chunks", ["--gpus", "2", "--tp", "2", "--tp-comm-chunks", "4"]),
                      ("tp2_sp_chunks", ["--gpus", "2", "--tp", "2", "--sequence-parallel", "--tp-comm-chunks", "4"])]:
        r = _run([*args, *base], timeout=300)
        assert r.returncode == 0, r.stderr[-4000:]
        losses[tag] = _json_lines(r.stdout)[0]["config"]["loss"]
    assert all(math.isfinite(v) for v in losses.values()), losses
    for tag in ("tp2", "tp2_sp", "tp2_chunks", "tp2_sp_chunks"):
        assert losses[tag] == pytest.approx(losses["tp1"], rel=2e-2), losses
    assert losses["tp2_chunks"] == pytest.approx(losses["tp2"], rel=2e-3), losses
    assert losses["tp2_sp_chunks"] == pytest.approx(losses["tp2_sp"], rel=2e-3), losses


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
@pytest.mark.parametrize("mp,pp,world", [(2, 2, 4), (1, 2, 4), (2, 1, 4)])
def test_rehearsal_train_resume_bit_exact_gpu(tmp_path, mp, pp, world):
    """The training entry point (data pipeline -> 3D engine -> ZeRO-1 -> checkpoint at step 6) on GPU ranks sharing
    the MI355X, bf16 + flash attention: resuming from the step-6 checkpoint reproduces steps 7-10 exactly."""
    import numpy as np

    from tests.test_training import _config, _make_data, _run as _train

    _make_data(tmp_path / "data")
    cfg = _config(tmp_path, mp, pp, world, precision="bfloat16", masked_softmax={"kernel": "flash_attention"},
                  hidden_size=128, sequence_length=128)
    cfg["topology"]["backend"] = "gloo"
    cfg["topology"]["gloo_on_gpu"] = True
    full = _train(tmp_path, cfg, world, "full")
    assert len(full) == 10 and all(np.isfinite(m["training/loss"]) for m in full)
    cfg["trainer"]["assert_checkpoint_loaded"] = True
    resumed = _train(tmp_path, cfg, world, "resumed")
    assert [m["training/loss"] for m in resumed] == [m["training/loss"] for m in full[-4:]]


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
@pytest.mark.parametrize(
    "args,env",
    [
        (["--gpus", "1", "--backend", "auto"], {}),                            # overlapped step on its side stream
        (["--gpus", "1", "--backend", "auto"], {"SCALING_AMD_WGRAD_STREAM": "1"}),  # + weight-gradient stream
        (["--gpus", "2"], {}),                                                 # DP comm stream
        (["--gpus", "2"], {"SCALING_AMD_COMM_DELAY_US": "1000"}),              # ... running 1 ms late per collective
        (["--gpus", "4", "--grad-acc", "2"], {"SCALING_AMD_COMM_DELAY_US": "1000"}),
        (["--gpus", "8", "--tp", "2", "--pp", "2", "--grad-acc", "2"], {}),
        # RCCL lifetimes (core/topology/gloo_gpu.py, asynchronous mode): every collective only enqueued, its input
        # read and its output written when the stream gets there / the peers are done
        (["--gpus", "2"], {"SCALING_AMD_REHEARSAL_ASYNC": "1"}),
        (["--gpus", "4", "--grad-acc", "2"], {"SCALING_AMD_REHEARSAL_ASYNC": "1", "SCALING_AMD_COMM_DELAY_US": "1000"}),
        # TP2 + SP with the row-parallel GEMMs in 4 pieces on the TP communication stream, async input-gradient
        # all-reduce
        (["--gpus", "2", "--tp", "2", "--sequence-parallel", "--tp-comm-chunks", "4"], {"SCALING_AMD_REHEARSAL_ASYNC": "1"}),
        # TP2 x PP2: pipeline p2p with RCCL's lifetimes too (payload read when the stream gets there, sends in flight)
        (["--gpus", "4", "--tp", "2", "--pp", "2", "--grad-acc", "2"], {"SCALING_AMD_REHEARSAL_ASYNC": "1"}),
    ],
)
def test_race_check_multi_stream_equals_single_stream(args, env):
    """Race check: the multi-stream schedule (DP communication stream, overlapped optimizer step,
    optional weight-gradient stream, per-layer event waits) must leave bit-identical parameters and losses to
    the same run with every side stream folded onto the compute stream (SCALING_AMD_SINGLE_STREAM=1).  A missing
    stream / event dependency shows up as a different checksum -- and so does any kernel whose result depends on
    timing.  Both runs use library-side determinism (SCALING_AMD_DETERMINISTIC=1: torch deterministic algorithms,
    rocBLAS without atomics): with several ranks sharing the one GPU, the default vendor GEMM kernels' atomic
    accumulation order varies from run to run (profiles/race_repeat_dp2_r4.log).

    History: round 5 fixed a cross-wave LDS-DMA race in the attention loops (flash_attn.h: dma_barrier) and then ran the
    multi-rank cases on disjoint CU ranges; round 6 found what the ranks' shared CUs exposed: the SLP-packed fp32
    rotation of the RoPE kernels (v_pk_mul/fma_f32 with operand-select modifiers) returned a different last bit in
    2-8 % of attention backwards when another process's waves shared the GPU, 0 % built unpacked
    (profiles/race_forensics_r6.md) -- so every multi-rank case runs on shared CUs again.  The SCALING_AMD_REHEARSAL_ASYNC
    cases run the collectives with RCCL's lifetimes (core/topology/gloo_gpu.py): inputs read and outputs written when
    the stream gets there, long after the call returned, so a missing record_stream / early free shows up too."""
    base = ["--model", "llama_tiny", "--backend", "gloo-gpu", "--seq-len", "256", "--micro-batch", "2", "--steps", "3",
            "--warmup", "1"]
    out = {}
    for mode, extra in (("multi", {}), ("single", {"SCALING_AMD_SINGLE_STREAM": "1"})):
        r = _run([*base, *args], env_extra={**env, **extra, "SCALING_AMD_DETERMINISTIC": "1"}, timeout=300)
        assert r.returncode == 0, r.stderr[-4000:]
        res = _json_lines(r.stdout)[0]["config"]
        out[mode] = (res["param_checksum"], res["loss"])
    assert out["multi"] == out["single"], out


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
@pytest.mark.parametrize("before,after", [((2, 2, 8), (1, 1, 1)), ((1, 1, 1), (2, 2, 8)), ((1, 2, 4), (2, 1, 4))])
def test_rehearsal_layout_change_resume_gpu(tmp_path, before, after):
    """Layout-independent checkpoints on GPU ranks (bf16, flash attention, ZeRO-1): saved at step 6 under one
    (TP, PP, world) layout, resumed under another, the run continues (reference tolerance: 15 % on the loss;
    global batch kept constant through the data-parallel size x gradient accumulation)."""
    from tests.test_training import _config, _make_data, _run as _train

    _make_data(tmp_path / "data")

    def cfg_for(mp, pp, world):
        c = _config(tmp_path, mp, pp, world, precision="bfloat16", masked_softmax={"kernel": "flash_attention"},
                    hidden_size=128, sequence_length=128)
        dp = world // (mp * pp)
        c["topology"]["gradient_accumulation_steps"] = 4 // dp if dp <= 4 else 1
        c["topology"]["backend"] = "gloo"
        c["topology"]["gloo_on_gpu"] = True
        return c

    full = _train(tmp_path, cfg_for(*before), before[2], "full")
    c2 = cfg_for(*after)
    c2["trainer"]["assert_checkpoint_loaded"] = True
    resumed = _train(tmp_path, c2, after[2], "resumed")
    a = [m["training/loss"] for m in full][-4:]
    b = [m["training/loss"] for m in resumed]
    assert len(b) == 4 and all(abs(x - y) / x < 0.15 for x, y in zip(a, b)), (a, b)


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
@pytest.mark.parametrize("mp,pp,world,initial_scale", [(1, 1, 1, 16.0), (2, 1, 2, 16.0), (1, 1, 2, 2.0 ** 40)])
def test_rehearsal_fp16_loss_scaling_resume_bit_exact_gpu(tmp_path, mp, pp, world, initial_scale):
    """fp16 + dynamic loss scaling on the GPU path (flash attention in fp16, fp16 weight gradients through the
    hipBLASLt fallback of the bf16-only hand-written wgrad kernel, fused fp16 AdamW / grad-norm): trains, skips the
    overflowing steps of a 2^40 initial scale on every rank, and resumes bit-exactly from the step-6 checkpoint."""
    import numpy as np

    from tests.test_training import _config, _make_data, _run as _train

    _make_data(tmp_path / "data")
    cfg = _config(tmp_path, mp, pp, world, precision="float16", masked_softmax={"kernel": "flash_attention"},
                  hidden_size=128, sequence_length=128)
    cfg["optimizer"]["loss_scaler"] = {"enable": True, "initial_scale": initial_scale, "window": 3, "hysteresis": 1}
    cfg["topology"]["backend"] = "gloo"
    cfg["topology"]["gloo_on_gpu"] = True
    full = _train(tmp_path, cfg, world, "full")
    assert len(full) == 10 and all(np.isfinite(m["training/loss"]) for m in full)
    scales = [m["training/current_loss_scale"] for m in full]
    if initial_scale > 1e9:
        assert any(m["training/overflow"] for m in full) and scales[-1] < initial_scale
    else:
        assert max(scales) > initial_scale
    cfg["trainer"]["assert_checkpoint_loaded"] = True
    resumed = _train(tmp_path, cfg, world, "resumed")
    assert [m["training/loss"] for m in resumed] == [m["training/loss"] for m in full[-4:]]


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
@pytest.mark.parametrize("kernel", ["torch", "flash_attention"])
def test_deterministic_torch_training_gpu(tmp_path, kernel):
    """``training.use_deterministic_torch_algorithms: true`` (reference tests/transformer/test_training.py:845-862)
    trains on the GPU with every torch op passing the deterministic-algorithms check (the dense mask builder uses
    a sorted search, not a scatter-add), and two runs give bit-identical losses."""
    import numpy as np

    from tests.test_training import _config, _make_data, _run as _train

    _make_data(tmp_path / "data")
    cfg = _config(tmp_path, 1, 1, 1, precision="bfloat16", masked_softmax={"kernel": kernel},
                  hidden_size=128, sequence_length=128)
    cfg["training"]["use_deterministic_torch_algorithms"] = True
    cfg["trainer"]["save_dir"] = None
    cfg["trainer"]["load_dir"] = None
    a = _train(tmp_path, cfg, 1, "det_a")
    b = _train(tmp_path, cfg, 1, "det_b")
    assert len(a) == 10 and all(np.isfinite(m["training/loss"]) for m in a)
    assert [m["training/loss"] for m in a] == [m["training/loss"] for m in b]


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_keep_attention_checkpointing_gpu(tmp_path):
    """Per-layer checkpointing that keeps the flash-attention output + LSE: identical losses to plain per-layer
    checkpointing, rounding-close to no checkpointing (deterministic kernels, attention dropout on), and the backward's
    recompute runs no attention forward (one fa_fwd per layer and micro-batch instead of two)."""
    from scaling_amd.ops import _ext
    from tests.test_training import _config, _make_data, _run as _train

    _make_data(tmp_path / "data")
    losses = {}
    for ac in ("disabled", "every_layer", "every_layer_keep_attention", "every_layer_save_matmuls"):
        cfg = _config(tmp_path, 1, 1, 1, precision="bfloat16", masked_softmax={"kernel": "flash_attention"},
                      hidden_size=128, sequence_length=128, checkpointing=ac)
        cfg["trainer"]["save_dir"] = None
        cfg["trainer"]["load_dir"] = None
        losses[ac] = [m["training/loss"] for m in _train(tmp_path, cfg, 1, ac)]
    # keep-attention (and the selective recompute that also keeps the GEMM outputs) reproduces plain per-layer
    # checkpointing bit for bit; against no checkpointing the recompute re-associates some gradient sums (autograd
    # accumulation order at the checkpoint seams), so only rounding-close
    assert losses["every_layer_keep_attention"] == losses["every_layer"], losses
    assert losses["every_layer_save_matmuls"] == losses["every_layer"], losses
    assert losses["every_layer"][0] == losses["disabled"][0]
    assert all(abs(a - b) <= 2e-3 * abs(b) for a, b in zip(losses["every_layer"], losses["disabled"])), losses

    # fa_fwd calls of one checkpointed layer, forward + backward
    from scaling_amd.core.nn.parallel_module.activation_checkpointing import checkpoint_with_rng
    from scaling_amd.models import llama_architecture
    from scaling_amd.transformer.context.config import TransformerArchitectureConfig
    from scaling_amd.transformer.model.layers import TransformerLayer
    from scaling_amd.transformer.model.layers.base import TransformerLayerIO

    arch = TransformerArchitectureConfig(**llama_architecture("llama_tiny", sequence_length=128, vocab_size=512))
    layer = TransformerLayer(arch, layer_index=0).cuda()
    e = _ext.ext()
    real = e.fa_fwd
    calls = []

    def counting(*a, **k):
        calls.append(1)
        return real(*a, **k)

    for keep, want in ((False, 2), (True, 1)):
        calls.clear()
        x = torch.randn(2, 128, arch.hidden_size, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        cu = torch.tensor([0, 128, 256], dtype=torch.int32, device="cuda")
        pos = torch.arange(128, device="cuda").unsqueeze(0).expand(2, -1).contiguous()
        io = TransformerLayerIO(activations=x, position_ids=pos, cumulative_seq_lengths_padded=cu,
                                cumulative_seq_lengths=cu)
        e.fa_fwd = counting
        try:
            out = checkpoint_with_rng(layer._forward_tuple_input, None, True, *layer.input_to_tuple(io),
                                      keep_attention=keep)
            out.hidden().float().pow(2).mean().backward()
            torch.cuda.synchronize()
        finally:
            e.fa_fwd = real
        assert len(calls) == want, (keep, len(calls))
