"""Batch-1 greedy decode latency on one GPU: eager cached generation vs HIP-graph-captured decoding.

    python tools/decode_bench.py [--model llama2_7b] [--prompt 128] [--tokens 64]

Random-init weights of the named preset; the prompt is random token ids.  Per-token time excludes the prefill
(eager: generate(N+1) - generate(1); graph: the replay loop alone, capture reported separately).  Prints one
JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="llama2_7b")
    p.add_argument("--prompt", type=int, default=128)
    p.add_argument("--tokens", type=int, default=64)
    p.add_argument("--num-layers", type=int, default=None)
    a = p.parse_args()
    from scaling_amd.models import llama_architecture
    from scaling_amd.transformer.context.config import TransformerArchitectureConfig
    from scaling_amd.transformer.inference import TransformerInferenceModule, sample_argmax
    from scaling_amd.transformer.inference.graph_decode import GraphDecoder
    from scaling_amd.transformer.model.model import get_transformer_layer_specs
    from scaling_amd.utils.gemm_tuning import enable_tuned_gemms

    enable_tuned_gemms("use")
    arch_d = llama_architecture(a.model, sequence_length=max(4096, a.prompt + a.tokens))
    if a.num_layers is not None:
        arch_d["num_layers"] = a.num_layers
    arch = TransformerArchitectureConfig.from_dict(arch_d)
    torch.manual_seed(0)
    m = TransformerInferenceModule(get_transformer_layer_specs(arch), devices=(0,))
    prompt = torch.randint(1, arch.vocab_size, (a.prompt,)).tolist()

    def timed(fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        return time.perf_counter() - t, r

    m.generate(4, input_tokens=prompt, stop_tokens=[])  # warm-up (library handles, tables)
    t1, _ = timed(lambda: m.generate(1, input_tokens=prompt, stop_tokens=[]))
    tn, eager = timed(lambda: m.generate(a.tokens + 1, input_tokens=prompt, stop_tokens=[]))
    eager_ms = 1000.0 * (tn - t1) / a.tokens

    cur = m._pre_process_input(None, prompt, True)
    out = m.forward(cur)
    first = sample_argmax(out.activations)
    dec = GraphDecoder(m, a.prompt, a.tokens + 1, first, sample_argmax, out.activations[:, -1, :])
    tc, _ = timed(dec.capture)
    tg, (toks, _) = timed(lambda: dec.run([], check_every=a.tokens + 1))
    graph_ms = 1000.0 * tg / a.tokens
    same = toks == eager.completion_tokens
    print(json.dumps({
        "metric": "batch-1 greedy decode ms/token", "model": a.model, "layers": arch.num_layers, "prompt": a.prompt,
        "tokens": a.tokens, "eager_ms_per_token": round(eager_ms, 3), "graph_ms_per_token": round(graph_ms, 3),
        "speedup": round(eager_ms / graph_ms, 2), "graph_capture_ms": round(1000.0 * tc, 1),
        "graph_tokens_equal_eager": same, "weights_gib": round(sum(p.numel() * p.element_size() for p in m.parameters()) / 2**30, 2),
        "graph_gb_per_s": round(sum(p.numel() * p.element_size() for p in m.parameters()) / (graph_ms * 1e-3) / 1e9, 1),
    }), flush=True)


if __name__ == "__main__":
    main()
