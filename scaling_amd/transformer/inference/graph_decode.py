"""Token-by-token generation with the decode step captured as ONE HIP graph.

Eager cached generation (``TransformerInferenceModule.generate``, reference
``transformer/inference/inference_model.py``) runs every decode step through the Python layer stack: ~15 kernel
launches per layer plus the host work around them, for a batch-1 step whose GPU time is a few milliseconds
(7B: the weights stream once per token).  On a single device the step is a fixed program once the cache has a
fixed capacity, so it is captured once and replayed:

* every attention layer's growing ``KVCache`` becomes a ``StaticKVCache`` of capacity ``prompt + max_tokens``
  sharing one ``DecodeState`` (device-side position / key range): the step writes its K/V rows at the device
  position and the flash-decoding kernel reads a device-side key range over a fixed-size buffer;
* the graph feeds the static token buffer, samples the next token into it, records token and logits at the
  device-side step index and advances the position — the host only replays and, every ``check_every`` steps,
  reads the tokens back to honour stop tokens.

Sampling must be graph-safe (device ops, no host sync): ``sample_argmax`` is; samplers that draw random numbers
are not supported here (they would replay the same draws).
"""
from __future__ import annotations

from typing import Any, Callable, Optional, Sequence

import torch

from ...core.nn.attention.attention import DecodeState, KVCache, ParallelSelfAttention, StaticKVCache
from ..data import TextDatasetBatch
from ..data.inference_settings import InferenceSettings


class GraphDecoder:
    def __init__(self, module: Any, n_prompt: int, max_tokens: int, first_token: torch.Tensor,
                 sample_fn: Callable[[torch.Tensor], torch.Tensor], vocab_logits: torch.Tensor,
                 cache_index: int = 0) -> None:
        self.module = module
        dev = first_token.device
        self.n_prompt = n_prompt
        self.max_tokens = max_tokens
        self.state = DecodeState(n_prompt, dev)
        self.attns = [m for m in module.modules() if isinstance(m, ParallelSelfAttention)]
        assert self.attns, "no attention layers"
        capacity = n_prompt + max_tokens
        for a in self.attns:
            kv = a.cache.get(cache_index)
            assert isinstance(kv, KVCache), "graph decoding starts from a prefilled KV cache"
            a.cache[cache_index] = StaticKVCache.from_cache(kv, capacity, self.state)
        self.first = first_token.reshape(1, 1).to(torch.long)
        self.tok = self.first.clone()
        self.tokens = torch.zeros(max_tokens, dtype=torch.long, device=dev)
        self.logits = torch.zeros((max_tokens,) + tuple(vocab_logits.shape[-1:]), dtype=vocab_logits.dtype, device=dev)
        self.tokens[0] = self.first.reshape(())
        self.logits[0].copy_(vocab_logits.reshape(-1))
        settings = InferenceSettings(use_cache=True, reset_cache=False, cache_index=cache_index, embedding_layers=[-1])
        cu_q = torch.tensor([0, 1], dtype=torch.int32, device=dev)
        self.batch = TextDatasetBatch(input_token_ids=self.tok, position_ids=self.state.pos.view(1, 1),
                                      cumulative_seq_lengths=cu_q, cumulative_seq_lengths_padded=cu_q,
                                      inference_settings=settings)
        self.sample_fn = sample_fn
        self._step_idx = torch.zeros(1, dtype=torch.long, device=dev)
        self.graph: Optional[torch.cuda.CUDAGraph] = None

    def _step(self) -> None:
        """One decode step, device ops only: feed ``tok`` at ``pos``, sample into ``tok``, record, advance."""
        out = self.module.forward(self.batch)
        act = out.activations
        nxt = self.sample_fn(act).reshape(1, 1)
        self.tok.copy_(nxt)
        torch.sub(self.state.pos, self.n_prompt - 1, out=self._step_idx)  # step k feeds position n_prompt + k - 1
        self.tokens.index_copy_(0, self._step_idx, nxt.reshape(1))
        self.logits.index_copy_(0, self._step_idx, act[:, -1, :].reshape(1, -1))
        self.state.advance()

    def capture(self) -> None:
        side = torch.cuda.Stream(device=self.tok.device)
        side.wait_stream(torch.cuda.current_stream(self.tok.device))
        with torch.cuda.stream(side), torch.no_grad():
            self._step()  # warm-up: allocator, TunableOp / library handles, lazy module state
        torch.cuda.current_stream(self.tok.device).wait_stream(side)
        self._rewind()
        g = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(g):
            self._step()
        self._rewind()  # capture records the work; it also ran it once (the state is reset before replay)
        self.graph = g

    def _rewind(self) -> None:
        self.state.reset(self.n_prompt)
        self.tok.copy_(self.first)

    def run(self, stop_tokens: Sequence[int], check_every: int = 8) -> tuple[list[int], torch.Tensor]:
        """Replays steps 1 .. max_tokens-1 (step 0 is the prefill's token); returns tokens (through the first
        stop token) and their logits."""
        assert self.graph is not None
        stops = set(int(t) for t in stop_tokens)
        if int(self.first.item()) in stops or self.max_tokens == 1:
            return [int(self.first.item())], self.logits[:1]
        done = 1
        while done < self.max_tokens:
            n = min(check_every, self.max_tokens - done)
            for _ in range(n):
                self.graph.replay()
            done += n
            self.state.check()
            got = self.tokens[:done].tolist()
            hit = next((i for i, t in enumerate(got) if t in stops), None)
            if hit is not None:
                return got[: hit + 1], self.logits[: hit + 1]
        return self.tokens[: self.max_tokens].tolist(), self.logits[: self.max_tokens]
