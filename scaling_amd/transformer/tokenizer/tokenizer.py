"""Tokenizer wrapper over HF ``tokenizers`` (reference ``transformer/tokenizer/tokenizer.py``).

``load_tokenizers`` returns the tokenizer and a variant that does not insert a leading space
(needed to tokenize stop sequences / completions inside a prompt), with the Llama-2 normalizer /
decoder adjustments of the reference.  ``Tokenizer.default()`` resolves its vocabulary from
``$SCALING_AMD_TOKENIZER`` (no vocabulary file is bundled).
"""
from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Any, Union

from tokenizers import Tokenizer as HFTokenizer  # type: ignore

_EOS_CANDIDATES = ("<|endoftext|>", "</s>", "<eos>")


class Tokenizer:
    def __init__(self, tokenizer: HFTokenizer) -> None:
        self.tokenizer = tokenizer
        eos = None
        for cand in _EOS_CANDIDATES:
            eos = self.tokenizer.token_to_id(cand)
            if eos is not None:
                break
        assert eos is not None, f"tokenizer defines none of the end-of-text tokens {_EOS_CANDIDATES}"
        self.eos_token_id: int = eos

    @classmethod
    def from_file(cls, filename: Union[str, Path]) -> "Tokenizer":
        return cls(HFTokenizer.from_file(str(filename)))

    @classmethod
    def from_str(cls, json_str: str) -> "Tokenizer":
        return cls(HFTokenizer.from_str(json_str))

    @classmethod
    def default(cls) -> "Tokenizer":
        path = os.environ.get("SCALING_AMD_TOKENIZER")
        if not path:
            raise FileNotFoundError("no default vocabulary bundled: set SCALING_AMD_TOKENIZER to a tokenizer.json")
        return cls.from_file(path)

    def __len__(self) -> int:
        return self.tokenizer.get_vocab_size(with_added_tokens=False)

    @property
    def vocab_size(self) -> int:
        return len(self)

    def encode(self, text: str, add_special_tokens: bool = False) -> list[int]:
        return self.tokenizer.encode(text, add_special_tokens=add_special_tokens).ids

    def decode(self, token_ids: list[int], skip_special_tokens: bool = True) -> str:
        return self.tokenizer.decode(token_ids, skip_special_tokens=skip_special_tokens)


def _without_prefix_space(defn: dict[str, Any], llama_style: bool) -> dict[str, Any]:
    pre = defn.get("pre_tokenizer")
    if pre and pre.get("add_prefix_space"):
        pre["add_prefix_space"] = False
    if llama_style:
        dec = defn.get("decoder")
        if dec and dec.get("type") == "Sequence":
            dec["decoders"] = [d for d in dec["decoders"] if not (d.get("type") == "Strip" and d.get("content") == " ")]
        norm = defn.get("normalizer")
        if norm and norm.get("type") == "Sequence":
            norm["normalizers"] = [n for n in norm["normalizers"] if n.get("type") != "Prepend"]
    return defn


def load_tokenizers(tokenizer_file: Union[str, Path]) -> tuple[Tokenizer, Tokenizer]:
    tokenizer_file = Path(tokenizer_file)
    tok = Tokenizer.from_file(tokenizer_file)
    with open(tokenizer_file, "r", encoding="UTF-8") as f:
        defn = json.load(f)
    llama_style = "llama" in str(tokenizer_file)
    pre = defn.get("pre_tokenizer")
    if not llama_style and not (pre and pre.get("add_prefix_space")):
        return tok, tok
    return tok, Tokenizer.from_str(json.dumps(_without_prefix_space(defn, llama_style)))
