"""Builds the train/validation datasets from ``DataConfig`` (reference ``transformer/dataset_loader.py``)."""
from __future__ import annotations

from pathlib import Path
from typing import Any, Sequence

from ..core import BaseDataset
from .context.config import DataConfig, TransformerArchitectureConfig, TransformerConfig


def load_datasets(data_config: DataConfig, architecture_config: TransformerArchitectureConfig,
                  config: TransformerConfig) -> tuple[Sequence[BaseDataset], Sequence[BaseDataset]]:
    assert data_config.data_prefixes is not None, "path to data prefix not defined in Transformer context"

    def build(prefixes: list[Path]) -> list[Any]:
        return [_one(p, data_config, architecture_config, config) for p in prefixes]

    train = build(data_config.data_prefixes)
    val = build(data_config.validation_data_prefixes) if data_config.validation_data_prefixes else []
    return train, val


def _softprompt_tokens(a: TransformerArchitectureConfig) -> int:
    return 0 if a.softprompt_config is None else a.softprompt_config.n_tokens


def _tokenizers(a: TransformerArchitectureConfig) -> tuple[Any, Any]:
    from .tokenizer import load_tokenizers

    assert a.vocab_file is not None, "vocab_file needs to be set to load the vocabulary file."
    return load_tokenizers(a.vocab_file)


def _one(prefix: Path, d: DataConfig, a: TransformerArchitectureConfig, config: TransformerConfig) -> Any:
    seed = config.trainer.seed
    if d.finetuning_dataset:
        from .data.finetuning_text_dataset import FinetuningTextDataset

        assert d.use_mmap, "Finetuning is currently only supported with use_mmap set to true."
        tok, tok_nps = _tokenizers(a)
        return FinetuningTextDataset(data_prefix=prefix, sequence_length=a.sequence_length, seed=seed,
                                     softprompt_n_tokens=_softprompt_tokens(a), tokenizer=tok,
                                     tokenizer_no_prefix_space=tok_nps, memory_map_dataset=d.finetuning_dataset_memory_map)
    if d.finetuning_chat_dataset:
        from .data.finetuning_chat_dataset import FinetuningChatDataset

        tok, tok_nps = _tokenizers(a)
        return FinetuningChatDataset(data_path=prefix, sequence_length=a.sequence_length, seed=seed,
                                     softprompt_n_tokens=_softprompt_tokens(a), tokenizer=tok,
                                     tokenizer_no_prefix_space=tok_nps)
    from .data.text_dataset import TextDataset

    return TextDataset(data_prefix=prefix, sequence_length=a.sequence_length, seed=seed, legacy_dataset=d.legacy_dataset,
                       load_mmap_index_to_memory=d.load_mmap_index_to_memory,
                       load_data_item_mmap_index_to_memory=d.load_data_item_mmap_index_to_memory,
                       only_full_sequences=d.only_full_sequences,
                       allow_incomplete_sequences_every_n=d.allow_incomplete_sequences_every_n, use_mmap=d.use_mmap)
