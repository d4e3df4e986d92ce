"""Text <-> token ids."""
from .tokenizer import Tokenizer, load_tokenizers

__all__ = ["Tokenizer", "load_tokenizers"]
