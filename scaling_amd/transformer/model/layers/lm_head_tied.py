from .lm_head import TransformerLMHeadTied

__all__ = ["TransformerLMHeadTied"]
