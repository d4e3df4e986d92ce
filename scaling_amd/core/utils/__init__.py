from .param_merge import merge_parameter, split_parameter
from .port import find_free_port

__all__ = ["find_free_port", "merge_parameter", "split_parameter"]
