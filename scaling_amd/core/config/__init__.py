from .base import BaseConfig, overwrite_recursive

__all__ = ["BaseConfig", "overwrite_recursive"]
