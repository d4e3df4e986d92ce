from .llama import llama_architecture, preset_names

__all__ = ["llama_architecture", "preset_names"]
