from .clip import ClipModifiedResNet, clip_transform
from .image_encoder import ImageEncoder

__all__ = ["ClipModifiedResNet", "ImageEncoder", "clip_transform"]
