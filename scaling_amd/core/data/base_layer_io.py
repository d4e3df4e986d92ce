import torch


class BaseLayerIO:
    """Container passed between pipeline layers (reference ``core/data/base_layer_io.py:4``)."""

    def to_(self, device: torch.device) -> None:
        for name, attr in list(self.__dict__.items()):
            if isinstance(attr, torch.Tensor):
                setattr(self, name, attr.to(device, non_blocking=True))

    def contiguous_(self) -> None:
        for name, attr in list(self.__dict__.items()):
            if isinstance(attr, torch.Tensor):
                setattr(self, name, attr.contiguous())
