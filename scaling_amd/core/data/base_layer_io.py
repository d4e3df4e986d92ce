import torch


class BaseLayerIO:
    """Container passed between pipeline layers (reference ``core/data/base_layer_io.py:4``)."""

    def to_(self, device: torch.device) -> None:
        for name, attr in list(self.__dict__.items()):
            if isinstance(attr, torch.Tensor):
                # device-to-host copies must complete before the host reads them: only GPU targets are async
                setattr(self, name, attr.to(device, non_blocking=torch.device(device).type == "cuda"))

    def contiguous_(self) -> None:
        for name, attr in list(self.__dict__.items()):
            if isinstance(attr, torch.Tensor):
                setattr(self, name, attr.contiguous())
