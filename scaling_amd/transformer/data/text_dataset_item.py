import torch

from ...core import BaseDatasetItem


class TextDatasetItem(BaseDatasetItem):
    def __init__(self, token_ids: torch.Tensor):
        super().__init__()
        self.token_ids = token_ids
