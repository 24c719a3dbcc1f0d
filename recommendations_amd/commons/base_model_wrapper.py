"""Model API the trainer calls — same surface as commons/base_model_wrapper.py:9-72."""
from typing import Any, Dict, List, Optional, Tuple

import torch
import torch.nn as nn

DEFAULT_OPTIM_GROUP = "DEFAULT_OPTIM_GROUP"


class BaseModelWrapper(nn.Module):
    def __init__(self, dummy_params: bool = False, sparse: bool = False):
        super().__init__()
        if dummy_params:
            if sparse:
                self.dummy_dense_emb = nn.Embedding(1, 1)
            else:
                self.dummy_sparse_emb = nn.Embedding(1, 1, sparse=True)

    def train_step(self, batch: Dict[str, torch.Tensor], output: Any) -> Tuple[torch.Tensor, Dict[str, float]]:
        raise NotImplementedError("Subclasses must implement this method")

    def val_step(self, batch: Dict[str, torch.Tensor], output: Any) -> Tuple[torch.Tensor, Dict[str, float]]:
        raise NotImplementedError("Subclasses must implement this method")

    def is_sparse(self, param_name: str):
        return param_name == "dummy_sparse_emb"

    def inference_models(self, batch: Optional[Any] = None) -> List[torch.jit.ScriptModule]:
        raise NotImplementedError("Subclasses must implement this method")

    def get_weights(self) -> Dict[str, torch.Tensor]:
        return {k: v.cpu() for k, v in self.state_dict().items()}

    def set_weights(self, weights: Dict[str, torch.Tensor]) -> None:
        self.load_state_dict(weights)

    def get_gradients(self) -> List[Optional[torch.Tensor]]:
        return [None if p.grad is None else p.grad.data.cpu() for p in self.parameters()]

    def set_gradients(self, gradients: List[Optional[torch.Tensor]]) -> None:
        for g, p in zip(gradients, self.parameters()):
            if g is not None:
                p.grad = g

    def optim_group(self, parent_module: nn.Module, full_param_name: str, numel: int) -> Optional[str]:
        return None

    def optimizers_for_param_groups(self, param_groups: Dict[str, List[torch.nn.Parameter]]) -> \
            Optional[List[torch.optim.Optimizer]]:
        return None
