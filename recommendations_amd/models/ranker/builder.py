"""RankerModelBuilder — the ModelBuilder the reference's main_training.py:30-31 asks
the ranker config for (models/ranker/builder.py is an empty file in the reference)."""
from .model import RankerModelWrapper


class RankerModelBuilder:
    def __init__(self, model_config, stats=None):
        self.model_config = model_config
        self.stats = stats

    def build(self) -> RankerModelWrapper:
        return RankerModelWrapper(self.model_config)
