"""LTHMModelBuilder — models/lthm/builder.py:8-14 (ModelBuilder.build() -> the wrapper)."""
from .sequence.wrapper import LTHMModelWrapper


class LTHMModelBuilder:
    def __init__(self, stats, model_config):
        self.stats = stats
        self.model_config = model_config

    def build(self):
        return LTHMModelWrapper(model_config=self.model_config, stats=self.stats)
