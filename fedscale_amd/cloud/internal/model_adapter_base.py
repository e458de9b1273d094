"""ModelAdapterBase — the reference's adapter ABC (fedscale/cloud/internal/model_adapter_base.py:6-37)."""
import abc
from typing import Any


class ModelAdapterBase(abc.ABC):
    """An adapter that operates on a framework-specific model (same three abstract methods)."""

    @abc.abstractmethod
    def set_weights(self, weights, is_aggregator=True, client_training_results=None):
        """Set the model's weights (list in state_dict order); run the server optimizer if aggregating."""

    @abc.abstractmethod
    def get_weights(self):
        """The model's weights as a list in state_dict order."""

    @abc.abstractmethod
    def get_model(self) -> Any:
        """The framework-specific model."""
