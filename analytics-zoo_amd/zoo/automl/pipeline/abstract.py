"""Pipeline contract (Py/automl/pipeline/abstract.py:20-51)."""
from abc import ABC, abstractmethod


class Pipeline(ABC):
    @abstractmethod
    def evaluate(self, input_df, metrics=None, multioutput="raw_values"):
        """Metric values of the pipeline's predictions on ``input_df``."""

    @abstractmethod
    def predict(self, input_df):
        """Predictions (un-scaled, with datetimes) for ``input_df``."""

    @abstractmethod
    def save(self, ppl_file):
        """Persist the feature transformer, model and config."""
