"""BaseModel: the model contract the AutoML search engine trains and the pipelines
serve (Py/automl/model/abstract.py:20-105)."""
from abc import ABC, abstractmethod


class BaseModel(ABC):
    """``fit_eval`` trains on one configuration and returns the validation metric;
    ``save``/``restore`` move a trained trial between processes and pipelines."""

    check_optional_config = True
    future_seq_len = None

    @abstractmethod
    def fit_eval(self, x, y, validation_data=None, mc=False, verbose=0, **config):
        """Fit on (x, y) with ``config``; return the metric on ``validation_data`` (or the train set)."""

    @abstractmethod
    def evaluate(self, x, y, metric=None):
        """List of metric values on (x, y)."""

    @abstractmethod
    def predict(self, x, mc=False):
        """Predictions for x (``mc``: Monte-Carlo dropout active)."""

    @abstractmethod
    def save(self, model_path, config_path):
        """Write weights to ``model_path`` and the configuration to ``config_path``."""

    @abstractmethod
    def restore(self, model_path, **config):
        """Rebuild from ``config`` and load the weights at ``model_path``."""

    @abstractmethod
    def _get_required_parameters(self):
        """Set of config keys that must be present."""

    @abstractmethod
    def _get_optional_parameters(self):
        """Set of config keys that may be present."""

    def _check_config(self, **config):
        config_parameters = set(config.keys())
        missing = self._get_required_parameters() - config_parameters
        if missing:
            raise ValueError("Missing required parameters in configuration. Required parameters are: %s"
                             % sorted(missing))
        if self.check_optional_config:
            missing_opt = self._get_optional_parameters() - config_parameters
            if missing_opt:
                raise ValueError("Missing optional parameters in configuration. Optional parameters are: %s"
                                 % sorted(missing_opt))
        return True
