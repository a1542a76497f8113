"""Feature-transformer contract (Py/automl/feature/abstract.py:20-97)."""
from abc import ABC, abstractmethod


class BaseFeatureTransformer(ABC):
    check_optional_config = False

    @abstractmethod
    def fit_transform(self, input_df, **config):
        """Fit the scalers / feature selection on ``input_df`` and return model inputs."""

    @abstractmethod
    def transform(self, input_df, is_train=True):
        """Model inputs for ``input_df`` with the fitted state."""

    @abstractmethod
    def save(self, file_path, replace=False):
        """Persist the fitted state (scalers, selected features, window length)."""

    @abstractmethod
    def restore(self, **config):
        """Restore the fitted state from a saved config."""

    @abstractmethod
    def _get_required_parameters(self):
        return set()

    @abstractmethod
    def _get_optional_parameters(self):
        return set()

    def _check_config(self, **config):
        missing = self._get_required_parameters() - set(config)
        if missing:
            raise ValueError("Missing required parameters in configuration. Required parameters are: %s"
                             % sorted(missing))
        if self.check_optional_config:
            missing = self._get_optional_parameters() - set(config)
            if missing:
                raise ValueError("Missing optional parameters in configuration. Optional parameters are: %s"
                                 % sorted(missing))
        return True
