"""Search-engine contract and search-space markers (Py/automl/search/abstract.py:21-66)."""
from abc import ABC, abstractmethod


class GoodError(Exception):
    """Raised by a trial to stop the search early with a result that is good enough."""


class SearchEngine(ABC):
    """Hyper-parameter search engine: ``run`` the trials, then ``get_best_trials``."""

    @abstractmethod
    def run(self, *args, **kwargs):
        """Run the trials over the searched parameters."""

    @abstractmethod
    def get_best_trials(self, k):
        """The configs of the best ``k`` trials."""


class GridSearch(object):
    """Every value is tried (Cartesian product with the other grids)."""

    def __init__(self, values):
        self.values = list(values)


class RandomSample(object):
    """``func(spec)`` draws a value per sample (``spec`` = the config drawn so far)."""

    def __init__(self, func):
        self.func = func
        self.fn = func


class BayersianOpt(object):
    """Marker of the Bayesian-optimisation search algorithm (``search_alg="BayesOpt"``)."""

    def __init__(self):
        pass


class TrialOutput(object):
    def __init__(self, config, model_path):
        self.config = config
        self.model_path = model_path
