"""Hyper-parameter search (Py/automl/search/RayTuneSearchEngine.py, abstract.py).

Ray Tune is replaced by a local engine: the search space (fixed values,
``GridSearch`` lists, ``RandomSample`` functions) is expanded into
grid x ``num_samples`` trials; trials run in-process, or — with
``n_parallel > 1`` — in worker processes pinned one per GPU with
HIP_VISIBLE_DEVICES. The best trial by the metric wins.
"""
import itertools
import logging
import multiprocessing as mp
import os

import numpy as np

log = logging.getLogger("zoo.automl")


class GridSearch:
    def __init__(self, values):
        self.values = list(values)


class RandomSample:
    def __init__(self, fn):
        self.fn = fn


def expand(space, num_samples=1, seed=0):
    rng_state = np.random.get_state()
    np.random.seed(seed)
    grids = {k: v.values for k, v in space.items() if isinstance(v, GridSearch)}
    keys = list(grids)
    combos = list(itertools.product(*[grids[k] for k in keys])) or [()]
    out = []
    try:
        for combo in combos:
            for _ in range(num_samples):
                cfg = {}
                for k, v in space.items():
                    if isinstance(v, GridSearch):
                        cfg[k] = combo[keys.index(k)]
                    elif isinstance(v, RandomSample):
                        cfg[k] = v.fn(cfg)
                    else:
                        cfg[k] = v
                out.append(cfg)
    finally:
        np.random.set_state(rng_state)
    return out


def _run_trial(args):
    fn, cfg, gpu = args
    if gpu is not None:
        os.environ["HIP_VISIBLE_DEVICES"] = str(gpu)
    return fn(cfg)


class SearchEngine:
    def __init__(self, n_parallel=1, logs_dir=None):
        self.n_parallel, self.logs_dir = max(1, int(n_parallel)), logs_dir
        self.trials = []

    def run(self, trial_fn, space, num_samples=1, metric="mse", mode="min", seed=0):
        """trial_fn(config) -> {metric: value, ...}; returns (best_config, best_result)."""
        cfgs = expand(space, num_samples, seed)
        if self.n_parallel > 1:
            ctx = mp.get_context("spawn")
            with ctx.Pool(self.n_parallel) as pool:
                results = pool.map(_run_trial, [(trial_fn, c, i % self.n_parallel) for i, c in enumerate(cfgs)])
        else:
            results = [trial_fn(c) for c in cfgs]
        self.trials = list(zip(cfgs, results))
        sign = 1 if mode == "min" else -1
        best = min(self.trials, key=lambda t: sign * t[1][metric])
        log.info("best trial %s -> %s", best[0], best[1])
        return best
