"""Hyper-parameter search (Py/automl/search/RayTuneSearchEngine.py, abstract.py).

Ray Tune is replaced by a local engine: the search space (fixed values,
``GridSearch`` lists, ``RandomSample`` functions) is expanded into
grid x ``num_samples`` trials; trials run in-process, or — with
``n_parallel > 1`` — in worker processes pinned one per GPU with
HIP_VISIBLE_DEVICES. The best trial by the metric wins.

``search_alg="BayesOpt"`` (the reference's ray.tune BayesOptSearch,
RayTuneSearchEngine.py:92-107) runs sequential Bayesian optimisation over a box
space ``{name: (low, high)}``: a Gaussian process (Matern-5/2 + noise, sklearn) is
fitted to the rewards seen so far and the next point maximises the acquisition
(``utility_kwargs``: ucb with kappa, ei / poi with xi), batch-parallel over
``n_parallel`` GPUs with the kriging-believer heuristic.
"""
import itertools
import logging
import multiprocessing as mp
import os

import numpy as np

log = logging.getLogger("zoo.automl")


from zoo.automl.search.abstract import (BayersianOpt, GoodError, GridSearch, RandomSample,  # noqa: F401
                                       SearchEngine as _AbstractSearchEngine, TrialOutput)


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
                        cfg[k] = v.func(cfg)
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


class BayesOptSearch:
    """GP-based Bayesian optimisation over ``space = {name: (low, high)}`` (maximises reward)."""

    def __init__(self, space, utility_kwargs=None, n_init=None, seed=0, n_candidates=4096):
        self.names = sorted(space)
        self.lo = np.array([float(space[k][0]) for k in self.names])
        self.hi = np.array([float(space[k][1]) for k in self.names])
        u = dict(utility_kwargs or {"kind": "ucb", "kappa": 2.5, "xi": 0.0})
        self.kind, self.kappa, self.xi = u.get("kind", "ucb"), float(u.get("kappa", 2.5)), float(u.get("xi", 0.0))
        self.n_init = n_init
        self.rng = np.random.default_rng(seed)
        self.n_candidates = n_candidates
        self.X, self.y = [], []

    def _unit(self, x):
        return (np.asarray(x) - self.lo) / np.maximum(self.hi - self.lo, 1e-12)

    def _point(self, u):
        return {k: float(v) for k, v in zip(self.names, self.lo + u * (self.hi - self.lo))}

    def _acq(self, mu, sd, best):
        from scipy.stats import norm
        if self.kind == "ucb":
            return mu + self.kappa * sd
        z = (mu - best - self.xi) / np.maximum(sd, 1e-12)
        if self.kind == "ei":
            return (mu - best - self.xi) * norm.cdf(z) + sd * norm.pdf(z)
        if self.kind == "poi":
            return norm.cdf(z)
        raise ValueError("utility kind must be ucb, ei or poi")

    def suggest(self, n=1):
        """n points to evaluate next (dicts in the original units)."""
        d = len(self.names)
        n_init = self.n_init if self.n_init is not None else max(2, min(5, d + 1))
        out = []
        X, y = [self._unit(x) for x in self.X], list(self.y)
        for _ in range(n):
            if len(X) < n_init:
                u = self.rng.random(d)
            else:
                from sklearn.gaussian_process import GaussianProcessRegressor
                from sklearn.gaussian_process.kernels import ConstantKernel, Matern, WhiteKernel
                gp = GaussianProcessRegressor(ConstantKernel(1.0) * Matern(length_scale=np.full(d, 0.3), nu=2.5) +
                                              WhiteKernel(1e-3), normalize_y=True, n_restarts_optimizer=2,
                                              random_state=int(self.rng.integers(1 << 30)))
                gp.fit(np.asarray(X), np.asarray(y))
                cand = self.rng.random((self.n_candidates, d))
                top = np.asarray(X)[np.argsort(y)[-3:]]   # local refinement around the best points
                cand = np.vstack([cand, np.clip(top[self.rng.integers(len(top), size=512)] +
                                                0.05 * self.rng.standard_normal((512, d)), 0, 1)])
                mu, sd = gp.predict(cand, return_std=True)
                u = cand[int(np.argmax(self._acq(mu, sd, max(y))))]
                # kriging believer: pretend the suggestion returned its mean (batch suggestions)
                y.append(float(gp.predict(u[None])[0]))
                X.append(u)
                out.append(self._point(u))
                continue
            X.append(u)
            y.append(float(np.mean(y)) if y else 0.0)
            out.append(self._point(u))
        return out

    def observe(self, point, reward):
        self.X.append(np.array([point[k] for k in self.names]))
        self.y.append(float(reward))


class SearchEngine(_AbstractSearchEngine):
    """The local counterpart of RayTuneSearchEngine (RayTuneSearchEngine.py:28-458):
    trials in-process or in worker processes pinned one per GPU."""

    def __init__(self, n_parallel=1, logs_dir=None):
        self.n_parallel, self.logs_dir = max(1, int(n_parallel)), logs_dir
        self.trials = []
        self._mode = "min"
        self._metric = "mse"

    def get_best_trials(self, k=1):
        """Configs of the best ``k`` finished trials (by the last run's metric and mode)."""
        sign = 1 if self._mode == "min" else -1
        ranked = sorted(self.trials, key=lambda t: sign * t[1][self._metric])
        return [c for c, _ in ranked[:k]]

    def _map(self, trial_fn, cfgs):
        if self.n_parallel > 1:
            ctx = mp.get_context("spawn")
            with ctx.Pool(self.n_parallel) as pool:
                return pool.map(_run_trial, [(trial_fn, c, i % self.n_parallel) for i, c in enumerate(cfgs)])
        return [trial_fn(c) for c in cfgs]

    def run_bayes(self, trial_fn, space, num_samples=1, metric="mse", mode="min", seed=0, fixed_params=None,
                  utility_kwargs=None):
        """Sequential GP Bayesian optimisation; ``space`` = {name: (low, high)}. Each point is
        turned into a trial config by ``convert_bayes_configs`` plus ``fixed_params``."""
        from zoo.automl.common.util import convert_bayes_configs
        self._metric, self._mode = metric, mode
        opt = BayesOptSearch(space, utility_kwargs, seed=seed)
        sign = -1.0 if mode == "min" else 1.0
        self.trials = []
        done = 0
        while done < num_samples:
            pts = opt.suggest(min(self.n_parallel, num_samples - done))
            cfgs = [dict(convert_bayes_configs(p), **(fixed_params or {})) for p in pts]
            for p, c, r in zip(pts, cfgs, self._map(trial_fn, cfgs)):
                opt.observe(p, sign * float(r[metric]))
                self.trials.append((c, r))
            done += len(pts)
        best = min(self.trials, key=lambda t: -sign * t[1][metric])
        log.info("best trial %s -> %s", best[0], best[1])
        return best

    def run(self, trial_fn, space, num_samples=1, metric="mse", mode="min", seed=0, search_alg=None,
            search_alg_params=None, fixed_params=None):
        """trial_fn(config) -> {metric: value, ...}; returns (best_config, best_result)."""
        if search_alg == "BayesOpt":
            return self.run_bayes(trial_fn, space, num_samples, metric, mode, seed, fixed_params,
                                  (search_alg_params or {}).get("utility_kwargs"))
        self._metric, self._mode = metric, mode
        if fixed_params:
            space = dict(space, **fixed_params)
        cfgs = expand(space, num_samples, seed)
        results = self._map(trial_fn, cfgs)
        self.trials = list(zip(cfgs, results))
        sign = 1 if mode == "min" else -1
        best = min(self.trials, key=lambda t: sign * t[1][metric])
        log.info("best trial %s -> %s", best[0], best[1])
        return best

# the reference's driver (compile / run / get_best_trials -> TrialOutput) lives in the submodule
# of its name: zoo.automl.search.RayTuneSearchEngine.RayTuneSearchEngine
