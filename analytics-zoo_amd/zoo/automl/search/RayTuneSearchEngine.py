"""RayTuneSearchEngine (Py/automl/search/RayTuneSearchEngine.py:28-458) without Ray.

Same driver contract as the reference -- ``compile(input_df, search_space, num_samples, stop,
search_algorithm, search_algorithm_params, fixed_params, feature_transformers, future_seq_len,
validation_df, mc, metric)``, ``run()``, ``get_best_trials(k)`` -> ``TrialOutput(config,
model_path)``, ``test_run()`` -- with ray.tune replaced by the local engine of
zoo.automl.search: trials expand from GridSearch x RandomSample x ``num_samples`` (or are
suggested one by one by the GP ``BayesOptSearch``), run in-process or in worker processes
pinned one per GPU, and each trial is the reference's train function: up to 100 iterations of
``TimeSequenceModel.fit_eval``, a ``reward_metric`` (mse negated, r2 as is) reported per
iteration, the best iteration checkpointed as ``best.ckpt`` (feature transformer + model +
config zip, zoo.automl.common.util.save_zip) in the trial's log directory, and the ``stop``
criteria (``training_iteration``, ``reward_metric``: stop once reached) ending the loop.
"""
import copy
import os

import numpy as np
import pandas as pd

from zoo.automl.common.util import convert_bayes_configs, save_zip
from zoo.automl.model.time_sequence import TimeSequenceModel
from zoo.automl.search import BayesOptSearch, SearchEngine, expand
from zoo.automl.search.abstract import GoodError, GridSearch, RandomSample, TrialOutput


class _StopTrial(Exception):
    pass


class Trial:
    """What ray.tune keeps of a finished trial: config, log dir and the last reported result."""

    def __init__(self, config, logdir):
        self.config, self.logdir = config, logdir
        self.last_result = {}
        self.results = []


def _run_local_trial(args):
    train_func, config, logdir, stop, gpu = args
    if gpu is not None:
        os.environ["HIP_VISIBLE_DEVICES"] = str(gpu)
    trial = Trial(config, logdir)
    os.makedirs(logdir, exist_ok=True)

    def reporter(**kw):
        trial.last_result = dict(kw)
        trial.results.append(dict(kw))
        for k, v in (stop or {}).items():
            if k in kw and kw[k] >= v:
                raise _StopTrial()
    cwd = os.getcwd()
    os.chdir(logdir)                     # the train function checkpoints relative to its trial dir
    try:
        train_func(config, reporter)
    except _StopTrial:
        pass
    finally:
        os.chdir(cwd)
    return trial


class _TrialTrainer:
    """The per-trial train function (picklable, so spawned worker processes can run it):
    fit the trial's feature transformer, then train the model up to ``max_iters`` epochs of
    ``fit_eval``, reporting ``reward_metric`` (metric_op * mean metric) each epoch and keeping
    the best epoch's (transformer, model, config) in ``best.ckpt`` of the trial directory."""
    ckpt = "best.ckpt"
    max_iters = 100

    def __init__(self, input_df, feature_transformers, future_seq_len, validation_df, metric_op, mc):
        self.input_df, self.ft = input_df, feature_transformers
        self.future_seq_len, self.validation_df = future_seq_len, validation_df
        self.metric_op, self.mc = metric_op, mc

    def __call__(self, config, report):
        ft = copy.deepcopy(self.ft)
        model = TimeSequenceModel(check_optional_config=False, future_seq_len=self.future_seq_len)
        config = dict(convert_bayes_configs(config))
        x, y = ft.fit_transform(copy.deepcopy(self.input_df), **config)
        val = None if self.validation_df is None else ft.transform(copy.deepcopy(self.validation_df))
        best = None
        for epoch in range(1, self.max_iters + 1):
            metric = model.fit_eval(x, y, validation_data=val, mc=self.mc, **config)
            reward = self.metric_op * float(np.mean(metric))
            if best is None or reward > best:
                best = reward
                save_zip(self.ckpt, ft, model, config)
            report(training_iteration=epoch, reward_metric=reward, checkpoint=self.ckpt)


class RayTuneSearchEngine(SearchEngine):
    def __init__(self, logs_dir="", resources_per_trial=None, name="", remote_dir=None, n_parallel=1):
        super().__init__(n_parallel=n_parallel, logs_dir=logs_dir)
        self.pipeline = None
        self.train_func = None
        self.resources_per_trail = resources_per_trial
        self.trials = None
        self.remote_dir = remote_dir
        self.name = name or "automl"

    def compile(self, input_df, search_space, num_samples=1, stop=None, search_algorithm=None,
                search_algorithm_params=None, fixed_params=None, feature_transformers=None, future_seq_len=1,
                validation_df=None, mc=False, metric="mean_squared_error"):
        self.search_space = self._prepare_tune_config(search_space)
        self.stop_criteria = stop
        self.num_samples = num_samples
        if metric in ("mse", "mean_squared_error"):
            metric_op = -1
        elif metric == "r2":
            metric_op = 1
        else:
            raise ValueError("metric can only be \"mse\" or \"r2\"")
        self.search_algorithm = None
        if search_algorithm == "BayesOpt":
            self.search_algorithm = ("BayesOpt", (search_algorithm_params or {}).get("utility_kwargs"))
        self.fixed_params = fixed_params
        self.train_func = self._prepare_train_func(input_df, feature_transformers, future_seq_len, validation_df,
                                                   metric_op, mc, self.remote_dir)
        return self

    def _logdir(self, i):
        base = os.path.expanduser(self.logs_dir or "~/zoo_automl_logs")
        return os.path.join(base, self.name, "train_func_%d" % i)

    def run(self):
        stop = dict(self.stop_criteria or {})
        if not self.search_algorithm:
            cfgs = expand(self.search_space, self.num_samples)
            args = [(self.train_func, c, self._logdir(i), stop, (i % self.n_parallel) if self.n_parallel > 1
                     else None) for i, c in enumerate(cfgs)]
            self.trials = self._map_trials(args)
        else:
            _, utility = self.search_algorithm
            opt = BayesOptSearch(self.search_space, utility)
            self.trials = []
            i = 0
            while i < self.num_samples:
                pts = opt.suggest(min(self.n_parallel, self.num_samples - i))
                args = [(self.train_func, dict(p, **(self.fixed_params or {})), self._logdir(i + j), stop,
                         (j % self.n_parallel) if self.n_parallel > 1 else None) for j, p in enumerate(pts)]
                for p, t in zip(pts, self._map_trials(args)):
                    opt.observe(p, float(t.last_result.get("reward_metric", -1e30)))
                    self.trials.append(t)
                i += len(pts)
        return self

    def _map_trials(self, args):
        if self.n_parallel > 1:
            import multiprocessing as mp
            with mp.get_context("spawn").Pool(self.n_parallel) as pool:
                return pool.map(_run_local_trial, args)
        return [_run_local_trial(a) for a in args]

    def get_best_trials(self, k=1):
        ranked = self._get_sorted_trials(self.trials, metric="reward_metric")
        return [self._make_trial_output(t) for t in ranked[:k]]

    def _make_trial_output(self, trial):
        return TrialOutput(config=trial.config, model_path=os.path.join(trial.logdir, trial.last_result["checkpoint"]))

    # ---- trial ranking: higher reported metric is better (mse is reported negated) ----------
    @staticmethod
    def _score(trial, metric):
        return trial.last_result.get(metric, 0)

    @classmethod
    def _get_sorted_trials(cls, trial_list, metric):
        scored = [(cls._score(t, metric), n, t) for n, t in enumerate(trial_list)]
        scored.sort(key=lambda e: (-e[0], e[1]))       # stable: ties keep submission order
        return [t for _, _, t in scored]

    @classmethod
    def _get_best_trial(cls, trial_list, metric):
        ranked = cls._get_sorted_trials(trial_list, metric)
        return ranked[0] if ranked else None

    @classmethod
    def _get_best_result(cls, trial_list, metric):
        best = cls._get_best_trial(trial_list, metric)
        return {metric: best.last_result[metric]}

    def test_run(self):
        """Smoke-check the train function against a probe reporter: the first report must carry
        the reward metric and the checkpoint name (what run() and get_best_trials() rely on).
        Returns 1 when it does; raises otherwise."""
        seen = {}

        def probe(**report):
            seen.update(report)
            raise GoodError("train function reported")
        probe_config = {"out_units": 1, "selected_features": ["MONTH(datetime)", "WEEKDAY(datetime)"]}
        try:
            self.train_func(probe_config, probe)
        except GoodError:
            missing = [k for k in ("reward_metric", "checkpoint") if k not in seen]
            if missing:
                raise AssertionError("train function report lacks %s" % ", ".join(missing))
            return 1
        raise RuntimeError("train function returned without reporting a result")

    @staticmethod
    def _is_validation_df_valid(validation_df):
        """A usable validation set: a non-empty DataFrame, or a list holding at least one."""
        frames = validation_df if isinstance(validation_df, list) else [validation_df]
        return any(isinstance(f, pd.DataFrame) and not f.empty for f in frames)

    @staticmethod
    def _prepare_train_func(input_df, feature_transformers, future_seq_len, validation_df=None, metric_op=1,
                            mc=False, remote_dir=None):
        return _TrialTrainer(input_df, feature_transformers, future_seq_len,
                             validation_df if RayTuneSearchEngine._is_validation_df_valid(validation_df) else None,
                             metric_op, mc)

    def _prepare_tune_config(self, space):
        # GridSearch / RandomSample markers are expanded by the local engine as they are
        return {k: v for k, v in space.items()}


__all__ = ["RayTuneSearchEngine", "Trial", "GridSearch", "RandomSample"]
