"""TimeSequencePredictor (Py/automl/regression/time_sequence_predictor.py:32-296): search
feature selections / look-back windows / model hyper-parameters with a recipe; every trial
fits a TimeSequenceFeatureTransformer and a TimeSequenceModel (trained by this framework's
engine -- data-parallel over the initialised process group with ``distributed=True``) and
is scored on the validation frame; the best trial comes back as a TimeSequencePipeline."""
import logging

from zoo.automl.common.metrics import Evaluator
from zoo.automl.config.recipe import SmokeRecipe
from zoo.automl.feature.time_sequence import TimeSequenceFeatureTransformer

log = logging.getLogger("zoo.automl")


class TimeSequencePredictor:
    def __init__(self, name="automl", logs_dir="~/zoo_automl_logs", future_seq_len=1, dt_col="datetime",
                 target_col="value", extra_features_col=None, drop_missing=True):
        self.name, self.logs_dir = name, logs_dir
        self.future_seq_len, self.dt_col, self.target_col = int(future_seq_len), dt_col, target_col
        self.extra_features_col, self.drop_missing = extra_features_col, drop_missing
        self.pipeline = None
        self.trials = []

    def _ft(self):
        return TimeSequenceFeatureTransformer(self.future_seq_len, self.dt_col, self.target_col,
                                              self.extra_features_col, self.drop_missing)

    def _identity_config(self):
        return {"future_seq_len": self.future_seq_len, "dt_col": self.dt_col, "target_col": self.target_col,
                "extra_features_col": self.extra_features_col, "drop_missing": self.drop_missing}

    def fit(self, input_df, validation_df=None, metric="mse", recipe=None, mc=False, resources_per_trial=None,
            distributed=False, hdfs_url=None, n_parallel=1):
        """Search with ``recipe`` (the reference's _hp_search: RayTuneSearchEngine.compile / run,
        stop criteria = recipe.runtime_params() minus num_samples), then load the best trial's
        checkpoint (feature transformer + model + config) as the pipeline."""
        from zoo.automl.pipeline.time_sequence import load_ts_pipeline
        from zoo.automl.search.RayTuneSearchEngine import RayTuneSearchEngine
        Evaluator.check_metric(metric)
        self._check_input(input_df, validation_df)
        recipe = recipe or SmokeRecipe()
        feats = self._ft().get_feature_list(input_df[0] if isinstance(input_df, list) else input_df)
        runtime_params = dict(recipe.runtime_params())
        num_samples = runtime_params.pop("num_samples")
        searcher = RayTuneSearchEngine(logs_dir=self.logs_dir, resources_per_trial=resources_per_trial,
                                       name=self.name, n_parallel=n_parallel)
        fixed = recipe.fixed_params()
        if recipe.search_algorithm() == "BayesOpt":     # box space; constants ride in fixed_params
            space = recipe.search_space(feats)
            fixed = dict(fixed or {})
        else:
            space = dict(recipe.search_space(feats), **self._identity_config())
        searcher.compile(input_df, search_space=space, num_samples=num_samples, stop=runtime_params,
                         search_algorithm=recipe.search_algorithm(),
                         search_algorithm_params=recipe.search_algorithm_params(),
                         fixed_params=None if fixed is None else dict(fixed, **self._identity_config()),
                         feature_transformers=self._ft(), future_seq_len=self.future_seq_len,
                         validation_df=validation_df, mc=mc, metric=metric)
        searcher.run()
        best = searcher.get_best_trials(k=1)[0]
        self.trials = searcher.trials
        self.pipeline = load_ts_pipeline(best.model_path)
        self.pipeline.name = self.name
        return self.pipeline

    def _check_input(self, input_df, validation_df):
        import pandas as pd

        def cols(df):
            need = [self.dt_col, self.target_col] + list(self.extra_features_col or [])
            missing = set(need) - set(df.columns)
            if missing:
                raise ValueError("Missing Columns in the input data frame:" + ",".join(sorted(missing)))
        for d in (input_df if isinstance(input_df, list) else [input_df]):
            if not isinstance(d, pd.DataFrame):
                raise ValueError("input_df should be a data frame or a list of data frames")
            cols(d)
        if validation_df is not None:
            for d in (validation_df if isinstance(validation_df, list) else [validation_df]):
                cols(d)

    def evaluate(self, input_df, metric=("mse",)):
        return self.pipeline.evaluate(input_df, list(metric))

    def predict(self, input_df):
        return self.pipeline.predict(input_df)
