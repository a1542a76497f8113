"""TimeSequencePredictor (Py/automl/regression/time_sequence_predictor.py:32-296): search
feature selections / look-back windows / model hyper-parameters with a recipe; every trial
fits a TimeSequenceFeatureTransformer and a TimeSequenceModel (trained by this framework's
engine -- data-parallel over the initialised process group with ``distributed=True``) and
is scored on the validation frame; the best trial comes back as a TimeSequencePipeline."""
import logging

from zoo.automl.common.metrics import Evaluator
from zoo.automl.config.recipe import SmokeRecipe
from zoo.automl.feature.time_sequence import TimeSequenceFeatureTransformer
from zoo.automl.model.time_sequence import TimeSequenceModel
from zoo.automl.pipeline.time_sequence import TimeSequencePipeline
from zoo.automl.search import SearchEngine

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
        Evaluator.check_metric(metric)
        recipe = recipe or SmokeRecipe()
        feats = self._ft().get_feature_list(input_df)
        val_df = validation_df if validation_df is not None else input_df

        def trial(config):
            config = dict(config, **self._identity_config())
            ft = self._ft()
            x, y = ft.fit_transform(input_df, **config)
            vx, vy = ft.transform(val_df, is_train=True)
            model = TimeSequenceModel(check_optional_config=False, future_seq_len=self.future_seq_len)
            cfg = dict(config, epochs=int(config.get("epochs", 1)) * int(recipe.training_iteration))
            model.fit_eval(x, y, validation_data=(vx, vy), mc=mc, **cfg)
            ppl = TimeSequencePipeline(feature_transformers=ft, model=model, config=config, name=self.name)
            return {metric: float(ppl.evaluate(val_df, [metric], "uniform_average")[0]), "pipeline": ppl}

        engine = SearchEngine(n_parallel=n_parallel)
        mode = "max" if Evaluator.higher_is_better(metric) else "min"
        best_cfg, best = engine.run(trial, recipe.search_space(feats), recipe.num_samples, metric, mode,
                                    search_alg=recipe.search_algorithm(),
                                    search_alg_params=recipe.search_algorithm_params(),
                                    fixed_params=recipe.fixed_params())
        self.pipeline = best["pipeline"]
        self.trials = engine.trials
        return self.pipeline

    def evaluate(self, input_df, metric=("mse",)):
        return self.pipeline.evaluate(input_df, list(metric))

    def predict(self, input_df):
        return self.pipeline.predict(input_df)
