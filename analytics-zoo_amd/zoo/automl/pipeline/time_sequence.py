"""TimeSequencePipeline (Py/automl/pipeline/time_sequence.py:28-221): a fitted feature
transformer + a TimeSequenceModel + the trial config. fit (incremental) /
fit_with_fixed_configs (from scratch) / evaluate / predict / predict_with_uncertainty (MC
dropout) / save (zip bundle, zoo.automl.common.util.save_zip) / load_ts_pipeline."""
import os
import time

import pandas as pd

from zoo.automl.common.metrics import Evaluator
from zoo.automl.common.util import restore_zip, save_config, save_zip
from zoo.automl.feature.time_sequence import TimeSequenceFeatureTransformer
from zoo.automl.model.time_sequence import TimeSequenceModel
from zoo.automl.pipeline.abstract import Pipeline

DEFAULT_PPL_DIR = os.path.expanduser("~/zoo_automl_pipelines")
DEFAULT_CONFIG_DIR = os.path.expanduser("~/zoo_automl_configs")
DEFAULT_CONFIGS = {"dt_col": "datetime", "target_col": "value", "extra_features_col": None, "drop_missing": True,
                   "future_seq_len": 1, "past_seq_len": 2, "batch_size": 64, "lr": 0.001, "dropout": 0.2,
                   "epochs": 10, "metric": "mean_squared_error"}


class TimeSequencePipeline(Pipeline):
    def __init__(self, feature_transformers=None, model=None, config=None, name=None):
        self.feature_transformers = feature_transformers
        self.model = model
        self.config = config
        self.name = name
        self.time = time.strftime("%Y%m%d-%H%M%S")

    @property
    def ft(self):
        return self.feature_transformers

    def describe(self):
        keys = ["future_seq_len", "dt_col", "target_col", "extra_features_col", "drop_missing"]
        info = {k: (self.config or {}).get(k) for k in keys}
        print("**** Initialization info ****")
        for k, v in info.items():
            print("%s: %s" % (k, v))
        return info

    def fit(self, input_df, validation_df=None, mc=False, epoch_num=20):
        """Incremental fit of the current model on new data (same features / window)."""
        x, y = self.feature_transformers.transform(input_df, is_train=True)
        val = self.feature_transformers.transform(validation_df) if self._is_val_df_valid(validation_df) else None
        self.model.fit_eval(x, y, val, mc=mc, verbose=1, epochs=epoch_num)
        return self

    @staticmethod
    def _is_val_df_valid(validation_df):
        if isinstance(validation_df, pd.DataFrame):
            return not validation_df.empty
        if isinstance(validation_df, list):
            return bool(validation_df) and not all(d.empty for d in validation_df)
        return False

    def get_default_configs(self):
        return dict(DEFAULT_CONFIGS)

    def fit_with_fixed_configs(self, input_df, validation_df=None, mc=False, **user_configs):
        """Train from scratch with fixed configs (identity configs such as future_seq_len /
        dt_col / target_col plus tunable ones such as past_seq_len / batch_size)."""
        if self.config is None:
            self.config = self.get_default_configs()
        self.config.update(user_configs)
        for k, v in DEFAULT_CONFIGS.items():
            self.config.setdefault(k, v)
        ft_keys = ("future_seq_len", "dt_col", "target_col", "extra_features_col", "drop_missing")
        self.feature_transformers = TimeSequenceFeatureTransformer(**{k: self.config[k] for k in ft_keys})
        self.model = TimeSequenceModel(check_optional_config=False, future_seq_len=self.config["future_seq_len"])
        self.config["selected_features"] = self.feature_transformers.get_feature_list(input_df)
        x, y = self.feature_transformers.fit_transform(input_df, **self.config)
        val = self.feature_transformers.transform(validation_df) if self._is_val_df_valid(validation_df) else None
        self.model.fit_eval(x, y, validation_data=val, mc=mc, verbose=1, **self.config)
        return self

    def evaluate(self, input_df, metrics=("mse",), multioutput="raw_values"):
        if isinstance(metrics, str):
            metrics = [metrics]
        x, _ = self.feature_transformers.transform(input_df, is_train=True)
        y_pred = self.model.predict(x)
        if y_pred.ndim == 1 or y_pred.shape[1] == 1:
            multioutput = "uniform_average"
        y_true, y_hat = self.feature_transformers.post_processing(input_df, y_pred, is_train=True)
        return [Evaluator.evaluate(m, y_true, y_hat, multioutput=multioutput) for m in metrics]

    def predict(self, input_df):
        x, _ = self.feature_transformers.transform(input_df, is_train=False)
        return self.feature_transformers.post_processing(input_df, self.model.predict(x), is_train=False)

    def predict_with_uncertainty(self, input_df, n_iter=100):
        x, _ = self.feature_transformers.transform(input_df, is_train=False)
        y_pred, y_unc = self.model.predict_with_uncertainty(x, n_iter=n_iter)
        out = self.feature_transformers.post_processing(input_df, y_pred, is_train=False)
        return out, self.feature_transformers.unscale_uncertainty(y_unc)

    def save(self, ppl_file=None):
        ppl_file = ppl_file or os.path.join(DEFAULT_PPL_DIR, "%s_%s.ppl" % (self.name, self.time))
        save_zip(ppl_file, self.feature_transformers, self.model, self.config)
        return ppl_file

    def config_save(self, config_file=None):
        config_file = config_file or os.path.join(DEFAULT_CONFIG_DIR, "%s_%s.json" % (self.name, self.time))
        save_config(config_file, self.config, replace=True)
        return config_file


def load_ts_pipeline(file):
    ft = TimeSequenceFeatureTransformer()
    model = TimeSequenceModel(check_optional_config=False)
    all_config = restore_zip(file, ft, model)
    return TimeSequencePipeline(feature_transformers=ft, model=model, config=all_config)
