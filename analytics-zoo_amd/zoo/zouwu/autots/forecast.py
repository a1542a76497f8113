"""AutoTSTrainer / TSPipeline (Py/zouwu/autots/forecast.py:22-168): automated forecasting
on a datetime / target frame -- TimeSequencePredictor's recipe search underneath -- and the
resulting pipeline (incremental fit, predict, uncertainty, evaluate, save / load)."""
from zoo.automl.config.recipe import SmokeRecipe
from zoo.automl.pipeline.time_sequence import load_ts_pipeline
from zoo.automl.regression.time_sequence_predictor import TimeSequencePredictor


class AutoTSTrainer:
    def __init__(self, horizon=1, dt_col="datetime", target_col="value", extra_features_col=None):
        self.internal = TimeSequencePredictor(dt_col=dt_col, target_col=target_col, future_seq_len=horizon,
                                              extra_features_col=extra_features_col)

    def fit(self, train_df, validation_df=None, metric="mse", recipe=None, uncertainty=False, distributed=False,
            hdfs_url=None):
        ppl = TSPipeline()
        ppl.internal = self.internal.fit(train_df, validation_df, metric, recipe or SmokeRecipe(), mc=uncertainty,
                                         distributed=distributed, hdfs_url=hdfs_url)
        ppl.uncertainty = uncertainty
        return ppl


class TSPipeline:
    def __init__(self, internal=None):
        self.internal = internal
        self.uncertainty = False

    def save(self, pipeline_file):
        return self.internal.save(pipeline_file)

    @staticmethod
    def load(pipeline_file):
        return TSPipeline(load_ts_pipeline(pipeline_file))

    def fit(self, input_df, validation_df=None, uncertainty=False, epochs=1, **user_config):
        """Incremental fit; with ``user_config`` the pipeline is retrained from scratch with
        those fixed configs."""
        self.uncertainty = uncertainty
        if user_config:
            self.internal.fit_with_fixed_configs(input_df=input_df, validation_df=validation_df, mc=uncertainty,
                                                 epochs=epochs, **user_config)
        else:
            self.internal.fit(input_df=input_df, validation_df=validation_df, mc=uncertainty, epoch_num=epochs)
        return self

    def predict(self, input_df):
        if self.uncertainty:
            return self.internal.predict_with_uncertainty(input_df)
        return self.internal.predict(input_df)

    def predict_with_uncertainty(self, input_df, n_iter=100):
        return self.internal.predict_with_uncertainty(input_df, n_iter)

    def evaluate(self, input_df, metrics=("mse",), multioutput="raw_values"):
        return self.internal.evaluate(input_df, list(metrics), multioutput)
