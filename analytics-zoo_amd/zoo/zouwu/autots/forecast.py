"""AutoTSTrainer / TSPipeline (Py/zouwu/autots/forecast.py:22-168)."""
from zoo.automl.pipeline.time_sequence import load_ts_pipeline
from zoo.automl.regression.time_sequence_predictor import TimeSequencePredictor


class TSPipeline:
    def __init__(self, internal):
        self.internal = internal

    def fit(self, input_df, validation_df=None, uncertainty=False, epochs=1, **kw):
        self.internal.fit(input_df, validation_df, uncertainty, epochs)
        return self

    def predict(self, input_df):
        return self.internal.predict(input_df)

    def predict_with_uncertainty(self, input_df, n_iter=100):
        return self.internal.predict_with_uncertainty(input_df, n_iter)

    def evaluate(self, input_df, metrics=("mse",), multioutput="raw_values"):
        return self.internal.evaluate(input_df, list(metrics), multioutput)

    def save(self, pipeline_file):
        return self.internal.save(pipeline_file)

    @staticmethod
    def load(pipeline_file):
        return TSPipeline(load_ts_pipeline(pipeline_file))


class AutoTSTrainer:
    def __init__(self, dt_col="datetime", target_col="value", horizon=1, extra_features_col=None):
        self.internal = TimeSequencePredictor(dt_col=dt_col, target_col=target_col, future_seq_len=horizon,
                                              extra_features_col=extra_features_col)

    def fit(self, train_df, validation_df=None, metric="mse", recipe=None, uncertainty=False, distributed=False,
            hdfs_url=None):
        return TSPipeline(self.internal.fit(train_df, validation_df, metric, recipe, mc=uncertainty))
