"""TimeSequenceFeatureTransformer (Py/automl/feature/time_sequence.py:30-575).

Datetime features (MONTH, WEEKDAY, DAY, HOUR, IS_WEEKEND, IS_AWAKE,
IS_BUSY_HOURS — computed directly instead of through featuretools), feature
selection, standard scaling, rolling (past_seq_len -> future_seq_len)
windows, and post-processing back to a (datetime, value) frame."""
import json

import numpy as np
import pandas as pd

from zoo.automl.feature.abstract import BaseFeatureTransformer

DT_FEATURES = ["MONTH", "WEEKDAY", "DAY", "HOUR", "IS_WEEKEND", "IS_AWAKE", "IS_BUSY_HOURS"]


class TimeSequenceFeatureTransformer(BaseFeatureTransformer):
    def __init__(self, future_seq_len=1, dt_col="datetime", target_col="value", extra_features_col=None,
                 drop_missing=True):
        self.future_seq_len = int(future_seq_len)
        self.dt_col, self.target_col = dt_col, target_col
        self.extra_features_col = list(extra_features_col or [])
        self.drop_missing = drop_missing
        self.past_seq_len = None
        self.selected = None
        self.mean = self.std = None

    def get_feature_list(self, input_df=None):
        return DT_FEATURES + self.extra_features_col

    def _features(self, df):
        dt = pd.to_datetime(df[self.dt_col])
        hour = dt.dt.hour
        f = pd.DataFrame({"MONTH": dt.dt.month, "WEEKDAY": dt.dt.weekday, "DAY": dt.dt.day, "HOUR": hour,
                          "IS_WEEKEND": (dt.dt.weekday >= 5).astype(int),
                          "IS_AWAKE": (((hour >= 6) & (hour <= 23)) | (hour == 0)).astype(int),
                          "IS_BUSY_HOURS": (((hour >= 7) & (hour <= 9)) | ((hour >= 16) & (hour <= 19))).astype(int)},
                         index=df.index)
        for c in self.extra_features_col:
            f[c] = df[c]
        cols = [self.target_col] + list(self.selected)
        f[self.target_col] = df[self.target_col]
        return f[cols].astype(float).values

    def _check(self, df):
        if self.dt_col not in df or self.target_col not in df:
            raise ValueError("input_df needs columns %s and %s" % (self.dt_col, self.target_col))
        if self.drop_missing:
            df = df.dropna(subset=[self.target_col])
        return df

    def _roll(self, data, train=True):
        P, F = self.past_seq_len, self.future_seq_len
        n = len(data) - P - (F if train else 0) + 1
        if n <= 0:
            raise ValueError("time series shorter than past_seq_len + future_seq_len")
        idx = np.arange(P)[None, :] + np.arange(n)[:, None]
        x = data[idx]
        if not train:
            return x, None
        yidx = np.arange(F)[None, :] + np.arange(n)[:, None] + P
        return x, data[yidx, 0]

    def fit_transform(self, input_df, **config):
        df = self._check(input_df)
        self.past_seq_len = int(config.get("past_seq_len", 2))
        self.selected = list(config.get("selected_features", self.get_feature_list()))
        data = self._features(df)
        self.mean, self.std = data.mean(0), np.where(data.std(0) > 0, data.std(0), 1.0)
        return self._roll((data - self.mean) / self.std, True)

    def transform(self, input_df, is_train=True):
        df = self._check(input_df)
        data = (self._features(df) - self.mean) / self.std
        return self._roll(data, is_train)

    def _unscale(self, y):
        return y * self.std[0] + self.mean[0]

    def unscale_uncertainty(self, y_uncertainty):
        return y_uncertainty * self.std[0]

    def post_processing(self, input_df, y_pred, is_train):
        y = self._unscale(np.asarray(y_pred))
        if is_train:
            return y
        dts = pd.to_datetime(input_df[self.dt_col]).values[self.past_seq_len - 1:]
        out = pd.DataFrame({self.dt_col: dts[:len(y)]})
        if y.ndim == 1 or y.shape[1] == 1:
            out[self.target_col] = y.reshape(-1)
        else:
            for i in range(y.shape[1]):
                out["%s_%d" % (self.target_col, i)] = y[:, i]
        return out

    def state(self):
        return {"future_seq_len": self.future_seq_len, "dt_col": self.dt_col, "target_col": self.target_col,
                "extra_features_col": self.extra_features_col, "drop_missing": self.drop_missing,
                "past_seq_len": self.past_seq_len, "selected": self.selected,
                "mean": None if self.mean is None else self.mean.tolist(),
                "std": None if self.std is None else self.std.tolist()}

    @staticmethod
    def from_state(s):
        t = TimeSequenceFeatureTransformer(s["future_seq_len"], s["dt_col"], s["target_col"],
                                           s["extra_features_col"], s["drop_missing"])
        t.past_seq_len, t.selected = s["past_seq_len"], s["selected"]
        t.mean = None if s["mean"] is None else np.asarray(s["mean"])
        t.std = None if s["std"] is None else np.asarray(s["std"])
        return t

    def save(self, file_path, replace=False):
        with open(file_path, "w") as f:
            json.dump(self.state(), f)

    def restore(self, **config):
        """Restore from a saved state dict (``save`` file contents) merged into the config."""
        s = config.get("ft_state", config)
        if "file_path" in config:
            with open(config["file_path"]) as f:
                s = json.load(f)
        t = TimeSequenceFeatureTransformer.from_state(dict(self.state(), **{k: v for k, v in s.items()
                                                                             if k in self.state()}))
        self.__dict__.update(t.__dict__)
        return self

    def _get_required_parameters(self):
        return {"past_seq_len"}

    def _get_optional_parameters(self):
        return {"selected_features"}
