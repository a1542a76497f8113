"""TimeSequenceFeatureTransformer (Py/automl/feature/time_sequence.py:30-573).

Feature engineering for one target series sampled on a uniform datetime grid:

  * datetime features named like the reference's generated ones -- ``MONTH(dt)``,
    ``WEEKDAY(dt)`` (Monday = 0), ``DAY(dt)``, ``HOUR(dt)``, ``IS_WEEKEND(dt)``, ``IS_AWAKE(dt)``
    (06:00-23:59 and midnight), ``IS_BUSY_HOURS(dt)`` (07-09, 16-19) -- computed directly with
    pandas (the reference derives them with featuretools, which is not part of this stack),
    plus the user's extra feature columns;
  * the ``selected_features`` of a trial config (the target is always column 0) and
    ``past_seq_len``;
  * standard scaling fitted on the training frame(s) (population std, as sklearn's
    StandardScaler);
  * rolling into (x [N, past, 1 + features], y [N, future]) windows -- a window holding any NaN
    is dropped -- and back: ``post_processing`` unscales predictions and, for test frames,
    attaches the prediction datetimes;
  * input checks: datetime64 dtype, no NaT, uniform sampling, nothing in the future, enough rows;
  * ``save`` / ``restore`` through the shared config file (zoo.automl.common.util).

Every entry point accepts one frame or a list of frames (one series each).
"""
import numpy as np
import pandas as pd

from zoo.automl.common.util import save_config
from zoo.automl.feature.abstract import BaseFeatureTransformer

_DT_PRIMS = ["MONTH", "WEEKDAY", "DAY", "HOUR", "IS_WEEKEND", "IS_AWAKE", "IS_BUSY_HOURS"]


class _Scaler:
    """StandardScaler state (mean_, scale_) with the sklearn semantics the reference uses."""

    def __init__(self, mean=None, scale=None):
        self.mean_ = None if mean is None else np.asarray(mean, dtype=np.float64)
        self.scale_ = None if scale is None else np.asarray(scale, dtype=np.float64)

    def fit(self, data):
        a = np.asarray(data, dtype=np.float64)
        self.mean_ = np.nanmean(a, axis=0)
        std = np.nanstd(a, axis=0)
        self.scale_ = np.where(std > 0, std, 1.0)
        return self

    def transform(self, data):
        return (np.asarray(data, dtype=np.float64) - self.mean_) / self.scale_


def _extra_list(extra):
    if extra is None:
        return []
    return [extra] if isinstance(extra, str) else list(extra)


class TimeSequenceFeatureTransformer(BaseFeatureTransformer):
    def __init__(self, future_seq_len=1, dt_col="datetime", target_col="value", extra_features_col=None,
                 drop_missing=True):
        self.scaler = _Scaler()
        self.config = None
        self.dt_col = dt_col
        self.target_col = target_col
        self.extra_features_col = extra_features_col
        self.drop_missing = drop_missing
        self.past_seq_len = None
        self.future_seq_len = int(future_seq_len)

    # ------------------------------------------------------------------ features
    def _dt_names(self):
        return ["%s(%s)" % (p, self.dt_col) for p in _DT_PRIMS]

    def _generate_features(self, input_df):
        """All candidate feature columns (datetime features + every non-datetime column)."""
        df = input_df.reset_index(drop=True)
        dt = pd.to_datetime(df[self.dt_col])
        hour, wd = dt.dt.hour, dt.dt.weekday
        out = pd.DataFrame(index=df.index)
        vals = {"MONTH": dt.dt.month, "WEEKDAY": wd, "DAY": dt.dt.day, "HOUR": hour,
                "IS_WEEKEND": (wd >= 5).astype(int),
                "IS_AWAKE": (((hour >= 6) & (hour <= 23)) | (hour == 0)).astype(int),
                "IS_BUSY_HOURS": (((hour >= 7) & (hour <= 9)) | ((hour >= 16) & (hour <= 19))).astype(int)}
        for p in _DT_PRIMS:
            out["%s(%s)" % (p, self.dt_col)] = vals[p].values
        for c in df.columns:
            if c != self.dt_col:
                out[c] = df[c].values
        return out

    def get_feature_list(self, input_df=None):
        """Names a trial may select: the datetime features plus the extra feature columns."""
        return self._dt_names() + [c for c in _extra_list(self.extra_features_col)]

    def _get_features(self, input_df, config):
        fm = self._generate_features(input_df)
        cols = [self.target_col] + list(config.get("selected_features", []))
        missing = [c for c in cols if c not in fm.columns]
        if missing:
            raise ValueError("unknown feature(s) %s; available: %s" % (missing, list(fm.columns)))
        return fm[cols].astype(float)

    def _get_feat_config(self, **config):
        self._check_config(**config)
        feat = {k: config[k] for k in ("selected_features", "past_seq_len") if k in config}
        self.past_seq_len = int(feat.get("past_seq_len", 1))
        return feat

    # ------------------------------------------------------------------ checks
    def _check_input(self, input_df, mode="train"):
        df = input_df.reset_index(drop=True)
        if self.dt_col not in df.columns or self.target_col not in df.columns:
            raise ValueError("input frame needs the datetime column %r and the target column %r"
                             % (self.dt_col, self.target_col))
        dt = df[self.dt_col]
        if not np.issubdtype(dt.dtype, np.datetime64):
            raise ValueError("The dtype of datetime column is required to be np.datetime64!")
        if pd.isna(dt).any():
            raise ValueError("Missing datetime in input dataframe!")
        if len(dt) > 1:
            d = np.diff(dt.values.astype("datetime64[ns]").astype(np.int64))
            if not np.all(d == d[0]):
                raise ValueError("Input time sequence intervals are not uniform!")
        if not self.drop_missing and pd.isna(df).any(axis=None):
            raise ValueError("Missing values in input dataframe!")
        if len(dt) and dt.iloc[-1] > pd.Timestamp.now():
            raise ValueError("Last date time is bigger than current time!")
        if mode == "test":
            need = self.past_seq_len
            msg = ("Length of {m} data should be larger than the past sequence length selected by automl.\n"
                   "{m} data length: {n}\npast sequence length selected: {p}\n"
                   .format(m=mode, n=len(df), p=self.past_seq_len))
        else:
            need = self.past_seq_len + self.future_seq_len
            msg = ("Length of {m} data should be larger than the sequence length you want to predict plus "
                   "the past sequence length selected by automl.\n{m} data length: {n}\n"
                   "predict sequence length: {f}\npast sequence length selected: {p}\n"
                   .format(m=mode, n=len(df), f=self.future_seq_len, p=self.past_seq_len))
        if len(df) < need:
            raise ValueError(msg)
        return df

    # ------------------------------------------------------------------ rolling
    @staticmethod
    def _roll_data(data, seq_len):
        a = np.asarray(data, dtype=np.float64)
        n = len(a) - seq_len + 1
        if n <= 0:
            return np.empty((0, seq_len) + a.shape[1:]), np.zeros(0, bool)
        idx = np.arange(seq_len)[None, :] + np.arange(n)[:, None]
        win = a[idx]
        mask = ~np.isnan(win.reshape(n, -1)).any(1)
        return win, mask

    def _roll_train(self, dataframe, past_seq_len, future_seq_len):
        """x: windows of past_seq_len rows of all columns; y: the next future_seq_len target
        values ([N, future]); windows with a NaN in x or y are dropped."""
        df = pd.DataFrame(dataframe)
        x_src = df.values[:len(df) - future_seq_len] if future_seq_len > 0 else df.values
        y_src = df.iloc[past_seq_len:, 0].values
        x, mx = self._roll_data(x_src, past_seq_len)
        y, my = self._roll_data(y_src, future_seq_len)
        n = min(len(x), len(y))
        mask = mx[:n] & my[:n]
        return x[:n][mask], y[:n][mask]

    def _roll_test(self, dataframe, past_seq_len):
        vals = dataframe.values if hasattr(dataframe, "values") else np.asarray(dataframe)
        x, mask = self._roll_data(vals, past_seq_len)
        return x[mask]

    # ------------------------------------------------------------------ API
    def _scale(self, feature_data):
        return pd.DataFrame(self.scaler.transform(feature_data))

    def _fit_transform(self, input_df):
        df = self._check_input(input_df, mode="train")
        feats = self._get_features(df, self.config)
        self.scaler.fit(feats.values)
        return self._roll_train(self._scale(feats.values), self.past_seq_len, self.future_seq_len)

    def fit_transform(self, input_df, **config):
        """Fit the scaler (on the last frame of a list, as the reference does frame by frame)
        and roll every frame into (x, y)."""
        self.config = self._get_feat_config(**config)
        if isinstance(input_df, list):
            xs, ys = zip(*[self._fit_transform(df) for df in input_df])
            return np.concatenate(xs, 0), np.concatenate(ys, 0)
        return self._fit_transform(input_df)

    def _transform(self, input_df, mode):
        df = self._check_input(input_df, mode)
        data = self._scale(self._get_features(df, self.config).values)
        if mode == "val":
            return self._roll_train(data, self.past_seq_len, self.future_seq_len)
        return self._roll_test(data, self.past_seq_len), None

    def transform(self, input_df, is_train=True):
        if self.config is None or self.past_seq_len is None:
            raise Exception("Needs to call fit_transform or restore first before calling transform")
        mode = "val" if is_train else "test"
        if isinstance(input_df, list):
            outs = [self._transform(df, mode) for df in input_df]
            x = np.concatenate([o[0] for o in outs], 0)
            y = np.concatenate([o[1] for o in outs], 0) if mode == "val" else None
            return x, y
        return self._transform(input_df, mode)

    def _unscale(self, y):
        return np.asarray(y) * self.scaler.scale_[0] + self.scaler.mean_[0]

    def unscale_uncertainty(self, y_uncertainty):
        return np.asarray(y_uncertainty) * self.scaler.scale_[0]

    def _pred_dt_df(self, input_df):
        """Prediction datetimes: every row from past_seq_len on, plus one step past the end."""
        dts = pd.to_datetime(input_df.reset_index(drop=True)[self.dt_col])
        step = dts.iloc[-1] - dts.iloc[-2]
        out = list(dts.iloc[self.past_seq_len:]) + [dts.iloc[-1] + step]
        return pd.DataFrame({self.dt_col: pd.to_datetime(out)})

    def _pred_df(self, dt_df, y):
        df = dt_df.copy()
        y = np.asarray(y)
        if self.future_seq_len > 1:
            for i in range(self.future_seq_len):
                df["%s_%d" % (self.target_col, i)] = y[:, i]
        else:
            df[self.target_col] = y.reshape(len(y), -1)[:, 0]
        return df

    def post_processing(self, input_df, y_pred, is_train):
        """is_train: (y_true_unscaled, y_pred_unscaled) over the rolled windows of input_df;
        otherwise a frame (or list of frames) {dt_col, target(_i)} of unscaled predictions."""
        y_pred = self._unscale(y_pred)
        frames = input_df if isinstance(input_df, list) else [input_df]
        if is_train:
            ys = [self._roll_train(df[[self.target_col]], self.past_seq_len, self.future_seq_len)[1]
                  for df in frames]
            return np.concatenate(ys, 0), y_pred
        outs, at = [], 0
        for df in frames:
            dt_df = self._pred_dt_df(df)
            n = min(len(dt_df), len(y_pred) - at)
            outs.append(self._pred_df(dt_df.iloc[:n].reset_index(drop=True), y_pred[at:at + n]))
            at += n
        return outs if isinstance(input_df, list) else outs[0]

    # ------------------------------------------------------------------ persistence
    def save(self, file_path, replace=False):
        save_config(file_path, {"mean": self.scaler.mean_.tolist(), "scale": self.scaler.scale_.tolist(),
                                "future_seq_len": self.future_seq_len, "dt_col": self.dt_col,
                                "target_col": self.target_col, "extra_features_col": self.extra_features_col,
                                "drop_missing": self.drop_missing}, replace=replace)

    def restore(self, **config):
        self.scaler = _Scaler(config["mean"], config["scale"])
        self.future_seq_len = int(config["future_seq_len"])
        self.dt_col = config["dt_col"]
        self.target_col = config["target_col"]
        self.extra_features_col = config.get("extra_features_col")
        self.drop_missing = config.get("drop_missing", True)
        self.config = self._get_feat_config(**config)
        return self

    def _get_optional_parameters(self):
        return {"past_seq_len"}

    def _get_required_parameters(self):
        return {"selected_features"}
