"""Time-series regression metrics (Py/automl/common/metrics.py)."""
import numpy as np

EPS = 1e-8


def _prep(y_true, y_pred):
    yt = np.asarray(y_true, np.float64)
    yp = np.asarray(y_pred, np.float64)
    if yt.shape != yp.shape:
        raise ValueError("y_true %s and y_pred %s shapes differ" % (yt.shape, yp.shape))
    if yt.ndim == 1:
        yt, yp = yt[:, None], yp[:, None]
    return yt.reshape(len(yt), -1), yp.reshape(len(yp), -1)


def _out(v, multioutput):
    return v if multioutput == "raw_values" else float(np.mean(v))


def sMAPE(y_true, y_pred, multioutput="raw_values"):  # noqa: N802
    t, p = _prep(y_true, y_pred)
    return _out(100 * np.mean(np.abs(t - p) / (np.abs(t) + np.abs(p) + EPS), 0), multioutput)


def MPE(y_true, y_pred, multioutput="raw_values"):  # noqa: N802
    t, p = _prep(y_true, y_pred)
    return _out(100 * np.mean((t - p) / (t + EPS), 0), multioutput)


def MAPE(y_true, y_pred, multioutput="raw_values"):  # noqa: N802
    t, p = _prep(y_true, y_pred)
    return _out(100 * np.mean(np.abs((t - p) / (t + EPS)), 0), multioutput)


def MDAPE(y_true, y_pred, multioutput="raw_values"):  # noqa: N802
    t, p = _prep(y_true, y_pred)
    return _out(100 * np.median(np.abs((t - p) / (t + EPS)), 0), multioutput)


def sMDAPE(y_true, y_pred, multioutput="raw_values"):  # noqa: N802
    t, p = _prep(y_true, y_pred)
    return _out(100 * np.median(np.abs(t - p) / (np.abs(t) + np.abs(p) + EPS), 0), multioutput)


def ME(y_true, y_pred, multioutput="raw_values"):  # noqa: N802
    t, p = _prep(y_true, y_pred)
    return _out(np.mean(t - p, 0), multioutput)


def MSPE(y_true, y_pred, multioutput="raw_values"):  # noqa: N802
    t, p = _prep(y_true, y_pred)
    return _out(100 * np.mean(((t - p) / (t + EPS)) ** 2, 0), multioutput)


def MSE(y_true, y_pred, multioutput="raw_values"):  # noqa: N802
    t, p = _prep(y_true, y_pred)
    return _out(np.mean((t - p) ** 2, 0), multioutput)


def RMSE(y_true, y_pred, multioutput="raw_values"):  # noqa: N802
    return _out(np.sqrt(MSE(y_true, y_pred)), multioutput)


def MAE(y_true, y_pred, multioutput="raw_values"):  # noqa: N802
    t, p = _prep(y_true, y_pred)
    return _out(np.mean(np.abs(t - p), 0), multioutput)


def R2(y_true, y_pred, multioutput="raw_values"):  # noqa: N802
    t, p = _prep(y_true, y_pred)
    ss_res = ((t - p) ** 2).sum(0)
    ss_tot = ((t - t.mean(0)) ** 2).sum(0)
    return _out(1 - ss_res / np.maximum(ss_tot, EPS), multioutput)


METRICS = {"me": ME, "mae": MAE, "mse": MSE, "rmse": RMSE, "r2": R2, "smape": sMAPE, "mpe": MPE, "mape": MAPE,
           "mdape": MDAPE, "smdape": sMDAPE, "mspe": MSPE}
MAXIMIZE = {"r2"}
# Keras metric names accepted where a forecaster / pipeline was configured with them
ALIASES = {"mean_squared_error": "mse", "mean_absolute_error": "mae", "root_mean_squared_error": "rmse",
           "mean_absolute_percentage_error": "mape", "r_square": "r2"}


def _name(metric):
    m = metric.lower()
    return ALIASES.get(m, m)


class Evaluator:
    @staticmethod
    def evaluate(metric, y_true, y_pred, multioutput="raw_values"):
        Evaluator.check_metric(metric)
        return METRICS[_name(metric)](y_true, y_pred, multioutput)

    @staticmethod
    def check_metric(metric):
        if _name(metric) not in METRICS:
            raise ValueError("metric %s not supported (%s)" % (metric, sorted(METRICS)))

    @staticmethod
    def higher_is_better(metric):
        return _name(metric) in MAXIMIZE
