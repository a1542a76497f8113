"""Zouwu forecasters (Py/zouwu/model/forecast.py:26-166): LSTMForecaster and MTNetForecaster
over rolled (x [N, past, F], y [N, horizon]) windows.

Each forecaster wraps the AutoML network of the same name (zoo.automl.model._nets) as a
framework KerasNet (TorchNet) trained by this framework's engine: ``fit(...,
distributed=True)`` trains data-parallel over the initialised process group (RCCL on the GPU,
gloo on the CPU -- every rank passes the full arrays, the FeatureSet shards them), and
``uncertainty=True`` enables Monte-Carlo dropout for ``predict_with_uncertainty``.
"""
import logging

import numpy as np
import torch

from zoo.automl.model._nets import VanillaLSTMNet
from zoo.automl.model.MTNet_keras import MTNetNet

log = logging.getLogger("zoo.zouwu")

_LOSS = {"mean_squared_error": "mse", "mse": "mse", "mean_absolute_error": "mae", "mae": "mae"}


class Forecaster:
    """Base: ``_build()`` returns the torch network; the KerasNet wrapper is compiled with
    Adam(lr) and the metric's loss."""

    def __init__(self):
        from zoo.pipeline.api.keras.optimizers import Adam
        from zoo.pipeline.api.net import TorchNet
        self.module = self._build()
        self.net = TorchNet.from_pytorch(self.module)
        self.net.compile(optimizer=Adam(lr=float(self.lr)), loss=_LOSS.get(self.metric, "mse"))

    def _build(self):
        raise NotImplementedError

    def _prep(self, x):
        return np.asarray(x, np.float32)

    def fit(self, x, y=None, batch_size=32, epochs=1, validation_data=None, distributed=False):
        import torch.distributed as dist
        world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        if distributed and world == 1:
            log.info("fit(distributed=True) without an initialised process group: training on this process")
        x = self._prep(x)
        y = np.asarray(y, np.float32).reshape(len(x), -1)
        val = None
        if validation_data is not None:
            val = (self._prep(validation_data[0]), np.asarray(validation_data[1], np.float32).reshape(-1, y.shape[1]))
        self.net.fit(x, y, batch_size=batch_size, nb_epoch=epochs, validation_data=val, distributed=distributed)
        return self

    def predict(self, x, batch_size=256, distributed=False):
        x = self._prep(x)
        m = self.module
        was = m.training
        m.eval()
        dev = next(m.parameters()).device
        out = []
        with torch.no_grad():
            for i in range(0, len(x), batch_size):
                out.append(m(torch.from_numpy(x[i:i + batch_size]).to(dev)).float().cpu().numpy())
        m.train(was)
        return np.concatenate(out, 0)

    def predict_with_uncertainty(self, x, n_iter=100, batch_size=256):
        """(mean, std) over ``n_iter`` Monte-Carlo dropout passes (needs ``uncertainty=True``)."""
        if not self.uncertainty:
            raise ValueError("construct the forecaster with uncertainty=True for predict_with_uncertainty")
        x = self._prep(x)
        m = self.module
        was = m.training
        m.train(True)                                  # dropout active
        dev = next(m.parameters()).device
        runs = []
        with torch.no_grad():
            for _ in range(int(n_iter)):
                runs.append(np.concatenate([m(torch.from_numpy(x[i:i + batch_size]).to(dev)).float().cpu().numpy()
                                            for i in range(0, len(x), batch_size)], 0))
        m.train(was)
        runs = np.stack(runs)
        return runs.mean(0), runs.std(0)

    def evaluate(self, x, y, metrics=None, distributed=False):
        from zoo.automl.common.metrics import Evaluator
        p = self.predict(x)
        y = np.asarray(y, np.float32).reshape(p.shape)
        metrics = metrics or [self.metric]
        return [Evaluator.evaluate(m, y, p, "uniform_average") for m in metrics]


class LSTMForecaster(Forecaster):
    """Vanilla LSTM forecaster: LSTM(lstm_1_units) -> Dropout -> LSTM(lstm_2_units) -> Dropout
    -> Dense(horizon)."""

    def __init__(self, horizon=1, feature_dim=1, lstm_1_units=16, dropout_1=0.2, lstm_2_units=8, dropout_2=0.2,
                 metric="mean_squared_error", lr=0.001, uncertainty=False):
        self.horizon, self.feature_dim = int(horizon), int(feature_dim)
        self.metric, self.lr, self.uncertainty = metric, lr, bool(uncertainty)
        self.model_config = {"lstm_1_units": lstm_1_units, "dropout_1": dropout_1, "lstm_2_units": lstm_2_units,
                             "dropout_2": dropout_2}
        super().__init__()

    def _build(self):
        return VanillaLSTMNet(self.feature_dim, self.horizon, **self.model_config)


class MTNetForecaster(Forecaster):
    """MTNet forecaster: ``lb_long_steps`` long-term memory blocks of ``lb_long_stepsize`` steps
    plus one short-term block (look-back (lb_long_steps + 1) * lb_long_stepsize)."""

    def __init__(self, horizon=1, feature_dim=1, lb_long_steps=1, lb_long_stepsize=1, metric="mean_squared_error",
                 uncertainty=False, ar_window=None, cnn_height=None, cnn_hid_size=32, rnn_hid_sizes=(16, 32),
                 dropout=0.2, lr=0.001):
        self.horizon, self.feature_dim = int(horizon), int(feature_dim)
        self.long_num, self.time_step = int(lb_long_steps), int(lb_long_stepsize)
        self.past_seq_len = (self.long_num + 1) * self.time_step
        self.metric, self.lr, self.uncertainty = metric, lr, bool(uncertainty)
        self.model_config = {"time_step": self.time_step, "long_num": self.long_num,
                             "ar_window": int(ar_window or max(1, self.time_step)),
                             "cnn_height": int(cnn_height or max(1, min(2, self.time_step))),
                             "cnn_hid_size": cnn_hid_size, "rnn_hid_sizes": list(rnn_hid_sizes), "dropout": dropout}
        super().__init__()

    def _build(self):
        return MTNetNet(self.feature_dim, self.horizon, **self.model_config)

    def preprocess_input(self, x):
        """Rolled windows [N, (long+1)*step, F] -> (long_term [N, long, step, F],
        short_term [N, step, F])."""
        x = np.asarray(x, np.float32)
        if x.shape[1] != self.past_seq_len:
            raise ValueError("MTNet expects a look-back of (lb_long_steps + 1) * lb_long_stepsize = %d steps, got %d"
                             % (self.past_seq_len, x.shape[1]))
        n, t = self.long_num, self.time_step
        return (x[:, :n * t].reshape(-1, n, t, x.shape[-1]), x[:, n * t:].reshape(-1, t, x.shape[-1]))

    def _prep(self, x):
        if isinstance(x, (list, tuple)) and len(x) == 2:
            long_x, short_x = (np.asarray(v, np.float32) for v in x)
            return np.concatenate([long_x.reshape(len(long_x), -1, long_x.shape[-1]), short_x], 1)
        return np.asarray(x, np.float32)
