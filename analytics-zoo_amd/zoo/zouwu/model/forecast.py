"""Zouwu forecasters (Py/zouwu/model/forecast.py:26-166): LSTMForecaster and
MTNetForecaster over (x [N, past, F], y [N, horizon]) numpy windows."""
import numpy as np
import torch

from zoo.automl.model import MTNetNet as MTNet, VanillaLSTMNet as VanillaLSTM


class Forecaster:
    def __init__(self, module, lr=1e-3, loss="mse", optimizer="adam"):
        from zoo.pipeline.api.keras.optimizers import Adam, to_optim_method
        from zoo.pipeline.api.net import TorchNet
        self.module = module
        self.net = TorchNet.from_pytorch(module)
        self.net.compile(optimizer=Adam(lr=lr) if optimizer == "adam" else to_optim_method(optimizer), loss=loss)

    def fit(self, x, y, batch_size=32, epochs=1, validation_data=None, distributed=False):
        self.net.fit(np.asarray(x, np.float32), np.asarray(y, np.float32), batch_size=batch_size, nb_epoch=epochs,
                     validation_data=validation_data)
        return self

    def evaluate(self, x, y, metrics=("mse",)):
        from zoo.automl.common.metrics import Evaluator
        p = self.predict(x)
        return [Evaluator.evaluate(m, np.asarray(y).reshape(p.shape), p, "uniform_average") for m in metrics]

    def predict(self, x, batch_size=256):
        return self.net.predict(np.asarray(x, np.float32), batch_size=batch_size)


class LSTMForecaster(Forecaster):
    def __init__(self, target_dim=1, feature_dim=1, lstm_1_units=16, dropout_1=0.2, lstm_2_units=8, dropout_2=0.2,
                 metric="mean_squared_error", lr=0.001, loss="mse", optimizer="adam"):
        super().__init__(VanillaLSTM(feature_dim, target_dim, lstm_1_units, dropout_1, lstm_2_units, dropout_2),
                         lr, loss, optimizer)


class MTNetForecaster(Forecaster):
    def __init__(self, target_dim=1, feature_dim=1, long_series_num=1, series_length=1, ar_window_size=1,
                 cnn_height=1, cnn_hid_size=32, rnn_hid_sizes=(16, 32), lr=0.001, loss="mae", cnn_dropout=0.2,
                 rnn_dropout=0.2, metric="mean_squared_error", uncertainty=False):
        super().__init__(MTNet(feature_dim, target_dim, series_length, long_series_num, cnn_height, cnn_hid_size,
                               list(rnn_hid_sizes), ar_window_size, cnn_dropout), lr, loss)
        self.long_series_num, self.series_length = long_series_num, series_length

    def preprocess_input(self, x):
        """Windows must hold (long_series_num + 1) * series_length steps (MTNet layout)."""
        need = (self.long_series_num + 1) * self.series_length
        x = np.asarray(x, np.float32)
        if x.shape[1] != need:
            raise ValueError("MTNet expects past length %d, got %d" % (need, x.shape[1]))
        return x
