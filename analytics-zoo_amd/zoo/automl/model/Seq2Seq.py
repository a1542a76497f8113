"""LSTMSeq2Seq (Py/automl/model/Seq2Seq.py:27-345): LSTM encoder-decoder forecaster.

Training is teacher-forced as in the reference: the encoder LSTM (``latent_dim`` units, input
dropout) reads the past window, its (h, c) state initialises the decoder LSTM, which reads the
lagged target series (``_get_decoder_inputs``: sample i's decoder input is sample i-1's target
window -- consecutive rolled samples are one step apart -- and sample 0 starts from the last
observed target) and a Dense maps every decoder step to ``target_col_num`` values; loss MSE,
RMSprop(lr). Inference (``_decode_sequence``) runs the decoder autoregressively for
``future_seq_len`` steps from the last observed target values.

Both inputs travel to the engine as one tensor (past window, then the decoder inputs zero-padded
to the feature width) so the network trains as a plain TorchNet on this framework's engine.
"""
import numpy as np
import torch
import torch.nn as nn

from zoo.automl.common.metrics import Evaluator
from zoo.automl.model.abstract import BaseModel


class LSTMSeq2SeqNet(nn.Module):
    """Encoder / decoder LSTMs + Dense. ``forward(packed)`` is the teacher-forced training
    graph; ``decode(x, steps)`` the autoregressive inference loop."""

    def __init__(self, feature_num, target_col_num=1, latent_dim=128, dropout=0.2, past_seq_len=None):
        super().__init__()
        self.Fd, self.T = int(feature_num), int(target_col_num)
        self.past = past_seq_len
        self.enc = nn.LSTM(self.Fd, int(latent_dim), batch_first=True)
        self.dec = nn.LSTM(self.T, int(latent_dim), batch_first=True)
        self.drop = nn.Dropout(float(dropout))
        self.dense = nn.Linear(int(latent_dim), self.T)
        from zoo.automl.model._nets import _to_native
        _to_native(self)

    def encode(self, x):
        _, (h, c) = self.enc(self.drop(x))
        return h, c

    def forward(self, packed):
        x, dec_in = packed[:, :self.past], packed[:, self.past:, :self.T]
        h, c = self.encode(x)
        o, _ = self.dec(self.drop(dec_in), (h, c))
        return self.dense(o)

    def decode(self, x, steps):
        h, c = self.encode(x)
        tgt = x[:, -1:, :self.T]
        outs = []
        for _ in range(int(steps)):
            o, (h, c) = self.dec(self.drop(tgt), (h, c))
            tgt = self.dense(o)
            outs.append(tgt)
        return torch.cat(outs, 1)


class LSTMSeq2Seq(BaseModel):
    def __init__(self, check_optional_config=True, future_seq_len=2):
        self.model = None
        self.net = None
        self.past_seq_len = None
        self.future_seq_len = future_seq_len
        self.feature_num = None
        self.target_col_num = None
        self.metric = None
        self.latent_dim = None
        self.batch_size = None
        self.dropout = None
        self.lr = None
        self.check_optional_config = check_optional_config
        self.config = {}

    # ------------------------------------------------------------------ graph
    def _build_train(self, mc=False, **config):
        from zoo.pipeline.api.keras.optimizers import RMSprop
        from zoo.pipeline.api.net import TorchNet
        super()._check_config(**config)
        self.metric = config.get("metric", "mean_squared_error")
        self.latent_dim = config.get("latent_dim", 128)
        self.dropout = config.get("dropout", 0.2)
        self.lr = config.get("lr", 0.001)
        self.batch_size = config.get("batch_size", 64)
        self.model = LSTMSeq2SeqNet(self.feature_num, self.target_col_num, self.latent_dim, self.dropout,
                                    self.past_seq_len)
        self.net = TorchNet.from_pytorch(self.model)
        self.net.compile(optimizer=RMSprop(learningrate=float(self.lr), decayrate=0.9, epsilon=1e-7), loss="mse")
        return self.model

    def _decode_sequence(self, input_seq, mc=False):
        m = self.model
        was = m.training
        m.train(bool(mc))
        dev = next(m.parameters()).device
        x = np.asarray(input_seq, np.float32)
        with torch.no_grad():
            out = np.concatenate([m.decode(torch.from_numpy(x[i:i + 1024]).to(dev), self.future_seq_len)
                                  .float().cpu().numpy() for i in range(0, len(x), 1024)], 0)
        m.train(was)
        return out

    # ------------------------------------------------------------------ data
    def _get_decoder_inputs(self, x, y):
        """Teacher-forcing decoder inputs: the target series shifted back by one sample (sample i
        reads sample i-1's targets); sample 0 has no predecessor and reads its own targets one
        step late, led by the last observed target of the final input window."""
        tc = self.target_col_num
        head = np.concatenate([x[-1:, -1:, :tc], y[:1, :-1]], axis=1)
        return np.concatenate([head, y[:-1]], axis=0).astype(np.float32)

    def _get_len(self, x, y):
        (_, self.past_seq_len, self.feature_num), self.target_col_num = x.shape, y.shape[2]

    @staticmethod
    def _expand_y(y):
        y = np.asarray(y, np.float32)
        return y.reshape(y.shape + (1,) * max(0, 3 - y.ndim))

    def _pack(self, x, dec):
        n, f = len(x), max(self.feature_num, self.target_col_num)
        out = np.zeros((n, self.past_seq_len + dec.shape[1], f), np.float32)
        out[:, :self.past_seq_len, :x.shape[2]] = x
        out[:, self.past_seq_len:, :dec.shape[2]] = dec
        return out

    def _pre_processing(self, x, y, validation_data):
        x = np.asarray(x, np.float32)
        y = self._expand_y(y)
        self._get_len(x, y)
        decoder_input_data = self._get_decoder_inputs(x, y)
        if validation_data is not None:
            val_x, val_y = validation_data
            val_x = np.asarray(val_x, np.float32)
            val_y = self._expand_y(val_y)
            validation_data = (val_x, val_y, self._get_decoder_inputs(val_x, val_y))
        return x, y, decoder_input_data, validation_data

    # ------------------------------------------------------------------ BaseModel
    def fit_eval(self, x, y, validation_data=None, mc=False, verbose=0, **config):
        x, y, dec, validation_data = self._pre_processing(x, y, validation_data)
        self.config.update(config)
        if self.model is None:
            self._build_train(mc=mc, **self.config)
        self.net.fit(self._pack(x, dec), y, batch_size=max(1, min(int(self.batch_size), len(x))),
                     nb_epoch=int(config.get("epochs", 10)))
        # the reference reports the (teacher-forced) Keras metric of the last epoch
        vx, vy, vdec = validation_data if validation_data is not None else (x, y, dec)
        m = self.model
        was = m.training
        m.eval()
        dev = next(m.parameters()).device
        with torch.no_grad():
            pred = m(torch.from_numpy(self._pack(vx, vdec)).to(dev)).float().cpu().numpy()
        m.train(was)
        return float(np.mean(Evaluator.evaluate(self.metric, vy.reshape(len(vy), -1), pred.reshape(len(vy), -1),
                                                multioutput="uniform_average")))

    def evaluate(self, x, y, metric=("mse",)):
        y_pred = self.predict(x)
        y = np.asarray(y, np.float32).reshape(y_pred.shape)
        return [Evaluator.evaluate(m, y, y_pred) for m in metric]

    def predict(self, x, mc=False):
        if self.model is None:
            raise RuntimeError("fit_eval or restore the model first")
        return np.squeeze(self._decode_sequence(x, mc=mc), axis=2)

    def predict_with_uncertainty(self, x, n_iter=100):
        result = np.stack([self.predict(x, mc=True) for _ in range(int(n_iter))])
        return result.mean(axis=0), result.std(axis=0)

    def save(self, model_path, config_path):
        from zoo.automl.common.util import save_config
        torch.save({k: v.detach().cpu() for k, v in self.model.state_dict().items()}, model_path)
        save_config(config_path, {"past_seq_len": self.past_seq_len, "feature_num": self.feature_num,
                                  "future_seq_len": self.future_seq_len, "target_col_num": self.target_col_num,
                                  "metric": self.metric, "latent_dim": self.latent_dim,
                                  "batch_size": self.batch_size, "dropout": self.dropout, "lr": self.lr})

    def restore(self, model_path, **config):
        self.past_seq_len = config["past_seq_len"]
        self.feature_num = config["feature_num"]
        self.future_seq_len = config["future_seq_len"]
        self.target_col_num = config["target_col_num"]
        self.config.update(config)
        chk, self.check_optional_config = self.check_optional_config, False
        try:
            self._build_train(**config)
        finally:
            self.check_optional_config = chk
        self.model.load_state_dict(torch.load(model_path, weights_only=True))
        return self

    def _get_required_parameters(self):
        return set()

    def _get_optional_parameters(self):
        # the reference's set literal concatenates the first three names (missing commas):
        # 'past_seq_lenlatent_dimdropout', 'metric', 'lr', 'epochs', 'batch_size'
        return {"past_seq_len" "latent_dim" "dropout", "metric", "lr", "epochs", "batch_size"}


__all__ = ["LSTMSeq2Seq", "LSTMSeq2SeqNet"]
