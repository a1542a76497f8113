"""MTNetKeras (Py/automl/model/MTNet_keras.py:95-606): the Memory Time-series Network.

The look-back window is ``(long_num + 1) * time_step`` steps: ``long_num`` long-term memory
blocks and one short-term block. Each block goes through the same encoder structure

    Conv2D(cnn_height x feature_num, relu) -> Dropout -> stacked GRU cells (relu) wrapped by an
    input-attention RNN (``AttentionRNN``: at every step the cell input is
    [x_t, sum_k softmax_k(V^T tanh-free additive score(X W1 + b2 + h W2)) X_k] W3 + b3)

with separate weights for the memory, context and query encoders. The query attends over the
memory encodings (softmax over the ``long_num`` blocks -- the reference applies its Softmax to
a size-1 axis, i.e. uniform weights; the attention is taken over the blocks here), weights the
context encodings, and a Dense over [weighted context, query] is added to the autoregressive
Dense over the last ``ar_window`` steps of the short-term block. Loss MAE, Adam(lr).

The network runs as a TorchNet trained by this framework's engine (fused optimizer; the GRU
recurrence on the native kernels on the GPU where the cell shapes allow).
"""
import time

import numpy as np
import torch
import torch.nn as nn

from zoo.automl.common.metrics import Evaluator
from zoo.automl.model.abstract import BaseModel


def _trunc_normal_(t, std=0.1):
    with torch.no_grad():
        nn.init.trunc_normal_(t, 0.0, std, -2 * std, 2 * std)
    return t


def _mm(a, w, b=None):
    """a @ w (+ b) with w [in, out] on the native MFMA GEMM (zoo.ops.linear)."""
    from zoo import ops
    return ops.linear(a, w.t().contiguous(), b)


class AttentionRNN(nn.Module):
    """Stacked GRU cells (relu activation, input dropout) driven through the reference's
    AttentionRNNWrapper step: additive attention of the last cell state over the whole input
    sequence, the attended input concatenated to x_t and projected back to the input width."""

    def __init__(self, input_dim, hid_sizes, dropout=0.2):
        super().__init__()
        d = int(input_dim)
        self.W1 = nn.Parameter(_trunc_normal_(torch.empty(d, d)))
        self.W2 = nn.Parameter(_trunc_normal_(torch.empty(int(hid_sizes[-1]), d)))
        self.W3 = nn.Parameter(_trunc_normal_(torch.empty(2 * d, d)))
        self.b2 = nn.Parameter(_trunc_normal_(torch.empty(d)))
        self.b3 = nn.Parameter(_trunc_normal_(torch.empty(d)))
        self.V = nn.Parameter(_trunc_normal_(torch.empty(d, 1)))
        sizes = [d] + [int(h) for h in hid_sizes]
        self.cells = nn.ModuleList([nn.GRUCell(sizes[i], sizes[i + 1]) for i in range(len(hid_sizes))])
        self.drop = nn.Dropout(float(dropout))

    @staticmethod
    def _relu_gru(cell, x, h):
        # GRUCell with relu instead of tanh for the candidate (Keras GRUCell(activation="relu")):
        # on the GPU one native input GEMM + one recurrent-kernel step (reset-after GRU cell)
        from zoo.pipeline.api.net.native_lower import gru_cell_native
        y = gru_cell_native(x, h, cell.weight_ih, cell.weight_hh, cell.bias_ih, cell.bias_hh, act="relu")
        if y is not None:
            return y.to(x.dtype)
        gi = nn.functional.linear(x, cell.weight_ih, cell.bias_ih)
        gh = nn.functional.linear(h, cell.weight_hh, cell.bias_hh)
        ir, iz, in_ = gi.chunk(3, 1)
        hr, hz, hn = gh.chunk(3, 1)
        r = torch.sigmoid(ir + hr)
        z = torch.sigmoid(iz + hz)
        n = torch.relu(in_ + r * hn)
        return (1 - z) * n + z * h

    def forward(self, X):                                     # X [B, T, d] -> [B, hid[-1]]
        B, T, _ = X.shape
        hs = [X.new_zeros(B, c.hidden_size) for c in self.cells]
        mm = _mm if X.is_cuda else (lambda a, w, b=None: a @ w if b is None else a @ w + b)
        xw = mm(X, self.W1, self.b2)                             # [B, T, d]
        for t in range(T):
            score = mm(xw + mm(hs[-1], self.W2)[:, None], self.V)     # [B, T, 1]
            att = torch.softmax(score, dim=1)
            xa = (att * X).sum(1)
            inp = mm(torch.cat([X[:, t], xa], 1), self.W3, self.b3)
            for i, cell in enumerate(self.cells):
                hs[i] = self._relu_gru(cell, self.drop(inp), hs[i])
                inp = hs[i]
        return hs[-1]


class _Encoder(nn.Module):
    def __init__(self, feature_num, time_step, cnn_height, cnn_hid_size, rnn_hid_sizes, dropout):
        super().__init__()
        self.conv = nn.Conv2d(1, int(cnn_hid_size), (int(cnn_height), int(feature_num)))
        _trunc_normal_(self.conv.weight)
        nn.init.constant_(self.conv.bias, 0.1)
        self.drop = nn.Dropout(float(dropout))
        self.rnn = AttentionRNN(cnn_hid_size, rnn_hid_sizes, dropout)

    def forward(self, x):                                     # [B, num, T, F] -> [B, num, H]
        B, num, T, Fd = x.shape
        c = torch.relu(self.conv(x.reshape(B * num, 1, T, Fd)))  # [B*num, C, Tc, 1]
        c = self.drop(c).squeeze(-1).transpose(1, 2)            # [B*num, Tc, C]
        return self.rnn(c).reshape(B, num, -1)


class MTNetNet(nn.Module):
    """The MTNet graph on one input ``x [B, (long_num + 1) * time_step, feature_num]`` (split
    into the long-term blocks and the short-term block as ``_reshape_input_x`` does)."""

    def __init__(self, feature_num, output_dim, time_step=1, long_num=7, ar_window=1, cnn_height=1,
                 cnn_hid_size=32, rnn_hid_sizes=(16, 32), dropout=0.2):
        super().__init__()
        self.T, self.n, self.ar, self.F = int(time_step), int(long_num), int(ar_window), int(feature_num)
        args = (feature_num, time_step, cnn_height, cnn_hid_size, list(rnn_hid_sizes), dropout)
        self.memory, self.context, self.query = _Encoder(*args), _Encoder(*args), _Encoder(*args)
        last = int(list(rnn_hid_sizes)[-1])
        self.out = nn.Linear(last * (self.n + 1), int(output_dim))
        _trunc_normal_(self.out.weight)
        nn.init.constant_(self.out.bias, 0.1)
        self.ar_fc = None
        if self.ar > 0:
            self.ar_fc = nn.Linear(self.ar * self.F, int(output_dim))
            _trunc_normal_(self.ar_fc.weight)
            nn.init.constant_(self.ar_fc.bias, 0.1)
        from zoo.automl.model._nets import _to_native
        _to_native(self)

    def forward(self, x):
        B = x.shape[0]
        long_x = x[:, :self.n * self.T].reshape(B, self.n, self.T, self.F)
        short_x = x[:, self.n * self.T:(self.n + 1) * self.T]
        mem = self.memory(long_x)                              # [B, n, H]
        ctx = self.context(long_x)
        q = self.query(short_x[:, None])                       # [B, 1, H]
        prob = torch.softmax((mem * q).sum(-1, keepdim=True), dim=1)   # [B, n, 1] attention over the blocks
        pred_x = torch.cat([ctx * prob, q], 1).reshape(B, -1)
        y = self.out(pred_x)
        if self.ar_fc is not None:
            y = y + self.ar_fc(short_x[:, -self.ar:].reshape(B, -1))
        return y


class MTNetKeras(BaseModel):
    """BaseModel API of the reference (apply_config / fit_eval / evaluate / predict /
    predict_with_uncertainty / save / restore)."""

    def __init__(self, check_optional_config=False, future_seq_len=1):
        self.check_optional_config = check_optional_config
        self.future_seq_len = future_seq_len
        self.config = None
        self.time_step = self.cnn_height = self.long_num = self.ar_window = None
        self.feature_num = self.output_dim = None
        self.cnn_hid_size = self.rnn_hid_sizes = self.last_rnn_size = None
        self.dropout = self.lr = self.batch_size = None
        self.saved_configs = {"cnn_height", "long_num", "time_step", "ar_window", "cnn_hid_size", "rnn_hid_sizes",
                              "dropout", "lr", "batch_size", "epochs", "metrics", "mc", "feature_num", "output_dim"}
        self.model = None
        self.net = None
        self.metrics = None
        self.mc = None
        self.epochs = None

    # ------------------------------------------------------------------ config
    def apply_config(self, rs=False, config=None):
        super()._check_config(**config)
        if rs and not set(config.keys()).issuperset(self.saved_configs):
            raise ValueError("restore needs the saved configs %s" % sorted(self.saved_configs - set(config)))
        self.epochs = config.get("epochs")
        self.metrics = config.get("metrics", ["mean_squared_error"])
        self.mc = config.get("mc")
        self.feature_num = config["feature_num"]
        self.output_dim = config["output_dim"]
        self.time_step = config.get("time_step", 1)
        self.long_num = config.get("long_num", 7)
        self.ar_window = config.get("ar_window", 1)
        self.cnn_height = config.get("cnn_height", 1)
        self.cnn_hid_size = config.get("cnn_hid_size", 32)
        self.rnn_hid_sizes = config.get("rnn_hid_sizes", [16, 32])
        self.last_rnn_size = self.rnn_hid_sizes[-1]
        self.dropout = config.get("dropout", 0.2)
        self.batch_size = config.get("batch_size", 64)
        self.lr = config.get("lr", 0.001)
        self._check_configs()

    def _check_configs(self):
        if not self.time_step >= 1:
            raise ValueError("Invalid configuration value. 'time_step' must be larger than 1")
        if not self.time_step >= self.ar_window:
            raise ValueError("Invalid configuration value. 'ar_window' must not exceed 'time_step'")
        if not isinstance(self.rnn_hid_sizes, list):
            raise ValueError("Invalid configuration value. 'rnn_hid_sizes' must be a list of integers")

    def build(self):
        from zoo.pipeline.api.keras.optimizers import Adam
        from zoo.pipeline.api.net import TorchNet
        self.model = MTNetNet(self.feature_num, self.output_dim, self.time_step, self.long_num, self.ar_window,
                              self.cnn_height, self.cnn_hid_size, self.rnn_hid_sizes, self.dropout)
        self.net = TorchNet.from_pytorch(self.model)
        self.net.compile(optimizer=Adam(lr=float(self.lr)), loss="mae")
        return self.model

    # ------------------------------------------------------------------ data
    def _reshape_input_x(self, x):
        long_term = np.reshape(x[:, :self.time_step * self.long_num], [-1, self.long_num, self.time_step, x.shape[-1]])
        short_term = np.reshape(x[:, self.time_step * self.long_num:], [-1, self.time_step, x.shape[-1]])
        return long_term, short_term

    def _flat(self, x):
        """(long, short) inputs or a rolled window -> the net's [N, (long+1)*T, F] input."""
        if isinstance(x, (list, tuple)):
            lt, st = (np.asarray(v, np.float32) for v in x)
            return np.concatenate([lt.reshape(len(lt), -1, lt.shape[-1]), st], 1)
        x = np.asarray(x, np.float32)
        need = (self.long_num + 1) * self.time_step
        if x.shape[1] != need:
            raise ValueError("MTNet needs a look-back of (long_num + 1) * time_step = %d steps, got %d"
                             % (need, x.shape[1]))
        return x

    def _add_config_attributes(self, config, **new_attributes):
        if self.config is None:
            self.config = config
        elif config:
            raise ValueError("You can only pass new configuations for 'mc', 'epochs' and 'metrics' during "
                             "incremental fitting. Additional configs passed are {}".format(config))
        if new_attributes["metrics"] is None:
            del new_attributes["metrics"]
        self.config.update(new_attributes)

    def _check_input(self, x, y):
        input_feature_num = np.asarray(x[1] if isinstance(x, (list, tuple)) else x).shape[-1]
        input_output_dim = np.asarray(y).shape[-1]
        if self.feature_num is not None and self.feature_num != input_feature_num:
            raise ValueError("input x has different feature number (the shape of last dimension) {} with the "
                             "fitted model, which is {}.".format(input_feature_num, self.feature_num))
        if self.output_dim is not None and self.output_dim != input_output_dim:
            raise ValueError("input y has different prediction size (the shape of last dimension) of {} with "
                             "the fitted model, which is {}.".format(input_output_dim, self.output_dim))
        return input_feature_num, input_output_dim

    # ------------------------------------------------------------------ BaseModel
    def fit_eval(self, x, y, validation_data=None, mc=False, metrics=None, epochs=10, verbose=0, **config):
        y = np.asarray(y, np.float32)
        if y.ndim == 1:
            y = y[:, None]
        feature_num, output_dim = self._check_input(x, y)
        self._add_config_attributes(config, epochs=epochs, mc=mc, metrics=metrics, feature_num=feature_num,
                                    output_dim=output_dim)
        self.apply_config(config=self.config)
        xin = self._flat(x)
        if self.model is None:
            st = time.time()
            self.build()
            if verbose == 1:
                print("Build model took {}s".format(time.time() - st))
        st = time.time()
        self.net.fit(xin, y, batch_size=max(1, min(int(self.batch_size), len(xin))), nb_epoch=int(self.epochs))
        if verbose == 1:
            print("Fit model took {}s".format(time.time() - st))
        if validation_data is None:
            vx, vy = x, y
        else:
            vx, vy = validation_data
        return self.evaluate(vx, vy, [self.metrics[0]])[0]

    def evaluate(self, x, y, metrics=("mse",)):
        y_pred = self.predict(x)
        y = np.asarray(y, np.float32).reshape(y_pred.shape)
        multioutput = "uniform_average" if y_pred.shape[1] == 1 else "raw_values"
        return [Evaluator.evaluate(m, y, y_pred, multioutput=multioutput) for m in metrics]

    def predict(self, x, mc=False):
        if self.model is None:
            raise RuntimeError("fit_eval or restore the model first")
        xin = self._flat(x)
        m = self.model
        was = m.training
        m.train(bool(mc))
        dev = next(m.parameters()).device
        with torch.no_grad():
            out = np.concatenate([m(torch.from_numpy(xin[i:i + 1024]).to(dev)).float().cpu().numpy()
                                  for i in range(0, len(xin), 1024)], 0)
        m.train(was)
        return out

    def predict_with_uncertainty(self, x, n_iter=100):
        result = np.stack([self.predict(x, mc=True) for _ in range(int(n_iter))])
        return result.mean(axis=0), result.std(axis=0)

    def save(self, model_path, config_path):
        from zoo.automl.common.util import save_config
        torch.save({k: v.detach().cpu() for k, v in self.model.state_dict().items()}, model_path)
        config_to_save = {"cnn_height": self.cnn_height, "long_num": self.long_num, "time_step": self.time_step,
                          "ar_window": self.ar_window, "cnn_hid_size": self.cnn_hid_size,
                          "rnn_hid_sizes": self.rnn_hid_sizes, "dropout": self.dropout, "lr": self.lr,
                          "batch_size": self.batch_size, "epochs": self.epochs, "metrics": self.metrics,
                          "mc": self.mc, "feature_num": self.feature_num, "output_dim": self.output_dim}
        assert set(config_to_save) == self.saved_configs
        save_config(config_path, config_to_save)

    def restore(self, model_path, **config):
        self.config = config
        self.apply_config(rs=True, config=config)
        self.build()
        self.model.load_state_dict(torch.load(model_path, weights_only=True))
        return self

    def _get_optional_parameters(self):
        return {"batch_size", "dropout", "time_step", "filter_size", "long_num", "ar_size"}

    def _get_required_parameters(self):
        return {"feature_num", "output_dim"}

    @staticmethod
    def past_seq_len(long_num, time_step):
        return (int(long_num) + 1) * int(time_step)


__all__ = ["MTNetKeras", "MTNetNet", "AttentionRNN"]
