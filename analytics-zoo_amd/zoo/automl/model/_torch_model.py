"""Shared trainer of the AutoML time-series models: a torch network from ``_nets``
trained by this framework's engine (TorchNet -> TrainingEngine with the fused
optimizers; on the GPU the LSTM/GRU layers run the native recurrent kernels), with
Monte-Carlo-dropout uncertainty and state-dict save/restore."""
import json
import os

import numpy as np
import torch

from zoo.automl.common.metrics import Evaluator
from zoo.automl.model.abstract import BaseModel


def _jsonable(v):
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, np.integer):
        return int(v)
    if isinstance(v, np.floating):
        return float(v)
    if isinstance(v, (list, tuple)):
        return [_jsonable(e) for e in v]
    return v


class TorchTSModel(BaseModel):
    """Subclasses set ``net_cls`` and the parameter sets."""
    net_cls = None
    required = set()
    optional = set()
    default_batch_size = 32

    def _optimizer(self, cfg):
        from zoo.pipeline.api.keras.optimizers import Adam
        return Adam(lr=float(cfg.get("lr", 1e-3)))

    def __init__(self, check_optional_config=False, future_seq_len=1):
        self.check_optional_config = check_optional_config
        self.future_seq_len = int(future_seq_len)
        self.model = None
        self.net = None
        self.config = {}
        self.input_dim = None

    # -- subclass hooks
    def _net_kwargs(self, config):
        return {k: v for k, v in config.items() if k in self.required | self.optional}

    def _reshape_input(self, x):
        return np.asarray(x, np.float32)

    def _build(self, input_dim, config):
        kw = {k: v for k, v in self._net_kwargs(config).items()
              if k not in ("lr", "batch_size", "epochs", "metric", "loss")}
        self.model = self.net_cls(input_dim=input_dim, future_seq_len=self.future_seq_len, **kw)
        self.input_dim = int(input_dim)
        return self.model

    # -- BaseModel
    def fit_eval(self, x, y, validation_data=None, mc=False, verbose=0, **config):
        from zoo.pipeline.api.net import TorchNet
        self.config.update(config)
        cfg = self.config
        x = self._reshape_input(x)
        y = np.asarray(y, np.float32).reshape(len(x), -1)
        if self.model is None:
            self._check_config(**cfg)
            self._build(x.shape[-1], cfg)
        if self.net is None:
            self.net = TorchNet.from_pytorch(self.model, input_shape=x.shape[1:])
            self.net.compile(optimizer=self._optimizer(cfg), loss=cfg.get("loss", "mse"))
        # a batch larger than the data trains on all of it (Keras' partial last batch)
        bs = max(1, min(int(cfg.get("batch_size", self.default_batch_size)), len(x)))
        self.net.fit(x, y, batch_size=bs, nb_epoch=int(cfg.get("epochs", 1)))
        metric = cfg.get("metric", "mse")
        vx, vy = validation_data if validation_data is not None else (x, y)
        return float(self.evaluate(vx, vy, [metric])[0])

    def evaluate(self, x, y, metric=None):
        metric = list(metric or ["mse"])
        pred = self.predict(x)
        y = np.asarray(y, np.float32).reshape(pred.shape)
        return [float(np.mean(Evaluator.evaluate(m, y, pred, "raw_values"))) for m in metric]

    def predict(self, x, mc=False):
        if self.model is None:
            raise RuntimeError("fit_eval or restore the model first")
        x = self._reshape_input(x)
        m = self.model
        was = m.training
        m.train(bool(mc))
        dev = next(m.parameters()).device
        out = []
        with torch.no_grad():
            for i in range(0, len(x), 1024):
                out.append(m(torch.from_numpy(x[i:i + 1024]).to(dev)).float().cpu().numpy())
        m.train(was)
        return np.concatenate(out, 0)

    def predict_with_uncertainty(self, x, n_iter=100):
        preds = np.stack([self.predict(x, mc=True) for _ in range(int(n_iter))])
        return preds.mean(0), preds.std(0)

    def state_dict(self):
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items()}

    def save(self, model_path, config_path):
        d = os.path.dirname(os.path.abspath(model_path))
        os.makedirs(d, exist_ok=True)
        torch.save(self.state_dict(), model_path)
        cfg = dict(self.config, input_dim=self.input_dim, future_seq_len=self.future_seq_len)
        # merged into the bundle's shared config file (feature transformer state + trial config)
        from zoo.automl.common.util import save_config
        save_config(config_path, {k: _jsonable(v) for k, v in cfg.items()})

    def restore(self, model_path, **config):
        self.config.update(config)
        self.future_seq_len = int(self.config.get("future_seq_len", self.future_seq_len))
        self._build(int(self.config["input_dim"]), self.config)
        self.model.load_state_dict(torch.load(model_path, weights_only=True))
        self.net = None
        return self

    def _get_required_parameters(self):
        return set(self.required)

    def _get_optional_parameters(self):
        return set(self.optional)
