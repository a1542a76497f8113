"""TimeSequencePipeline (Py/automl/pipeline/time_sequence.py): feature transformer +
model + config; fit / evaluate / predict / predict_with_uncertainty (MC dropout) /
save / load."""
import json
import os

import numpy as np
import torch

from zoo.automl.common.metrics import Evaluator
from zoo.automl.feature.time_sequence import TimeSequenceFeatureTransformer
from zoo.automl.model import build_model
from zoo.automl.pipeline.abstract import Pipeline


def _train(module, x, y, config, epochs=None):
    from zoo.pipeline.api.keras.optimizers import Adam
    from zoo.pipeline.api.net import TorchNet
    net = TorchNet.from_pytorch(module, input_shape=x.shape[1:])
    net.compile(optimizer=Adam(lr=float(config.get("lr", 1e-3))), loss="mse")
    net.fit(x.astype(np.float32), y.astype(np.float32), batch_size=int(config.get("batch_size", 32)),
            nb_epoch=int(epochs if epochs is not None else config.get("epochs", 1)))
    return net


class TimeSequencePipeline(Pipeline):
    def __init__(self, feature_transformers=None, model=None, config=None, name=None):
        self.ft, self.model, self.config, self.name = feature_transformers, model, dict(config or {}), name
        self.net = None

    def describe(self):
        return {"name": self.name, "config": self.config}

    def fit(self, input_df, validation_df=None, mc=False, epoch_num=20):
        x, y = self.ft.transform(input_df, is_train=True)
        self.net = _train(self.model, x, y, self.config, epoch_num)
        return self

    def fit_with_fixed_configs(self, input_df, validation_df=None, mc=False, **user_configs):
        self.config.update(user_configs)
        x, y = self.ft.fit_transform(input_df, **self.config)
        self.model = build_model(self.config, x.shape[-1], self.ft.future_seq_len)
        self.net = _train(self.model, x, y, self.config)
        return self

    def _predict_scaled(self, x, mc=False):
        m = self.model
        was = m.training
        m.train(mc)
        dev = next(m.parameters()).device
        with torch.no_grad():
            out = m(torch.from_numpy(x.astype(np.float32)).to(dev)).cpu().numpy()
        m.train(was)
        return out

    def evaluate(self, input_df, metrics=("mse",), multioutput="raw_values"):
        x, y = self.ft.transform(input_df, is_train=True)
        pred = self.ft.post_processing(input_df, self._predict_scaled(x), True)
        truth = self.ft.post_processing(input_df, y, True)
        return [Evaluator.evaluate(m, truth, pred, multioutput) for m in metrics]

    def predict(self, input_df):
        x, _ = self.ft.transform(input_df, is_train=False)
        return self.ft.post_processing(input_df, self._predict_scaled(x), False)

    def predict_with_uncertainty(self, input_df, n_iter=100):
        x, _ = self.ft.transform(input_df, is_train=False)
        preds = np.stack([self._predict_scaled(x, mc=True) for _ in range(n_iter)])
        mean = self.ft.post_processing(input_df, preds.mean(0), False)
        return mean, self.ft.unscale_uncertainty(preds.std(0))

    def save(self, ppl_file):
        os.makedirs(ppl_file, exist_ok=True)
        with open(os.path.join(ppl_file, "pipeline.json"), "w") as f:
            json.dump({"config": {k: (v.tolist() if isinstance(v, np.ndarray) else
                                      (int(v) if isinstance(v, np.integer) else
                                       (float(v) if isinstance(v, np.floating) else v)))
                                  for k, v in self.config.items()},
                       "ft": self.ft.state(), "name": self.name}, f)
        torch.save({k: v.detach().cpu() for k, v in self.model.state_dict().items()},
                   os.path.join(ppl_file, "model.pt"))
        return ppl_file

    def config_save(self, config_file):
        with open(config_file, "w") as f:
            json.dump(self.describe(), f, default=str)


def load_ts_pipeline(ppl_file):
    with open(os.path.join(ppl_file, "pipeline.json")) as f:
        d = json.load(f)
    ft = TimeSequenceFeatureTransformer.from_state(d["ft"])
    n_feat = 1 + len(ft.selected)
    model = build_model(d["config"], n_feat, ft.future_seq_len)
    model.load_state_dict(torch.load(os.path.join(ppl_file, "model.pt"), weights_only=True))
    return TimeSequencePipeline(ft, model, d["config"], d.get("name"))
