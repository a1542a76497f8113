"""KerasModel (Py/tfpark/model.py:KerasModel): fit/evaluate/predict + on-batch APIs over a
zoo Keras model (or any torch module), trained by the TrainingEngine."""
import numpy as np
import torch

from zoo.tfpark.tf_dataset import TFDataset


class KerasModel:
    def __init__(self, model, model_dir=None, optimizer="adam", loss="mse", metrics=None):
        from zoo.pipeline.api.keras.engine.topology import KerasNet
        if not isinstance(model, KerasNet):
            from zoo.pipeline.api.net import TorchNet
            model = TorchNet.from_pytorch(model)
        self.model = model
        self.model_dir = model_dir
        if getattr(model, "_criterion", None) is None:
            model.compile(optimizer, loss, metrics)

    @property
    def metrics_names(self):
        return ["loss"] + [m.name for m in (self.model._metrics or [])]

    def get_weights(self):
        return [p.detach().cpu().numpy().copy() for p in self.model.parameters()]

    def set_weights(self, weights):
        with torch.no_grad():
            for p, w in zip(self.model.parameters(), weights):
                p.copy_(torch.as_tensor(w).reshape(p.shape))

    def save_weights(self, filepath, overwrite=True, save_format=None):
        from zoo.utils.checkpoint import save_object
        save_object({k: v.detach().cpu() for k, v in self.model.state_dict().items()}, filepath, overwrite)

    def load_weights(self, filepath, by_name=False):
        from zoo.utils.checkpoint import load_object
        self.model.load_state_dict(load_object(filepath), strict=not by_name)
        eng = getattr(self.model, "_engine", None)
        if eng is not None:
            eng.flat.refresh_bf16()

    def save_model(self, path):
        self.model.save(path, over_write=True)

    @staticmethod
    def load_model(path):
        from zoo.pipeline.api.keras.serialization import load_model
        return KerasModel(load_model(path))

    def set_train_summary(self, summary):
        self.model._tb = (summary, self.model._tb[1] if self.model._tb else summary)

    def set_val_summary(self, summary):
        self.model._tb = (self.model._tb[0] if self.model._tb else summary, summary)

    def fit(self, x=None, y=None, batch_size=None, epochs=1, validation_split=0.0, validation_data=None,
            distributed=False, **kwargs):
        if isinstance(x, TFDataset):
            val = x.get_validation_data()
            self.model.fit(x.get_training_data(), None, nb_epoch=epochs, validation_data=val)
        else:
            if validation_split and validation_data is None:
                n = int(len(x) * (1 - validation_split))
                x, y, validation_data = x[:n], y[:n], (x[n:], y[n:])
            self.model.fit(x, y, batch_size=batch_size or 32, nb_epoch=epochs, validation_data=validation_data)
        return self

    def evaluate(self, x=None, y=None, batch_per_thread=None, distributed=False):
        if isinstance(x, TFDataset):
            return self.model.evaluate(x.get_evaluation_data())
        return self.model.evaluate(x, y, batch_size=batch_per_thread or 32)

    def predict(self, x, batch_per_thread=None, distributed=False):
        if isinstance(x, TFDataset):
            return self.model.predict(x.get_prediction_data())
        return self.model.predict(x, batch_size=batch_per_thread or 256)

    def train_on_batch(self, x, y=None, sample_weight=None, class_weight=None, reset_metrics=True):
        eng = self.model._get_engine()
        dev = eng.device
        xt = [torch.as_tensor(np.asarray(t)).to(dev) for t in x] if isinstance(x, list) else \
            torch.as_tensor(np.asarray(x)).to(dev)
        return float(eng.train_step(xt, torch.as_tensor(np.asarray(y)).to(dev)))

    def test_on_batch(self, x, y=None, sample_weight=None, reset_metrics=True):
        return self.model.evaluate(x, y, batch_size=len(x))

    def predict_on_batch(self, x):
        return self.model.predict(x, batch_size=len(x) if not isinstance(x, list) else len(x[0]))
