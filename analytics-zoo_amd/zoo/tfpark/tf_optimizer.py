"""TFOptimizer / TFEstimator / ZooOptimizer (Py/tfpark/tf_optimizer.py, estimator.py,
zoo_optimizer.py) on the TrainingEngine."""
import torch

from zoo.common import triggers as T


class ZooOptimizer:
    """Wraps an optimizer spec so gradients are aggregated by the engine (zoo_optimizer.py:20-81)."""

    def __init__(self, optimizer="adam"):
        from zoo.pipeline.api.keras.optimizers import to_optim_method
        self.optim = to_optim_method(optimizer)


class TFOptimizer:
    def __init__(self, model, optim_method=None, dataset=None, clip=None):
        self.model, self.dataset = model, dataset
        if optim_method is not None:
            from zoo.pipeline.api.keras.optimizers import to_optim_method
            model._optim = to_optim_method(optim_method.optim if isinstance(optim_method, ZooOptimizer)
                                           else optim_method)
            model._engine = None

    @classmethod
    def from_keras(cls, keras_model, dataset, optim_method=None, val_split=0.0, **kwargs):
        m = keras_model.model if hasattr(keras_model, "model") and hasattr(keras_model, "fit") and \
            not hasattr(keras_model, "_get_engine") else keras_model
        return cls(m, optim_method, dataset)

    @classmethod
    def from_loss(cls, *a, **k):
        raise NotImplementedError("from_loss needs a TensorFlow graph; use from_keras with a zoo/torch model")

    @classmethod
    def from_train_op(cls, *a, **k):
        raise NotImplementedError("from_train_op needs a TensorFlow graph; use from_keras with a zoo/torch model")

    def set_constant_gradient_clipping(self, min_value, max_value):
        self.model.set_constant_gradient_clipping(min_value, max_value)

    def set_gradient_clipping_by_l2_norm(self, clip_norm):
        self.model.set_gradient_clipping_by_l2_norm(clip_norm)

    def set_train_summary(self, summary):
        self.model._tb = (summary, self.model._tb[1] if self.model._tb else summary)

    def optimize(self, end_trigger=None, checkpoint_trigger=None):
        eng = self.model._get_engine()
        eng.fit(self.dataset.get_training_data(), end_trigger=end_trigger or T.MaxEpoch(1),
                validation=self.dataset.get_validation_data(), val_methods=self.model._metrics or None)
        return self


class TFEstimatorSpec:
    def __init__(self, mode, predictions=None, loss=None):
        self.mode, self.predictions, self.loss = mode, predictions, loss


class TFEstimator:
    """``model_fn(features, labels, mode, params)`` returns a TFEstimatorSpec whose
    ``loss`` is a torch scalar (train/eval) and ``predictions`` a tensor. The
    module(s) it uses are passed as ``modules`` so their parameters are optimized."""

    def __init__(self, model_fn, modules, optimizer="adam", model_dir=None, params=None):
        from zoo.parallel.flat import FlatParams
        from zoo.pipeline.api.keras.optimizers import to_optim_method
        from zoo.common.nncontext import get_nncontext
        self.model_fn, self.params = model_fn, params or {}
        self.modules = torch.nn.ModuleList(modules)
        self.device = get_nncontext().device
        self.modules.to(self.device)
        self.flat = FlatParams(list(self.modules.parameters()), device=self.device,
                               bf16_copy=self.device.type == "cuda")
        self.optim = to_optim_method(optimizer)

    @classmethod
    def from_model_fn(cls, model_fn, modules, optimizer="adam", model_dir=None, params=None):
        return cls(model_fn, modules, optimizer, model_dir, params)

    def train(self, input_fn, steps=None):
        n = 0
        self.modules.train()
        while steps is None or n < steps:
            for x, y in input_fn():
                self.flat.grad.zero_()
                spec = self.model_fn(x.to(self.device), y.to(self.device), "train", self.params)
                spec.loss.backward()
                self.optim.step(self.flat.master, self.flat.grad, self.flat.bf16, 1.0)
                n += 1
                if steps is not None and n >= steps:
                    break
            if steps is None:
                break
        return self

    @torch.no_grad()
    def evaluate(self, input_fn, eval_methods=None):
        self.modules.eval()
        tot, cnt = 0.0, 0
        for x, y in input_fn():
            spec = self.model_fn(x.to(self.device), y.to(self.device), "eval", self.params)
            tot += float(spec.loss) * x.shape[0]
            cnt += x.shape[0]
        return {"loss": tot / max(cnt, 1)}

    @torch.no_grad()
    def predict(self, input_fn):
        self.modules.eval()
        out = []
        for batch in input_fn():
            x = batch[0] if isinstance(batch, (list, tuple)) else batch
            out.append(self.model_fn(x.to(self.device), None, "infer", self.params).predictions.cpu())
        return torch.cat(out).numpy()
