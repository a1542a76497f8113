"""TFPredictor (Py/tfpark/tf_predictor.py:30-77): batch prediction of a model
over every element of a TFDataset. The reference freezes a TF session into a
TFNet; here the model is a zoo Keras model, a torch module or a TFNet and runs
directly on the device."""
import numpy as np
import torch


class TFPredictor:
    def __init__(self, model, outputs=None, inputs=None, dataset=None):
        if dataset is None:
            raise ValueError("TFPredictor needs a TFDataset (set batch_per_thread on it for prediction)")
        if getattr(dataset, "batch_per_thread", -1) <= 0 and getattr(dataset, "batch_size", -1) <= 0:
            raise ValueError("You should set batch_per_thread on TFDataset instead of batch_size for prediction")
        self.model, self.dataset = model, dataset

    @classmethod
    def from_keras(cls, keras_model, dataset):
        return cls(getattr(keras_model, "model", keras_model), dataset=dataset)

    @classmethod
    def from_outputs(cls, sess, outputs):
        raise NotImplementedError("from_outputs needs a TF session; use from_keras or pass a TFNet / module")

    @torch.no_grad()
    def predict(self):
        from zoo.common.nncontext import get_nncontext
        dev = get_nncontext().device
        m = self.model
        if isinstance(m, torch.nn.Module):
            m = m.to(dev).eval()
        outs = []
        for batch in self.dataset.get_prediction_data().data(train=False):
            x = batch[0] if isinstance(batch, (list, tuple)) else batch
            xs = [t.to(dev) for t in x] if isinstance(x, (list, tuple)) else x.to(dev)
            o = m(*xs) if isinstance(xs, list) else m(xs)
            outs.append([t.float().cpu().numpy() for t in (o if isinstance(o, (list, tuple)) else [o])])
        res = [np.concatenate([o[k] for o in outs]) for k in range(len(outs[0]))]
        return res[0] if len(res) == 1 else res
