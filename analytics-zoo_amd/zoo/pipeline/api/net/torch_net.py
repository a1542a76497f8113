"""TorchNet / TorchModel / TorchCriterion (Zs/pipeline/api/net/TorchNet.scala:39-242,
TorchCriterion.scala; Py/pipeline/api/net/torch_net.py ``TorchNet.from_pytorch``).

The reference pushes JVM-held weights into libtorch on every forward. Here a
TorchNet adopts the nn.Module as a Keras layer: its parameters join the engine's
flat fp32 master / gradient buffers like any other layer (bucketed RCCL
all-reduce, fused optimizer), and ``from_pytorch`` swaps its standard layers for
the native-kernel twins of zoo.pipeline.api.net.native_lower.
"""
import io

import torch

from zoo.pipeline.api.keras.base import Layer
from zoo.pipeline.api.keras.engine.topology import KerasNet
from zoo.pipeline.api.keras.objectives import TorchLoss


class TorchNet(KerasNet):
    def __init__(self, module, input_shape=None, name=None):
        super().__init__(name=name)
        self.module = module
        self._input_shape = None if input_shape is None else (None,) + tuple(input_shape)
        self.built = True

    @staticmethod
    def from_pytorch(module, input_shape=None, sample_input=None, native=True):
        """Wrap an nn.Module (``sample_input`` is accepted for API parity; no tracing needed).
        ``native``: the module's conv / linear / pooling / batch-norm / activation / LRN / LSTM
        submodules get their native twins IN PLACE (zoo.pipeline.api.net.native_lower swaps
        the class only: parameters, state_dict keys and behaviour off the GPU are unchanged; the
        reference instead pushes JVM-held weights into libtorch, TorchNet.scala:86-113).
        TorchScript modules are wrapped as they are."""
        if sample_input is not None and input_shape is None:
            input_shape = tuple(sample_input.shape[1:])
        if native and not isinstance(module, torch.jit.ScriptModule):
            from zoo.pipeline.api.net.native_lower import lower_module
            module = lower_module(module, training=module.training)
        return TorchNet(module, input_shape)

    @staticmethod
    def load(path):
        """TorchScript archive (torch.jit.save) -> TorchNet."""
        return TorchNet(torch.jit.load(path, map_location="cpu"))

    def save_torchscript(self, path, example):
        torch.jit.trace(self.module, example).save(path)

    def compute_output_shape(self, input_shape):
        if input_shape is None or any(d is None for d in input_shape[1:]):
            return None
        with torch.no_grad():
            dev = next(self.module.parameters(), torch.zeros(0)).device
            out = self.module(torch.zeros((1,) + tuple(input_shape[1:]), device=dev))
        return (None,) + tuple(out.shape[1:])

    def call(self, x):
        return self.module(x)

    def forward(self, x, *rest):
        return self.module(x, *rest)

    def _layer_list(self):
        return []

    def get_weights(self):
        return [p.detach().cpu().numpy().copy() for p in self.module.parameters()]

    def set_weights(self, weights):
        with torch.no_grad():
            for p, w in zip(self.module.parameters(), weights):
                p.copy_(torch.as_tensor(w).reshape(p.shape))

    def state_bytes(self):
        buf = io.BytesIO()
        torch.save(self.module.state_dict(), buf)
        return buf.getvalue()


TorchModel = TorchNet


class TorchCriterion(TorchLoss):
    @staticmethod
    def from_pytorch(loss, input_shape=None, label_shape=None):
        return TorchCriterion(loss)


class TorchLayer(Layer):
    """A single nn.Module as a Keras layer inside Sequential / functional graphs."""

    def __init__(self, module, output_shape=None, **kwargs):
        super().__init__(**kwargs)
        self.module = module
        self._fixed_out = output_shape

    def compute_output_shape(self, input_shape):
        if self._fixed_out is not None:
            return (None,) + tuple(self._fixed_out)
        with torch.no_grad():
            out = self.module(torch.zeros((1,) + tuple(input_shape[1:])))
        return (None,) + tuple(out.shape[1:])

    def call(self, x):
        return self.module(x)

    def _keras_params(self):
        return list(self.module.parameters())
