"""ZooModel / KerasZooModel base (Zs/models/common/ZooModel.scala:38-154,
KerasZooModel.scala:32-183; Py/models/common/zoo_model.py).

A ZooModel owns a Keras graph built by ``build_model()`` and exposes the
KerasNet API (compile/fit/evaluate/predict/summary/save) by delegation.
``save_model``/``load_model`` write/read the reference's BigDL/Zoo ``.model``
protobuf (zoo.utils.bigdl_model: constructor config + every tensor).
"""
from zoo.pipeline.api.keras.engine.topology import KerasNet


class ZooModel(KerasNet):
    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.model = None

    def build_model(self):
        raise NotImplementedError

    def _init_model(self):
        self.model = self.build_model()
        self.built = True
        self._input_shape = self.model.get_input_shape()
        self._output_shape = self.model.get_output_shape()
        return self

    def build(self, input_shape):
        pass

    def compute_output_shape(self, input_shape):
        return self._output_shape

    def call(self, x):
        return self.model(x)

    def forward(self, x, *rest):
        if rest:
            x = [x] + list(rest)
        return self.model(x)

    def _layer_list(self):
        return [self.model]

    def save_model(self, path, weight_path=None, over_write=False):
        self.save(path, over_write)

    @classmethod
    def load_model(cls, path, weight_path=None):
        from zoo.pipeline.api.keras.serialization import load_model
        return load_model(path)

    def quantize(self):
        """int8 inference copy of the model in place (AbstractModule.quantize,
        ImageModel.scala:133-145): see zoo.ops.quant."""
        from zoo.ops.quant import quantize
        return quantize(self)

    def get_model(self):
        return self.model


KerasZooModel = ZooModel
