"""Net: model loaders (Zs/pipeline/api/Net.scala:44-260; Py/pipeline/api/net/net_load.py).

  Net.load(path)                 zoo Keras / ZooModel file
  Net.load_bigdl(path, weights)  BigDL protobuf ``.model`` -> GraphNet
  Net.load_caffe(def, model)     Caffe prototxt + caffemodel -> GraphNet
  Net.load_onnx(path)            ONNX ModelProto -> GraphNet
  Net.load_torch(path)           TorchScript or Lua Torch7 .t7 -> TorchNet
  Net.load_tf(path, in, out)     TF frozen graph / SavedModel -> TFNet
  Net.load_keras(json, hdf5)     Keras 1.2 / 2.x definition + HDF5 weights -> zoo Keras model
"""


class Net:
    @staticmethod
    def load(model_path, weight_path=None):
        from zoo.pipeline.api.keras.serialization import load_model
        return load_model(model_path)

    @staticmethod
    def load_bigdl(model_path, weight_path=None, bigdl_type="float", native=True):
        """``native``: run the imported graph on the zoo kernels (GraphNet.to_native); False keeps
        the plain torch modules (the fp32 reference path)."""
        from zoo.pipeline.api.net.bigdl_loader import load_bigdl
        return _native(load_bigdl(model_path, weight_path), native)

    @staticmethod
    def load_caffe(def_path, model_path, bigdl_type="float", native=True):
        from zoo.pipeline.api.net.caffe_loader import load_caffe
        return _native(load_caffe(def_path, model_path), native)

    @staticmethod
    def load_onnx(model_path, native=True):
        from zoo.pipeline.api.onnx.onnx_loader import load_onnx
        return _native(load_onnx(model_path), native)

    @staticmethod
    def load_torch(path, bigdl_type="float", native=True):
        """TorchScript archive -> TorchNet; a Lua Torch7 ``.t7`` nn model (Net.loadTorch,
        BigDL TorchFile) -> torch module rebuilt from the decoded objects."""
        with open(path, "rb") as f:
            magic = f.read(4)
        if magic[:2] != b"PK":   # not a zip archive: Torch7 binary serialisation
            from zoo.pipeline.api.net.torch7 import load_torch7
            from zoo.pipeline.api.net.torch_net import TorchNet
            return TorchNet.from_pytorch(load_torch7(path), native=native)
        from zoo.pipeline.api.net.torch_net import TorchNet
        return TorchNet.load(path)

    @staticmethod
    def load_tf(path, inputs=None, outputs=None, **kw):
        """Frozen GraphDef / export folder / SavedModel -> TFNet (torch executor
        of the TF graph, zoo.pipeline.api.net.tf_graph)."""
        from zoo.tfpark.tfnet import TFNet
        return TFNet(path, inputs, outputs, **kw)

    @staticmethod
    def load_keras(json_path=None, hdf5_path=None, by_name=False):
        """Keras model definition (json, or the model_config of a full-model HDF5 file) and
        HDF5 weights -> zoo Keras Sequential / Model (zoo.pipeline.api.keras.keras_import;
        HDF5 read by the built-in codec, no h5py)."""
        from zoo.pipeline.api.keras.keras_import import load_keras
        return load_keras(json_path, hdf5_path, by_name)


def _native(graph, native):
    """GraphNet loaders: swap in the native twins (in inference form; a later ``fit`` keeps the
    fused BatchNorm in training mode inside the native conv node)."""
    if native and hasattr(graph, "to_native"):
        graph.to_native()
    return graph
