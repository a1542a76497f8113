"""TFPark on the MI355X engine (Py/tfpark/*: TFDataset, KerasModel, TFOptimizer,
TFEstimator, gan/GANEstimator; Zs/tfpark/GanOptimMethod.scala).

There is no TensorFlow runtime here ("TFPark becomes a thin
shim that imports TF/Keras/ONNX graphs into our module graph"). The TFPark
front-end API is kept and backed by the framework itself:

  * ``TFDataset``    -> FeatureSet construction (ndarrays / ImageSet / TextSet /
                        FeatureSet / pandas DataFrame), per-rank sharded
  * ``KerasModel``   -> any zoo Keras model or torch module, trained by the
                        TrainingEngine (RCCL all-reduce across ranks)
  * ``TFOptimizer.from_keras`` -> the same, driven by an end trigger
  * ``TFEstimator``  -> model_fn(features, labels, mode) returning a
                        (module-output, loss) spec, run by the engine
  * ``GanOptimMethod`` / ``GANEstimator`` -> alternating D / G steps over two
                        slices of ONE flat parameter buffer (generator first)
  * ``TFNet``        -> a TF frozen graph / export_tf folder / SavedModel decoded
                        from protobuf and executed op-by-op on torch (tfnet.py)
Graph-building paths that need a live TF session (``from_loss``,
``from_train_op``, ``TFNet.from_session``) raise: save the graph and load it
with TFNet instead.
"""
from zoo.tfpark.gan import GANEstimator, GanOptimMethod  # noqa: F401
from zoo.tfpark.model import KerasModel  # noqa: F401
from zoo.tfpark.tf_dataset import TFDataset  # noqa: F401
from zoo.tfpark.tf_optimizer import TFEstimator, TFEstimatorSpec, TFOptimizer, ZooOptimizer  # noqa: F401
from zoo.tfpark.tfnet import TFNet  # noqa: F401
