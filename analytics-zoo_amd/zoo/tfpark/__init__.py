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
Graph-import paths (``from_loss``, ``from_train_op``, frozen ``.pb``) need TF
and raise; export such graphs to ONNX and use zoo.pipeline.api.onnx.
"""
from zoo.tfpark.gan import GANEstimator, GanOptimMethod  # noqa: F401
from zoo.tfpark.model import KerasModel  # noqa: F401
from zoo.tfpark.tf_dataset import TFDataset  # noqa: F401
from zoo.tfpark.tf_optimizer import TFEstimator, TFEstimatorSpec, TFOptimizer, ZooOptimizer  # noqa: F401
