"""zoo — an MI355X-native (gfx950) rebuild of Analytics Zoo.

Same user-facing API as the reference's ``pyzoo/zoo`` package
(``init_nncontext``, ``zoo.pipeline.api.keras``, ``Estimator``, ``NNEstimator``,
``InferenceModel``, TFPark/TorchModel shims, Cluster Serving, model zoo), with
the compute path on hand-written CDNA4 HIP kernels (``zoo._C``) and the
distributed path on RCCL over xGMI (one process per GPU).
"""
from zoo.common.nncontext import init_nncontext, get_nncontext, init_spark_on_local, init_spark_on_yarn, \
    ZooConfig, ZooContext

__version__ = "0.8.0.dev0+mi355x"
