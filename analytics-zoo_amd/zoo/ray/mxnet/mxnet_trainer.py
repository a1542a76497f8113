"""Import-path compatibility with the reference module ``zoo.ray.mxnet.mxnet_trainer`` (Py/ray/mxnet/mxnet_trainer.py):
the implementations live in the modules imported below."""
from zoo.ray.mxnet import MXNetTrainer  # noqa: F401
