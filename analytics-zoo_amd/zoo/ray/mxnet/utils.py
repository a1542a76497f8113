"""Import-path compatibility with the reference module ``zoo.ray.mxnet.utils`` (Py/ray/mxnet/utils.py):
the implementations live in the modules imported below."""
from zoo.ray.mxnet import find_free_port, create_trainer_config  # noqa: F401
