"""Import-path compatibility with the reference module ``zoo.tfpark.zoo_optimizer`` (Py/tfpark/zoo_optimizer.py):
the implementations live in the modules imported below."""
from zoo.tfpark.tf_optimizer import ZooOptimizer  # noqa: F401
