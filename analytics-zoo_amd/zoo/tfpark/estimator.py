"""Import-path compatibility with the reference module ``zoo.tfpark.estimator`` (Py/tfpark/estimator.py):
the implementations live in the modules imported below."""
from zoo.tfpark.tf_optimizer import TFEstimator  # noqa: F401
