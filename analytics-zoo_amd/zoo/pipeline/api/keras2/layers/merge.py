"""Import-path compatibility with the reference module ``zoo.pipeline.api.keras2.layers.merge`` (Py/pipeline/api/keras2/layers/merge.py):
the implementations live in the modules imported below."""
from zoo.pipeline.api.keras2.layers import Maximum, Minimum, Average, maximum, minimum, average  # noqa: F401
