"""Import-path compatibility with the reference module ``zoo.pipeline.nnframes.nn_image_schema`` (Py/pipeline/nnframes/nn_image_schema.py):
the implementations live in the modules imported below."""
from zoo.pipeline.nnframes.nn_image_reader import with_origin_column  # noqa: F401
