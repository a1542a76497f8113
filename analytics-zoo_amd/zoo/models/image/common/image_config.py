"""Import-path compatibility with the reference module ``zoo.models.image.common.image_config`` (Py/models/image/common/image_config.py):
the implementations live in the modules imported below."""
from zoo.models.image.imageclassification.image_classifier import ImageConfigure  # noqa: F401
