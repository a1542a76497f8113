"""Import-path compatibility with the reference module ``zoo.models.image.common.image_model`` (Py/models/image/common/image_model.py):
the implementations live in the modules imported below."""
from zoo.models.image.imageclassification.image_classifier import ImageModel  # noqa: F401
