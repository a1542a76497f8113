"""Import-path compatibility with the reference module ``zoo.models.image.imageclassification.image_classification`` (Py/models/image/imageclassification/image_classification.py):
the implementations live in the modules imported below."""
from zoo.models.image.imageclassification.image_classifier import ImageClassifier, LabelOutput  # noqa: F401
