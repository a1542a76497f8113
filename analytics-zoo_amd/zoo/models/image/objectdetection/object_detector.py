"""Import-path compatibility with the reference module ``zoo.models.image.objectdetection.object_detector`` (Py/models/image/objectdetection/object_detector.py):
the implementations live in the modules imported below."""
from zoo.models.image.objectdetection.ssd import ObjectDetector  # noqa: F401
