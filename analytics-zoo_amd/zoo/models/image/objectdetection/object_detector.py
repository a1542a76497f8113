"""Import-path compatibility with the reference module ``zoo.models.image.objectdetection.object_detector`` (Py/models/image/objectdetection/object_detector.py):
the implementations live in the modules imported below."""
from zoo.models.image.objectdetection.ssd import ObjectDetector  # noqa: F401
from zoo.models.image.objectdetection.postprocess import (DecodeOutput, ImInfo, ScaleDetection, Visualizer,  # noqa: F401,E501
                                                          read_coco_label_map, read_pascal_label_map)
