from zoo.models.image.objectdetection.ssd import (SSD, DetectionOutputSSD, MultiBoxLoss, NormalizeScale,  # noqa: F401
                                                  ObjectDetector, SSDConfig, decode, encode, iou_matrix,
                                                  mean_average_precision, nms, prior_boxes)
