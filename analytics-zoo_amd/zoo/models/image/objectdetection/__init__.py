from zoo.models.image.objectdetection.ssd import (SSD, DetectionOutputSSD, MultiBoxLoss, NormalizeScale,  # noqa: F401
                                                  ObjectDetector, SSDConfig, decode, encode, iou_matrix,
                                                  mean_average_precision, nms, prior_boxes)
from zoo.models.image.objectdetection.ssd import FrcnnDetector, SSDMobileNet  # noqa: F401,E402
from zoo.models.image.objectdetection.frcnn import (DetectionOutputFrcnn, FasterRCNN, Proposal,  # noqa: F401,E402
                                                    generate_anchors, roi_pool)
from zoo.models.image.objectdetection.postprocess import (DecodeOutput, ImInfo, ScaleDetection,  # noqa: F401,E402
                                                          Visualizer, read_coco_label_map,
                                                          read_pascal_label_map)
