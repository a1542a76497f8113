"""Detection post-processing and label maps (Zs/models/image/objectdetection/
Postprocessor.scala:30-75, LabelReader.scala; Py/models/image/objectdetection/
object_detector.py: ImInfo, DecodeOutput, ScaleDetection, Visualizer,
read_pascal_label_map, read_coco_label_map)."""
import numpy as np

PASCAL_CLASSES = ["__background__", "aeroplane", "bicycle", "bird", "boat", "bottle", "bus", "car", "cat", "chair",
                  "cow", "diningtable", "dog", "horse", "motorbike", "person", "pottedplant", "sheep", "sofa",
                  "train", "tvmonitor"]

COCO_CLASSES = ["__background__", "person", "bicycle", "car", "motorcycle", "airplane", "bus", "train", "truck",
                "boat", "traffic light", "fire hydrant", "stop sign", "parking meter", "bench", "bird", "cat", "dog",
                "horse", "sheep", "cow", "elephant", "bear", "zebra", "giraffe", "backpack", "umbrella", "handbag",
                "tie", "suitcase", "frisbee", "skis", "snowboard", "sports ball", "kite", "baseball bat",
                "baseball glove", "skateboard", "surfboard", "tennis racket", "bottle", "wine glass", "cup", "fork",
                "knife", "spoon", "bowl", "banana", "apple", "sandwich", "orange", "broccoli", "carrot", "hot dog",
                "pizza", "donut", "cake", "chair", "couch", "potted plant", "bed", "dining table", "toilet", "tv",
                "laptop", "mouse", "remote", "keyboard", "cell phone", "microwave", "oven", "toaster", "sink",
                "refrigerator", "book", "clock", "vase", "scissors", "teddy bear", "hair drier", "toothbrush"]


def read_pascal_label_map():
    return {i: n for i, n in enumerate(PASCAL_CLASSES)}


def read_coco_label_map():
    return {i: n for i, n in enumerate(COCO_CLASSES)}


class ImInfo:
    """im_info = (height, width, scale_h, scale_w) of the network input vs the original image."""

    def __call__(self, image, original_hw):
        h, w = image.shape[:2]
        return np.asarray([h, w, h / float(original_hw[0]), w / float(original_hw[1])], np.float32)


class DecodeOutput:
    """Flat detection output [n, (label, score, x1, y1, x2, y2)...] -> [K, 6] (BboxUtil.decodeRois)."""

    def __call__(self, detection):
        d = np.asarray(detection, np.float32).reshape(-1)
        if d.size == 0:
            return np.zeros((0, 6), np.float32)
        n = int(d[0])
        return d[1:1 + 6 * n].reshape(n, 6) if d.size >= 1 + 6 * n and n * 6 + 1 == d.size else d.reshape(-1, 6)


class ScaleDetection:
    """Normalised boxes ([0, 1]) -> original-image pixels, clipped first."""

    def __call__(self, detection, original_hw):
        d = np.asarray(detection, np.float32).copy()
        if d.size == 0:
            return d.reshape(0, 6)
        d[:, 2:6] = np.clip(d[:, 2:6], 0.0, 1.0)
        h, w = original_hw
        d[:, [2, 4]] *= w
        d[:, [3, 5]] *= h
        return d


class Visualizer:
    """Draw detections above ``thresh`` as 2-pixel boxes on an HWC uint8 copy of the image."""

    def __init__(self, label_map=None, thresh=0.3, color=(0, 255, 0)):
        self.label_map, self.thresh, self.color = label_map or {}, float(thresh), np.asarray(color, np.uint8)

    def __call__(self, image, detection):
        img = np.array(image, dtype=np.uint8, copy=True)
        H, W = img.shape[:2]
        for lab, score, x1, y1, x2, y2 in np.asarray(detection).reshape(-1, 6):
            if score < self.thresh:
                continue
            x1, x2 = int(max(0, min(W - 1, x1))), int(max(0, min(W - 1, x2)))
            y1, y2 = int(max(0, min(H - 1, y1))), int(max(0, min(H - 1, y2)))
            img[y1:y1 + 2, x1:x2 + 1] = self.color
            img[max(y2 - 1, 0):y2 + 1, x1:x2 + 1] = self.color
            img[y1:y2 + 1, x1:x1 + 2] = self.color
            img[y1:y2 + 1, max(x2 - 1, 0):x2 + 1] = self.color
        return img
