"""Cluster Serving client (Py/serving/client.py:25-150).

``InputQueue.enqueue_image(uri, img)`` resizes the image to the configured
shape, JPEG-encodes it, base64s it and XADDs it to ``image_stream`` — with
back-pressure when the queue server's memory is above 60 % of ``maxmemory``.
``enqueue_tensor`` sends raw float32 tensors. ``OutputQueue.dequeue()``
collects and deletes every ``result:*`` hash; ``query(uri)`` waits for one.
"""
import base64
import io
import time

import numpy as np

from zoo.serving.resp import connect
from zoo.serving.server import GROUP, STREAM, load_config


class API:
    def __init__(self, config_path="config.yaml", host=None, port=None):
        try:
            cfg = load_config(config_path)
        except FileNotFoundError:
            cfg = {"host": "127.0.0.1", "port": 6379, "image_shape": [3, 224, 224]}
        self.db = connect(host or cfg["host"], port or cfg["port"])
        try:
            self.db.xgroup_create(STREAM, GROUP, id="0", mkstream=True)
        except Exception:  # noqa: BLE001 - group exists
            pass
        self.data_shape = list(cfg["image_shape"])


class InputQueue(API):
    def __init__(self, config_path="config.yaml", host=None, port=None):
        super().__init__(config_path, host, port)
        self.input_threshold = 0.6
        self.interval_if_error = 1
        self.c = self.h = self.w = None
        for num in self.data_shape:
            if num <= 0:
                raise ValueError("invalid image shape %s: no negative value is allowed" % self.data_shape)
            if 0 < num < 5:
                self.c = num
            elif self.h is None:
                self.h = num
            else:
                self.w = num

    def _full(self):
        try:
            inf = self.db.info()
            return inf.get("maxmemory", 0) and inf["used_memory"] >= inf["maxmemory"] * self.input_threshold
        except Exception:  # noqa: BLE001
            return False

    def _push(self, fields, retries=3):
        for _ in range(retries):
            if self._full():
                time.sleep(self.interval_if_error)
                continue
            try:
                return self.db.xadd(STREAM, fields)
            except Exception as e:  # noqa: BLE001 - OOM from the server
                print(e, "queue memory is full, please dequeue or delete.")
                time.sleep(self.interval_if_error)
        raise RuntimeError("serving queue is full")

    def enqueue_image(self, uri, img):
        from PIL import Image
        if isinstance(img, str):
            img = np.asarray(Image.open(img).convert("RGB"))[:, :, ::-1]  # BGR like cv2.imread
        img = np.asarray(img)
        rgb = img[:, :, ::-1] if img.ndim == 3 and img.shape[2] == 3 else img
        im = Image.fromarray(np.ascontiguousarray(rgb.astype(np.uint8)))
        if self.h and self.w:
            im = im.resize((self.w, self.h), Image.BILINEAR)
        buf = io.BytesIO()
        im.save(buf, format="JPEG", quality=95)
        return self._push({"uri": uri, "image": base64.b64encode(buf.getvalue()).decode()})

    def enqueue_encoded(self, uri, jpeg_bytes):
        """Enqueue an already-encoded JPEG/PNG (skips the client-side resize)."""
        return self._push({"uri": uri, "image": base64.b64encode(bytes(jpeg_bytes)).decode()})

    def enqueue_tensor(self, uri, data):
        a = np.ascontiguousarray(np.asarray(data, np.float32))
        return self._push({"uri": uri, "tensor": base64.b64encode(a.tobytes()).decode(),
                           "shape": ",".join(str(s) for s in a.shape)})

    @staticmethod
    def base64_encode_image(img_bytes):
        return base64.b64encode(img_bytes).decode("utf-8")


class OutputQueue(API):
    def dequeue(self):
        out = {}
        for key in self.db.keys("result:*"):
            k = key.decode() if isinstance(key, bytes) else key
            d = self.db.hgetall(k)
            v = d.get(b"value", d.get("value"))
            out[k.split(":", 1)[1]] = v.decode() if isinstance(v, bytes) else v
            self.db.delete(k)
        return out

    def query(self, uri, timeout=10.0, poll=0.01):
        deadline = time.time() + timeout
        while time.time() < deadline:
            v = self.db.hget("result:" + uri, "value")
            if v is not None:
                self.db.delete("result:" + uri)
                return v.decode() if isinstance(v, bytes) else v
            time.sleep(poll)
        return None
