"""HTTP front end for Cluster Serving (FastAPI): POST /predict with
{"instances": [{"uri": ..., "tensor": [[...]]} | {"uri": ..., "image": "<base64 jpeg>"}]}
enqueues every instance and waits for its result; GET /health."""
import base64
import uuid

import numpy as np


def create_app(config_path="config.yaml", host=None, port=None, timeout=30.0):
    from fastapi import FastAPI, HTTPException

    from zoo.serving.client import InputQueue, OutputQueue
    app = FastAPI(title="zoo cluster serving")
    inq = InputQueue(config_path, host, port)
    outq = OutputQueue(config_path, host, port)

    @app.get("/health")
    def health():
        return {"status": "ok"}

    @app.post("/predict")
    def predict(body: dict):
        uris = []
        for inst in body.get("instances", []):
            uri = str(inst.get("uri") or uuid.uuid4())
            if "tensor" in inst:
                inq.enqueue_tensor(uri, np.asarray(inst["tensor"], np.float32))
            elif "image" in inst:
                inq._push({"uri": uri, "image": inst["image"]})
            else:
                raise HTTPException(400, "instance needs 'tensor' or 'image'")
            uris.append(uri)
        preds = []
        for u in uris:
            v = outq.query(u, timeout=timeout)
            if v is None:
                raise HTTPException(504, "timed out waiting for %s" % u)
            preds.append({"uri": u, "value": v})
        return {"predictions": preds}

    return app


def encode_image_file(path):
    with open(path, "rb") as f:
        return base64.b64encode(f.read()).decode()
