from zoo.pipeline.api.onnx.onnx_loader import OnnxLoader, load_onnx, supported_ops  # noqa: F401
