from zoo.pipeline.inference.inference_model import InferenceModel  # noqa: F401
