from zoo.pipeline.api.keras2 import layers  # noqa: F401
