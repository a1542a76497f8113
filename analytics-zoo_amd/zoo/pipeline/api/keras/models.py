"""zoo.pipeline.api.keras.models (Py/pipeline/api/keras/models.py)."""
from zoo.pipeline.api.keras.engine.topology import KerasNet, Model, Sequential  # noqa: F401


def load_model(path):
    from zoo.pipeline.api.keras.serialization import load_model as _load
    return _load(path)
