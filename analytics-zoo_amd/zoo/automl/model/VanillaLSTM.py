"""Import-path compatibility with the reference module ``zoo.automl.model.VanillaLSTM`` (Py/automl/model/VanillaLSTM.py):
the implementations live in the modules imported below."""
from zoo.automl.model import VanillaLSTM  # noqa: F401
