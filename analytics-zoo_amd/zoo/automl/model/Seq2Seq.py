"""Import-path compatibility with the reference module ``zoo.automl.model.Seq2Seq`` (Py/automl/model/Seq2Seq.py):
the implementations live in the modules imported below."""
from zoo.automl.model import LSTMSeq2Seq  # noqa: F401
