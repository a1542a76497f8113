"""AutoML time-series models (Py/automl/model/*.py): BaseModel wrappers
(VanillaLSTM, LSTMSeq2Seq, MTNetKeras, TimeSequenceModel) over the torch networks
in ``_nets`` (VanillaLSTMNet, LSTMSeq2SeqNet, MTNetNet; ``build_model`` builds one
from a trial config)."""
from zoo.automl.model._nets import MODELS, LSTMSeq2SeqNet, MTNetNet, VanillaLSTMNet, build_model  # noqa: F401
from zoo.automl.model.abstract import BaseModel  # noqa: F401
from zoo.automl.model.VanillaLSTM import VanillaLSTM  # noqa: F401,E402
from zoo.automl.model.Seq2Seq import LSTMSeq2Seq  # noqa: F401,E402
from zoo.automl.model.MTNet_keras import MTNetKeras  # noqa: F401,E402
from zoo.automl.model.time_sequence import TimeSequenceModel  # noqa: F401,E402

MTNet = MTNetNet  # network class under its short name
