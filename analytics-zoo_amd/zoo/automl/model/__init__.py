"""AutoML time-series models (Py/automl/model/*.py): VanillaLSTM, LSTMSeq2Seq (teacher-forced
encoder-decoder), MTNetKeras (memory network with attention RNN encoders) and the
TimeSequenceModel dispatcher, each a BaseModel over its torch network trained by the engine."""
from zoo.automl.model._nets import MODELS, VanillaLSTMNet, build_model  # noqa: F401
from zoo.automl.model.abstract import BaseModel  # noqa: F401
from zoo.automl.model.VanillaLSTM import VanillaLSTM  # noqa: F401,E402
from zoo.automl.model.Seq2Seq import LSTMSeq2Seq, LSTMSeq2SeqNet  # noqa: F401,E402
from zoo.automl.model.MTNet_keras import MTNetKeras, MTNetNet  # noqa: F401,E402
from zoo.automl.model.time_sequence import TimeSequenceModel  # noqa: F401,E402

MTNet = MTNetNet  # network class under its short name
