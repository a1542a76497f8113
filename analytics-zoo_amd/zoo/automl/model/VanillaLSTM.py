"""VanillaLSTM (Py/automl/model/VanillaLSTM.py:28-205): two stacked LSTMs with dropout
and a dense head over the last step, predicting ``future_seq_len`` values."""
from zoo.automl.model._nets import VanillaLSTMNet
from zoo.automl.model._torch_model import TorchTSModel


class VanillaLSTM(TorchTSModel):
    net_cls = VanillaLSTMNet
    required = set()
    optional = {"lstm_1_units", "dropout_1", "lstm_2_units", "dropout_2", "lr", "batch_size", "epochs", "metric"}


__all__ = ["VanillaLSTM"]
