"""LSTMSeq2Seq (Py/automl/model/Seq2Seq.py:27-345): an LSTM encoder over the past window
and an LSTM decoder unrolled ``future_seq_len`` steps on its own predictions."""
from zoo.automl.model._nets import LSTMSeq2SeqNet
from zoo.automl.model._torch_model import TorchTSModel


class LSTMSeq2Seq(TorchTSModel):
    net_cls = LSTMSeq2SeqNet
    required = set()
    optional = {"latent_dim", "dropout", "lr", "batch_size", "epochs", "metric"}


__all__ = ["LSTMSeq2Seq"]
