"""The VanillaLSTM network (Py/automl/model/VanillaLSTM.py) and ``build_model`` (a trial config's
network); the Seq2Seq and MTNet networks live with their models (Seq2Seq.py, MTNet_keras.py)."""
import torch
import torch.nn as nn


def _to_native(net):
    """LSTM / Linear / Conv2d submodules -> the persistent recurrent kernel and the MFMA GEMMs
    (zoo.pipeline.api.net.native_lower; parameters shared, CPU falls back to torch)."""
    from zoo.pipeline.api.net.native_lower import lower_module
    return lower_module(net)


class VanillaLSTMNet(nn.Module):
    """LSTM(lstm_1_units) -> Dropout -> LSTM(lstm_2_units) -> Dropout -> Dense(future_seq_len)."""

    def __init__(self, input_dim, future_seq_len=1, lstm_1_units=20, dropout_1=0.2, lstm_2_units=10, dropout_2=0.2,
                 **_):
        super().__init__()
        self.l1 = nn.LSTM(input_dim, int(lstm_1_units), batch_first=True)
        self.d1 = nn.Dropout(float(dropout_1))
        self.l2 = nn.LSTM(int(lstm_1_units), int(lstm_2_units), batch_first=True)
        self.d2 = nn.Dropout(float(dropout_2))
        self.fc = nn.Linear(int(lstm_2_units), int(future_seq_len))
        _to_native(self)

    def forward(self, x):
        h, _ = self.l1(x)
        h, _ = self.l2(self.d1(h))
        return self.fc(self.d2(h[:, -1]))


def build_model(config, input_dim, future_seq_len):
    """The torch network of a trial config (model LSTM / Seq2seq / MTNet)."""
    from zoo.automl.model.MTNet_keras import MTNetNet
    from zoo.automl.model.Seq2Seq import LSTMSeq2SeqNet
    name = config.get("model", "LSTM")
    cfg = {k: v for k, v in config.items() if k not in ("model", "input_dim", "future_seq_len")}
    if name == "LSTM":
        return VanillaLSTMNet(input_dim=input_dim, future_seq_len=future_seq_len, **cfg)
    if name == "Seq2seq":
        return LSTMSeq2SeqNet(input_dim, 1, cfg.get("latent_dim", 128), cfg.get("dropout", 0.2),
                              cfg.get("past_seq_len"))
    if name == "MTNet":
        keys = ("time_step", "long_num", "ar_window", "cnn_height", "cnn_hid_size", "rnn_hid_sizes", "dropout")
        return MTNetNet(input_dim, future_seq_len, **{k: cfg[k] for k in keys if k in cfg})
    raise ValueError("unknown model %s" % name)


MODELS = ("LSTM", "Seq2seq", "MTNet")
