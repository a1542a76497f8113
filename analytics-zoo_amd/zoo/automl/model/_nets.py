"""The torch networks behind the AutoML time-series models (Py/automl/model/{VanillaLSTM,Seq2Seq,MTNet_keras}.py);
the BaseModel wrappers (fit_eval / evaluate / predict / save / restore) live in the modules named after them."""
import torch
import torch.nn as nn


class VanillaLSTMNet(nn.Module):
    """LSTM(lstm_1_units) -> Dropout -> LSTM(lstm_2_units) -> Dropout -> Dense(future_seq_len)."""

    def __init__(self, input_dim, future_seq_len=1, lstm_1_units=16, dropout_1=0.2, lstm_2_units=8, dropout_2=0.2,
                 **_):
        super().__init__()
        self.l1 = nn.LSTM(input_dim, int(lstm_1_units), batch_first=True)
        self.d1 = nn.Dropout(float(dropout_1))
        self.l2 = nn.LSTM(int(lstm_1_units), int(lstm_2_units), batch_first=True)
        self.d2 = nn.Dropout(float(dropout_2))
        self.fc = nn.Linear(int(lstm_2_units), int(future_seq_len))

    def forward(self, x):
        h, _ = self.l1(x)
        h, _ = self.l2(self.d1(h))
        return self.fc(self.d2(h[:, -1]))


class LSTMSeq2SeqNet(nn.Module):
    """Encoder LSTM -> decoder LSTM unrolled future_seq_len steps on its own predictions."""

    def __init__(self, input_dim, future_seq_len=1, latent_dim=32, dropout=0.2, **_):
        super().__init__()
        self.F = int(future_seq_len)
        self.enc = nn.LSTM(input_dim, int(latent_dim), batch_first=True)
        self.dec = nn.LSTM(1, int(latent_dim), batch_first=True)
        self.drop = nn.Dropout(float(dropout))
        self.fc = nn.Linear(int(latent_dim), 1)

    def forward(self, x):
        _, (h, c) = self.enc(x)
        inp = x[:, -1:, :1]
        outs = []
        for _ in range(self.F):
            o, (h, c) = self.dec(inp, (h, c))
            y = self.fc(self.drop(o))
            outs.append(y[:, :, 0])
            inp = y
        return torch.cat(outs, 1)


class MTNetNet(nn.Module):
    """Memory time-series network (MTNet_keras.py): the past window is split into
    ``long_num`` memory blocks + one short block of ``time_step``; each block is
    encoded by Conv1D + GRU, the short-term encoding attends over the memory
    encodings, and an autoregressive linear term on the target is added."""

    def __init__(self, input_dim, future_seq_len=1, time_step=2, long_num=2, cnn_height=2, cnn_hid_size=16,
                 rnn_hid_sizes=(16,), ar_window=2, dropout=0.2, **_):
        super().__init__()
        self.T, self.n, self.F = int(time_step), int(long_num), int(future_seq_len)
        self.ar = int(ar_window)
        k = min(int(cnn_height), self.T)
        rh = int(rnn_hid_sizes[-1] if isinstance(rnn_hid_sizes, (list, tuple)) else rnn_hid_sizes)

        def encoder():
            return nn.ModuleDict({"conv": nn.Conv1d(input_dim, int(cnn_hid_size), k),
                                  "gru": nn.GRU(int(cnn_hid_size), rh, batch_first=True)})
        self.m_enc, self.c_enc, self.q_enc = encoder(), encoder(), encoder()
        self.drop = nn.Dropout(float(dropout))
        self.out = nn.Linear(2 * rh, self.F)
        self.ar_fc = nn.Linear(self.ar, self.F)

    def _encode(self, enc, blocks):
        b, t, d = blocks.shape
        h = torch.relu(enc["conv"](blocks.transpose(1, 2))).transpose(1, 2)
        _, last = enc["gru"](self.drop(h))
        return last[-1]

    def forward(self, x):
        B, L, D = x.shape
        need = (self.n + 1) * self.T
        if L < need:
            x = torch.cat([x[:, :1].expand(B, need - L, D), x], 1)
        x = x[:, -need:]
        mem = x[:, :self.n * self.T].reshape(B * self.n, self.T, D)
        short = x[:, self.n * self.T:]
        m = self._encode(self.m_enc, mem).reshape(B, self.n, -1)
        c = self._encode(self.c_enc, mem).reshape(B, self.n, -1)
        q = self._encode(self.q_enc, short)
        att = torch.softmax((m * q[:, None]).sum(-1), 1)
        o = (att[:, :, None] * c).sum(1)
        y = self.out(torch.cat([o, q], 1))
        return y + self.ar_fc(x[:, -self.ar:, 0])


MODELS = {"LSTM": VanillaLSTMNet, "Seq2seq": LSTMSeq2SeqNet, "MTNet": MTNetNet}


def build_model(config, input_dim, future_seq_len):
    name = config.get("model", "LSTM")
    if name not in MODELS:
        raise ValueError("unknown model %s" % name)
    cfg = {k: v for k, v in config.items() if k not in ("model", "input_dim", "future_seq_len")}
    return MODELS[name](input_dim=input_dim, future_seq_len=future_seq_len, **cfg)
