"""TextKerasModel (Py/tfpark/text/keras/text_model.py:21-51) and the shared
building blocks of the text taggers (word + character features, BiLSTM, CRF).

The reference wraps nlp-architect's TF-Keras models; those are rebuilt here on
the framework's layers (embedding gather kernel, LSTM kernels, MFMA Dense) and
trained by the TrainingEngine. Save/load keeps the reference's contract: the
constructor arguments plus the weights go to one file, and ``load_model``
rebuilds the same architecture before loading the weights.
"""
import numpy as np
import torch
import torch.nn as nn

from zoo import ops
from zoo.ops.crf import crf_decode, crf_nll
from zoo.pipeline.api.keras.layers import LSTM, Bidirectional


def bilstm(in_dim, hidden, return_sequences=True):
    """Bidirectional LSTM built eagerly (parameters exist before the first call,
    so a saved state dict loads into a fresh model)."""
    layer = Bidirectional(LSTM(hidden, return_sequences=return_sequences))
    layer._ensure_built((None, None, in_dim))
    return layer


class CharWordEncoder(nn.Module):
    """word ids [B, T] + char ids [B, T, W] -> [B, T, word_emb + 2*char_lstm]."""

    def __init__(self, word_vocab_size, char_vocab_size, word_emb_dim, char_emb_dim, char_lstm_dim, dropout):
        super().__init__()
        self.word = nn.Parameter(torch.empty(word_vocab_size, word_emb_dim).uniform_(-0.05, 0.05))
        self.char = nn.Parameter(torch.empty(char_vocab_size, char_emb_dim).uniform_(-0.05, 0.05))
        self.char_lstm = bilstm(char_emb_dim, char_lstm_dim, return_sequences=False)
        self.dropout = dropout
        self.out_dim = word_emb_dim + 2 * char_lstm_dim

    def forward(self, words, chars):
        B, T = words.shape
        w = ops.embedding(words.long(), self.word)
        c = ops.embedding(chars.long().reshape(B * T, -1), self.char)          # [B*T, W, Dc]
        cf = self.char_lstm(c).reshape(B, T, -1)
        x = torch.cat([w, cf.to(w.dtype)], -1)
        return nn.functional.dropout(x, self.dropout, self.training)


class CRF(nn.Module):
    def __init__(self, num_tags):
        super().__init__()
        self.transitions = nn.Parameter(torch.zeros(num_tags, num_tags))
        self.start = nn.Parameter(torch.zeros(num_tags))
        self.end = nn.Parameter(torch.zeros(num_tags))

    def nll(self, emissions, tags, mask=None):
        return crf_nll(emissions, tags, self.transitions, mask, self.start, self.end)

    def decode(self, emissions, mask=None):
        return crf_decode(emissions, self.transitions, mask, self.start, self.end)


def _np_list(x):
    return [np.asarray(v) for v in (x if isinstance(x, (list, tuple)) else [x])]


class TextKerasModel:
    """fit / evaluate / predict / save_model over a tagger module whose
    ``loss(inputs, labels)`` and ``infer(inputs)`` define the task."""

    def __init__(self, module, optimizer=None, **config):
        from zoo.common.nncontext import get_nncontext
        self.module = module
        self.config = config
        self.optimizer = optimizer or "adam"
        self.device = get_nncontext().device
        self._engine = None

    # -- engine ------------------------------------------------------------
    def _eng(self):
        if self._engine is None:
            from zoo.pipeline.api.keras.optimizers import to_optim_method
            from zoo.pipeline.engine import TrainingEngine

            class _Loss:
                def __call__(s, out, labels):
                    return out

            mod = self.module
            self._engine = TrainingEngine(mod, _Loss(), to_optim_method(self.optimizer), device=self.device,
                                          model_forward=lambda m, batch: m.loss(batch[0], batch[1]))
        return self._engine

    def _tensors(self, arrays):
        return [torch.as_tensor(a).to(self.device) for a in arrays]

    def fit(self, x, y, batch_size=32, epochs=1, validation_data=None, shuffle=True):
        xs, ys = _np_list(x), _np_list(y)
        n = len(xs[0])
        eng = self._eng()
        hist = []
        for _ in range(int(epochs)):
            order = np.random.permutation(n) if shuffle else np.arange(n)
            tot, cnt = 0.0, 0
            for s in range(0, n, batch_size):
                idx = order[s:s + batch_size]
                bx = self._tensors([a[idx] for a in xs])
                by = self._tensors([a[idx] for a in ys])
                loss = eng.train_step((bx, by), torch.zeros(1, device=self.device))
                tot += float(loss) * len(idx)
                cnt += len(idx)
            hist.append(tot / max(cnt, 1))
        return hist

    @torch.no_grad()
    def predict(self, x, batch_per_thread=128):
        xs = _np_list(x)
        self.module.to(self.device).eval()
        outs = []
        for s in range(0, len(xs[0]), batch_per_thread):
            o = self.module.infer(self._tensors([a[s:s + batch_per_thread] for a in xs]))
            outs.append([t.float().cpu().numpy() for t in (o if isinstance(o, (list, tuple)) else [o])])
        res = [np.concatenate([o[k] for o in outs]) for k in range(len(outs[0]))]
        return res[0] if len(res) == 1 else res

    @torch.no_grad()
    def evaluate(self, x, y, batch_per_thread=128):
        xs, ys = _np_list(x), _np_list(y)
        self.module.to(self.device).eval()
        tot, cnt = 0.0, 0
        for s in range(0, len(xs[0]), batch_per_thread):
            bx = self._tensors([a[s:s + batch_per_thread] for a in xs])
            by = self._tensors([a[s:s + batch_per_thread] for a in ys])
            tot += float(self.module.loss(bx, by)) * len(bx[0])
            cnt += len(bx[0])
        return {"loss": tot / max(cnt, 1)}

    # -- persistence -----------------------------------------------------------
    def save_model(self, path):
        from zoo.utils.checkpoint import save_object
        save_object({"class": type(self).__name__, "config": self.config,
                     "weights": {k: v.detach().cpu() for k, v in self.module.state_dict().items()}}, path, True)

    @classmethod
    def _load(cls, path):
        from zoo.utils.checkpoint import load_object
        d = load_object(path)
        m = cls(**d["config"])
        m.module.load_state_dict(d["weights"])
        return m

    @classmethod
    def load_model(cls, path):
        return cls._load(path)
