"""NER (Py/tfpark/text/keras/ner.py:21-73): word + character (BiLSTM) features ->
BiLSTM tagger -> linear-chain CRF. Inputs: word ids [B, T], char ids [B, T, W]
(+ sequence lengths [B, 1] in ``crf_mode='pad'``). Output: entity tags one-hot
[B, T, num_entities] from Viterbi decoding."""
import torch
import torch.nn as nn

from zoo import ops
from zoo.tfpark.text.keras.text_model import CRF, CharWordEncoder, TextKerasModel, bilstm


def _mask(inputs, T, crf_mode):
    if crf_mode == "pad" and len(inputs) > 2:
        lengths = inputs[2].reshape(-1, 1).long()
        return (torch.arange(T, device=lengths.device).unsqueeze(0) < lengths).float()
    return None


class _NERNet(nn.Module):
    def __init__(self, num_entities, word_vocab_size, char_vocab_size, word_length, word_emb_dim, char_emb_dim,
                 tagger_lstm_dim, dropout, crf_mode, char_lstm_dim=25):
        super().__init__()
        self.enc = CharWordEncoder(word_vocab_size, char_vocab_size, word_emb_dim, char_emb_dim, char_lstm_dim,
                                   dropout)
        self.tagger = bilstm(self.enc.out_dim, tagger_lstm_dim)
        self.out_w = nn.Parameter(torch.empty(num_entities, 2 * tagger_lstm_dim).uniform_(-0.05, 0.05))
        self.out_b = nn.Parameter(torch.zeros(num_entities))
        self.crf = CRF(num_entities)
        self.crf_mode, self.n = crf_mode, num_entities

    def emissions(self, inputs):
        h = self.tagger(self.enc(inputs[0], inputs[1]))
        return ops.linear(h, self.out_w, self.out_b).float()

    def loss(self, inputs, labels):
        e = self.emissions(inputs)
        tags = labels[0]
        if tags.dim() == 3:  # one-hot labels as in the reference
            tags = tags.argmax(-1)
        return self.crf.nll(e, tags, _mask(inputs, e.shape[1], self.crf_mode))

    def infer(self, inputs):
        e = self.emissions(inputs)
        path = self.crf.decode(e, _mask(inputs, e.shape[1], self.crf_mode))
        return torch.nn.functional.one_hot(path, self.n).float()


class NER(TextKerasModel):
    def __init__(self, num_entities, word_vocab_size, char_vocab_size, word_length=12, word_emb_dim=100,
                 char_emb_dim=30, tagger_lstm_dim=100, dropout=0.5, crf_mode="reg", optimizer=None):
        cfg = dict(num_entities=num_entities, word_vocab_size=word_vocab_size, char_vocab_size=char_vocab_size,
                   word_length=word_length, word_emb_dim=word_emb_dim, char_emb_dim=char_emb_dim,
                   tagger_lstm_dim=tagger_lstm_dim, dropout=dropout, crf_mode=crf_mode)
        if crf_mode not in ("reg", "pad"):
            raise ValueError("crf_mode must be 'reg' or 'pad'")
        super().__init__(_NERNet(num_entities, word_vocab_size, char_vocab_size, word_length, word_emb_dim,
                                 char_emb_dim, tagger_lstm_dim, dropout, crf_mode), optimizer, **cfg)

    @staticmethod
    def load_model(path):
        return NER._load(path)
