"""SequenceTagger (Py/tfpark/text/keras/pos_tagging.py:21-75): POS tagging and
chunking. Word (+ optional character) features -> stacked BiLSTMs; POS is read
from the first layer, chunk tags from the last (softmax, or CRF with
``classifier='crf'``). Outputs: [pos probabilities [B, T, P], chunk [B, T, C]]."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo import ops
from zoo.tfpark.text.keras.text_model import CRF, CharWordEncoder, TextKerasModel, bilstm


class _TaggerNet(nn.Module):
    def __init__(self, num_pos_labels, num_chunk_labels, word_vocab_size, char_vocab_size, word_length,
                 feature_size, dropout, classifier, num_lstm_layers):
        super().__init__()
        self.use_chars = char_vocab_size is not None
        if self.use_chars:
            self.enc = CharWordEncoder(word_vocab_size, char_vocab_size, feature_size, 25, 25, dropout)
            d = self.enc.out_dim
        else:
            self.word = nn.Parameter(torch.empty(word_vocab_size, feature_size).uniform_(-0.05, 0.05))
            d = feature_size
        self.layers = nn.ModuleList([bilstm(d if i == 0 else 2 * feature_size, feature_size)
                                     for i in range(max(int(num_lstm_layers), 1))])
        self.pos_w = nn.Parameter(torch.empty(num_pos_labels, 2 * feature_size).uniform_(-0.05, 0.05))
        self.pos_b = nn.Parameter(torch.zeros(num_pos_labels))
        self.chunk_w = nn.Parameter(torch.empty(num_chunk_labels, 2 * feature_size).uniform_(-0.05, 0.05))
        self.chunk_b = nn.Parameter(torch.zeros(num_chunk_labels))
        self.crf = CRF(num_chunk_labels) if classifier == "crf" else None
        self.dropout, self.n_chunk, self.in_dim = dropout, num_chunk_labels, d

    def _heads(self, inputs):
        if self.use_chars:
            x = self.enc(inputs[0], inputs[1])
        else:
            x = F.dropout(ops.embedding(inputs[0].long(), self.word), self.dropout, self.training)
        first = None
        for layer in self.layers:
            x = layer(x)
            first = x if first is None else first
        pos = ops.linear(first, self.pos_w, self.pos_b).float()
        chunk = ops.linear(x, self.chunk_w, self.chunk_b).float()
        return pos, chunk

    def loss(self, inputs, labels):
        pos, chunk = self._heads(inputs)
        yp = labels[0].argmax(-1) if labels[0].dim() == 3 else labels[0]
        yc = labels[1].argmax(-1) if labels[1].dim() == 3 else labels[1]
        lp = F.cross_entropy(pos.reshape(-1, pos.shape[-1]), yp.reshape(-1).long())
        if self.crf is not None:
            return lp + self.crf.nll(chunk, yc)
        return lp + F.cross_entropy(chunk.reshape(-1, chunk.shape[-1]), yc.reshape(-1).long())

    def infer(self, inputs):
        pos, chunk = self._heads(inputs)
        c = F.one_hot(self.crf.decode(chunk), self.n_chunk).float() if self.crf is not None \
            else torch.softmax(chunk, -1)
        return [torch.softmax(pos, -1), c]


class SequenceTagger(TextKerasModel):
    def __init__(self, num_pos_labels, num_chunk_labels, word_vocab_size, char_vocab_size=None, word_length=12,
                 feature_size=100, dropout=0.2, classifier="softmax", optimizer=None, num_lstm_layers=2):
        if classifier not in ("softmax", "crf"):
            raise ValueError("classifier must be 'softmax' or 'crf'")
        cfg = dict(num_pos_labels=num_pos_labels, num_chunk_labels=num_chunk_labels,
                   word_vocab_size=word_vocab_size, char_vocab_size=char_vocab_size, word_length=word_length,
                   feature_size=feature_size, dropout=dropout, classifier=classifier,
                   num_lstm_layers=num_lstm_layers)
        super().__init__(_TaggerNet(num_pos_labels, num_chunk_labels, word_vocab_size, char_vocab_size, word_length,
                                    feature_size, dropout, classifier, num_lstm_layers), optimizer, **cfg)

    @staticmethod
    def load_model(path):
        return SequenceTagger._load(path)


POSTagger = SequenceTagger
