"""IntentEntity (Py/tfpark/text/keras/intent_extraction.py:21-73): joint intent
classification and slot filling. Shared word + char features -> BiLSTM; the
intent head reads the final states, the slot head a second BiLSTM + CRF.
Outputs: [intent probabilities [B, num_intents], entity tags one-hot [B, T, num_entities]]."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo import ops
from zoo.tfpark.text.keras.text_model import CRF, CharWordEncoder, TextKerasModel, bilstm


class _IntentNet(nn.Module):
    def __init__(self, num_intents, num_entities, word_vocab_size, char_vocab_size, word_length, word_emb_dim,
                 char_emb_dim, char_lstm_dim, tagger_lstm_dim, dropout):
        super().__init__()
        self.enc = CharWordEncoder(word_vocab_size, char_vocab_size, word_emb_dim, char_emb_dim, char_lstm_dim,
                                   dropout)
        self.shared = bilstm(self.enc.out_dim, tagger_lstm_dim)
        self.slot_lstm = bilstm(2 * tagger_lstm_dim, tagger_lstm_dim)
        H = 2 * tagger_lstm_dim
        self.intent_w = nn.Parameter(torch.empty(num_intents, H).uniform_(-0.05, 0.05))
        self.intent_b = nn.Parameter(torch.zeros(num_intents))
        self.slot_w = nn.Parameter(torch.empty(num_entities, H).uniform_(-0.05, 0.05))
        self.slot_b = nn.Parameter(torch.zeros(num_entities))
        self.crf = CRF(num_entities)
        self.n_ent, self.dropout, self.H = num_entities, dropout, tagger_lstm_dim

    def _heads(self, inputs):
        h = self.shared(self.enc(inputs[0], inputs[1]))
        # intent from the forward direction's last state and the backward direction's first
        summary = torch.cat([h[:, -1, :self.H], h[:, 0, self.H:]], -1)
        intent = ops.linear(F.dropout(summary, self.dropout, self.training), self.intent_w, self.intent_b).float()
        s = self.slot_lstm(h)
        slots = ops.linear(s, self.slot_w, self.slot_b).float()
        return intent, slots

    def loss(self, inputs, labels):
        intent, slots = self._heads(inputs)
        yi, ys = labels[0], labels[1]
        yi = yi.argmax(-1) if yi.dim() > 1 and yi.shape[-1] > 1 else yi.reshape(-1)
        ys = ys.argmax(-1) if ys.dim() == 3 else ys
        return F.cross_entropy(intent, yi.long()) + self.crf.nll(slots, ys)

    def infer(self, inputs):
        intent, slots = self._heads(inputs)
        return [torch.softmax(intent, -1), F.one_hot(self.crf.decode(slots), self.n_ent).float()]


class IntentEntity(TextKerasModel):
    def __init__(self, num_intents, num_entities, word_vocab_size, char_vocab_size, word_length=12,
                 word_emb_dim=100, char_emb_dim=30, char_lstm_dim=30, tagger_lstm_dim=100, dropout=0.2,
                 optimizer=None):
        cfg = dict(num_intents=num_intents, num_entities=num_entities, word_vocab_size=word_vocab_size,
                   char_vocab_size=char_vocab_size, word_length=word_length, word_emb_dim=word_emb_dim,
                   char_emb_dim=char_emb_dim, char_lstm_dim=char_lstm_dim, tagger_lstm_dim=tagger_lstm_dim,
                   dropout=dropout)
        super().__init__(_IntentNet(num_intents, num_entities, word_vocab_size, char_vocab_size, word_length,
                                    word_emb_dim, char_emb_dim, char_lstm_dim, tagger_lstm_dim, dropout),
                         optimizer, **cfg)

    @staticmethod
    def load_model(path):
        return IntentEntity._load(path)
