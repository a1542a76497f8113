"""Seq2seq (Zs/models/seq2seq/Seq2seq.scala:50-302, RNNEncoder.scala, RNNDecoder.scala,
Bridge.scala; Py seq2seq.py:30-300).

model([encoder_input, decoder_input]) = generator(decoder(decoder_input,
bridge(encoder_final_states))); ``infer`` decodes greedily by feeding the
last predicted step back (Seq2seq.scala:114-165)."""
import numpy as np
import torch
import torch.nn as nn

from zoo.models.common.zoo_model import ZooModel
from zoo.pipeline.api.keras.base import Layer
from zoo.pipeline.api.keras.engine.topology import KerasNet
from zoo.pipeline.api.keras.layers import GRU, LSTM, Dense, SimpleRNN


def create_rnn(rnn_type, nlayers, hidden_size):
    t = rnn_type.lower()
    cls = {"lstm": LSTM, "gru": GRU, "simplernn": SimpleRNN}.get(t)
    if cls is None:
        raise ValueError("Only support lstm|gru|simplernn, got %s" % rnn_type)
    return [cls(hidden_size, return_sequences=True, return_state=True) for _ in range(nlayers)]


class RNNEncoder(Layer):
    def __init__(self, rnns, embedding=None, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.rnns = nn.ModuleList(rnns)
        self.embedding = embedding

    @classmethod
    def initialize(cls, rnn_type, nlayers, hidden_size, embedding=None, input_shape=None):
        return cls(create_rnn(rnn_type, nlayers, hidden_size), embedding, input_shape)

    def call(self, x):
        h = self.embedding(x) if self.embedding is not None else x
        states = []
        for r in self.rnns:
            out = r(h)
            h, st = out[0], out[1:]
            states.append(st)
        return h, states


class RNNDecoder(Layer):
    def __init__(self, rnns, embedding=None, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.rnns = nn.ModuleList(rnns)
        self.embedding = embedding

    @classmethod
    def initialize(cls, rnn_type, nlayers, hidden_size, embedding=None, input_shape=None):
        return cls(create_rnn(rnn_type, nlayers, hidden_size), embedding, input_shape)

    def call(self, x, init_states=None):
        if init_states is None and isinstance(x, (list, tuple)):
            x, init_states = x[0], x[1]
        h = self.embedding(x) if self.embedding is not None else x
        for i, r in enumerate(self.rnns):
            st = init_states[i] if init_states is not None and i < len(init_states) else None
            out = r([h] + list(st)) if st is not None else r(h)
            h = out[0]
        return h


class Bridge(Layer):
    """Maps encoder final states to decoder initial states: "dense" (linear),
    "densenonlinear" (tanh) or a custom layer applied to every state."""

    def __init__(self, bridge_type="dense", decoder_hidden_size=None, bridge=None, **kwargs):
        super().__init__(**kwargs)
        t = (bridge_type or "customized").lower()
        if bridge is None and t not in ("dense", "densenonlinear"):
            raise ValueError("Only support dense | densenonlinear as bridgeType")
        self.bridge_type, self.hidden = t, decoder_hidden_size
        self.custom = bridge
        self.maps = nn.ModuleList()

    @classmethod
    def initialize(cls, bridge_type, decoder_hidden_size):
        return cls(bridge_type, decoder_hidden_size)

    @classmethod
    def initialize_from_keras_layer(cls, bridge):
        return cls("customized", None, bridge)

    def call(self, states):
        flat = [s for layer in states for s in layer]
        if self.custom is not None:
            mapped = [self.custom(s) for s in flat]
        else:
            while len(self.maps) < len(flat):
                d = Dense(self.hidden, activation="tanh" if self.bridge_type == "densenonlinear" else None)
                d._ensure_built((None, flat[len(self.maps)].shape[-1]))
                self.maps.append(d.to(flat[0].device))
            mapped = [m(s) for m, s in zip(self.maps, flat)]
        out, i = [], 0
        for layer in states:
            out.append(mapped[i:i + len(layer)])
            i += len(layer)
        return out

    def build_for(self, states_shapes):
        """Create the dense maps eagerly (so they are registered before the optimizer)."""
        if self.custom is not None:
            return
        for d_in in states_shapes:
            d = Dense(self.hidden, activation="tanh" if self.bridge_type == "densenonlinear" else None)
            d._ensure_built((None, d_in))
            self.maps.append(d)


class Seq2seq(ZooModel):
    def __init__(self, encoder, decoder, input_shape, output_shape, bridge=None, generator=None, **kwargs):
        super().__init__(**kwargs)
        self.encoder, self.decoder, self.bridge, self.generator = encoder, decoder, bridge, generator
        self.in_shape, self.out_shape = tuple(input_shape), tuple(output_shape)
        self._build()

    def _build(self):
        enc_dim = self.in_shape[-1]
        d = enc_dim
        for r in self.encoder.rnns:
            r._ensure_built((None, self.in_shape[0], d))
            d = r.output_dim
        dec_dim = self.out_shape[-1]
        d = dec_dim
        for r in self.decoder.rnns:
            r._ensure_built((None, self.out_shape[0], d))
            d = r.output_dim
        if self.bridge is not None:
            shapes = [r.output_dim for r in self.encoder.rnns for _ in range(r._n_state)]
            self.bridge.build_for(shapes)
        if self.generator is not None:
            self.generator._ensure_built((None, self.out_shape[0], d))
        self.model = _Seq2seqNet(self)
        self.built = True
        self._input_shape = [(None,) + self.in_shape, (None,) + self.out_shape]

    def build_model(self):
        return self.model

    def forward(self, x, *rest):
        if rest:
            x = [x] + list(rest)
        return self.model(x)

    def infer(self, input, start_sign, max_seq_len=30, stop_sign=None, build_output=None):  # noqa: A002
        """Greedy decoding: feed the model's last output step back as the next decoder input."""
        dev = next(self.parameters()).device
        was = self.training
        self.eval()
        with torch.no_grad():
            src = torch.as_tensor(np.asarray(input), dtype=torch.float32, device=dev)
            if src.dim() == len(self.in_shape):
                src = src.unsqueeze(0)
            cur = torch.as_tensor(np.asarray(start_sign), dtype=torch.float32, device=dev).reshape(
                (1, 1) + tuple(np.asarray(start_sign).shape[-1:]))
            stop = None if stop_sign is None else torch.as_tensor(np.asarray(stop_sign), dtype=torch.float32,
                                                                   device=dev).reshape(-1)
            for _ in range(max_seq_len):
                out = self.model([src, cur])
                gen = build_output(out) if build_output is not None else out
                pred = gen[:, -1:]
                cur = torch.cat([cur, pred], 1)
                if stop is not None and torch.allclose(pred.reshape(-1), stop, atol=1e-8):
                    break
        self.train(was)
        return cur.cpu().numpy()


class _Seq2seqNet(KerasNet):
    def __init__(self, owner):
        super().__init__()
        self.encoder, self.decoder = owner.encoder, owner.decoder
        self.bridge, self.generator = owner.bridge, owner.generator
        self.built = True

    def _layer_list(self):
        return [m for m in (self.encoder, self.decoder, self.bridge, self.generator) if m is not None]

    def compute_output_shape(self, input_shape):
        return None

    def call(self, x):
        enc_in, dec_in = x
        _, states = self.encoder(enc_in)
        if self.bridge is not None:
            states = self.bridge(states)
        out = self.decoder(dec_in, states)
        return self.generator(out) if self.generator is not None else out

    def forward(self, x, *rest):
        if rest:
            x = [x] + list(rest)
        return self.call(x)
