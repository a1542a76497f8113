"""KNRM kernel-pooling text matcher (Zs/models/textmatching/KNRM.scala:60-192, Py knrm.py:32-130).

The translation matrix (query x doc cosine of normalised embeddings) is one
batched GEMM; the K RBF kernels, the per-query log-sum and the sum over
query terms are one vectorised pass (:class:`KernelPooling`) instead of K
separate elementwise graphs."""
import torch

from zoo.models.textmatching.text_matcher import TextMatcher, prepare_embedding
from zoo.pipeline.api.keras.base import Layer
from zoo.pipeline.api.keras.engine.topology import Model
from zoo.pipeline.api.keras.layers import Dense, Embedding, Input


class KernelPooling(Layer):
    def __init__(self, text1_length, text2_length, kernel_num=21, sigma=0.1, exact_sigma=0.001, **kwargs):
        super().__init__(**kwargs)
        self.l1, self.l2, self.k = int(text1_length), int(text2_length), int(kernel_num)
        mus, sigmas = [], []
        for i in range(self.k):
            mu = 1.0 / (self.k - 1) + (2.0 * i) / (self.k - 1) - 1.0
            s = sigma
            if mu > 1.0:  # exact match kernel
                mu, s = 1.0, exact_sigma
            mus.append(mu)
            sigmas.append(s)
        self.register_buffer("mu", torch.tensor(mus))
        self.register_buffer("sigma", torch.tensor(sigmas))

    def compute_output_shape(self, input_shape):
        return (None, self.k)

    def call(self, emb):
        q, d = emb[:, :self.l1], emb[:, self.l1:self.l1 + self.l2]
        mm = torch.bmm(q.float(), d.float().transpose(1, 2))                      # [B, L1, L2]
        diff = mm.unsqueeze(-1) - self.mu                                            # [B, L1, L2, K]
        k = torch.exp(-0.5 * diff * diff / (self.sigma * self.sigma))
        return torch.log(k.sum(2) + 1.0).sum(1)                                      # [B, K]


class KNRM(TextMatcher):
    def __init__(self, text1_length, text2_length, embedding_file=None, word_index=None, train_embed=True,
                 kernel_num=21, sigma=0.1, exact_sigma=0.001, target_mode="ranking", embed_weights=None, **kwargs):
        if embed_weights is None:
            embed_weights = prepare_embedding(embedding_file, word_index, randomize_unknown=True, normalize=True)
        vocab, dim = embed_weights.shape
        super().__init__(text1_length, vocab, dim, embed_weights, train_embed, target_mode, **kwargs)
        if kernel_num <= 1:
            raise ValueError("kernel_num must be an int larger than 1")
        self.text2_length, self.kernel_num = int(text2_length), int(kernel_num)
        self.sigma, self.exact_sigma = float(sigma), float(exact_sigma)
        self._init_model()

    def build_model(self):
        inp = Input(shape=(self.text1_length + self.text2_length,))
        emb = Embedding(self.vocab_size, self.embed_size, weights=[self.embed_weights],
                        trainable=self.train_embed)(inp)
        phi = KernelPooling(self.text1_length, self.text2_length, self.kernel_num, self.sigma,
                            self.exact_sigma)(emb)
        act = None if self.target_mode == "ranking" else "sigmoid"
        return Model(inp, Dense(1, init="uniform", activation=act)(phi))
