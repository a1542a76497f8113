"""SessionRecommender (Zs/models/recommendation/SessionRecommender.scala:45-209,
Py session_recommender.py:30-140): GRU stack over the session's item
embeddings (+ optional MLP over the summed purchase-history embeddings),
softmax over items."""
import numpy as np

from zoo.models.recommendation.recommender import Recommender
from zoo.pipeline.api.keras.engine.topology import Model, merge
from zoo.pipeline.api.keras.layers import GRU, Activation, Dense, Embedding, Input, Lambda


class SessionRecommender(Recommender):
    def __init__(self, item_count, item_embed, rnn_hidden_layers=(40, 20), session_length=0, include_history=False,
                 mlp_hidden_layers=(40, 20), history_length=0, **kwargs):
        super().__init__(**kwargs)
        if session_length <= 0:
            raise ValueError("session_length should align with input features")
        if include_history and history_length <= 0:
            raise ValueError("history_length should align with input features")
        self.item_count, self.item_embed = int(item_count), int(item_embed)
        self.rnn_hidden_layers = [int(u) for u in rnn_hidden_layers]
        self.mlp_hidden_layers = [int(u) for u in mlp_hidden_layers]
        self.session_length, self.history_length = int(session_length), int(history_length)
        self.include_history = include_history
        self._init_model()

    def build_model(self):
        inp = Input(shape=(self.session_length,))
        h = Embedding(self.item_count + 1, self.item_embed, init="uniform")(inp)
        for u in self.rnn_hidden_layers[:-1]:
            h = GRU(u, return_sequences=True)(h)
        h = GRU(self.rnn_hidden_layers[-1], return_sequences=False)(h)
        rnn = Dense(self.item_count)(h)
        if not self.include_history:
            return Model(inp, Activation("softmax")(rnn))
        hist = Input(shape=(self.history_length,))
        t = Embedding(self.item_count + 1, self.item_embed, init="uniform")(hist)
        s = Lambda(lambda x: x.sum(1), output_shape=(self.item_embed,))(t)
        for u in self.mlp_hidden_layers:
            s = Dense(u, activation="relu")(s)
        mlp = Dense(self.item_count)(s)
        return Model([inp, hist], Activation("softmax")(merge([rnn, mlp], mode="sum")))

    def recommend_for_user(self, *a, **k):
        raise NotImplementedError("recommend_for_user: Unsupported for SessionRecommender")

    def recommend_for_item(self, *a, **k):
        raise NotImplementedError("recommend_for_item: Unsupported for SessionRecommender")

    def predict_user_item_pair(self, *a, **k):
        raise NotImplementedError("predict_user_item_pair: Unsupported for SessionRecommender")

    def recommend_for_session(self, sessions, max_items, zero_based_label=True):
        """-> per session: [(item, probability)] top ``max_items`` (1-based items unless zero_based)."""
        probs = np.asarray(self.predict(sessions))
        out = []
        for p in probs:
            top = np.argsort(-p, kind="stable")[:max_items]
            out.append([(int(i) + (0 if zero_based_label else 1), float(p[i])) for i in top])
        return out
