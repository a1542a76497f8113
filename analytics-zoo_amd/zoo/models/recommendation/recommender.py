"""Recommender base + UserItemFeature / UserItemPrediction
(Zs/models/recommendation/Recommender.scala:36-105, Py/models/recommendation/recommender.py)."""
import numpy as np

from zoo.models.common.zoo_model import ZooModel


class UserItemFeature:
    def __init__(self, user_id, item_id, sample):
        self.user_id, self.item_id, self.sample = int(user_id), int(item_id), sample

    def __repr__(self):
        return "UserItemFeature[user_id: %s, item_id: %s]" % (self.user_id, self.item_id)


class UserItemPrediction:
    def __init__(self, user_id, item_id, prediction, probability):
        self.user_id, self.item_id = int(user_id), int(item_id)
        self.prediction, self.probability = int(prediction), float(probability)

    def __repr__(self):
        return "UserItemPrediction[user_id: %s, item_id: %s, prediction: %s, probability: %s]" % (
            self.user_id, self.item_id, self.prediction, self.probability)


class Recommender(ZooModel):
    def _predict_features(self, features):
        xs = [f.sample[0] if isinstance(f.sample, (list, tuple)) else f.sample for f in features]
        if isinstance(xs[0], (list, tuple)):
            x = [np.stack([np.asarray(s[i]) for s in xs]) for i in range(len(xs[0]))]
        else:
            x = np.stack([np.asarray(s) for s in xs])
        probs = self.predict(x)
        return probs

    def predict_user_item_pair(self, features):
        features = list(features)
        probs = self._predict_features(features)
        out = []
        for f, p in zip(features, probs):
            c = int(np.argmax(p))
            out.append(UserItemPrediction(f.user_id, f.item_id, c + 1, float(p[c])))
        return out

    def recommend_for_user(self, features, max_items):
        preds = self.predict_user_item_pair(features)
        by_user = {}
        for p in preds:
            by_user.setdefault(p.user_id, []).append(p)
        out = []
        for u, ps in by_user.items():
            ps.sort(key=lambda q: (q.prediction, q.probability), reverse=True)
            out.extend(ps[:max_items])
        return out

    def recommend_for_item(self, features, max_users):
        preds = self.predict_user_item_pair(features)
        by_item = {}
        for p in preds:
            by_item.setdefault(p.item_id, []).append(p)
        out = []
        for i, ps in by_item.items():
            ps.sort(key=lambda q: (q.prediction, q.probability), reverse=True)
            out.extend(ps[:max_users])
        return out
