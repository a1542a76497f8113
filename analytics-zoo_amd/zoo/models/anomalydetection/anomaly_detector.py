"""AnomalyDetector (Zs/models/anomalydetection/AnomalyDetector.scala:40-222,
Py anomaly_detector.py:30-190): stacked LSTM regression over unrolled
windows; ``detect_anomalies`` flags the points with the largest
|truth - prediction|."""
import numpy as np

from zoo.models.common.zoo_model import ZooModel
from zoo.pipeline.api.keras.layers import LSTM, Dense, Dropout
from zoo.pipeline.api.keras.models import Sequential


class FeatureLabelIndex:
    def __init__(self, feature, label, index):
        self.feature, self.label, self.index = np.asarray(feature, np.float32), float(label), int(index)

    def __repr__(self):
        return "FeatureLabelIndex(index=%d, label=%s)" % (self.index, self.label)


class AnomalyDetector(ZooModel):
    def __init__(self, feature_shape, hidden_layers=(8, 32, 15), dropouts=(0.2, 0.2, 0.2), **kwargs):
        super().__init__(**kwargs)
        if len(hidden_layers) != len(dropouts):
            raise ValueError("sizes of dropouts and hidden_layers should be equal")
        self.feature_shape = tuple(int(s) for s in feature_shape)
        self.hidden_layers = [int(h) for h in hidden_layers]
        self.dropouts = [float(d) for d in dropouts]
        self._init_model()

    def build_model(self):
        m = Sequential()
        m.add(LSTM(self.hidden_layers[0], return_sequences=True, input_shape=self.feature_shape))
        m.add(Dropout(self.dropouts[0]))
        for h, d in zip(self.hidden_layers[1:-1], self.dropouts[1:-1]):
            m.add(LSTM(h, return_sequences=True))
            m.add(Dropout(d))
        m.add(LSTM(self.hidden_layers[-1], return_sequences=False))
        m.add(Dropout(self.dropouts[-1]))
        m.add(Dense(1))
        return m

    @staticmethod
    def unroll(data, unroll_length, predict_step=1):
        """[T, F] series -> FeatureLabelIndex windows: feature = rows [i, i+L), label = data[i+L+step-1, 0]."""
        a = np.asarray(data, np.float32)
        a = a.reshape(len(a), -1)
        out = []
        for i in range(len(a) - unroll_length - predict_step + 1):
            out.append(FeatureLabelIndex(a[i:i + unroll_length], a[i + unroll_length + predict_step - 1, 0], i))
        return out

    @staticmethod
    def to_arrays(unrolled):
        return (np.stack([u.feature for u in unrolled]), np.array([u.label for u in unrolled], np.float32),
                np.array([u.index for u in unrolled]))

    @staticmethod
    def detect_anomalies(ytruth, ypredict, anomaly_size=5):
        """-> [(truth, predict, is_anomaly)] marking the ``anomaly_size`` largest distances."""
        t = np.asarray(ytruth, np.float64).reshape(-1)
        p = np.asarray(ypredict, np.float64).reshape(-1)
        dist = np.abs(t - p)
        thr = np.sort(dist)[-anomaly_size] if anomaly_size > 0 else np.inf
        return [(float(a), float(b), bool(d >= thr)) for a, b, d in zip(t, p, dist)]

    @staticmethod
    def standard_scale(x):
        x = np.asarray(x, np.float64)
        return (x - x.mean(0)) / np.where(x.std(0) > 0, x.std(0), 1.0)

    @staticmethod
    def train_test_split(unrolled, test_size):
        n = len(unrolled) - int(test_size) if test_size >= 1 else int(len(unrolled) * (1 - test_size))
        return unrolled[:n], unrolled[n:]
