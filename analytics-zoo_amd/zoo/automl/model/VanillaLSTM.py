"""VanillaLSTM (Py/automl/model/VanillaLSTM.py:28-205): two stacked LSTMs with dropout
and a dense head over the last step, predicting ``future_seq_len`` values."""
from zoo.automl.model._nets import VanillaLSTMNet
from zoo.automl.model._torch_model import TorchTSModel


class VanillaLSTM(TorchTSModel):
    """Reference defaults: lstm_1_units 20, lstm_2_units 10, dropouts 0.2, batch 1024, MSE with
    RMSprop(lr 0.001)."""
    net_cls = VanillaLSTMNet
    default_batch_size = 1024

    def _optimizer(self, cfg):
        from zoo.pipeline.api.keras.optimizers import RMSprop
        return RMSprop(learningrate=float(cfg.get("lr", 1e-3)), decayrate=0.9, epsilon=1e-7)
    required = set()
    optional = {"lstm_1_units", "dropout_1", "lstm_2_units", "dropout_2", "lr", "batch_size", "epochs", "metric"}


__all__ = ["VanillaLSTM"]
