"""MTNetKeras (Py/automl/model/MTNet_keras.py:95-606): the memory time-series network.
The past window is ``(long_num + 1) * time_step`` steps: ``long_num`` memory blocks and
one short-term block, each encoded by Conv1D + GRU; the short-term encoding attends
over the memory encodings and an autoregressive term on the target is added."""
import numpy as np

from zoo.automl.model._nets import MTNetNet
from zoo.automl.model._torch_model import TorchTSModel


class MTNetKeras(TorchTSModel):
    net_cls = MTNetNet
    required = {"long_num", "time_step"}
    optional = {"ar_window", "cnn_height", "cnn_hid_size", "rnn_hid_sizes", "dropout", "lr", "batch_size",
                "epochs", "metric"}

    def _reshape_input(self, x):
        x = np.asarray(x, np.float32)
        cfg = self.config
        if "long_num" in cfg and "time_step" in cfg:
            need = (int(cfg["long_num"]) + 1) * int(cfg["time_step"])
            if x.shape[1] < need:
                raise ValueError("MTNet needs a past window of (long_num + 1) * time_step = %d steps, got %d"
                                 % (need, x.shape[1]))
            x = x[:, -need:]
        return x

    @staticmethod
    def past_seq_len(long_num, time_step):
        return (int(long_num) + 1) * int(time_step)


__all__ = ["MTNetKeras"]
