"""TimeSequenceModel (Py/automl/model/time_sequence.py:28-136): picks the concrete
model from ``config["model"]`` (LSTM, Seq2seq, MTNet) and forwards the BaseModel calls;
multi-step horizons (future_seq_len > 1) default to Seq2seq."""
from zoo.automl.model.abstract import BaseModel
from zoo.automl.model.MTNet_keras import MTNetKeras
from zoo.automl.model.Seq2Seq import LSTMSeq2Seq
from zoo.automl.model.VanillaLSTM import VanillaLSTM

MODEL_MAP = {"LSTM": VanillaLSTM, "Seq2seq": LSTMSeq2Seq, "MTNet": MTNetKeras}


class TimeSequenceModel(BaseModel):
    def __init__(self, check_optional_config=False, future_seq_len=None):
        self.check_optional_config = check_optional_config
        self.future_seq_len = future_seq_len
        self.model = None
        self.selected_model = None

    def _sel_model(self, config, verbose=0):
        name = config.get("model", "LSTM" if (self.future_seq_len or 1) == 1 else "Seq2seq")
        if name not in MODEL_MAP:
            raise ValueError("unknown model %r (one of %s)" % (name, sorted(MODEL_MAP)))
        self.selected_model = name
        return MODEL_MAP[name](check_optional_config=self.check_optional_config,
                               future_seq_len=self.future_seq_len or 1)

    def fit_eval(self, x, y, validation_data=None, mc=False, verbose=0, **config):
        if self.model is None:
            self.model = self._sel_model(config, verbose)
        return self.model.fit_eval(x, y, validation_data, mc=mc, verbose=verbose, **config)

    def evaluate(self, x, y, metric=("mse",)):
        return self.model.evaluate(x, y, list(metric))

    def predict(self, x, mc=False):
        return self.model.predict(x, mc=mc)

    def predict_with_uncertainty(self, x, n_iter=100):
        return self.model.predict_with_uncertainty(x, n_iter)

    def save(self, model_path, config_path):
        self.model.config["model"] = self.selected_model
        self.model.save(model_path, config_path)

    def restore(self, model_path, **config):
        self.future_seq_len = int(config.get("future_seq_len", self.future_seq_len or 1))
        self.model = self._sel_model(config)
        self.model.restore(model_path, **config)
        return self

    def _get_required_parameters(self):
        return self.model._get_required_parameters() if self.model else set()

    def _get_optional_parameters(self):
        return self.model._get_optional_parameters() if self.model else set()
