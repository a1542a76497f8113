"""Search recipes (Py/automl/config/recipe.py:22-460)."""
import numpy as np

from zoo.automl.search import GridSearch, RandomSample


class Recipe:
    num_samples = 1
    training_iteration = 1

    def search_space(self, all_available_features):
        raise NotImplementedError

    def runtime_params(self):
        return {"training_iteration": self.training_iteration, "num_samples": self.num_samples}

    def fixed_params(self):
        return {}

    def search_algorithm(self):
        return None

    def search_algorithm_params(self):
        return None


def _past(look_back):
    """past_seq_len search config from ``look_back``: an int >= 2, or an (min, max) int tuple
    sampled uniformly (a min below 2 is raised to 2) -- recipe.py:117-152 semantics."""
    if isinstance(look_back, tuple) and len(look_back) == 2 and all(isinstance(v, int) and not isinstance(v, bool)
                                                                   for v in look_back):
        lo, hi = look_back
        if hi < 2:
            raise ValueError("The max look back value should be at least 2")
        lo = max(2, lo)
        return RandomSample(lambda spec: int(np.random.randint(lo, hi + 1)))
    if isinstance(look_back, int) and not isinstance(look_back, bool):
        if look_back < 2:
            raise ValueError("look back value should not be smaller than 2. Current value is %s" % look_back)
        return look_back
    raise ValueError("look back is %r.\n look_back should be either a tuple with 2 int values: (min_len, max_len) "
                     "or a single int" % (look_back,))


class SmokeRecipe(Recipe):
    def search_space(self, all_available_features):
        return {"selected_features": list(all_available_features), "model": "LSTM",
                "lstm_1_units": RandomSample(lambda s: int(np.random.choice([32, 64]))),
                "dropout_1": RandomSample(lambda s: float(np.random.uniform(0.2, 0.5))),
                "lstm_2_units": RandomSample(lambda s: int(np.random.choice([32, 64]))),
                "dropout_2": RandomSample(lambda s: float(np.random.uniform(0.2, 0.5))),
                "lr": 0.001, "batch_size": 1024, "epochs": 1, "past_seq_len": 2}


class MTNetSmokeRecipe(Recipe):
    def search_space(self, all_available_features):
        return {"selected_features": list(all_available_features), "model": "MTNet", "lr": 0.001,
                "batch_size": 16, "epochs": 1, "dropout": 0.2, "time_step": 2, "long_num": 2, "ar_window": 2,
                "cnn_height": 2, "cnn_hid_size": 16, "rnn_hid_sizes": [16], "past_seq_len": 6}


def _random_features(all_features):
    def f(spec):
        n = len(all_features)
        k = int(np.random.randint(min(3, n), n + 1)) if n > 0 else 0
        return list(np.random.choice(all_features, size=k, replace=False)) if k else []
    return RandomSample(f)


class GridRandomRecipe(Recipe):
    def __init__(self, num_rand_samples=1, look_back=2, epochs=5, training_iteration=10):
        self.num_samples, self.training_iteration, self.epochs = num_rand_samples, training_iteration, epochs
        self.past = _past(look_back)

    def search_space(self, all_available_features):
        return {"selected_features": _random_features(all_available_features),
                "model": RandomSample(lambda s: str(np.random.choice(["LSTM", "Seq2seq"]))),
                "lstm_1_units": GridSearch([16, 32]), "dropout_1": 0.2, "lstm_2_units": GridSearch([16, 32]),
                "dropout_2": RandomSample(lambda s: float(np.random.uniform(0.2, 0.5))),
                "latent_dim": GridSearch([32, 64]),
                "dropout": RandomSample(lambda s: float(np.random.uniform(0.2, 0.5))),
                "lr": RandomSample(lambda s: float(np.random.uniform(0.001, 0.01))),
                "batch_size": RandomSample(lambda s: int(np.random.choice([32, 64]))),
                "epochs": self.epochs, "past_seq_len": self.past}


class LSTMGridRandomRecipe(Recipe):
    def __init__(self, num_rand_samples=1, epochs=5, training_iteration=10, look_back=2, lstm_1_units=(16, 32),
                 lstm_2_units=(8, 16), batch_size=(32, 64)):
        self.num_samples, self.training_iteration, self.epochs = num_rand_samples, training_iteration, epochs
        self.past = _past(look_back)
        self.l1, self.l2, self.bs = list(lstm_1_units), list(lstm_2_units), list(batch_size)

    def search_space(self, all_available_features):
        return {"selected_features": _random_features(all_available_features), "model": "LSTM",
                "lstm_1_units": GridSearch(self.l1), "dropout_1": 0.2, "lstm_2_units": GridSearch(self.l2),
                "dropout_2": RandomSample(lambda s: float(np.random.uniform(0.2, 0.5))),
                "lr": RandomSample(lambda s: float(np.random.uniform(0.001, 0.01))),
                "batch_size": GridSearch(self.bs), "epochs": self.epochs, "past_seq_len": self.past}


class MTNetGridRandomRecipe(Recipe):
    def __init__(self, num_rand_samples=1, epochs=5, training_iteration=10, time_step=(3, 4), long_num=(3, 4),
                 cnn_height=(2, 3), cnn_hid_size=(32, 50), ar_size=(2, 3), batch_size=(32, 64)):
        self.num_samples, self.training_iteration, self.epochs = num_rand_samples, training_iteration, epochs
        self.time_step, self.long_num, self.cnn_height = list(time_step), list(long_num), list(cnn_height)
        self.cnn_hid, self.ar, self.bs = list(cnn_hid_size), list(ar_size), list(batch_size)

    def search_space(self, all_available_features):
        ts, ln = self.time_step, self.long_num
        return {"selected_features": _random_features(all_available_features), "model": "MTNet",
                "lr": 0.001, "batch_size": GridSearch(self.bs), "epochs": self.epochs,
                "dropout": RandomSample(lambda s: float(np.random.uniform(0.2, 0.5))),
                "time_step": RandomSample(lambda s: int(np.random.choice(ts))),
                "long_num": RandomSample(lambda s: int(np.random.choice(ln))),
                "cnn_height": RandomSample(lambda s: int(np.random.choice(self.cnn_height))),
                "cnn_hid_size": RandomSample(lambda s: int(np.random.choice(self.cnn_hid))),
                "ar_window": RandomSample(lambda s: int(np.random.choice(self.ar))),
                "rnn_hid_sizes": [16],
                "past_seq_len": RandomSample(lambda s: (s["long_num"] + 1) * s["time_step"])}


class RandomRecipe(Recipe):
    def __init__(self, num_rand_samples=1, look_back=2, epochs=5, reward_metric=-0.05, training_iteration=10):
        self.num_samples, self.training_iteration, self.epochs = num_rand_samples, training_iteration, epochs
        self.past = _past(look_back)

    def search_space(self, all_available_features):
        return {"selected_features": _random_features(all_available_features),
                "model": RandomSample(lambda s: str(np.random.choice(["LSTM", "Seq2seq"]))),
                "lstm_1_units": RandomSample(lambda s: int(np.random.choice([8, 16, 32, 64, 128]))),
                "dropout_1": RandomSample(lambda s: float(np.random.uniform(0.2, 0.5))),
                "lstm_2_units": RandomSample(lambda s: int(np.random.choice([8, 16, 32, 64, 128]))),
                "dropout_2": RandomSample(lambda s: float(np.random.uniform(0.2, 0.5))),
                "latent_dim": RandomSample(lambda s: int(np.random.choice([32, 64, 128, 256]))),
                "dropout": RandomSample(lambda s: float(np.random.uniform(0.2, 0.5))),
                "lr": RandomSample(lambda s: float(np.random.uniform(0.001, 0.01))),
                "batch_size": RandomSample(lambda s: int(np.random.choice([32, 64, 1024]))),
                "epochs": self.epochs, "past_seq_len": self.past}


class BayesRecipe(Recipe):
    """Bayesian-optimisation recipe (Py/automl/config/recipe.py:423-518): a continuous box
    space searched by GP-UCB (zoo.automl.search.BayesOptSearch). Feature selection is a
    ``bayes_feature_<f>`` in (0.3, 1) thresholded at 0.5; integer knobs are ``*_float``
    ranges truncated to int; the batch size is 2**``batch_size_log``."""

    def __init__(self, num_samples=1, look_back=2, epochs=5, reward_metric=-0.05, training_iteration=5):
        self.num_samples, self.reward_metric = int(num_samples), reward_metric
        self.training_iteration, self.epochs = training_iteration, epochs
        if isinstance(look_back, tuple) and len(look_back) == 2 and all(isinstance(v, int) for v in look_back):
            if look_back[1] < 2:
                raise ValueError("The max look back value should be at least 2")
            self.bayes_past = {"past_seq_len_float": (max(2, look_back[0]), look_back[1])}
            self.fixed_past = {}
        elif isinstance(look_back, int):
            if look_back < 2:
                raise ValueError("look back value should not be smaller than 2")
            self.bayes_past, self.fixed_past = {}, {"past_seq_len": look_back}
        else:
            raise ValueError("look_back should be either a tuple with 2 int values (min_len, max_len) "
                             "or a single int")

    def search_space(self, all_available_features):
        space = {"bayes_feature_%s" % f: (0.3, 1) for f in all_available_features}
        space.update({"lstm_1_units_float": (8, 128), "dropout_1": (0.2, 0.5), "lstm_2_units_float": (8, 128),
                      "dropout_2": (0.2, 0.5), "lr": (0.001, 0.01), "batch_size_log": (5, 10)})
        space.update(self.bayes_past)
        return space

    def fixed_params(self):
        return dict({"epochs": self.epochs, "model": "LSTM"}, **self.fixed_past)

    def search_algorithm_params(self):
        return {"utility_kwargs": {"kind": "ucb", "kappa": 2.5, "xi": 0.0}}

    def search_algorithm(self):
        return "BayesOpt"
