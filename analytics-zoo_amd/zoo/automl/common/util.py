"""Py/automl/common/util.py helpers used by the search engine."""


def convert_bayes_configs(config):
    """A point of a Bayesian-optimisation space (all floats) -> a trial config
    (Py/automl/common/util.py:242): ``bayes_feature_<f>`` >= 0.5 selects feature f,
    ``batch_size_log`` -> 2**x, ``<name>_float`` -> int(<name>)."""
    selected, out = [], {}
    for k, v in config.items():
        if k.startswith("bayes_feature_"):
            if v >= 0.5:
                selected.append(k[len("bayes_feature_"):])
        elif k == "batch_size_log":
            out["batch_size"] = int(2 ** v)
        elif k.endswith("_float"):
            out[k[:-len("_float")]] = int(v)
        else:
            out[k] = v
    if selected:
        out["selected_features"] = selected
    return out
