"""Py/automl/common/util.py helpers: train / validation / test splitting of a time series
frame, JSON config files (merged on save), and the feature-transformer + model + config
save / restore bundle (a directory, or a zip of it) that pipelines are persisted as.

Reference: pyzoo/zoo/automl/common/util.py:28-263."""
import json
import os
import shutil
import tempfile
import zipfile

import numpy as np
import pandas as pd

CONFIG_FILE = "config.json"
MODEL_FILE = "weights_tune.h5"      # name kept for bundle compatibility; holds a torch state dict


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


def split_input_df(input_df, ts_col="timestamp", overlap=0, val_split_ratio=0, test_split_ratio=0.1):
    """Split a frame in time order into train / val / test (the tail); the time-stamp column
    becomes a ``datetime`` (datetime64) column in front. ``overlap`` rows of history are
    repeated at the start of val and test (the look-back a model needs there)."""
    df = input_df.copy()
    dt = pd.to_datetime(df[ts_col])
    df = df.drop(columns=ts_col)
    df.insert(0, "datetime", dt.values)
    n = len(df)
    val_n, test_n = int(n * val_split_ratio), int(n * test_split_ratio)
    train_df = df.iloc[:n - (val_n + test_n)]
    val_df = df.iloc[max(0, n - (val_n + test_n) - overlap):n - test_n].reset_index(drop=True)
    test_df = df.iloc[max(0, n - test_n - overlap):].reset_index(drop=True)
    return train_df, val_df, test_df


class NumpyEncoder(json.JSONEncoder):
    """numpy scalars / arrays -> JSON."""

    def default(self, obj):
        if isinstance(obj, np.integer):
            return int(obj)
        if isinstance(obj, np.floating):
            return float(obj)
        if isinstance(obj, np.bool_):
            return bool(obj)
        if isinstance(obj, np.ndarray):
            return obj.tolist()
        return super().default(obj)


def save_config(file_path, config, replace=False):
    """Write ``config`` as JSON; unless ``replace``, keys already in the file are kept and
    updated (so the feature transformer, the model and the trial config share one file)."""
    if os.path.isfile(file_path) and not replace:
        with open(file_path) as f:
            old = json.load(f)
        old.update(config)
        config = old
    d = os.path.dirname(os.path.abspath(file_path))
    os.makedirs(d, exist_ok=True)
    with open(file_path, "w") as f:
        json.dump(config, f, cls=NumpyEncoder)


def load_config(file_path):
    with open(file_path) as f:
        return json.load(f)


def save(file_path, feature_transformers=None, model=None, config=None):
    """Bundle directory: ``config.json`` (transformer state + model config + trial config)
    and the model weights."""
    os.makedirs(file_path, exist_ok=True)
    config_path = os.path.join(file_path, CONFIG_FILE)
    if feature_transformers is not None:
        feature_transformers.save(config_path, replace=True)
    if model is not None:
        model.save(os.path.join(file_path, MODEL_FILE), config_path)
    if config is not None:
        save_config(config_path, config)


def restore(file_path, feature_transformers=None, model=None, config=None):
    """Inverse of :func:`save`; ``config`` (if given) is overridden by the saved values.
    Returns the merged config."""
    local = load_config(os.path.join(file_path, CONFIG_FILE))
    all_config = dict(config or {})
    all_config.update(local)
    if model is not None:
        model.restore(os.path.join(file_path, MODEL_FILE), **all_config)
    if feature_transformers is not None:
        feature_transformers.restore(**all_config)
    return all_config


def save_zip(file, feature_transformers=None, model=None, config=None):
    d = os.path.dirname(os.path.abspath(file))
    os.makedirs(d, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix="automl_save_")
    try:
        save(tmp, feature_transformers=feature_transformers, model=model, config=config)
        with zipfile.ZipFile(file, "w") as zf:
            for name in sorted(os.listdir(tmp)):
                zf.write(os.path.join(tmp, name), name)
    finally:
        shutil.rmtree(tmp)
    return file


def restore_zip(file, feature_transformers=None, model=None, config=None):
    tmp = tempfile.mkdtemp(prefix="automl_restore_")
    try:
        with zipfile.ZipFile(file) as zf:
            for name in zf.namelist():      # flat bundle: refuse paths that leave the directory
                if os.path.isabs(name) or ".." in name.replace("\\", "/").split("/"):
                    raise ValueError("unsafe entry %r in %s" % (name, file))
            zf.extractall(tmp)
        return restore(tmp, feature_transformers, model, config)
    finally:
        shutil.rmtree(tmp)
