#!/usr/bin/env python3
"""Anomaly detection on a time series (pyzoo/zoo/examples/anomalydetection/
anomaly_detection.py on NYC taxi): standardise, unroll into windows, train the LSTM
AnomalyDetector to predict the next value, flag the points with the largest prediction
error. ``--data nyc_taxi.csv`` (timestamp,value) or a synthetic daily-seasonal series with
injected spikes."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401
import numpy as np  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--data", default=None)
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--unroll", type=int, default=24)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--anomalies", type=int, default=5)
    a = ap.parse_args(argv)
    from zoo.common.nncontext import init_nncontext
    from zoo.models.anomalydetection import AnomalyDetector
    from zoo.pipeline.api.keras.optimizers import Adam
    init_nncontext("anomaly_detection")
    if a.data:
        import pandas as pd
        v = pd.read_csv(a.data)["value"].values.astype(np.float32)
    else:
        t = np.arange(a.n)
        v = (np.sin(2 * np.pi * t / 48) + 0.3 * np.sin(2 * np.pi * t / 336)).astype(np.float32)
        v += np.random.default_rng(0).normal(0, 0.05, a.n).astype(np.float32)
        for k in (a.n // 3, a.n // 2, 3 * a.n // 4):
            v[k] += 3.0
    v = (v - v.mean()) / v.std()
    un = AnomalyDetector.unroll(v.reshape(-1, 1), a.unroll)
    x, y, _ = AnomalyDetector.to_arrays(un)
    m = AnomalyDetector((a.unroll, 1), hidden_layers=(8, 32, 15), dropouts=(0.2, 0.2, 0.2))
    m.compile(optimizer=Adam(lr=0.005), loss="mse")
    m.fit(x, y, batch_size=a.batch, nb_epoch=a.epochs)
    pred = m.predict(x).reshape(-1)
    flags = AnomalyDetector.detect_anomalies(y, pred, anomaly_size=a.anomalies)
    found = [i + a.unroll for i, f in enumerate(flags) if f[2]]
    print("anomalies at:", found)
    return found


if __name__ == "__main__":
    main()
