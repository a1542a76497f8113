from zoo.models.anomalydetection.anomaly_detector import AnomalyDetector, FeatureLabelIndex  # noqa: F401
