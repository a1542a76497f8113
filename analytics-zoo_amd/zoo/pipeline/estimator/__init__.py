from zoo.pipeline.estimator.estimator import Estimator, LocalEstimator, MultiOptimMethod, Predictor  # noqa: F401
