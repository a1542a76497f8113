from zoo.automl.regression.time_sequence_predictor import TimeSequencePredictor  # noqa: F401
