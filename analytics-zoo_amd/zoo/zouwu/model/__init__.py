from zoo.zouwu.model.forecast import LSTMForecaster, MTNetForecaster  # noqa: F401
