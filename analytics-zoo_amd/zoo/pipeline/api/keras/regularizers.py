from zoo.pipeline.api.keras.base import Regularizer, l1, l2, l1l2  # noqa: F401

L1L2Regularizer = Regularizer
