from zoo.pipeline.nnframes.nn_classifier import (NNClassifier, NNClassifierModel, NNEstimator, NNModel,  # noqa: F401
                                                 Pipeline, PipelineModel)
from zoo.pipeline.nnframes.nn_image_reader import NNImageReader, with_origin_column  # noqa: F401
