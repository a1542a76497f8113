from zoo.models.recommendation.recommender import Recommender, UserItemFeature, UserItemPrediction  # noqa: F401
from zoo.models.recommendation.neuralcf import NeuralCF  # noqa: F401
