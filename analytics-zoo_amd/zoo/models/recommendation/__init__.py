from zoo.models.recommendation.neuralcf import NeuralCF  # noqa: F401
from zoo.models.recommendation.recommender import Recommender, UserItemFeature, UserItemPrediction  # noqa: F401
from zoo.models.recommendation.session_recommender import SessionRecommender  # noqa: F401
from zoo.models.recommendation.wide_and_deep import ColumnFeatureInfo, WideAndDeep  # noqa: F401
