from zoo.models.common.zoo_model import ZooModel, KerasZooModel  # noqa: F401
from zoo.models.common.ranker import Ranker  # noqa: F401
