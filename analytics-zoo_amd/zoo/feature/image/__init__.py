from zoo.feature.image.imageset import DistributedImageSet, ImageSet, LocalImageSet  # noqa: F401
from zoo.feature.image.transforms import *  # noqa: F401,F403
