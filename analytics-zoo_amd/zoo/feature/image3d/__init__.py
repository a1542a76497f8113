from zoo.feature.image3d.transformation import (AffineTransform3D, CenterCrop3D, Crop3D, ImageFeature3D,  # noqa: F401
                                                RandomCrop3D, Rotate3D, Warp)
