from zoo.models.image.imageclassification.image_classifier import (ImageClassifier, ImageConfigure,  # noqa: F401
                                                                   ImageModel, LabelOutput)
