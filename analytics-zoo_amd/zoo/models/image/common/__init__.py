from zoo.models.image.imageclassification.image_classifier import ImageConfigure, ImageModel  # noqa: F401
