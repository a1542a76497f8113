from zoo.models.textclassification.text_classifier import TextClassifier  # noqa: F401
