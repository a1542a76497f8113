"""Import-path compatibility with the reference module ``zoo.feature.text.text_feature`` (Py/feature/text/text_feature.py):
the implementations live in the modules imported below."""
from zoo.feature.text.text_set import TextFeature  # noqa: F401
