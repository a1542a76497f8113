"""Import-path compatibility with the reference module ``zoo.feature.text.transformer`` (Py/feature/text/transformer.py):
the implementations live in the modules imported below."""
from zoo.feature.text.text_set import Tokenizer, Normalizer, WordIndexer, SequenceShaper, TextFeatureToSample  # noqa: F401
