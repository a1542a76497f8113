"""Import-path compatibility with the reference module ``zoo.automl.search.abstract`` (Py/automl/search/abstract.py):
the implementations live in the modules imported below."""
from zoo.automl.search import SearchEngine, GridSearch, RandomSample  # noqa: F401
