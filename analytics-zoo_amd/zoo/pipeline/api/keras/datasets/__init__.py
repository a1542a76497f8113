"""Bundled dataset loaders (Py/pipeline/api/keras/datasets/{mnist,imdb,reuters,boston_housing}.py).

There is no network access: every loader reads files already present in
``dest_dir`` (the reference downloads them there first). Formats:
  mnist          the four IDX files (optionally .gz) of the original release
  imdb / reuters ``imdb.npz`` / ``reuters.npz`` with x_train, y_train, x_test, y_test
                 (object arrays are refused: sequences must be stored padded, or as
                 ``*_lengths`` + flat ``*_flat`` int arrays)
  boston_housing ``boston_housing.npz`` with x, y
Pickled files are never loaded.
"""
from zoo.pipeline.api.keras.datasets import boston_housing, imdb, mnist, reuters  # noqa: F401
