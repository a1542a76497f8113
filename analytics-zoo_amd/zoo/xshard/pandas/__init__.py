from zoo.xshard.pandas.preprocessing import read_csv, read_json, RayPandasShard  # noqa: F401
