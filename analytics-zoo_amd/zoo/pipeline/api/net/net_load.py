"""Import-path compatibility with the reference module ``zoo.pipeline.api.net.net_load`` (Py/pipeline/api/net/net_load.py):
the implementations live in the modules imported below."""
from zoo.pipeline.api.net.net import Net  # noqa: F401
