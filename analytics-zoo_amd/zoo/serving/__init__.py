"""Cluster Serving: RESP queue server, serving workers, client queues, CLI, HTTP front end."""
from zoo.serving.client import InputQueue, OutputQueue  # noqa: F401
from zoo.serving.resp import RespClient, RespServer  # noqa: F401
from zoo.serving.server import ClusterServing, load_config, post_process  # noqa: F401
