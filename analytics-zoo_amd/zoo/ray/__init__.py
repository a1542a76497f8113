"""Ray-style task/actor runtime (Py/ray/*: RayContext, ProcessMonitor, utils) and
distributed trainers on top of it (Py/ray/mxnet/*). See raycontext.py."""
from zoo.ray.process import ProcessInfo, ProcessMonitor, session_execute  # noqa: F401
from zoo.ray.raycontext import (ActorHandle, ObjectRef, RayContext, get, put, remote,  # noqa: F401
                                wait)
from zoo.ray.utils import is_local, resource_to_bytes, to_list  # noqa: F401
