from zoo.common.nncontext import *  # noqa: F401,F403
