from zoo.zouwu.autots.forecast import AutoTSTrainer, TSPipeline  # noqa: F401
