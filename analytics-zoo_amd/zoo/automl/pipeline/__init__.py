from zoo.automl.pipeline.time_sequence import TimeSequencePipeline, load_ts_pipeline  # noqa: F401
