"""Keras-1 style API (zoo.pipeline.api.keras) on the MI355X engine."""
