"""Zouwu time-series toolkit (Py/zouwu)."""
