"""Py/util/*: nest (structure flatten/pack), engine (env prep), tf (graph export)."""
