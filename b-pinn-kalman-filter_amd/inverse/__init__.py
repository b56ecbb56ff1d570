"""Measurement operators of the inverse / PINN pipelines (reference inverse/)."""
