"""Inverse-problem configs (reference: configs/inverse/**)."""
