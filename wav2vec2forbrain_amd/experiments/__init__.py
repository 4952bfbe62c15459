"""Experiment layer (reference src/experiments): run.py builds one of these by name."""
