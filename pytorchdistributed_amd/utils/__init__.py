"""Utilities: logging, timing, profiling ranges, checkpoints, fault injection, config, model summary."""
