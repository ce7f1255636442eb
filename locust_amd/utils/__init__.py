"""Utilities: independent oracle, synthetic text generator, metrics."""
