"""Kernel-level operations exposed for tests and tools (device string library, sort)."""
from .strings import itoa, pack_key, strcmp, strtok_r_tokens

__all__ = ["itoa", "pack_key", "strcmp", "strtok_r_tokens"]
