"""MI355X-native engine for the Swin-T + 8-layer decoder greedy-decode hot path."""
from . import synth  # noqa: F401
