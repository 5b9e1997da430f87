"""MI355X-native engine for the Swin-T + 8-layer decoder greedy-decode hot path of
PTD504/handwritten-math-ocr-api.

The package directory name contains hyphens, so import it with
``importlib.import_module("handwritten-math-ocr-api_amd")``.
"""
from . import config, im2latex, inference, parallel, pipeline, predict, preprocess, synth, utils, weights  # noqa: F401
from .engine import DecodeResult, Engine, MocrError, load_library  # noqa: F401
