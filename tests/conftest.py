import importlib
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

# Load torch (and its HIP runtime) before libmathocr.so so that one runtime is shared.
import torch  # noqa: E402,F401

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmathocr.so)")


@pytest.fixture(scope="session")
def pkg():
    return importlib.import_module("handwritten-math-ocr-api_amd")


def load_golden(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    out = {k: z[k] for k in z.files}
    out["meta"] = json.loads(str(out["meta"]))
    return out


@pytest.fixture(scope="session")
def golden():
    return load_golden
