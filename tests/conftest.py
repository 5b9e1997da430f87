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


LOGIT_TOL = 1e-3  # the north star's "logits within 1e-3"


def check_logit_windows(logits, g, row0=0, label=""):
    """Teacher-forced logits at the fixture's late windows (``win_steps``, 8 steps each, full
    rows for its first ``win_logits.shape[0]`` rows; ``oracle/gen_golden.py`` windows) against
    the reference's: max |d| per window printed as a PARITY_RECORD and held to 1e-3.  ``row0``:
    the fixture's first row in ``logits`` (a chain that holds other images first)."""
    ws, ref = g["win_steps"], g["win_logits"]
    assert ws.size and ref.shape[1] == ws.size, "fixture without late windows"
    got = logits[row0:row0 + ref.shape[0]][:, ws]
    d = np.abs(got - ref).max(axis=(0, 2))
    per = {f"{int(ws[i])}-{int(ws[i + 7])}": float(d[i:i + 8].max()) for i in range(0, ws.size, 8)}
    print("PARITY_RECORD", json.dumps({"logit_windows": label, "rows": int(ref.shape[0]), "row0": row0,
                                       "max_abs_err": per}))
    assert float(d.max()) < LOGIT_TOL, (label, per)
    return per
