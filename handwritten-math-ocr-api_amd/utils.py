"""Tokenizer / vocabulary helpers of the serving path (``app/src/utils.py``).

These are the reference's host-side string functions, restated so that the engine's
token ids turn into the same strings the reference returns:

* ``tokenize_latex``     — ``app/src/utils.py:5-8`` (LaTeX command, brace/script/special
  character, digit run, letter run, or any other non-space character);
* ``load_vocab``         — ``app/src/utils.py:10-15`` (``vocab.json`` with ``vocab`` and
  ``idx2char``; idx2char keys become ints);
* ``tokens_to_latex``    — ``app/src/utils.py:17-20`` (drop sos/eos/pad and ids missing
  from the vocabulary, join with single spaces);
* ``clean_latex_output`` — ``app/src/utils.py:22-27`` (four regex fix-ups);
* ``detokenize``         — ``src/inference.py:29-40`` (batched path: skip sos/pad, stop at
  eos, join with spaces).
"""
from __future__ import annotations

import json
import re

SOS, EOS, PAD, UNK = "<sos>", "<eos>", "<pad>", "<unk>"
SPECIAL_TOKENS = [PAD, SOS, EOS, UNK]

_TOKEN_RE = re.compile(r"(\\[a-zA-Z]+|[{}_^$%&#]|[0-9]+|[a-zA-Z]+|[^\s])")

# (pattern, replacement) applied in order by clean_latex_output
_CLEANUPS = (
    (re.compile(r"\\begin\s+\{"), r"\\begin{"),          # "\begin {" -> "\begin{"
    (re.compile(r"\\end\s+\{"), r"\\end{"),              # "\end {"   -> "\end{"
    (re.compile(r"\{(\s+)([a-zA-Z]+)(\s+)\}"), r"{\2}"),  # "{ word }" -> "{word}"
    (re.compile(r"\\\s+\\"), r"\\\\"),                   # "\ \"      -> "\\"
)


def tokenize_latex(formula: str) -> list:
    return _TOKEN_RE.findall(formula)


def load_vocab(filepath: str):
    with open(filepath, "r", encoding="utf-8") as f:
        data = json.load(f)
    return data["vocab"], {int(k): v for k, v in data["idx2char"].items()}


def tokens_to_latex(token_ids, idx2char: dict) -> str:
    dropped = (SOS, EOS, PAD)
    return " ".join(idx2char[t] for t in token_ids if t in idx2char and idx2char[t] not in dropped)


def clean_latex_output(latex_str: str) -> str:
    for pattern, repl in _CLEANUPS:
        latex_str = pattern.sub(repl, latex_str)
    return latex_str


def detokenize(seq, idx2char: dict) -> str:
    out = []
    for idx in seq:
        tok = idx2char[int(idx)]
        if tok == EOS:
            break
        if tok not in (SOS, PAD):
            out.append(tok)
    return " ".join(out)
