"""ORACLE — test infrastructure only.

CPU fp32 restatement of the reference hot path.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import anything under ``oracle/``; the product package never does, and the
engine fails loudly instead of falling back to it.
"""
