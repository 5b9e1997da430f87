#!/bin/bash
# beam 4 (config 4): the round-2 tree (tmp_r02, built from commit 42abab6) vs the current tree, same box
set -o pipefail
for rep in 1 2; do
  (cd tmp_r02 && timeout -k 10 400 python -u bench.py --beam 4 --batch 32 --tokens 256 --no-cpu-baseline --steps 24 2>/dev/null | cut -c1-200) || exit 1
  timeout -k 10 400 python -u bench.py --beam 4 --batch 32 --tokens 256 --no-cpu-baseline --steps 24 2>/dev/null | cut -c1-200 || exit 1
done
