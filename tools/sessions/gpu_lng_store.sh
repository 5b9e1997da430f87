#!/bin/bash
# lngemm384 output stores: op times and one WRITE_SIZE pass of an encode
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/lngst; mkdir -p $O
timeout -k 10 200 python tools/op_times.py --batch 256 --variants production --filter s3.,merge 2>&1 | grep -v amdgpu.ids || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o run -- \
  python3 tools/profile_encoder.py --batch 256 > $O/pmc_w.log 2>&1 || { echo "PMC W FAILED"; exit 1; }
python3 - <<'PY'
import csv
rows = [r for r in csv.DictReader(open("gpurun_out/lngst/pmc_w/run_counter_collection.csv")) if "lngemm384" in r["Kernel_Name"]]
print("lngemm384 WRITE_SIZE MB per launch:", [round(float(r["Counter_Value"]) * 1024 / 1e6, 1) for r in rows])
PY
