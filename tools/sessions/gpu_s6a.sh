#!/bin/bash
# Round 6, first call: the driver-form bench on this round's starting tree (baseline on
# this box), the FETCH_SIZE calibration of the decode step's access patterns
# (tools/fetch_calib.hip: FETCH_SIZE, the four TCC request-size counters, WRITE_SIZE),
# and the request-size counters of one 640-image encode + 8 greedy steps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s6a; mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { echo "BENCH FAILED"; tail $O/bench_driver.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_driver.json')); print('driver', d['value'], d['ms_per_step'], d['roofline']['avg_step_ms'])"
REQ="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/cal_f -o run -- tools/fetch_calib > $O/cal_f.log 2>&1 || { echo "CAL F FAILED"; tail $O/cal_f.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc $REQ --output-format csv -d $O/cal_r -o run -- tools/fetch_calib > $O/cal_r.log 2>&1 || { echo "CAL R FAILED"; tail $O/cal_r.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc TCC_BUBBLE_sum TCC_EA0_RDREQ_sum --output-format csv -d $O/cal_b -o run -- tools/fetch_calib > $O/cal_b.log 2>&1 || { echo "CAL B FAILED"; tail $O/cal_b.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/cal_w -o run -- tools/fetch_calib > $O/cal_w.log 2>&1 || { echo "CAL W FAILED"; tail $O/cal_w.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc $REQ --output-format csv -d $O/dec_r -o run -- \
  python3 tools/profile_encoder.py --batch 640 --decode-steps 8 > $O/dec_r.log 2>&1 || { echo "DEC R FAILED"; tail $O/dec_r.log; exit 1; }
echo done
