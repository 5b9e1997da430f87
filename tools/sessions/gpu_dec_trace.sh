set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/dtr
for R in 1 3; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dtr/r$R -o run -- python3 tools/decode_replicas.py $R > gpurun_out/dtr/r$R.log 2>&1 || { echo "R=$R failed"; tail -5 gpurun_out/dtr/r$R.log; exit 1; }
  python3 tools/trace_gaps.py gpurun_out/dtr/r$R/run_kernel_trace.csv > gpurun_out/dtr/gaps_r$R.txt
  rm -f gpurun_out/dtr/r$R/run_kernel_trace.csv
  cat gpurun_out/dtr/gaps_r$R.txt
done
