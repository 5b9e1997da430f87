set -o pipefail
mkdir -p gpurun_out/rep
for cfg in "--replicas 2 --chain-batches 4" "--replicas 3 --chain-batches 4" "--replicas 3 --chain-batches 2" "--replicas 4 --chain-batches 2"; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-isolated $cfg > gpurun_out/rep/b.json 2>gpurun_out/rep/b.err || { tail gpurun_out/rep/b.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/rep/b.json')); print('$cfg', round(d['value']), {k:v for k,v in d.items() if 'p50' in k})"
done
