set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_check.sh r03j nobench || exit 1
timeout -k 10 400 python -u bench.py --arch res18trans > gpurun_out/r03j_bench_c5.json 2> gpurun_out/r03j_bench_c5.err || { tail -5 gpurun_out/r03j_bench_c5.err; exit 1; }
cut -c1-200 gpurun_out/r03j_bench_c5.json
timeout -k 10 500 python -u bench.py --beam 4 --batch 32 --tokens 256 > gpurun_out/r03j_bench_c4.json 2> gpurun_out/r03j_bench_c4.err || { tail -5 gpurun_out/r03j_bench_c4.err; exit 1; }
cut -c1-200 gpurun_out/r03j_bench_c4.json
timeout -k 10 300 python tools/stop_batch_probe.py --reps 5 --eos-boost 0,5 > gpurun_out/r03j_stop_probe.json 2>/dev/null
