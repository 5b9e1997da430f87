"""Print tools/gemm_ab.py result lines (gpurun_out/ab.log) as a per-class table."""
import json
import sys

runs = [json.loads(l) for l in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab.log") if l.startswith("{")]
keys = sorted({k for r in runs for k in r["us_tflops"]})
print("%-10s" % "class" + "".join("%16s" % f'{r["ring"]}/{r["precision"]}' for r in runs))
print("%-10s" % "encoder" + "".join("%13.2f ms" % r["encoder_ms"] for r in runs))
for k in keys:
    print("%-10s" % k + "".join("%9.0f %4.0fT" % tuple(r["us_tflops"].get(k, (0, 0))) for r in runs))
