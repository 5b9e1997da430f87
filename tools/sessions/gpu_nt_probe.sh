set -o pipefail
mkdir -p gpurun_out
L0=handwritten-math-ocr-api_amd/lib_var/nt0/libmathocr.so
for lib in $L0 handwritten-math-ocr-api_amd/lib/libmathocr.so $L0 handwritten-math-ocr-api_amd/lib/libmathocr.so; do
  timeout -k 10 200 python -u tools/pipeline_probe.py --lib $lib --replicas 1 --modes decode --steps 4 || exit 1
  timeout -k 10 300 python -u tools/pipeline_probe.py --lib $lib --replicas 4 --modes decode,both --steps 16 || exit 1
done
