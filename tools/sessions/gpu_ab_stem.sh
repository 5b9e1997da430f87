L=handwritten-math-ocr-api_amd
O=gpurun_out/ab_stem2.log; : > $O
for lib in $L/lib_var/prev/libmathocr.so $L/lib/libmathocr.so $L/lib_var/stem1k/libmathocr.so $L/lib_var/prev/libmathocr.so $L/lib/libmathocr.so $L/lib_var/stem1k/libmathocr.so; do
  echo "== $lib" >> $O
  timeout -k 10 180 python tools/op_times.py --lib $lib --variants production --filter stem >> $O 2>&1 || exit 1
done
timeout -k 10 180 python tests/probes/stage_diff.py $L/lib_var/prev/libmathocr.so gpurun_out/sd_a.npz >> $O 2>&1 || exit 1
timeout -k 10 180 python tests/probes/stage_diff.py $L/lib_var/stem1k/libmathocr.so gpurun_out/sd_b.npz >> $O 2>&1 || exit 1
python -c "
import numpy as np
a=np.load('gpurun_out/sd_a.npz'); b=np.load('gpurun_out/sd_b.npz')
bad=[k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('stage maps bitwise equal' if not bad else 'DIFFER: %s' % bad)" >> $O
grep -v amdgpu $O | grep -v "^op\|total"
