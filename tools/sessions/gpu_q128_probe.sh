O=gpurun_out/gemm_q128.log; : > $O
for rep in 1 2; do for b in ./tools/gemm_bench ./tools/gemm_bench_nostore; do for k in 10 12; do
echo "$b k$k | $(timeout -k 5 60 $b 36864 1536 384 3 1 30 1 $k)" >> $O || exit 1; done; done; done; cat $O
