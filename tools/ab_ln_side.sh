set -e
B="python -u bench.py --no-cpu-baseline --no-census --no-generate"
for i in 1 2; do
 for v in 0 1; do CHARPT_LN_REDUCE_SIDE=$v timeout -k 10 120 $B > gpurun_out/ab_c2_$v.txt 2>&1; echo "c2 side=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_c2_$v.txt)"; done
done
for v in 0 1; do CHARPT_LN_REDUCE_SIDE=$v timeout -k 10 150 $B --config c4 --steps 10 --warmup 3 > gpurun_out/ab_c4_$v.txt 2>&1; echo "c4 side=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_c4_$v.txt)"; done
for v in 0 1; do CHARPT_LN_REDUCE_SIDE=$v timeout -k 10 150 $B --config c4 --steps 10 --warmup 3 > gpurun_out/ab_c4_$v.txt 2>&1; echo "c4 side=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_c4_$v.txt)"; done
