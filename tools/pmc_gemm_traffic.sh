cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in c2 c4; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcg_$c -o fetch -- python3 $R/tools/pmc_gemm.py run $c > $R/gpurun_out/pmcg_${c}_f.log 2>&1 || exit 3
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcg_$c -o write -- python3 $R/tools/pmc_gemm.py run $c > $R/gpurun_out/pmcg_${c}_w.log 2>&1 || exit 3
done
echo done
