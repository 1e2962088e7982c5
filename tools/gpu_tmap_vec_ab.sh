# Parity and A/B of the vectorized run-piece kernel (PNCX_TMAP_VEC).
#   bash tools/gpu_tmap_vec_ab.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
for v in 1 0; do
  PNCX_TMAP_VEC=$v timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_flex.py $R/tests/test_gpu_reftests_file.py -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/$1_flex_v$v.txt 2>&1 || { echo FAIL $v; tail -30 $R/gpurun_out/$1_flex_v$v.txt; exit 1; }
  tail -1 $R/gpurun_out/$1_flex_v$v.txt
done
for v in 0 1 0 1; do
  PNCX_TMAP_VEC=$v timeout -k 10 300 python3 $R/tools/flex_bench.py --big > $R/gpurun_out/$1_fb_v$v.txt 2>&1 || exit 2
  grep "halo\|vector256\|short_runs\"" $R/gpurun_out/$1_fb_v$v.txt | sed "s/^/vec=$v /"
done
