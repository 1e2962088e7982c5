# Parity and A/B of lattice tables as varm (PNCX_TMAP_IMAP).
#   bash tools/gpu_lattice_ab.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_flex.py $R/tests/test_gpu_reftests_file.py $R/tests/test_gpu_c_api.py -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/$1_tests.txt 2>&1 || { echo FAIL; tail -30 $R/gpurun_out/$1_tests.txt; exit 1; }
tail -1 $R/gpurun_out/$1_tests.txt
for v in 0 1 0 1; do
  PNCX_TMAP_IMAP=$v timeout -k 10 300 python3 $R/tools/flex_bench.py --big > $R/gpurun_out/$1_fb_i$v.txt 2>&1 || exit 2
  grep "halo" $R/gpurun_out/$1_fb_i$v.txt | sed "s/^/tmap_imap=$v /"
done
