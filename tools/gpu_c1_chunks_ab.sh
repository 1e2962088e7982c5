# C1 (2^20 NC_INT put_vara_int_all + get_vara_int_all through libpnetcdf.so
# on /dev/shm, host buffers) by pipeline chunk count (PNCX_MIN_CHUNKS) and
# I/O threads, alternating; the file-layer GPU tests first.
#   bash tools/gpu_c1_chunks_ab.sh <tag> [rounds]
# (PNCX_MIN_CHUNKS existed only in the A/B build; the product keeps one chunk per slot.)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c1_ab_$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_ncfile.py $R/tests/test_gpu_c_api.py $R/tests/test_gpu_large_reqs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { echo TESTS_FAIL; tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in $(seq 1 ${2:-3}); do
  for t in 1 8; do
    for c in 1 4 8; do
      PNCX_IO_THREADS=$t PNCX_MIN_CHUNKS=$c timeout -k 10 60 $R/tests/mpi/api_check c1bench /dev/shm/c1ab_$$.nc 1048576 41 0 > $O/t$t.c$c.$i.json 2>&1 || { echo FAIL $t $c; cat $O/t$t.c$c.$i.json; exit 2; }
      echo "io=$t chunks=$c rep=$i $(tail -1 $O/t$t.c$c.$i.json)"
    done
  done
done
rm -f /dev/shm/c1ab_*.nc
