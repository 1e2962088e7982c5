# The reference's own benchmarks/C/pnetcdf_put_vara.c (built unchanged from
# /root/reference by `make -C oracle ref-bench`, linked with libpnetcdf.so)
# on the GPU box: CDF-5, 8 NC_FLOAT variables of 2048 x 2048 per rank,
# 4 records, blocking and nonblocking, 1 and 4 ranks on the one GPU; the
# file in /dev/shm (REFBENCH_DIR overrides).
#   tools/ref_bench_run.sh <out.txt>
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$1
D=$(mktemp -d ${REFBENCH_DIR:-/dev/shm}/refbench.XXXXXX)
for np in 1 4; do
  for mode in "" "-i"; do
    echo "== nprocs $np mode ${mode:-blocking}" >> $out
    timeout -k 10 240 /opt/conda/bin/mpiexec -n $np $R/oracle/_ref/pnetcdf_put_vara -k 5 -l 2048 -n 8 -t 4 $mode \
        $D/out.nc >> $out 2>&1 || { echo "FAILED rc=$?" >> $out; rm -rf $D; exit 1; }
    rm -f $D/out.nc
  done
done
rm -rf $D
