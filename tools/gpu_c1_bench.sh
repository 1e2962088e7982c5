# C1 through libpnetcdf.so (tests/mpi/api_check c1bench: 2^20 NC_INT
# put_vara_int_all + get_vara_int_all on /dev/shm, median of 41) with host
# buffers at 1 and 8 I/O threads and with device buffers, a few rounds.
#   bash tools/gpu_c1_bench.sh <tag> [rounds]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c1_$1
mkdir -p $O
for i in $(seq 1 ${2:-3}); do
  for t in 1 8; do
    for d in 0 1; do
      PNCX_IO_THREADS=$t timeout -k 10 60 $R/tests/mpi/api_check c1bench /dev/shm/c1b_$$.nc 1048576 41 $d > $O/t$t.d$d.$i.json 2>&1 || { echo FAIL $t $d; cat $O/t$t.d$d.$i.json; exit 2; }
      echo "io=$t dev=$d rep=$i $(tail -1 $O/t$t.d$d.$i.json | sed 's/"mode": "c1bench", "n": 1048576, "reps": 41, //')"
    done
  done
done
rm -f /dev/shm/c1b_*.nc
