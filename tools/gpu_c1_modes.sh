# C1 through libpnetcdf.so by host-chunk mode (PNCX_HOST_ZC 0/1/2) and I/O
# threads, alternating, plus the reference's sequence in C (tools/c1_probe).
#   bash tools/gpu_c1_modes.sh <tag> [rounds]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c1m_$1
mkdir -p $O
for i in $(seq 1 ${2:-2}); do
  for z in 0 1 2; do
    for t in 1 8; do
      PNCX_HOST_ZC=$z PNCX_IO_THREADS=$t timeout -k 10 60 $R/tests/mpi/api_check c1bench /dev/shm/c1m_$$.nc 1048576 41 0 > $O/z$z.t$t.$i.json 2>&1 || { echo FAIL $z $t; cat $O/z$z.t$t.$i.json; exit 2; }
      echo "zc=$z io=$t rep=$i $(tail -1 $O/z$z.t$t.$i.json | sed 's/"mode": "c1bench", "n": 1048576, "reps": 41, "dev": 0, "var_offset": 512, //')"
    done
  done
done
for z in 1 2; do
  PNCX_PHASES=1 PNCX_HOST_ZC=$z PNCX_IO_THREADS=1 timeout -k 10 60 $R/tests/mpi/api_check c1bench /dev/shm/c1m_$$.nc 1048576 41 0 > $O/ph_z$z.json 2>&1 || exit 2
done
rm -f /dev/shm/c1m_*.nc
timeout -k 10 120 $R/tools/c1_probe /dev/shm/c1p_$$.nc 4194304 41 > $O/probe_4m.txt 2>&1 || exit 2
grep reference_ $O/probe_4m.txt
