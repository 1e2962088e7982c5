# C1 per-phase breakdown (tests/mpi/api_check c1bench with PNCX_PHASES=1:
# host clock per phase + HIP events around H2D / kernel / D2H of the staged
# conversion) at 1 and 8 I/O threads, then tools/c1_probe (every candidate
# piece timed alone on the same box).
#   bash tools/gpu_c1_phases.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c1ph_$1
mkdir -p $O
for t in 1 8; do
  for i in 1 2; do
    PNCX_PHASES=1 PNCX_IO_THREADS=$t timeout -k 10 60 $R/tests/mpi/api_check c1bench /dev/shm/c1ph_$$.nc 1048576 41 0 > $O/ph_t$t.$i.json 2>&1 || { echo FAIL phases $t; cat $O/ph_t$t.$i.json; exit 2; }
    echo "io=$t phases: $(tail -1 $O/ph_t$t.$i.json)"
  done
  PNCX_IO_THREADS=$t timeout -k 10 60 $R/tests/mpi/api_check c1bench /dev/shm/c1ph_$$.nc 1048576 41 0 > $O/noph_t$t.json 2>&1 || { echo FAIL nophases $t; exit 2; }
  echo "io=$t plain: $(tail -1 $O/noph_t$t.json)"
done
rm -f /dev/shm/c1ph_*.nc
timeout -k 10 120 $R/tools/c1_probe /dev/shm/c1p_$$.nc 4194304 41 > $O/probe_4m.txt 2>&1 || { echo FAIL probe; cat $O/probe_4m.txt; exit 2; }
cat $O/probe_4m.txt
timeout -k 10 120 $R/tools/c1_probe /dev/shm/c1p_$$.nc 1048576 41 > $O/probe_1m.txt 2>&1 || { echo FAIL probe1m; exit 2; }
