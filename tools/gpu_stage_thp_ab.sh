# (historical: PNCX_STAGE_THP was an experiment removed after this run, profiles/r06o_stage_thp_ab.txt)
# Staging area on 2 MiB transparent huge pages (PNCX_STAGE_THP=1, experiment)
# against hipHostMalloc: whole c1first processes with per-phase times,
# alternating, host and device buffers.
set -o pipefail
out=${OUT:-gpurun_out/r06o_stage_thp_ab.txt}
mkdir -p gpurun_out
: > "$out"
echo "thp_enabled: $(cat /sys/kernel/mm/transparent_hugepage/enabled 2>/dev/null)" >> "$out"
echo "thp_defrag: $(cat /sys/kernel/mm/transparent_hugepage/defrag 2>/dev/null)" >> "$out"
F=/dev/shm/thp_ab_$$.nc
for round in ${ROUNDS:-1 2 3 4}; do
  for dev in 0 1; do
    order="0 1"; [ $((round % 2)) = 0 ] && order="1 0"
    for thp in $order; do
      if [ $thp = 1 ]; then
        r=$(PNCX_STAGE_THP=1 PNCX_PHASES=1 timeout -k 10 60 tests/mpi/api_check c1first $F 1048576 32 $dev) || { echo "FAIL thp $thp dev $dev" >> "$out"; exit 1; }
      else
        r=$(PNCX_PHASES=1 timeout -k 10 60 tests/mpi/api_check c1first $F 1048576 32 $dev) || { echo "FAIL thp $thp dev $dev" >> "$out"; exit 1; }
      fi
      echo "{\"round\": $round, \"dev\": $dev, \"thp\": $thp, \"c1first\": $r}" >> "$out"
    done
  done
done
rm -f $F
