# Cache-pull helpers (PNCX_PULL) on the C1 first-touch put: in-process A/B
# (api_check c1ab alternates the knob record by record, A B B A ...) and
# whole processes with per-phase times (api_check c1first, PNCX_PHASES=1)
# (historical: the knob it A/Bs was removed after the run; kept as the record of how its profiles/ file was made)
set -o pipefail
out=${OUT:-gpurun_out/r06d_pull_ab.txt}
mkdir -p gpurun_out
: > "$out"
F=/dev/shm/pull_ab_$$.nc
for round in 1 2 3; do
  for dev in 0 1; do
    r=$(timeout -k 10 60 tests/mpi/api_check c1ab $F 1048576 32 PULL 0 3 $dev) || { echo "FAIL c1ab dev $dev" >> "$out"; exit 1; }
    echo "{\"round\": $round, \"dev\": $dev, \"ab\": $r}" >> "$out"
  done
  for pull in 0 3; do
    r=$(PNCX_PULL=$pull PNCX_PHASES=1 timeout -k 10 60 tests/mpi/api_check c1first $F 1048576 32 0) || { echo "FAIL c1first pull $pull" >> "$out"; exit 1; }
    echo "{\"round\": $round, \"pull\": $pull, \"c1first\": $r}" >> "$out"
  done
done
rm -f $F
