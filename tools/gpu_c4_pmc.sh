#!/bin/bash
# C4 (k_batch_swapmix over 256 variables) against the same bytes as two
# segments and as one flat swap (k_tile): occupancy, DRAM credit stalls and
# request counts per dispatch, to tell ramp/drain from placement.
#   bash tools/gpu_c4_pmc.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1_c4pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for mode in batch flat2 flat; do
  timeout -k 10 120 python3 $R/tools/c4_pmc_probe.py $mode --reps 30 > $O/$mode.time.json 2>$O/$mode.time.log \
      || { echo "TIME_FAIL $mode"; tail -5 $O/$mode.time.log; exit 2; }
  k=0
  for grp in "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ_DRAM_CREDIT_STALL TCC_EA0_RDREQ_LEVEL TCC_EA0_WRREQ_LEVEL" \
             "TCC_EA0_RDREQ TCC_EA0_WRREQ TCC_EA0_WRREQ_64B GRBM_GUI_ACTIVE"; do
    k=$((k+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
        -d $O/$mode.$k -o p -- python3 $R/tools/c4_pmc_probe.py $mode --reps 10 > $O/$mode.$k.log 2>&1 \
        || { echo "PMC_FAIL $mode $k"; tail -5 $O/$mode.$k.log; exit 2; }
  done
done
python3 $R/tools/c4_pmc_summary.py $O
