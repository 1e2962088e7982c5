#!/bin/bash
# Counters of the short-run scatter against the gather (tools/scatter_probe.hip):
# one rocprofv3 --pmc pass per counter group and mode, each under its own limit.
#   bash tools/gpu_scatter_pmc.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1_scatter_pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/tools/scatter_probe > $O/rates.txt 2>&1 || { echo RATES_FAIL; cat $O/rates.txt; exit 1; }
groups=("TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_EA0_RDREQ TCC_EA0_WRREQ_STALL"
        "TCC_EA0_WRREQ_DRAM_CREDIT_STALL TCC_WRITE_SECTORS TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_DRAM"
        "TCC_EA0_WRREQ_DRAM TCC_EA0_WRREQ_WRITE_DRAM_32B TCC_EA0_WR_UNCACHED_32B TCC_WRITE"
        "TA_BUSY TD_TD_BUSY GRBM_GUI_ACTIVE GRBM_COUNT")
for m in ${MODES:-gather nt wb touch touch2 touch2nt fill}; do
  k=0
  for grp in "${groups[@]}"; do
    k=$((k+1))
    MODE=$m REPS=5 timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/$m.$k -o p -- $R/tools/scatter_probe > $O/$m.$k.log 2>&1 || { echo "PMC_FAIL $m $k"; tail -5 $O/$m.$k.log; exit 2; }
  done
done
find $O -name "*counter_collection.csv" | head -3
