#!/bin/bash
# DRAM credit stalls and queue levels of the varm transposes (k_imap_tile),
# x254 against x256, put and get: where the x254 cycles go below the L2.
#   bash tools/gpu_xpose_stalls.sh <tag> [shape ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1_xstall
shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for shape in "${@:-1024x1024x256 1024x1024x254}"; do
  for dir in put get; do
    k=0
    for grp in "TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ_DRAM_CREDIT_STALL TCC_EA0_RDREQ_LEVEL TCC_EA0_WRREQ_LEVEL" \
               "TCC_EA0_RDREQ TCC_EA0_WRREQ TCC_EA0_WRREQ_64B GRBM_GUI_ACTIVE"; do
      k=$((k+1))
      PROBE_DIR=$dir timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
          -d $O/$shape.$dir.$k -o p -- python3 $R/tools/transpose_probe.py $shape > $O/$shape.$dir.$k.log 2>&1 \
          || { echo "PMC_FAIL $shape $dir $k"; tail -5 $O/$shape.$dir.$k.log; exit 2; }
    done
  done
done
