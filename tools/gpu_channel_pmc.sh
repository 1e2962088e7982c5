#!/bin/bash
# Per-channel L2->memory request counts (TCC_EA0_WRREQ / _RDREQ per TCC
# instance, summed over the XCDs; tools/pmc_channels.yaml) for the varm
# transposes, ×254 against ×256 and the 2-D shapes: does the packed column
# stride pile the requests onto a few channels?  (VERDICT r04 "Next" 6)
#   bash tools/gpu_channel_pmc.sh <tag> [shape ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1_channels
shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
WR=$(seq -f "WR_CH%02g" 0 15 | tr '\n' ' ')
RD=$(seq -f "RD_CH%02g" 0 15 | tr '\n' ' ')
for shape in "${@:-1024x1024x256 1024x1024x254}"; do
  for dir in put get; do
    for grp in WR RD; do
      ctrs=$([ $grp = WR ] && echo "$WR" || echo "$RD")
      PROBE_DIR=$dir timeout -s KILL 120 rocprofv3 -E $R/tools/pmc_channels.yaml --pmc $ctrs --kernel-trace --output-format csv \
          -d $O/$shape.$dir.$grp -o p -- python3 $R/tools/transpose_probe.py $shape > $O/$shape.$dir.$grp.log 2>&1 \
          || { echo "PMC_FAIL $shape $dir $grp"; tail -5 $O/$shape.$dir.$grp.log; exit 2; }
    done
  done
done
ls $O
