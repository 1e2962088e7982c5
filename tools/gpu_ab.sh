#!/bin/bash
# The one parameterised A/B runner for GPU measurements (replaces round 1-4's
# one-off tools/gpu_*_ab.sh scripts; they remain in git history before
# commit "tools: one A/B runner").  Runs COMMAND once per environment setting
# per pass, settings interleaved so that box drift hits all of them alike,
# each run under its own time limit; stops at the first failure.
#
#   tools/gpu_ab.sh TAG PASSES "ENV=V,ENV2=V2" "ENV=W" ... -- COMMAND [ARGS...]
#
# An empty setting ("") runs the defaults.  Output: gpurun_out/TAG.txt, one
# "# pass P env SETTING" header before each run's stdout+stderr.
# Examples:
#   tools/gpu_ab.sh r05_tile 3 "" "PNCX_TILE_U=1" -- python tools/matrix_bench.py --pairs float:int64
#   tools/gpu_ab.sh r05_xp 2 "PNCX_XPOSE_ORDER=0" "PNCX_XPOSE_ORDER=8" -- python tools/transpose_probe.py 1024x1024x254
set -o pipefail
tag=$1; passes=$2; shift 2
envs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
shift
[ $# -gt 0 ] || { echo "usage: $0 TAG PASSES SETTING... -- COMMAND" >&2; exit 2; }
export TMPDIR=${TMPDIR:-/tmp}
out=gpurun_out/$tag.txt
mkdir -p gpurun_out
: > "$out"
for ((p = 1; p <= passes; p++)); do
  for e in "${envs[@]}"; do
    echo "# pass $p env $e" >> "$out"
    env $(echo "$e" | tr ',' ' ') timeout -k 10 ${AB_TIMEOUT:-300} "$@" >> "$out" 2>&1 || { echo "FAILED: env $e" | tee -a "$out"; exit 1; }
  done
done
tail -n 20 "$out"
