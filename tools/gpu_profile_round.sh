# Round evidence on the GPU box, small enough to come back through
# gpurun_out/ (< 64 MiB): tools/gpu_profile.sh, then the kernel stats and
# PMC summary (tools/pmc_summary.py) into gpurun_out/<tag>_sum/, the C4
# NC_ERANGE kernel trace beside them, and the bulky rocprof output removed.
#   bash tools/gpu_profile_round.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
S=$R/gpurun_out/$1_sum
mkdir -p $S
bash $R/tools/gpu_profile.sh > $S/profile.txt 2>&1 || { echo PROFILE_FAIL; tail -20 $S/profile.txt; exit 1; }
cp $R/profiles/pmc_traffic.json $S/
python3 $R/tools/pmc_summary.py $R/gpurun_out/prof $1 $S > $S/summary.json || exit 2
cp $R/gpurun_out/prof/trace/c4_erange_kernel_trace.csv $S/$1_c4_erange_kernel_trace.csv 2>/dev/null
cp $R/gpurun_out/prof/trace_*.json $S/ 2>/dev/null
rm -rf $R/gpurun_out/prof
ls $S
