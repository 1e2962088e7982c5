# round 6 evidence: rocprof kernel stats + PMC passes (tools/gpu_profile_round.sh),
# the C-level synchronous C4 call timing, and the default bench line
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_profile_round.sh r06k || exit 1
timeout -k 10 120 tools/c4_call_c 200 20 > gpurun_out/r06k_c4_call_c.json 2>&1 || exit 2
timeout -k 10 120 tools/c4_call_c 200 20 >> gpurun_out/r06k_c4_call_c.json 2>&1 || exit 3
timeout -k 10 600 python -u bench.py > gpurun_out/r06k_bench.json 2> gpurun_out/r06k_bench.err || exit 4
cp profiles/bench_detail_last.json gpurun_out/r06k_bench_detail.json
