# round 6: the new GPU tests (pthread, warm-up/preload, first-touch fault
# injection) and the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_first_touch.py::test_failed_append_cuts_the_file_back tests/test_gpu_warmup.py -p no:cacheprovider > gpurun_out/r06c_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r06c_bench.json 2> gpurun_out/r06c_bench.err || exit 2
cp profiles/bench_detail_last.json gpurun_out/r06c_bench_detail.json
