S="1024x1024x256 1024x1024x250 1024x1024x252 1024x1024x254 1000x1000x268 1024x1000x256 512x512x1000 1000x1024x256"
timeout -k 10 300 python -u -m pytest tests/test_gpu_imap.py tests/test_gpu_flex.py tests/test_gpu_reftests_file.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03p_imap.txt 2>&1; echo pytest_rc=$?; tail -2 gpurun_out/r03p_imap.txt
for mg in 0 1; do for d in put get; do PROBE_DIR=$d PNCX_XPOSE_MERGE=$mg timeout -k 10 200 python tools/transpose_probe.py $S > gpurun_out/r03p_xpose_m$mg.$d.jsonl || exit 1; done; done
timeout -k 10 300 python tools/flex_bench.py --big > gpurun_out/r03p_flex_big.txt 2>&1
