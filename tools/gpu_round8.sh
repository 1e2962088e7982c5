set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k large_pinned > gpurun_out/t_pin.log 2>&1 || { tail -30 gpurun_out/t_pin.log; exit 1; }
for mb in 16 32 64; do PNCX_CHUNK_MB=$mb timeout -k 10 300 python tools/host_roundtrip.py --gib 4 > gpurun_out/host_rt_$mb.json 2>&1 || exit 2; done
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 3; }
tail -3 gpurun_out/t_pin.log gpurun_out/t_all.log
grep -v amdgpu gpurun_out/host_rt_*.json
