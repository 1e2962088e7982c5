set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/pcie_probe.py > gpurun_out/pcie.json 2>&1 || { cat gpurun_out/pcie.json; exit 1; }
for mb in 16 64 256; do PNCX_CHUNK_MB=$mb timeout -k 10 300 python tools/host_roundtrip.py --gib 4 > gpurun_out/host_rt_$mb.json 2>&1 || exit 2; done
grep -v amdgpu gpurun_out/pcie.json gpurun_out/host_rt_*.json
