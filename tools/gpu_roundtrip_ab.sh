# Host round trip (tools/host_roundtrip.py, 2 GiB) of the round-3 library
# (abcmp/r03/libpncx.so, built from f840f2f) against this build, alternating,
# plus the raw PCIe link (tools/pcie_probe.py) on the same box.
#   bash tools/gpu_roundtrip_ab.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rtab_$1
mkdir -p $O
timeout -k 10 120 python3 $R/tools/pcie_probe.py > $O/pcie.json 2>&1 || { echo PCIE_FAIL; tail -5 $O/pcie.json; }
tail -3 $O/pcie.json
for i in 1 2; do
  PNCX_LIB_PATH=$R/abcmp/r03/libpncx.so timeout -k 10 200 python3 $R/tools/host_roundtrip.py --gib 2 > $O/r03.$i.json 2> $O/r03.$i.err || { echo FAIL r03; tail -5 $O/r03.$i.err; exit 2; }
  timeout -k 10 200 python3 $R/tools/host_roundtrip.py --gib 2 > $O/r04.$i.json 2> $O/r04.$i.err || { echo FAIL r04; tail -5 $O/r04.$i.err; exit 2; }
  for b in r03 r04; do echo "$b.$i $(python3 -c "import json;d=json.loads(open('$O/$b.$i.json').read().strip().splitlines()[-1]);print({k:(v.get('slab_GiBps') or v.get('moved_GiBps')) for k,v in d.items() if isinstance(v,dict)})")"; done
done
