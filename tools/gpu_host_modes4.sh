# One box: host round trip (tools/host_roundtrip.py, 2 GiB) of the round-3
# library against this build's zero copy (PNCX_HOST_ZC=2) and SDMA copies on
# alternating streams (3, round 3's pipeline since the mode stopped taking
# zero-copy stores), and file_bench with both.
#   bash tools/gpu_host_modes3.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/hm4_$1
mkdir -p $O
for i in 1 2; do
  PNCX_LIB_PATH=$R/abcmp/r03/libpncx.so timeout -k 10 200 python3 $R/tools/host_roundtrip.py --gib 2 > $O/rt_r03.$i.json 2> $O/rt_r03.$i.err || { echo FAIL r03; tail -5 $O/rt_r03.$i.err; exit 2; }
  echo "r03.$i $(python3 -c "import json;d=json.loads(open('$O/rt_r03.$i.json').read().strip().splitlines()[-1]);print({k:(v.get('slab_GiBps') or v.get('moved_GiBps')) for k,v in d.items() if isinstance(v,dict)})")"
  for z in 2 3; do
    PNCX_HOST_ZC=$z timeout -k 10 200 python3 $R/tools/host_roundtrip.py --gib 2 > $O/rt_z$z.$i.json 2> $O/rt_z$z.$i.err || { echo FAIL rt $z; tail -5 $O/rt_z$z.$i.err; exit 2; }
    echo "z$z.$i $(python3 -c "import json;d=json.loads(open('$O/rt_z$z.$i.json').read().strip().splitlines()[-1]);print({k:(v.get('slab_GiBps') or v.get('moved_GiBps')) for k,v in d.items() if isinstance(v,dict)})")"
  done
done
for z in 2 3; do
  PNCX_HOST_ZC=$z timeout -k 10 300 python3 $R/tools/file_bench.py --reps 3 > $O/fb_z$z.json 2> $O/fb_z$z.err || { echo FAIL fb $z; tail -5 $O/fb_z$z.err; exit 2; }
  echo "fb zc=$z $(python3 -c "import json;d=json.loads(open('$O/fb_z$z.json').read().strip().splitlines()[-1]);b=d['INT_big_ours'];print('bigput',b['put_GiBps_external'],'bigget',b['get_GiBps_external'],'c3',d['C3_file_get_vara_double']['ours_GiBps_external'],'c4',d['C4_file_iput_wait_all']['ours_GiBps_external'],'c1',d['C1_ours']['put_s'],d['C1_ours']['get_s'])")"
done
