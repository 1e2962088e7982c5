# Round trip by stager mode 0..3, then file_bench's 1 GiB put/get with 8 I/O
# threads by mode and MAP_POPULATE.
#   bash tools/gpu_host_modes2.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/hm2_$1
mkdir -p $O
for z in 3 0 1 2; do
  PNCX_HOST_ZC=$z timeout -k 10 200 python3 $R/tools/host_roundtrip.py --gib 2 > $O/rt_z$z.json 2> $O/rt_z$z.err || { echo FAIL rt $z; tail -5 $O/rt_z$z.err; exit 2; }
  echo "rt zc=$z $(python3 -c "import json;d=json.loads(open('$O/rt_z$z.json').read().strip().splitlines()[-1]);print({k:(v.get('slab_GiBps') or v.get('moved_GiBps')) for k,v in d.items() if isinstance(v,dict)})")"
done
for z in 3 2; do
  for pop in 1 0; do
    PNCX_IO_POPULATE=$pop PNCX_HOST_ZC=$z PNCX_IO_THREADS=8 timeout -k 10 300 python3 $R/tools/file_bench.py --reps 3 > $O/fb_z$z.p$pop.json 2> $O/fb_z$z.p$pop.err || { echo FAIL fb $z; tail -5 $O/fb_z$z.p$pop.err; exit 2; }
    echo "fb zc=$z pop=$pop $(python3 -c "import json;d=json.loads(open('$O/fb_z$z.p$pop.json').read().strip().splitlines()[-1]);b=d['INT_big_ours'];print(b['put_GiBps_external'],b['get_GiBps_external'],d['C3_file_get_vara_double']['ours_GiBps_external'],d['C4_file_iput_wait_all']['ours_GiBps_external'])")"
  done
done
