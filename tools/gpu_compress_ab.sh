set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r06g_compress_ab.txt
: > $O
for r in 1 2 3; do
  for lib in plain z; do
    if [ $lib = plain ]; then L=$PWD/pnetcdf_amd/lib/plain/libpncx.so; else L=$PWD/pnetcdf_amd/lib/libpncx.so; fi
    echo "round $r lib $lib" >> $O
    PNCX_LIB_PATH=$L timeout -k 10 120 python3 tools/first_launch_probe.py spgd >> $O 2>&1 || exit 1
  done
done
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_warmup.py -p no:cacheprovider >> $O 2>&1 || exit 2
