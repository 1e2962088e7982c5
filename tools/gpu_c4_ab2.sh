# batch-kernel change check: GPU parity tests of the batch paths, the kernel
# ablation and the in-process A/B of the in-tree build against tools/ab/libpncx.so
set -o pipefail
R=$GRAFT_REPO_ROOT
tag=${1:-c4ab2}
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > $R/gpurun_out/${tag}_tests.txt 2>&1 || { tail -20 $R/gpurun_out/${tag}_tests.txt; exit 1; }
tail -1 $R/gpurun_out/${tag}_tests.txt
timeout -k 10 200 $R/tools/c4_kernel_ablation > $R/gpurun_out/${tag}_ablation.txt 2>&1 || exit 1
timeout -k 10 500 python -u $R/tools/c4_ab.py --b $R/tools/ab/libpncx.so --rounds 7 > $R/gpurun_out/${tag}_ab.txt 2>&1 || { tail -5 $R/gpurun_out/${tag}_ab.txt; exit 1; }
cat $R/gpurun_out/${tag}_ablation.txt
cut -c1-120 $R/gpurun_out/${tag}_ab.txt
