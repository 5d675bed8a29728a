#!/bin/bash
# round-4 batch p: the 128 x 128 kernel (weight gradients) with its next-tile loads spread evenly
# over the 48 MFMAs (g10), with s_setprio 1 around the MFMA phase (g01), both (g11), vs in-tree.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4p; mkdir -p $O
b() { "$@" || { rc=$?; echo "stopping: rc=$rc"; exit $rc; }; }
LIBS="in-tree $PWD/variants/g10/libmst_hip.so $PWD/variants/g01/libmst_hip.so $PWD/variants/g11/libmst_hip.so"
for r in 1 2; do
  for lib in $LIBS; do
    l=$lib; [ "$l" = in-tree ] && l=""
    for shp in "--B 32 --T 252 --cin 1536 --cout 1536" "--B 32 --T 15 --cin 4096 --cout 4096"; do
      echo "== lib $lib $shp" >> $O/micro.txt
      b env MST_LIB_PATH=$l timeout -k 10 120 python -u tools/gemm_micro.py $shp --kinds wgrad --reps 20 >> $O/micro.txt 2>> $O/micro.err
    done
  done
done
echo "micro ok"
b env MST_LIB_PATH=$PWD/variants/g11/libmst_hip.so timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad or gemm or conv" > $O/pytest_g11.log 2>&1
for r in 1 2; do
  for lib in $LIBS; do
    l=$lib; [ "$l" = in-tree ] && l=""
    echo "== lib $lib" >> $O/ab_step.jsonl
    b env MST_LIB_PATH=$l timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
      >> $O/ab_step.jsonl 2>> $O/ab_step.err
  done
done
echo "all ok"
