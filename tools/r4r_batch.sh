#!/bin/bash
# round-4 batch r: parity of the load-spread build (in-tree), then a re-sweep of the wide kernel's
# LDS-store spacing (d1, d3) and split VALU per MFMA (v4) on top of it.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4r; mkdir -p $O
t() { local log=$1; shift; "$@" > "$O/$log" 2>&1; local rc=$?; echo "$log rc=$rc";
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $log rc=$rc"; exit $rc; fi; }
b() { "$@" || { rc=$?; echo "stopping: rc=$rc"; exit $rc; }; }
t pytest_gemm.log timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_bench_shapes.py tests/test_gpu_knobs.py
LIBS="in-tree $PWD/variants/d1/libmst_hip.so $PWD/variants/d3/libmst_hip.so $PWD/variants/v4/libmst_hip.so"
for r in 1 2; do
  for lib in $LIBS; do
    l=$lib; [ "$l" = in-tree ] && l=""
    for shp in "--B 32 --T 252 --cin 1536 --cout 1536" "--B 32 --T 15 --cin 4096 --cout 4096"; do
      echo "== lib $lib $shp" >> $O/micro.txt
      b env MST_LIB_PATH=$l timeout -k 10 120 python -u tools/gemm_micro.py $shp --reps 20 >> $O/micro.txt 2>> $O/micro.err
    done
  done
done
echo "micro ok"
for r in 1 2; do
  for lib in $LIBS; do
    l=$lib; [ "$l" = in-tree ] && l=""
    echo "== lib $lib" >> $O/ab_step.jsonl
    b env MST_LIB_PATH=$l timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
      >> $O/ab_step.jsonl 2>> $O/ab_step.err
  done
done
echo "all ok"
