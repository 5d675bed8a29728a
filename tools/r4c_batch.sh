#!/bin/bash
# round-4 batch c. In-tree = control (round-3 InstanceNorm kernels, 128x128 GEMM only);
# variants/next = chunk-staged InstanceNorm + the wide conv GEMM (MST_GEMM_WIDE=1/2);
# variants/m16 = 16x16x32 MFMA GEMM build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c; mkdir -p $O
V=variants/next/libmst_hip.so
# test steps: test failures (exit 1) are recorded and the batch goes on; anything else
# (a crash, a GPU fault, a timeout) ends the batch
t() { local log=$1; shift; "$@" > "$O/$log" 2>&1; local rc=$?; echo "$log rc=$rc";
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $log rc=$rc"; exit $rc; fi; }
b() { "$@" || { rc=$?; echo "stopping: bench rc=$rc"; exit $rc; }; }
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
t pytest_next.log env MST_LIB_PATH=$V timeout -k 10 500 $PT tests -m gpu
t pytest_wide1.log env MST_LIB_PATH=$V MST_GEMM_WIDE=1 timeout -k 10 400 $PT tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_bench_shapes.py
t pytest_wide2.log env MST_LIB_PATH=$V MST_GEMM_WIDE=2 timeout -k 10 400 $PT tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_bench_shapes.py
t pytest_m16.log env MST_LIB_PATH=variants/m16/libmst_hip.so timeout -k 10 400 $PT tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_bench_shapes.py
for r in 1; do
  for cfg in "in-tree::0" "$V::0" "$V::1" "$V::2" "variants/m16/libmst_hip.so::0"; do
    lib=${cfg%%::*}; w=${cfg##*::}; [ "$lib" = in-tree ] && lib=""
    echo "== lib ${lib:-in-tree} wide $w" >> $O/ab_step.jsonl
    b env MST_LIB_PATH=$lib MST_GEMM_WIDE=$w timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
      >> $O/ab_step.jsonl 2>> $O/ab_step.err
  done
done
echo "ab ok"
