#!/bin/bash
# round-4 batch t: weight gradients on the 128 x 256 kernel (variants/wgw with MST_GEMM_WIDE_WG=1)
# vs the 128 x 128 kernel (same library, knob off, and in-tree): parity first, then gemm_micro and
# the step.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4t; mkdir -p $O
V=$PWD/variants/wgw/libmst_hip.so
t() { local log=$1; shift; "$@" > "$O/$log" 2>&1; local rc=$?; echo "$log rc=$rc";
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $log rc=$rc"; exit $rc; fi; }
b() { "$@" || { rc=$?; echo "stopping: rc=$rc"; exit $rc; }; }
t pytest_wgw.log env MST_LIB_PATH=$V MST_GEMM_WIDE_WG=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_bench_shapes.py
if grep -q " failed" $O/pytest_wgw.log; then echo "parity failed"; exit 0; fi
for r in 1 2; do
  for w in 0 1; do
    for shp in "--B 32 --T 252 --cin 1536 --cout 1536" "--B 32 --T 15 --cin 4096 --cout 4096" "--B 32 --T 126 --cin 2048 --cout 2048"; do
      echo "== wide_wg $w $shp" >> $O/micro.txt
      b env MST_LIB_PATH=$V MST_GEMM_WIDE_WG=$w timeout -k 10 120 python -u tools/gemm_micro.py $shp --kinds wgrad --reps 20 >> $O/micro.txt 2>> $O/micro.err
    done
  done
done
echo "micro ok"
for r in 1 2; do
  for w in 0 1; do
    echo "== wide_wg $w" >> $O/ab_step.jsonl
    b env MST_LIB_PATH=$V MST_GEMM_WIDE_WG=$w timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
      >> $O/ab_step.jsonl 2>> $O/ab_step.err
  done
done
echo "all ok"
