#!/bin/bash
# round-4 batch g: conflict-free plane swizzle (variants/swz; wide conv GEMM on by default there)
# vs the in-tree build; bias gradients on the side stream (MST_BIAS_SIDE) A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4g; mkdir -p $O
V=$PWD/variants/swz/libmst_hip.so
t() { local log=$1; shift; "$@" > "$O/$log" 2>&1; local rc=$?; echo "$log rc=$rc";
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $log rc=$rc"; exit $rc; fi; }
b() { "$@" || { rc=$?; echo "stopping: rc=$rc"; exit $rc; }; }
PT="python -u -m pytest -q --timeout 120 --timeout-method thread"
t pytest_swz_w1.log env MST_LIB_PATH=$V MST_GEMM_WIDE=1 timeout -k 10 500 $PT tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_bench_shapes.py
t pytest_swz_w0.log env MST_LIB_PATH=$V MST_GEMM_WIDE=0 timeout -k 10 300 $PT tests/test_gpu_kernels.py
for r in 1 2 3; do
  for cfg in "in-tree:1:0" "$V:1:0" "$V:1:1" "$V:0:1"; do
    IFS=: read lib w bs <<< "$cfg"; [ "$lib" = in-tree ] && lib=""
    echo "== lib ${lib:-in-tree} wide $w bias_side $bs" >> $O/ab_step.jsonl
    b env MST_LIB_PATH=$lib MST_GEMM_WIDE=$w MST_BIAS_SIDE=$bs timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
      >> $O/ab_step.jsonl 2>> $O/ab_step.err
  done
done
echo "ab ok"
b env MST_LIB_PATH=$V MST_GEMM_WIDE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_swz1 -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-aux --kernel-timing-steps 0 > $O/prof_swz1.json 2> $O/prof_swz1.err
echo "prof ok"
b env MST_LIB_PATH=$V MST_GEMM_WIDE=1 bash tools/pmc_cmd.sh $O/pmc_gemm bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-aux --kernel-timing-steps 0
echo "all ok"
