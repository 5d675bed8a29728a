#!/bin/bash
# round-4 batch e. In-tree library = control (HEAD kernels); variants/mssf = chunk-staged
# InstanceNorm, new bias kernels, wide conv GEMM (MST_GEMM_WIDE=1), fused small-size MSS.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4e; mkdir -p $O
V=$PWD/variants/mssf/libmst_hip.so
t() { local log=$1; shift; "$@" > "$O/$log" 2>&1; local rc=$?; echo "$log rc=$rc";
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $log rc=$rc"; exit $rc; fi; }
b() { "$@" || { rc=$?; echo "stopping: rc=$rc"; exit $rc; }; }
PT="python -u -m pytest -q --timeout 120 --timeout-method thread"
t pytest_mssf.log env MST_LIB_PATH=$V timeout -k 10 700 $PT tests -m gpu
t pytest_mssf_wide1.log env MST_LIB_PATH=$V MST_GEMM_WIDE=1 timeout -k 10 400 $PT tests/test_gpu_kernels.py tests/test_gpu_model.py -k "conv or gemm or dgrad or forward or backward"
for r in 1 2; do
  for cfg in "in-tree::0" "$V::0" "$V::1"; do
    lib=${cfg%%::*}; w=${cfg##*::}; [ "$lib" = in-tree ] && lib=""
    echo "== lib ${lib:-in-tree} wide $w" >> $O/ab_step.jsonl
    b env MST_LIB_PATH=$lib MST_GEMM_WIDE=$w timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
      >> $O/ab_step.jsonl 2>> $O/ab_step.err
  done
  for lib in "" $V; do
    echo "== lib ${lib:-in-tree}" >> $O/ab_mss.jsonl
    b env MST_LIB_PATH=$lib timeout -k 10 200 python -u bench_aux.py --workload mss --no-cpu-baseline --steps 10 --warmup 2 \
      >> $O/ab_mss.jsonl 2>> $O/ab_mss.err
  done
done
echo "ab ok"
for cfg in "in-tree::0" "$V::0" "$V::1"; do
  lib=${cfg%%::*}; w=${cfg##*::}; [ "$lib" = in-tree ] && lib=""; tag=$([ -z "$lib" ] && echo tree || echo mssf)$w
  b env MST_LIB_PATH=$lib MST_GEMM_WIDE=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$tag -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-aux > $O/prof_$tag.json 2> $O/prof_$tag.err
done
echo "prof ok"
b env MST_LIB_PATH=$V bash tools/gpu_measure.sh r4e pmcgl pmcmss
echo "all ok"
