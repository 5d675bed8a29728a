#!/bin/bash
# round-4 batch k: InstanceNorm with paired 8-byte loads/stores for even T (variants/inev) and
# MSS twiddles/window from a compile-time table (both variants), and
# the same plus static priority for the wide GEMM's younger half (variants/prio) vs in-tree.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4k; mkdir -p $O
V1=$PWD/variants/inev/libmst_hip.so; V2=$PWD/variants/prio/libmst_hip.so
t() { local log=$1; shift; "$@" > "$O/$log" 2>&1; local rc=$?; echo "$log rc=$rc";
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $log rc=$rc"; exit $rc; fi; }
b() { "$@" || { rc=$?; echo "stopping: rc=$rc"; exit $rc; }; }
PT="python -u -m pytest -q --timeout 120 --timeout-method thread"
t pytest_prio.log env MST_LIB_PATH=$V2 timeout -k 10 500 $PT tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_bench_shapes.py
t pytest_mss.log env MST_LIB_PATH=$V1 timeout -k 10 300 $PT tests/test_gpu_spectral.py -k "multiscale or mss"
for r in 1 2 3; do
  for lib in "" $V1 $V2; do
    echo "== lib ${lib:-in-tree}" >> $O/ab_step.jsonl
    b env MST_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
      >> $O/ab_step.jsonl 2>> $O/ab_step.err
  done
done
for r in 1 2; do
  for lib in "" $V1; do
    echo "== lib ${lib:-in-tree}" >> $O/ab_mss.jsonl
    b env MST_LIB_PATH=$lib timeout -k 10 200 python -u bench_aux.py --workload mss --no-cpu-baseline --steps 10 --warmup 2 \
      >> $O/ab_mss.jsonl 2>> $O/ab_mss.err
  done
done
echo "ab ok"
for lib in "" $V2; do
  tag=$([ -z "$lib" ] && echo tree || echo prio)
  b env MST_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$tag -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-aux --kernel-timing-steps 0 > $O/prof_$tag.json 2> $O/prof_$tag.err
done
echo "all ok"
