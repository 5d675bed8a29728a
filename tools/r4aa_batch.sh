#!/bin/bash
# round-4 batch aa: wgrad dwordx4 loads in unmasked unit-stride K classes (MST_WG_VEC, default 1)
# vs dword loads (MST_WG_VEC=0): parity, gemm_micro wgrad per shape, then the training step.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4aa; mkdir -p $O
b() { "$@" || { rc=$?; echo "stopping: rc=$rc"; exit $rc; }; }
b timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_bench_shapes.py tests/test_gpu_model.py > $O/pytest.log 2>&1
echo "pytest ok"
for r in 1 2; do
  for v in 1 0; do
    for shp in "--B 32 --T 252 --cin 1536 --cout 1536" "--B 32 --T 126 --cin 2048 --cout 2048" \
               "--B 32 --T 63 --cin 2048 --cout 2048" "--B 32 --T 31 --cin 4096 --cout 4096"; do
      echo "== vec $v $shp" >> $O/micro.txt
      b env MST_WG_VEC=$v timeout -k 10 120 python -u tools/gemm_micro.py $shp --kinds wgrad --reps 20 >> $O/micro.txt 2>> $O/micro.err
    done
  done
done
echo "micro ok"
for r in 1 2; do
  for v in 1 0; do
    echo "== vec $v" >> $O/ab_step.jsonl
    b env MST_WG_VEC=$v timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
      >> $O/ab_step.jsonl 2>> $O/ab_step.err
  done
done
echo "all ok"
