#!/bin/bash
# round-4 batch ab: wgrad dwordx4 loads with the class setup per branch (fewer spills):
# every GPU test, a gemm_micro A/B against MST_WG_VEC=0, smoke, bench, rocprof stats, GEMM SQ counters.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4ab; mkdir -p $O
b() { "$@" || { rc=$?; echo "stopping: rc=$rc"; exit $rc; }; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1 2; do
  for v in 1 0; do
    for shp in "--B 32 --T 252 --cin 1536 --cout 1536" "--B 32 --T 63 --cin 2048 --cout 2048"; do
      echo "== vec $v $shp" >> $O/micro.txt
      b env MST_WG_VEC=$v timeout -k 10 120 python -u tools/gemm_micro.py $shp --kinds wgrad --reps 20 >> $O/micro.txt 2>> $O/micro.err
    done
  done
done
echo "micro ok"
bash tools/gpu_measure.sh r4ab smoke bench prof && \
  bash tools/pmc_cmd.sh $O/pmc_gemm bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-aux --kernel-timing-steps 0
