#!/bin/bash
# round-4 batch y: split-K cost-model constants re-checked on the final kernels (env only).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4z; mkdir -p $O
b() { "$@" || { rc=$?; echo "stopping: rc=$rc"; exit $rc; }; }
for r in 1 2; do
  for cfg in "3.4e-6:8e12" "4.8e-6:8e12" "6.5e-6:8e12" "9e-6:8e12"; do
    tau=${cfg%%:*}; bw=${cfg##*:}
    echo "== tau $tau bw $bw" >> $O/ab_step.jsonl
    b env MST_SPLITK_TAU=$tau MST_SPLITK_BW=$bw timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
      >> $O/ab_step.jsonl 2>> $O/ab_step.err
  done
done
echo "all ok"
