#!/bin/bash
# round-4 batch ac: same-box training-step A/B of the wgrad dwordx4 loads (MST_WG_VEC 1 vs 0).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4ac; mkdir -p $O
b() { "$@" || { rc=$?; echo "stopping: rc=$rc"; exit $rc; }; }
for r in 1 2 3; do
  for v in 1 0; do
    echo "== vec $v" >> $O/ab_step.jsonl
    b env MST_WG_VEC=$v timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
      >> $O/ab_step.jsonl 2>> $O/ab_step.err
  done
done
echo "all ok"
