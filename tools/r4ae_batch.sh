#!/bin/bash
# round-4 batch ae: Adam inside backward (--adam-overlap) re-measured on the round-4 kernels,
# and the hipGraph-replayed step (--graph), same-box triples against the default.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4ae; mkdir -p $O
b() { "$@" || { rc=$?; echo "stopping: rc=$rc"; exit $rc; }; }
for r in 1 2 3; do
  echo "== overlap" >> $O/ab_step.jsonl
  b timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 --adam-overlap \
    >> $O/ab_step.jsonl 2>> $O/ab_step.err
  echo "== graph" >> $O/ab_step.jsonl
  b timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 --graph \
    >> $O/ab_step.jsonl 2>> $O/ab_step.err
  echo "== default" >> $O/ab_step.jsonl
  b timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
    >> $O/ab_step.jsonl 2>> $O/ab_step.err
done
echo "all ok"
