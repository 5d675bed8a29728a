#!/bin/bash
# round-4 batch ad: the final tree's default bench line (aux legs and CPU baseline included),
# three back-to-back runs on one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4ad; mkdir -p $O
b() { "$@" || { rc=$?; echo "stopping: rc=$rc"; exit $rc; }; }
for r in 1 2 3; do
  b timeout -k 10 400 python -u bench.py >> $O/bench_repeat3.jsonl 2>> $O/bench.err
  echo "run $r ok"
done
echo "all ok"
