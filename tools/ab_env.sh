#!/bin/bash
# Same-box A/B of the training step: the default build vs the same build with one knob set
# (environment), alternated N times (dev tool; via gpurun).  tools/ab_env.sh TAG "VAR=val [VAR2=val]" [N]
set -e -o pipefail
OUT=gpurun_out/${1:?tag}; mkdir -p "$OUT"
KNOB=${2:?knob}
N=${3:-3}
for i in $(seq 1 "$N"); do
  for k in "" "$KNOB"; do
    echo "== knob ${k:-default}" >> "$OUT/ab_env.jsonl"
    env $k timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
      >> "$OUT/ab_env.jsonl" 2>> "$OUT/ab_env.err"
  done
done
echo "ab ok"
