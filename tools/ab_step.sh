#!/bin/bash
# Same-box A/B of the training step (dev tool; via gpurun from the repo root): optional GPU tests on
# the in-tree build first, then bench.py alternating the in-tree library with VAR (default
# variants/base/libmst_hip.so, e.g. the previous commit's build), N rounds.
#   tools/ab_step.sh TAG [tests-selection] ; env: VAR, ROUNDS (2), STEPS (20)
set -e -o pipefail
OUT=gpurun_out/${1:?tag}; mkdir -p "$OUT"
V=${VAR:-variants/base/libmst_hip.so}
export TMPDIR=/tmp
if [ -n "$2" ]; then
  timeout -k 10 700 python -u -m pytest $2 -x -v --timeout 120 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1
  echo "tests ok"
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "" $V; do
    echo "== lib ${lib:-in-tree}" >> "$OUT/ab_step.jsonl"
    MST_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps ${STEPS:-20} \
      --warmup 3 >> "$OUT/ab_step.jsonl" 2>> "$OUT/ab_step.err"
  done
done
echo "bench ok"
