#!/bin/bash
# Same-box A/B of the training step between two environment settings of the in-tree build (dev
# tool; via gpurun from the repo root): optional GPU tests first, then bench.py alternating
# "A" (no extra env) and "B" (the KNOB=VALUE in $ENVB), ROUNDS rounds.
#   ENVB="MST_GEMM_BCL=0" tools/ab_env_step.sh TAG [tests-selection]
set -e -o pipefail
OUT=gpurun_out/${1:?tag}; mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$2" ]; then
  timeout -k 10 800 python -u -m pytest $2 -x -v --timeout 200 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1
  echo "tests ok"
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for arm in A B; do
    echo "== arm $arm ${ENVB:?}" >> "$OUT/ab_step.jsonl"
    if [ $arm = A ]; then
      timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps ${STEPS:-20} --warmup 3 \
        >> "$OUT/ab_step.jsonl" 2>> "$OUT/ab_step.err"
    else
      env $ENVB timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps ${STEPS:-20} \
        --warmup 3 >> "$OUT/ab_step.jsonl" 2>> "$OUT/ab_step.err"
    fi
  done
done
echo "bench ok"
