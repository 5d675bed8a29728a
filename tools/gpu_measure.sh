#!/bin/bash
# One GPU-box measurement pass (run via gpurun from the repo root). Each GPU step has its own
# time limit and the steps are chained: the first failure ends the script.
#   tools/gpu_measure.sh TAG [tests] [bench] [prof] [pmc] [aux]
set -e -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for what in "$@"; do
  case $what in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 ;;
    bench)
      timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
        python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-aux > "$OUT/prof_bench.json" 2> "$OUT/prof.err" ;;
    pmc)
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-aux --kernel-timing-steps 0 > "$OUT/pmc_fetch.log" 2>&1
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-aux --kernel-timing-steps 0 > "$OUT/pmc_write.log" 2>&1 ;;
    pmcaux)
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcaux_fetch" -o run -- \
        python3 bench_aux.py --workload frontend --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/pmcaux_fetch.log" 2>&1
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmcaux_write" -o run -- \
        python3 bench_aux.py --workload frontend --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/pmcaux_write.log" 2>&1 ;;
    pmcgl)
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcgl_fetch" -o run -- \
        python3 bench_aux.py --workload griffinlim --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/pmcgl_fetch.log" 2>&1
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmcgl_write" -o run -- \
        python3 bench_aux.py --workload griffinlim --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/pmcgl_write.log" 2>&1 ;;
    pmcmss)
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcmss_fetch" -o run -- \
        python3 bench_aux.py --workload mss --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/pmcmss_fetch.log" 2>&1
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmcmss_write" -o run -- \
        python3 bench_aux.py --workload mss --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/pmcmss_write.log" 2>&1 ;;
    micro)
      make -C tools/micro > "$OUT/micro_build.log" 2>&1
      timeout -k 10 60 tools/micro/permlane_check > "$OUT/permlane_check.txt" 2>&1
      timeout -k 10 120 tools/micro/store_pattern > "$OUT/store_pattern.txt" 2>&1
      timeout -k 10 120 tools/micro/stft_stamps > "$OUT/stft_stamps.txt" 2>&1 ;;
    aux)
      timeout -k 10 400 python -u bench_aux.py > "$OUT/bench_aux.jsonl" 2> "$OUT/bench_aux.err" ;;
    layers)
      timeout -k 10 300 python -u tools/gemm_layers.py > "$OUT/gemm_layers.txt" 2> "$OUT/gemm_layers.err" ;;
    msstest)
      timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        -k "multiscale or mss" > "$OUT/pytest_mss.log" 2>&1 ;;
    gltest)
      timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        -k "griffinlim or istft or stft or mel" > "$OUT/pytest_gl.log" 2>&1 ;;
    auxgl)
      timeout -k 10 300 python -u bench_aux.py --workload griffinlim --no-cpu-baseline > "$OUT/aux_gl.json" 2> "$OUT/aux_gl.err" ;;
    auxmss)
      timeout -k 10 300 python -u bench_aux.py --workload mss --no-cpu-baseline > "$OUT/aux_mss.json" 2> "$OUT/aux_mss.err" ;;
    profaux)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profaux" -o run -- \
        python3 bench_aux.py --no-cpu-baseline --steps 5 --warmup 2 > "$OUT/profaux.json" 2> "$OUT/profaux.err" ;;
    abstft)
      for v in 2 4; do
        MST_STFT_WAVE=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_spectral.py -x -v --timeout 120 \
          --timeout-method thread -k "stft or logpow or power" > "$OUT/pytest_stftwave$v.log" 2>&1
      done
      for v in 0 2 4 0 2 4; do
        MST_STFT_WAVE=$v timeout -k 10 180 python -u bench_aux.py --workload frontend --no-cpu-baseline \
          >> "$OUT/ab_stftwave$v.jsonl" 2>> "$OUT/ab_stft.err"
      done ;;
    abmss2)
      for lib in "" variants/mss_head/libmst_hip.so "" variants/mss_head/libmst_hip.so; do
        echo "== lib ${lib:-in-tree}" >> "$OUT/ab_mss2.jsonl"
        MST_LIB_PATH=$lib timeout -k 10 180 python bench_aux.py --workload mss --no-cpu-baseline --steps 10 --warmup 2 \
          >> "$OUT/ab_mss2.jsonl" 2>> "$OUT/ab_mss2.err"
      done ;;
    abpk)
      MST_STFT_PK=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_inference.py -x -v --timeout 120 \
        --timeout-method thread > "$OUT/pytest_pk.log" 2>&1
      for v in 0 1 0 1; do
        MST_STFT_PK=$v timeout -k 10 180 python -u bench_aux.py --workload frontend --no-cpu-baseline \
          >> "$OUT/ab_pk$v.jsonl" 2>> "$OUT/ab_pk.err"
      done ;;
    abtau)
      for t in 3.4e-6 2.6e-6 4.2e-6 3.4e-6 2.6e-6 4.2e-6; do
        echo "== tau $t" >> "$OUT/ab_tau.jsonl"
        MST_SPLITK_TAU=$t timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
          >> "$OUT/ab_tau.jsonl" 2>> "$OUT/ab_tau.err"
      done ;;
    abin)
      timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
        -k "instnorm" > "$OUT/pytest_in.log" 2>&1
      for v in 0 1 0 1; do
        echo "== MST_IN_SEG=$v" >> "$OUT/ab_in.jsonl"
        MST_IN_SEG=$v timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
          >> "$OUT/ab_in.jsonl" 2>> "$OUT/ab_in.err"
      done ;;
    abgl)
      for lib in "" variants/gl_head/libmst_hip.so "" variants/gl_head/libmst_hip.so; do  # in-tree vs HEAD fft.hip
        echo "== lib ${lib:-in-tree}" >> "$OUT/ab_gl.jsonl"
        MST_LIB_PATH=$lib timeout -k 10 200 python -u bench_aux.py --workload griffinlim --no-cpu-baseline \
          >> "$OUT/ab_gl.jsonl" 2>> "$OUT/ab_gl.err"
      done ;;
    abcx)
      timeout -k 10 300 python -u -m pytest tests/test_gpu_spectral.py tests/test_istft_grad.py tests/test_gpu_inference.py \
        -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_cx.log" 2>&1
      for v in 1 0 1 0; do
        echo "== MST_STFT_CX_FM=$v" >> "$OUT/ab_cx.jsonl"
        MST_STFT_CX_FM=$v timeout -k 10 200 python -u bench_aux.py --workload griffinlim --no-cpu-baseline \
          >> "$OUT/ab_cx.jsonl" 2>> "$OUT/ab_cx.err"
      done ;;
    abgltab)
      timeout -k 10 300 python -u -m pytest tests/test_gpu_spectral.py -x -v --timeout 120 --timeout-method thread \
        -k "griffinlim" > "$OUT/pytest_gltab.log" 2>&1
      for v in 1 0 1 0; do
        echo "== MST_GL_TABS=$v" >> "$OUT/ab_gltab.jsonl"
        MST_GL_TABS=$v timeout -k 10 200 python -u bench_aux.py --workload griffinlim --no-cpu-baseline \
          >> "$OUT/ab_gltab.jsonl" 2>> "$OUT/ab_gltab.err"
      done ;;
    abmel)
      for lib in "" variants/mel_head/libmst_hip.so "" variants/mel_head/libmst_hip.so; do
        echo "== lib ${lib:-in-tree}" >> "$OUT/ab_mel.jsonl"
        MST_LIB_PATH=$lib timeout -k 10 200 python -u bench_aux.py --workload frontend --no-cpu-baseline \
          >> "$OUT/ab_mel.jsonl" 2>> "$OUT/ab_mel.err"
      done ;;
    abmssreg)
      timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        -k "multiscale or mss" > "$OUT/pytest_mssreg.log" 2>&1
      for v in 1 0 1 0; do
        echo "== MST_MSS_REG=$v" >> "$OUT/ab_mssreg.jsonl"
        MST_MSS_REG=$v timeout -k 10 180 python bench_aux.py --workload mss --no-cpu-baseline --steps 10 --warmup 2 \
          >> "$OUT/ab_mssreg.jsonl" 2>> "$OUT/ab_mssreg.err"
      done ;;
    abmssil)
      timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        -k "multiscale or mss" > "$OUT/pytest_mssil.log" 2>&1
      for v in 1 0 1 0; do
        echo "== MST_MSS_IL=$v" >> "$OUT/ab_mssil.jsonl"
        MST_MSS_IL=$v timeout -k 10 180 python bench_aux.py --workload mss --no-cpu-baseline --steps 10 --warmup 2 \
          >> "$OUT/ab_mssil.jsonl" 2>> "$OUT/ab_mssil.err"
      done ;;
    abbr)
      timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -v --timeout 120 \
        --timeout-method thread > "$OUT/pytest_br.log" 2>&1
      for lib in "" variants/br_head/libmst_hip.so "" variants/br_head/libmst_hip.so; do
        echo "== lib ${lib:-in-tree}" >> "$OUT/ab_br.jsonl"
        MST_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
          >> "$OUT/ab_br.jsonl" 2>> "$OUT/ab_br.err"
      done ;;
    msst)
      timeout -k 10 400 python -u -m pytest tests/test_gpu_spectral.py -x -v --timeout 120 --timeout-method thread \
        -k "multiscale or mss" > "$OUT/pytest_mss.log" 2>&1 ;;
    profmss)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profmss" -o run -- \
        python3 bench_aux.py --workload mss --no-cpu-baseline --no-parity --steps 5 --warmup 2 > "$OUT/profmss.json" 2> "$OUT/profmss.err" ;;
    adamab)
      MST_ADAM_VARIANT=2n timeout -k 10 200 python -u tools/adam_micro.py > "$OUT/adam_micro.jsonl" 2>&1
      MST_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_nows" -o run -- \
        python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-aux > "$OUT/prof_nows.json" 2> "$OUT/prof_nows.err" ;;
    abws)
      for v in 1 0 1 0 1 0; do
        echo "== MST_WGRAD_STREAM=$v" >> "$OUT/ab_ws.jsonl"
        MST_WGRAD_STREAM=$v timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
          >> "$OUT/ab_ws.jsonl" 2>> "$OUT/ab_ws.err"
      done ;;
    gemmt)
      timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_bench_shapes.py -x -q \
        --timeout 120 --timeout-method thread > "$OUT/pytest_gemm.log" 2>&1 ;;
    abprev)
      for lib in "" variants/prev/libmst_hip.so "" variants/prev/libmst_hip.so "" variants/prev/libmst_hip.so; do
        echo "== lib ${lib:-in-tree}" >> "$OUT/ab_prev.jsonl"
        MST_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
          >> "$OUT/ab_prev.jsonl" 2>> "$OUT/ab_prev.err"
      done ;;
    abfm16)
      MST_LIB_PATH=variants/fm16/libmst_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_config2.py \
        -x -q --timeout 120 --timeout-method thread -k "stft or mel or logpow or process_spectrum" > "$OUT/pytest_fm16.log" 2>&1
      for lib in "" variants/fm16/libmst_hip.so "" variants/fm16/libmst_hip.so; do
        echo "== lib ${lib:-in-tree}" >> "$OUT/ab_fm16.jsonl"
        MST_LIB_PATH=$lib timeout -k 10 200 python -u bench_aux.py --workload frontend --no-cpu-baseline \
          >> "$OUT/ab_fm16.jsonl" 2>> "$OUT/ab_fm16.err"
      done ;;
    abfm16gl)
      MST_LIB_PATH=variants/fm16/libmst_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_config2.py \
        tests/test_istft_grad.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_fm16_all.log" 2>&1
      for lib in "" variants/fm16/libmst_hip.so "" variants/fm16/libmst_hip.so; do
        echo "== lib ${lib:-in-tree}" >> "$OUT/ab_fm16_gl.jsonl"
        MST_LIB_PATH=$lib timeout -k 10 200 python -u bench_aux.py --workload griffinlim --no-cpu-baseline --no-parity \
          >> "$OUT/ab_fm16_gl.jsonl" 2>> "$OUT/ab_fm16_gl.err"
        MST_LIB_PATH=$lib timeout -k 10 200 python -u bench_aux.py --workload frontend --no-cpu-baseline --no-parity \
          >> "$OUT/ab_fm16_gl.jsonl" 2>> "$OUT/ab_fm16_gl.err"
      done ;;
    biasab)
      timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 120 \
        --timeout-method thread > "$OUT/pytest_bias.log" 2>&1
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
        python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-aux > "$OUT/prof_bench.json" 2> "$OUT/prof.err" ;;
    abprealloc)
      for v in 0 1 0 1 0 1; do
        echo "== MST_BENCH_PREALLOC=$v" >> "$OUT/ab_prealloc.jsonl"
        MST_BENCH_PREALLOC=$v timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
          >> "$OUT/ab_prealloc.jsonl" 2>> "$OUT/ab_prealloc.err"
      done ;;
    pmcmsssq)
      timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv \
        -d "$OUT/pmcmss_sq" -o run -- python3 bench_aux.py --workload mss --no-cpu-baseline --no-parity \
        --steps 2 --warmup 1 > "$OUT/pmcmss_sq.log" 2>&1 ;;
    abmssprev)
      for lib in "" variants/prev/libmst_hip.so "" variants/prev/libmst_hip.so "" variants/prev/libmst_hip.so; do
        echo "== lib ${lib:-in-tree}" >> "$OUT/ab_mss_prev.jsonl"
        MST_LIB_PATH=$lib timeout -k 10 200 python -u bench_aux.py --workload mss --no-cpu-baseline --no-parity \
          --steps 20 --warmup 3 >> "$OUT/ab_mss_prev.jsonl" 2>> "$OUT/ab_mss_prev.err"
      done ;;
    mssprobe)
      timeout -k 10 300 python -u tools/mss_probe.py > "$OUT/mss_probe.txt" 2>&1 ;;
    benchnoaux)
      timeout -k 10 300 python -u bench.py --no-aux > "$OUT/bench_noaux.json" 2> "$OUT/bench_noaux.err" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    *) echo "unknown step $what"; exit 2 ;;
  esac
  echo "step $what ok"
done
