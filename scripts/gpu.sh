#!/bin/bash
# One entry point for GPU runs through gpurun (replaces the per-experiment gpu_*.sh files of
# rounds 1-6; those remain in the git history and the profiles/ notes name them).
#
#   gpurun --timeout 1200 -- 'bash scripts/gpu.sh <task> [args]'
#
# tasks (output under gpurun_out/<tag>/, every GPU step under its own time limit, chained so
# that the first failure ends the call):
#   tests [pytest -k expr]     the GPU test tier (-m gpu), verbose, per-test timeout
#   smoke                      __graft_entry__.smoke()
#   bench [bench.py args]      the headline bench (default: bench.py's own defaults)
#   final                      tests + smoke + bench twice (the round-end sequence)
#   prof [bench.py args]       rocprofv3 --kernel-trace --stats over a short bench; stats copied
#   pmc <driver.py>            counter passes over a launch driver (scripts/gpu_pmc_run.sh)
#   arrivals [rates...]        open-loop Poisson arrivals (bench.py --arrival-rate), default 90 60,
#                              burst heuristics on and off
#   mixtral                    Mixtral-8x7B HTTP C=256 + engine C=1
#   ab <ENV=val> [bench args]  the headline bench with and without one environment setting
#   tp                         TP tests on one card (ranks share the GPU) + the sampling rehearsal
#   gemm [bs_bench.py args]    decode / prefill GEMM microbenchmarks (scripts/bs_bench.py)
set -o pipefail
export PYTHONUNBUFFERED=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
source scripts/gpu_heartbeat.sh
task=${1:-tests}
shift
O=gpurun_out/${GPU_TAG:-$task}
mkdir -p "$O"

run_tests() {
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 420 --timeout-method thread --durations=15 \
    "$@" > "$O/tests.log" 2>&1
  local rc=$?
  tail -20 "$O/tests.log"
  return $rc
}

run_bench() {
  local name=$1
  shift
  timeout -k 10 600 python -u bench.py "$@" > "$O/$name.log" 2> "$O/$name.err"
  local rc=$?
  echo "$name rc=$rc"
  tail -1 "$O/$name.log"
  [ $rc -ne 0 ] && tail -5 "$O/$name.err"
  return $rc
}

case $task in
  tests)
    run_tests "$@" ;;
  smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
    rc=$?; tail -5 "$O/smoke.log"; exit $rc ;;
  bench)
    run_bench bench "$@" ;;
  final)
    run_tests &&
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 &&
      run_bench bench1 && run_bench bench2 ;;
  prof)
    # kernel trace of one timed wave (engine or HTTP per the bench args) -> summary.md: whole-run
    # table, decode steady state per step and per (kernel, grid) (scripts/prof_summary.py)
    cd /tmp && export TMPDIR=/tmp
    rm -rf /tmp/prof
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run --output-format csv -- \
      python3 "$R/bench.py" --steps 1 --warmup 1 "$@" > "$R/$O/prof.log" 2>&1
    rc=$?
    cd "$R"
    cp $(find /tmp/prof -name "*kernel_stats.csv" | head -1) "$O/kernel_stats.csv" 2>/dev/null
    [ $rc -eq 0 ] && python3 scripts/prof_summary.py /tmp/prof "${PROF_TITLE:-kernel trace: bench.py $*}" \
      --steady 32 --by-grid 32 > "$O/summary.md"
    tail -2 "$O/prof.log"
    exit $rc ;;
  pmc)
    bash scripts/gpu_pmc_run.sh "$1" "$O" ;;
  arrivals)
    # each rate with the burst heuristics (admission window, prefill-first) on, then off
    rates=${*:-90 60}
    for rate in $rates; do
      run_bench "r${rate}_on" --warmup 1 --arrival-rate "$rate" --requests $((rate * 10)) || exit 1
      LOCALAI_AMD_ADMIT_WINDOW_MS=0 LOCALAI_AMD_PREFILL_FIRST_MS=0 \
        run_bench "r${rate}_off" --warmup 1 --arrival-rate "$rate" --requests $((rate * 10)) || exit 1
    done ;;
  mixtral)
    # BASELINE config 4's model: HTTP C=256 (headline layout), engine C=1; extra args go to the
    # C=256 run (e.g. an A/B setting through env)
    run_bench mx_http --preset mixtral-8x7b --steps 2 --warmup 1 "$@" &&
      run_bench mx_c1 --preset mixtral-8x7b --mode engine --concurrency 1 --steps 2 --warmup 1 ;;
  mixtral_ab)
    # Mixtral HTTP C=256 with the MoE variants pinned by one env setting, then the defaults
    setting=$1
    env $setting timeout -k 10 600 python -u bench.py --preset mixtral-8x7b --steps 2 --warmup 1 \
      > "$O/mx_ab.log" 2> "$O/mx_ab.err"
    rc=$?; echo "$setting rc=$rc"; tail -1 "$O/mx_ab.log"; [ $rc -ne 0 ] && exit $rc
    run_bench mx_http --preset mixtral-8x7b --steps 2 --warmup 1 ;;
  ab)
    setting=$1
    shift
    run_bench base "$@" && env "$setting" timeout -k 10 600 python -u bench.py "$@" > "$O/ab.log" 2> "$O/ab.err"
    rc=$?; echo "$setting rc=$rc"; tail -1 "$O/ab.log"; exit $rc ;;
  tp)
    timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tp_gpu.py \
      tests/test_tp_sample_gpu.py > "$O/tp_tests.log" 2>&1
    rc=$?; tail -12 "$O/tp_tests.log"; [ $rc -ne 0 ] && exit $rc
    python -c "from localai_amd.models import synth; synth.write_model('/tmp/tp.gguf', 'tiny-llama', exact=True)" &&
      TP_REHEARSAL_SAMPLING=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29611 scripts/tp_rehearsal.py /tmp/tp.gguf > "$O/rehearsal.log" 2>&1
    rc=$?; grep "TP_ROWS\|TP_OK\|TP texts" "$O/rehearsal.log"; exit $rc ;;
  gemm)
    timeout -k 10 600 python -u scripts/bs_bench.py "$@" > "$O/gemm.log" 2>&1
    rc=$?; tail -30 "$O/gemm.log"; exit $rc ;;
  *)
    echo "unknown task $task"; exit 2 ;;
esac
