#!/bin/bash
# One parameterised GPU-box runner (replaces the per-call tools/gpu_r0*.sh
# scripts of rounds 2-5).  Run through gpurun from the repo root:
#   gpurun --timeout 1200 -- tools/gpu_run.sh <tag> <step> [<step> ...]
# Every step writes under gpurun_out/<tag>/, runs under its own time limit,
# and the first failing step ends the call (no GPU step after a failure).
# Steps:
#   tests        the GPU suite (pytest -m gpu), as the driver runs it
#   testsk=EXPR  a subset of the GPU suite (pytest -k EXPR)
#   bench        the driver's command (python bench.py) -> bench20.json
#   bench200     the same at 200 steps -> bench200.json
#   f8 / f16 / f32   the N = 8 / 4 / 2 per-GPU shares, 20-step window -> f<n>.json
#   f8x200       the N = 8 share over 200 steps
#   e2e          bench.py --e2e (host-inclusive headline) -> e2e.json
#   profile      tools/profile_round.sh <tag> (rocprof window + PMC passes)
#   wire         tools/bench_wire.py (config 5 to the verifying loopback sink)
#   config5      tools/bench_config5.py (100 k files from tmpfs, end to end)
#   ab=ENV       bench.py with HBX_AB=1 and ENV (e.g. ab=HBX_K3_PSETS=2) -> ab_<ENV>.json
#   b=NAME,[VAR=VAL,..],--arg,val,..   bench.py with that environment and those arguments -> NAME.json
#   copystall, env=VAR=VAL   the e2e leg with the slow-submit trace (+ HIP runtime log / one runtime variable)
set -o pipefail
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
summ() {  # one line per bench JSON
  python3 - "$1" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
h = d.get("host_ms_per_step", {})
print(sys.argv[1], "value", d["value"], "check", d.get("check_vs_oracle"), "ms/step", d["ms_per_step"],
      "K3", d.get("roofline", {}).get("avg_launch_ms"), "K1", d.get("k1_roofline", {}).get("avg_launch_ms"),
      "submit", h.get("submit_ms_median_max"), "zipf", d.get("zipf", {}).get("value"),
      "e2e", d.get("e2e", {}).get("value"), "life", d.get("lifetime", {}).get("cycles_per_block"),
      d.get("lifetime", {}).get("launch_overhead"), d.get("lifetime", {}).get("staging"), flush=True)
EOF
}
run_bench() {  # name, limit, args...
  local name=$1 lim=$2
  shift 2
  timeout -k 10 $lim python bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -20 $O/$name.err; exit 1; }
  summ $O/$name.json
}
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
        || { tail -40 $O/gpu_tests.log; exit 1; }
      tail -3 $O/gpu_tests.log ;;
    testsk=*)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${step#testsk=}" > $O/gpu_tests_k.log 2>&1 \
        || { tail -40 $O/gpu_tests_k.log; exit 1; }
      tail -3 $O/gpu_tests_k.log ;;
    bench) run_bench bench20 300 --gpus 1 --steps 20 --warmup 5 ;;  # the driver's command
    bench200) run_bench bench200 400 --steps 200 ;;
    f8) run_bench f8 300 --files 8 --steps 20 --warmup 5 --e2e-steps 0 --no-cpu-baseline --no-lifetime ;;
    f16) run_bench f16 300 --files 16 --steps 20 --warmup 5 --e2e-steps 0 --no-cpu-baseline --no-lifetime ;;
    f32) run_bench f32 300 --files 32 --steps 20 --warmup 5 --e2e-steps 0 --no-cpu-baseline --no-lifetime ;;
    f8x200) run_bench f8x200 400 --files 8 --steps 200 --warmup 5 --e2e-steps 0 --no-cpu-baseline --no-lifetime ;;
    e2e) run_bench e2e 300 --e2e --steps 40 --no-cpu-baseline ;;
    profile) timeout -k 10 1100 tools/profile_round.sh $TAG || exit 1 ;;
    wire)
      timeout -k 10 700 python tools/bench_wire.py --sampled > $O/wire.json 2> $O/wire.err || { tail -20 $O/wire.err; exit 1; }
      cat $O/wire.json ;;
    config5)
      timeout -k 10 700 python tools/bench_config5.py > $O/config5.json 2> $O/config5.err || { tail -20 $O/config5.err; exit 1; }
      cat $O/config5.json ;;
    config5t)  # config 5 with the slow-submit trace (every submit or copy call over 1 ms prints its phases)
      HBX_TRACE_SLOW_SUBMIT=1 timeout -k 10 700 python tools/bench_config5.py > $O/config5t.json 2> $O/config5t.err || { tail -20 $O/config5t.err; exit 1; }
      grep -c "hbx slow" $O/config5t.err; grep -A1 "hbx slow submit" $O/config5t.err | head -40 | cut -c1-400 ;;
    copystall)  # the host stall in the SDMA copy call (verdict r05 item 2): trace + HIP runtime wait/signal log
      HBX_TRACE_SLOW_SUBMIT=1 AMD_LOG_LEVEL=4 timeout -k 10 300 python bench.py --e2e --steps 25 --warmup 5 \
        --no-cpu-baseline --no-check > $O/copystall.json 2> $O/copystall.err || { tail -20 $O/copystall.err; exit 1; }
      grep -E "hbx slow" $O/copystall.err | head -20; summ $O/copystall.json ;;
    env=*)  # bench.py --e2e with one runtime environment variable (e.g. env=ROC_SIGNAL_POOL_SIZE=256)
      kv=${step#env=}
      env HBX_TRACE_SLOW_SUBMIT=1 "$kv" timeout -k 10 300 python bench.py --e2e --steps 60 --warmup 5 --no-cpu-baseline \
        --no-check > $O/env_$kv.json 2> $O/env_$kv.err || { tail -20 $O/env_$kv.err; exit 1; }
      grep -E "hbx slow" $O/env_$kv.err | head -20; summ $O/env_$kv.json ;;
    b=*)  # b=NAME,[VAR=VAL,...],--bench-arg,value,... -> NAME.json (VAR=VAL: environment; HBX_* need HBX_AB=1)
      IFS=, read -ra toks <<< "${step#b=}"
      name=${toks[0]}
      envs=()
      args=()
      for t in "${toks[@]:1}"; do
        if [[ $t == --* || ${#args[@]} -gt 0 ]]; then args+=("$t"); else envs+=("$t"); fi
      done
      env "${envs[@]}" timeout -k 10 400 python bench.py "${args[@]}" > $O/$name.json 2> $O/$name.err \
        || { echo "FAIL $step"; tail -20 $O/$name.err; exit 1; }
      summ $O/$name.json ;;
    hbms=*)  # tools/ubench/hbm_streams cases by name (comma-separated), chains alone
      IFS=, read -ra cs <<< "${step#hbms=}"
      for cn in "${cs[@]}"; do
        timeout -k 10 120 tools/ubench/hbm_streams 128 $cn >> $O/hbm_streams.txt 2>&1 || { tail -5 $O/hbm_streams.txt; exit 1; }
      done
      grep -v "^#" $O/hbm_streams.txt ;;
    slowcu)  # per-launch K3 probe: slowest CUs, their cycles per block and stage-wait polls
      timeout -k 10 300 python tools/diag_slow_cu.py > $O/slow_cu.txt 2> $O/slow_cu.err || { tail -20 $O/slow_cu.err; exit 1; }
      tail -4 $O/slow_cu.txt | cut -c1-600 ;;
    ab=*)
      kv=${step#ab=}
      env HBX_AB=1 "$kv" timeout -k 10 300 python bench.py --e2e-steps 0 --no-cpu-baseline > $O/ab_$kv.json 2> $O/ab_$kv.err \
        || { echo "FAIL $step"; tail -20 $O/ab_$kv.err; exit 1; }
      summ $O/ab_$kv.json ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
