set -o pipefail
export TMPDIR=/tmp
for m in 2 1; do
  OUT=gpurun_out/tr8_$m; mkdir -p $OUT
  HBX_PLAN_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --files 8 --steps 100 --warmup 5 --workload random --no-cpu-baseline --no-check --join-lag 2 > $OUT/log 2>&1 || { tail -5 $OUT/log; exit 1; }
  KT=$(find $OUT -name "*kernel_trace.csv" | head -1)
  echo "== plan_mode=$m"; grep '^{' $OUT/log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
  python3 tools/trace_steps.py $KT -30 3
  python3 tools/window_timeline.py $KT 100 | head -4
done
