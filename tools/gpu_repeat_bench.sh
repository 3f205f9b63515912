#!/bin/bash
# The driver's bench command several times in one call (run-to-run spread on one box),
# then a long steady-state run.  usage: bash tools/gpu_repeat_bench.sh [repeats] [long_steps]
set -o pipefail
O=gpurun_out/repeat; mkdir -p $O
for i in $(seq 1 ${1:-3}); do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --workload random --no-cpu-baseline > $O/b20_$i.json 2> $O/b20_$i.err || { tail -3 $O/b20_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b20_$i.json').read().strip().splitlines()[-1]);print('20 steps', d['value'], d['ms_per_step'], d['check_vs_oracle'])"
done
timeout -k 10 400 python bench.py --steps ${2:-2000} --warmup 5 --workload random --no-cpu-baseline --no-check > $O/long.json 2> $O/long.err || { tail -3 $O/long.err; exit 1; }
python -c "import json;d=json.loads(open('$O/long.json').read().strip().splitlines()[-1]);print('long', d['steps'], d['value'], d['ms_per_step'], d['roofline']['frac'])"
