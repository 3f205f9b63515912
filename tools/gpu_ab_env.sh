#!/bin/bash
# A/B of environment switches on one build, alternating so drift shows.
# usage: ENVS="HBX_HASH_CUS=prio:hi;HBX_RES_CUS=prio:hi" BENCH_ARGS="--steps 20" tools/gpu_ab_env.sh
#        REPS=3 (default 2) alternations
set -o pipefail
export HBX_AB=1  # the library honours HBX_* A/B switches only with this
O=gpurun_out/abenv
mkdir -p $O
IFS=';' read -ra VS <<< "base;${ENVS}"
for rep in $(seq 1 ${REPS:-2}); do
  for v in "${VS[@]}"; do
    tag=$(echo "$v" | tr -c 'A-Za-z0-9' '_')
    if [ "$v" = base ]; then E=""; else E="$v"; fi
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-check --workload random $BENCH_ARGS > $O/$tag.$rep.json 2> $O/$tag.$rep.err || { tail -5 $O/$tag.$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$tag.$rep.json'));print('$v', d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"
  done
done
