#!/bin/bash
# Round 5: K1 LDS image transposed per 1 KiB (conflict-free reads): parity, PMC bank conflicts, A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v -k "tile or mixed or edge or schedule" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for z in 0 1; do
HBX_AB=1 HBX_K1_SWZ=$z timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --kernel-include-regex "hbx_k1_digest" --output-format csv -d $O/pmc$z -o run -- python3 bench.py --steps 40 --warmup 2 --workload random --no-cpu-baseline --no-check --e2e-steps 0 --no-lifetime > $O/pmc$z.log 2>&1 || { tail -5 $O/pmc$z.log; exit 1; }
F=$(find $O/pmc$z -name "*counter_collection.csv" | head -1)
python3 - "$F" $z <<'PY'
import csv, sys, collections
d = collections.defaultdict(float); n = set()
for r in csv.DictReader(open(sys.argv[1])):
    d[r["Counter_Name"]] += float(r["Counter_Value"]); n.add(r["Dispatch_Id"])
k = len(n); w = d["SQ_WAVE_CYCLES"]
print("swz", sys.argv[2], "K1 per dispatch: bank_conflict %.3g wait_any %.3f active_valu %.3f" % (d["SQ_LDS_BANK_CONFLICT"] / k, d["SQ_WAIT_ANY"] / w, d["SQ_ACTIVE_INST_VALU"] / w))
PY
done
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random --no-lifetime $BARGS > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));k=d['lib']['knobs']
print('$n', d['value'], d['check_vs_oracle'], 'swz', k['k1_swz'], d['kernel_ms_per_step']['k1_digest_scan'], d['kernel_ms_per_step']['k3_block_md5'])"
}
BARGS="--steps 100"
for r in 1 2; do
  run f64_s0_$r HBX_AB=1 HBX_K1_SWZ=0 || exit 1
  run f64_s1_$r HBX_AB=1 HBX_K1_SWZ=1 || exit 1
done
BARGS="--steps 400 --files 8"
for r in 1 2; do
  run f8_s0_$r HBX_AB=1 HBX_K1_SWZ=0 || exit 1
  run f8_s1_$r HBX_AB=1 HBX_K1_SWZ=1 || exit 1
done
