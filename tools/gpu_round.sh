#!/bin/bash
# GPU box: parity tests, then the pipelined bench at two slice sizes and the
# single-batch path.  Every GPU step has its own time limit; the chain stops at
# the first failure.
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 240 python bench.py --md5-slice 16384 --check > $O/bs16k.json 2> $O/bs16k.err || { tail -20 $O/bs16k.err; exit 1; }
cat $O/bs16k.json
timeout -k 10 240 python bench.py --md5-slice 8192 --no-cpu-baseline --check > $O/bs8k.json 2> $O/bs8k.err || { tail -20 $O/bs8k.err; exit 1; }
cat $O/bs8k.json
timeout -k 10 240 python bench.py --md5-slice 0 --steps 10 --warmup 2 --no-cpu-baseline > $O/bs0.json 2> $O/bs0.err || { tail -20 $O/bs0.err; exit 1; }
cat $O/bs0.json
HBX_ONE_STREAM=1 timeout -k 10 240 python bench.py --md5-slice 16384 --no-cpu-baseline > $O/bs16k_1s.json 2> $O/bs16k_1s.err || { tail -20 $O/bs16k_1s.err; exit 1; }
cat $O/bs16k_1s.json
# A/B: unaligned message loads in K3 (parity first)
UA=$PWD/build/variants/ua1/libhbxgpu.so
HBX_LIB=$UA timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q > $O/pytest_ua1.log 2>&1 || { tail -30 $O/pytest_ua1.log; exit 1; }
tail -1 $O/pytest_ua1.log
HBX_LIB=$UA timeout -k 10 240 python bench.py --md5-slice 16384 --no-cpu-baseline --check > $O/bs16k_ua1.json 2> $O/bs16k_ua1.err || { tail -20 $O/bs16k_ua1.err; exit 1; }
cat $O/bs16k_ua1.json
timeout -k 10 300 python bench.py --no-cpu-baseline --check > $O/bs_auto.json 2> $O/bs_auto.err || { tail -20 $O/bs_auto.err; exit 1; }
cat $O/bs_auto.json
