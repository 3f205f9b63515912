#!/bin/bash
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in r10 r12 dense; do
  HBX_LIB=$PWD/build/variants/$v/libhbxgpu.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "pipelined or edge or device_resident" > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
tools/ab_k3.sh
