#!/bin/bash
# Round 5: are a launch's slowest K3 waves slow in cycles per block (starved) or in clock?
set -o pipefail
O=gpurun_out/r05ad
mkdir -p $O
timeout -k 10 300 python tools/diag_slow_cu.py --steps 12 > $O/slow_cu.txt 2>&1 || { tail -20 $O/slow_cu.txt; exit 1; }
tail -13 $O/slow_cu.txt
