#!/bin/bash
# How much K1's VALU work (as opposed to its memory traffic) slows K3 beside
# it: the default build against a diagnostic build whose K1 skips its digest
# loop (HBX_K1_DIAG_NODIGEST=1, build/variants/nodigest; maxima wrong, so the
# bench runs without its oracle check), alternating on one box.
set -o pipefail
VARIANTS="nodigest" BENCH_ARGS="--steps 100 --workload random" bash tools/gpu_ab.sh
