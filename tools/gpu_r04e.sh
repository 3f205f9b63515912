#!/bin/bash
# Round 4's rocprof evidence and BASELINE configs on the final tree.
set -o pipefail
bash tools/profile_round.sh ${TAG:-r04z} || exit 1
bash tools/gpu_configs.sh || exit 1
echo done
