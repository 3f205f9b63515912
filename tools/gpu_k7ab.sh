#!/bin/bash
# K7a A/B over build flags (tools/ubench/k7_phases.hip, 256 MiB Zipf text): one line set per flag set.
set -o pipefail
O=gpurun_out/k7ab
mkdir -p $O
: > $O/k7ab.txt
i=0
for flags in "$@"; do
  i=$((i+1))
  hipcc --offload-arch=gfx950 -O3 -std=c++17 $flags -I${K7SRC:-hashbox_amd/csrc} -Ihashbox_amd/csrc -o $O/k7p_$i tools/ubench/k7_phases.hip || exit 1
  echo "## $flags" >> $O/k7ab.txt
  timeout -k 10 120 $O/k7p_$i 256 >> $O/k7ab.txt 2>&1 || { cat $O/k7ab.txt; exit 1; }
done
cat $O/k7ab.txt
