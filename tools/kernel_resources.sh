#!/bin/bash
# Register / scratch / occupancy of every narrow-phase kernel at the current source: the 12 parts of
# csrc/gjkepa_kernel.hip compiled in parallel with -Rpass-analysis=kernel-resource-usage (objects
# discarded), summarised by tools/resources.py.  usage: bash tools/kernel_resources.sh > out.txt
D=collision-detect-gjk-epa_amd
T=$(mktemp -d)
F="--offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 -Wno-unused-function -Rpass-analysis=kernel-resource-usage"
for p in 0 1 2 3 4 5 6 7 8 9 10 11; do
  /opt/rocm/bin/hipcc $F -DGK_PART=$p -c $D/csrc/gjkepa_kernel.hip -o $T/k$p.o 2> $T/r$p.txt &
done
wait
cat $T/r*.txt | c++filt | python3 tools/resources.py | sort -u
rm -rf $T
