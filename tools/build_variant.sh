#!/bin/bash
# Build a variant of libgjkepa_hip.so with overridden tier parameters (for A/B timing).  Only the
# narrow-phase kernels and the C-ABI are rebuilt; the other kernel objects come from build/.
# usage: tools/build_variant.sh NAME "-DGJKEPA_E0_MINW=3 ..."   (SRCDIR=<dir>: kernel sources from there,
# e.g. a committed revision's csrc/ exported with git archive, for an A/B against the working tree)
set -e
NAME=$1; shift
D=collision-detect-gjk-epa_amd
OUT=${VARDIR:-$D/build/variants}/$NAME
mkdir -p $OUT
S=${SRCDIR:-$D/csrc}
F="--offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 $*"
# the narrow-phase kernels in their parts (GK_PART, as the Makefile builds them), in parallel
# (SINGLE=1: one object without GK_PART, for diagnostics whose device globals must be one symbol,
# e.g. -DGJKEPA_DIAG_STAMPS)
PIDS=""
rm -f $OUT/k[0-9]*.o
if [ "${SINGLE:-0}" = 1 ]; then
  /opt/rocm/bin/hipcc $F -c $S/gjkepa_kernel.hip -o $OUT/k0.o & PIDS="$!"
else
  for p in 0 1 2 3 4 5 6 7 8 9 10 11; do
    /opt/rocm/bin/hipcc $F -DGK_PART=$p -c $S/gjkepa_kernel.hip -o $OUT/k$p.o & PIDS="$PIDS $!"
  done
fi
/opt/rocm/bin/hipcc $F -DGJKEPA_SRC_HASH="\"variant-$NAME\"" -c $S/gjkepa_capi.cpp -o $OUT/c.o
for pid in $PIDS; do wait $pid; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -fopenmp $OUT/k[0-9]*.o $OUT/c.o $D/build/hull_kernel.o \
    $D/build/broadphase_kernel.o $D/build/contacts_kernel.o $D/build/gjkepa_multi.o $D/build/synth.o -o $OUT/libgjkepa_hip.so -ldl -pthread -L/opt/rocm/lib -lrocprofiler-sdk-roctx
echo built $OUT/libgjkepa_hip.so
