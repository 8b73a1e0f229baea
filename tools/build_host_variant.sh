#!/bin/bash
# Build a variant of libgjkepa_hip.so that differs only in host-side (C-ABI) switches: the kernel
# objects come from build/, only gjkepa_capi.cpp is recompiled with the given -D flags.
# usage: tools/build_host_variant.sh NAME "-DGJKEPA_FORK_MASK=0x1F ..."
set -e
NAME=$1; shift
D=collision-detect-gjk-epa_amd
OUT=$D/build/variants/$NAME
mkdir -p $OUT
F="--offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 $*"
/opt/rocm/bin/hipcc $F -DGJKEPA_SRC_HASH="\"variant-$NAME\"" -c $D/csrc/gjkepa_capi.cpp -o $OUT/c.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -fopenmp $D/build/gjkepa_kernel.o $OUT/c.o $D/build/hull_kernel.o \
    $D/build/broadphase_kernel.o $D/build/contacts_kernel.o $D/build/gjkepa_multi.o $D/build/synth.o -o $OUT/libgjkepa_hip.so
echo built $OUT/libgjkepa_hip.so
