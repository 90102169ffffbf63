#!/bin/bash
# Build experimental variants of libdmlc_amd.so (lib/variants/<name>.so) with
# extra -D flags, for A/B timing via DMLC_AMD_LIB=... python bench.py.
# usage: tools/build_variants.sh name "-DFLAG=1" [name2 "-D..."]...
set -e
cd "$(dirname "$0")/../dmlc-core_amd"
mkdir -p lib/variants build/variants
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  d=build/variants/$name; mkdir -p $d
  for f in csrc/*.hip; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
      -fhip-fp32-correctly-rounded-divide-sqrt -I../include -Icsrc $flags -c $f -o $d/$(basename $f .hip).o &
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
    -fhip-fp32-correctly-rounded-divide-sqrt -I../include -Icsrc $flags -x hip -c csrc/capi.cpp -o $d/capi.o &
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/variants/$name.so $d/*.o
  echo built lib/variants/$name.so
done
