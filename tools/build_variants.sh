#!/bin/bash
# Build A/B variants of librt_hip.so into tools/variants/: NAME="-DKNOB=V ..." pairs.
#   bash tools/build_variants.sh a_base "" b_knob "-DRT_AO_FIRST=0"
cd "$(dirname "$0")/../tipe-raytracer_amd" || exit 1
rm -f ../tools/variants/*.so
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../include -Icsrc -shared csrc/rt_kernels.hip csrc/rt_api.cpp csrc/rt_bvh.cpp csrc/rt_rccl.cpp -ldl"
while [ $# -ge 2 ]; do
  /opt/rocm/bin/hipcc $F $2 -o ../tools/variants/$1.so &
  shift 2
done
wait
ls ../tools/variants
