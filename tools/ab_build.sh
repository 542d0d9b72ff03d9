#!/bin/bash
# Build the current csrc tree into ab/<name>.so (A/B probes: FMCW_LIB=ab/<name>.so)
#   tools/ab_build.sh <name> [extra hipcc flags, e.g. -DAB_HALF]
set -e
name=$1; shift
d=ab/build_$name
mkdir -p $d ab
make -s -j8 -C fmcw_radar_processing_amd/csrc OUT=$PWD/ab/$name.so BUILD=$PWD/$d \
  CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-result -mllvm -pragma-unroll-threshold=1000000 $*" >/dev/null
echo "built ab/$name.so"
