#!/bin/bash
# Build the current csrc tree into ab/<name>.so (A/B probes: FMCW_LIB=ab/<name>.so)
set -e
name=$1
d=ab/build_$name
mkdir -p $d ab
make -s -j8 -C fmcw_radar_processing_amd/csrc OUT=$PWD/ab/$name.so BUILD=$PWD/$d >/dev/null
echo "built ab/$name.so"
