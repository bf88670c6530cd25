#!/bin/bash
# Build ab/<name>.so: the product library with some objects recompiled with extra compiler flags (same-box
# A/B of code-generation options).  Usage: tools/flag_variant.sh <name> "<src.hip ...>" "<extra flags>"
set -e
cd "$(dirname "$0")/../hardnetnas_amd/csrc"
name=$1; srcs=$2; flags=$3
tmp=$(mktemp -d)
objs=""
for s in hn_api.hip hn_hardnet.hip hn_nas.hip hn_pairdist.hip hn_eval.hip hn_preprocess.hip hn_front.hip hn_irf.hip \
         hn_c12.hip hn_fdl.hip hn_train.hip hn_nas_train.hip hn_loss.hip hn_wino1.hip hn_c12w.hip; do
  o=build/${s%.hip}.o
  if [[ " $srcs " == *" $s "* ]]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../../include -Wall -Wno-unused-function \
      -fno-honor-nans $flags -c $s -o $tmp/${s%.hip}.o
    o=$tmp/${s%.hip}.o
  fi
  objs="$objs $o"
done
mkdir -p ../../ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../ab/$name.so $objs
rm -rf $tmp
echo built ab/$name.so
