#!/bin/bash
# Build a measurement copy of libgnca from a given gnca_k1_split.h (A/B runs, tools/ab_libs.sh):
#   tools/build_variant_lib.sh <k1 header> <out .so> [extra hipcc flags]
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
HDR=$1; OUT=$2; shift 2
D=$(mktemp -d)
cp "$ROOT"/graph_neural_cellular_automata_amd/csrc/* "$D"/
cp "$HDR" "$D"/gnca_k1_split.h
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -fno-slp-vectorize -Wno-unused-result "$@" \
  -I"$ROOT"/include "$D"/gnca_step.hip -o "$D"/step.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$D"/step.o "$ROOT"/build/obj/gnca_bwd.o "$ROOT"/build/obj/gnca_aux.o -o "$OUT"
rm -rf "$D"
