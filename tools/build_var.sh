#!/bin/bash
# Build the working tree's library with extra defines into tools/_ab/<name>/ (for tools/ab_libs.py A/B against the
# in-tree build).  usage: bash tools/build_var.sh <name> "-DRT_X=1 -DRT_Y=0"
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; defs=$2
tmp=$(mktemp -d)
cp -r "$ROOT/ray_tracer_fragment_shader_amd/csrc" "$ROOT/include" "$tmp/"
mkdir -p "$tmp/ray_tracer_fragment_shader_amd" && mv "$tmp/csrc" "$tmp/ray_tracer_fragment_shader_amd/"
make -C "$tmp/ray_tracer_fragment_shader_amd/csrc" -s -j8 ../lib/librt_amd.so \
    CXXFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function $defs"
mkdir -p "$ROOT/tools/_ab/$name"
cp "$tmp/ray_tracer_fragment_shader_amd/lib/librt_amd.so" "$ROOT/tools/_ab/$name/"
rm -rf "$tmp"
echo "built tools/_ab/$name ($defs)"
