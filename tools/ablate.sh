#!/bin/bash
# Build the instruction-count ablation libraries (rt_render.hpp RT_ABLATE: 1 the prologue alone, 2 trace without
# stores) into tools/_ab/ablate<k>/ — run them with RT_LIB_PATH=tools/_ab/ablate<k>/librt_amd.so tools/count.py under
# rocprofv3 --pmc (tools/count.sh LIBS=...).  Only depth 1 (c2) is built (RT_MAX_B=1).
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
for k in ${ABLATE:-1 2}; do
  tmp=$(mktemp -d)
  cp -r "$ROOT/ray_tracer_fragment_shader_amd/csrc" "$ROOT/include" "$tmp/"
  mkdir -p "$tmp/ray_tracer_fragment_shader_amd" && mv "$tmp/csrc" "$tmp/ray_tracer_fragment_shader_amd/"
  make -C "$tmp/ray_tracer_fragment_shader_amd/csrc" -s -j8 ../lib/librt_amd.so \
      CXXFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function -DRT_ABLATE=$k -DRT_MAX_B=1"
  mkdir -p "$ROOT/tools/_ab/ablate$k"
  cp "$tmp/ray_tracer_fragment_shader_amd/lib/librt_amd.so" "$ROOT/tools/_ab/ablate$k/"
  rm -rf "$tmp"
  echo "built tools/_ab/ablate$k"
done
