#!/bin/bash
# Build librt_amd.so of a git revision into tools/_ab/<name>/ (for same-box A/B with ab_variants.sh).
# Usage: bash tools/build_rev.sh <rev> <name>
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rev=$1; name=$2
tmp=$(mktemp -d)
git -C "$ROOT" archive "$rev" ray_tracer_fragment_shader_amd/csrc include | tar -x -C "$tmp"
make -C "$tmp/ray_tracer_fragment_shader_amd/csrc" -s -j8 ../lib/librt_amd.so
mkdir -p "$ROOT/tools/_ab/$name"
cp "$tmp/ray_tracer_fragment_shader_amd/lib/librt_amd.so" "$ROOT/tools/_ab/$name/"
rm -rf "$tmp"
echo "built $rev -> tools/_ab/$name"
