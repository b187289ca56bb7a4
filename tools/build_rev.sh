#!/bin/bash
# Build librt_amd.so of a git revision into tools/_var/<name>/ (for same-box A/B with ab_variants.sh).
# Usage: bash tools/build_rev.sh <rev> <name>
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rev=$1; name=$2
tmp=$(mktemp -d)
git -C "$ROOT" archive "$rev" ray_tracer_fragment_shader_amd/csrc include | tar -x -C "$tmp"
make -C "$tmp/ray_tracer_fragment_shader_amd/csrc" -s -j8 ../lib/librt_amd.so
mkdir -p "$ROOT/tools/_var/$name"
cp "$tmp/ray_tracer_fragment_shader_amd/lib/librt_amd.so" "$ROOT/tools/_var/$name/"
rm -rf "$tmp"
echo "built $rev -> tools/_var/$name"
