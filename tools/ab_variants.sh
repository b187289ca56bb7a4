#!/bin/bash
# Time each tools/_var/<name>/librt_amd.so against the in-tree build (tools/ab.py, one process each).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIB=ray_tracer_fragment_shader_amd/lib/librt_amd.so
cp "$LIB" /tmp/librt_amd.base.so
# base runs first and again last (the first process on a box tends to run ~1-2% faster at c2: compare a
# variant with both base lines)
for d in base tools/_var/*/ base; do
  name=$(basename "$d")
  if [ "$d" = base ]; then cp /tmp/librt_amd.base.so "$LIB"; else cp "$d/librt_amd.so" "$LIB"; fi
  timeout -k 10 120 python tools/ab.py ${AB_CFGS:-c2} base 2>/dev/null | sed "s/\"mode\": \"base\"/\"mode\": \"$name\"/" || { echo "variant $name failed"; break; }
done
cp /tmp/librt_amd.base.so "$LIB"
