#!/bin/bash
# Build experiment variants of the render library: tools/_var/<name>/librt_amd.so, one per
# "name=-DFLAG ..." argument (depth <= RT_MAX_B, default 3 = the c1..c5 kernels; the per-depth translation units
# of a variant compile in parallel).  Run them with tools/ab_variants.sh or tools/ab_libs.py on the GPU.
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/ray_tracer_fragment_shader_amd/csrc
LIB=$ROOT/ray_tracer_fragment_shader_amd/lib
make -C "$SRC" -s ../lib/rt_host.o ../lib/rt_screen.o ../lib/rt_group.o ../lib/rt_group_plan.o
UNITS="rt_kernel rt_render_b0 rt_render_b1 rt_render_b2 rt_render_b3 rt_render_b4 rt_render_b5 rt_render_b6 rt_render_b7"
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  d=$ROOT/tools/_var/$name; mkdir -p "$d"
  echo $UNITS | tr ' ' '\n' | (cd "$SRC" && xargs -P 8 -I{} /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off \
      -fno-fast-math -Wall -Wno-unused-function --offload-arch=gfx950 ${KERNARG_PRELOAD:+-mllvm -amdgpu-kernarg-preload-count=$KERNARG_PRELOAD} -DRT_MAX_B=${RT_MAX_B:-3} $flags -c {}.hip -o "$d/{}.o")
  objs=$(for u in $UNITS; do echo "$d/$u.o"; done)
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$d/librt_amd.so" $objs "$LIB/rt_host.o" "$LIB/rt_screen.o" \
      "$LIB/rt_group.o" "$LIB/rt_group_plan.o" -L/opt/rocm/lib -lrccl -lhsa-runtime64
  rm -f $objs
  echo "built $name"
done
