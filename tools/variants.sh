#!/bin/bash
# Build experiment variants of the render library: tools/_var/<name>/librt_amd.so, one per
# "name=-DFLAG ..." argument (compiled in parallel; depth <= RT_MAX_B, default 3 = the c1..c5 kernels).  Run them with tools/ab_variants.sh on the GPU.
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/ray_tracer_fragment_shader_amd/csrc
LIB=$ROOT/ray_tracer_fragment_shader_amd/lib
make -C "$SRC" -s ../lib/rt_host.o ../lib/rt_screen.o ../lib/rt_group.o
pids=()
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  d=$ROOT/tools/_var/$name; mkdir -p "$d"
  ( cd "$SRC" && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function \
      --offload-arch=gfx950 -DRT_MAX_B=${RT_MAX_B:-3} $flags -c rt_kernel.hip -o "$d/rt_kernel.o" && \
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$d/librt_amd.so" "$d/rt_kernel.o" "$LIB/rt_host.o" "$LIB/rt_screen.o" "$LIB/rt_group.o" -L/opt/rocm/lib -lrccl && \
    rm "$d/rt_kernel.o" && echo "built $name" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
