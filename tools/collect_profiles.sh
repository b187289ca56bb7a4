#!/bin/bash
# Copy a profile session's outputs (tools/gpu_r04_prof.sh, under gpurun_out/) into profiles/<round>/ and regenerate
# profiles/pmc_<cfg>.json.  usage: bash tools/collect_profiles.sh r04
set -eu
R=${1:?round}
cd "$(dirname "$0")/.."
D=profiles/$R; mkdir -p "$D"
cp gpurun_out/bench.json "$D/bench.json"
cp gpurun_out/gpu_tests.log "$D/gpu_tests.log"
for c in c2 c3 c5; do
  f=$(find gpurun_out/prof1_$c -name "*kernel_stats.csv" | head -1)
  cp "$f" "$D/${c}_kernel_stats_1stream.csv"
  cp gpurun_out/prof1_bench_$c.json "$D/${c}_bench_1stream.json"
  cp gpurun_out/pmc_$c/summary.json "$D/pmc_${c}_summary.json"
  python3 tools/pmc_profile.py $c gpurun_out/pmc_$c/summary.json "$R profile session (tools/gpu_r04_prof.sh)" > profiles/pmc_$c.json
done
ls -la "$D"
