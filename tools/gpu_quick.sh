#!/bin/bash
# Parity tests then the interleaved A/B timing (no profiling).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python tools/ab.py ${AB_CFGS:-c1,c2,c3,c5} ${AB_MODES:-base,RT_SCENE_IN_LDS=1} 2>&1 | tee gpurun_out/ab.log
