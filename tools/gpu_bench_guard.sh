#!/bin/bash
# bench.py checks: the N=1 line with its c4 leg, the c4 watchdog path (a leg that cannot finish in time still
# leaves the line), and a 2-rank gloo rehearsal of the N>1 path on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
show() { tail -1 "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], d.get('c4'))" | cut -c1-300; }
timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-extra > gpurun_out/b1.json 2> gpurun_out/b1.err || { echo "b1 failed"; tail -5 gpurun_out/b1.err; exit 3; }
show gpurun_out/b1.json
timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-extra --c4-timeout 0.5 > gpurun_out/b2.json 2> gpurun_out/b2.err
echo "watchdog rc=$?"; show gpurun_out/b2.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --backend gloo --steps 20 --warmup 3 > gpurun_out/b3.json 2> gpurun_out/b3.err \
    || { echo "b3 failed"; tail -5 gpurun_out/b3.err; exit 4; }
show gpurun_out/b3.json
