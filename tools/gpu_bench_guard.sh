#!/bin/bash
# bench.py checks: the N=1 line with its c4 leg; the c4 watchdog path (a leg that cannot finish in time still
# leaves the line, and the job exits 3); `--gpus 2` without a launcher: nccl on a one-GPU box is refused (exit 2),
# gloo self-launches two child ranks and prints one line with "n_gpus": 2; and the same rehearsal under
# torch.distributed.run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
show() { tail -1 "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], d.get('c4'))" | cut -c1-300; }
timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-extra > gpurun_out/b1.json 2> gpurun_out/b1.err || { echo "b1 failed"; tail -5 gpurun_out/b1.err; exit 3; }
show gpurun_out/b1.json
timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-extra --c4-timeout 0.5 > gpurun_out/b2.json 2> gpurun_out/b2.err
rc=$?; echo "watchdog rc=$rc (expected 3)"; show gpurun_out/b2.json
[ $rc -eq 3 ] || { tail -5 gpurun_out/b2.err; exit 5; }
timeout -k 10 120 python bench.py --gpus 2 --steps 5 > gpurun_out/b4.json 2> gpurun_out/b4.err
rc=$?; echo "nccl --gpus 2 on one GPU: rc=$rc (expected 2): $(tail -1 gpurun_out/b4.err)"
[ $rc -eq 2 ] || exit 6
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 20 --warmup 3 > gpurun_out/b5.json 2> gpurun_out/b5.err \
    || { echo "b5 failed"; tail -5 gpurun_out/b5.err; exit 7; }
show gpurun_out/b5.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --backend gloo --steps 20 --warmup 3 > gpurun_out/b3.json 2> gpurun_out/b3.err \
    || { echo "b3 failed"; tail -5 gpurun_out/b3.err; exit 4; }
show gpurun_out/b3.json
