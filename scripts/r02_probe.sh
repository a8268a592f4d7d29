#!/bin/bash
# Round-2 probe: lane-chain plan shapes on the det horizon, then the member-sharded EnKF on
# RCCL with two ranks sharing the one GPU of the box (nccl), compared with the one-session run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 bash scripts/chain_bench.sh "2:192 3:192 3:256 4:192 4:256" || exit 1
timeout -k 10 180 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 scripts/dist_enkf_check.py --backend nccl > gpurun_out/dist_nccl.log 2>&1
echo "nccl rc=$?"; tail -5 gpurun_out/dist_nccl.log
