#!/bin/bash
# Round-2 pass b: full GPU suite (incl. C3 multi-rank G=2/8), RCCL two-rank probe, u64-key C3 bench,
# C3-size GML ingest, full C1/C2 CPU baselines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r02b}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=20 \
    > $out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -24 $out/pytest_gpu.log
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 tools/rccl_two_ranks.py > $out/rccl_two_ranks_one_gpu.txt 2>&1; echo "rccl probe rc=$?"; tail -5 $out/rccl_two_ranks_one_gpu.txt
timeout -k 10 300 python -u bench.py --entry device --steps 3 --warmup 1 --no-cpu --lat-scale 1000 > $out/c3_u64.json 2> $out/c3_u64.err \
    && cat $out/c3_u64.json || { tail -20 $out/c3_u64.err; exit 1; }
timeout -k 10 400 python -u tools/ingest/ingest_bench.py --vertices 10000 --dir /tmp > $out/ingest_c3.json 2> $out/ingest.err \
    && cat $out/ingest_c3.json || { tail -20 $out/ingest.err; exit 1; }
timeout -k 10 600 python -u tools/cpu_full.py > $out/cpu_full.json 2> $out/cpu_full.err && cat $out/cpu_full.json
