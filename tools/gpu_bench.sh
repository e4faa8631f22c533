#!/bin/bash
# Bench lines for the configs (host-entry headline C3 with CPU baselines, C2, C1, C4, C5) + rocprof of C3.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-bench}
mkdir -p $out
timeout -k 10 300 python -u bench.py > $out/c3.json 2> $out/c3.err && cat $out/c3.json && \
timeout -k 10 200 python -u bench.py --config c2 --steps 5 > $out/c2.json 2> $out/c2.err && cat $out/c2.json && \
timeout -k 10 200 python -u bench.py --config c1 --steps 5 > $out/c1.json 2> $out/c1.err && cat $out/c1.json && \
timeout -k 10 300 python -u bench.py --config c4 --steps 3 --cpu-seconds 20 > $out/c4.json 2> $out/c4.err && cat $out/c4.json && \
timeout -k 10 200 python -u bench.py --config c5 --steps 5 > $out/c5.json 2> $out/c5.err && cat $out/c5.json
