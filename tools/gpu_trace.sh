#!/bin/bash
# rocprofv3 kernel trace (timestamps) of one simulated rank's bench run: tools/gpu_trace.sh TAG G:r [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=$1; sr=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- \
    python3 -u bench.py --steps 1 --warmup 1 --no-cpu --no-verify --simulate-rank $sr "$@" > $out/sim.json 2> $out/sim.err || { echo "trace failed"; tail -20 $out/sim.err; exit 1; }
cat $out/sim.json
