#!/bin/bash
# rocprofv3 kernel stats of bench runs: C3 host entry (1 GPU) and simulated ranks (G:r list)
# usage: tools/gpu_prof.sh TAG [G:r ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c3 -o run -- \
    python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-verify > $out/c3.json 2> $out/c3.err || { echo "c3 profile failed"; tail -20 $out/c3.err; exit 1; }
cat $out/c3.json
for sr in "$@"; do
    timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-verify --simulate-rank $sr > $out/sim_${sr/:/_}.json 2> $out/sim_${sr/:/_}.err || { echo "sim $sr failed"; tail -20 $out/sim_${sr/:/_}.err; exit 1; }
    cat $out/sim_${sr/:/_}.json
done
