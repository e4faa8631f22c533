#!/bin/bash
# round 4 probes: integer atomicMin throughput on device memory; host u32 -> u64 widening rate
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-probes}
mkdir -p $out
timeout -k 10 120 ./tools/atomic_probe > $out/atomic_probe.txt 2>&1 || { echo "atomic probe failed"; cat $out/atomic_probe.txt; exit 1; }
cat $out/atomic_probe.txt
for t in 8 16; do timeout -k 10 60 ./tools/host_widen_probe $t 1; done > $out/host_widen.txt 2>&1
timeout -k 10 60 ./tools/host_widen_probe 16 0 >> $out/host_widen.txt 2>&1
cat $out/host_widen.txt
