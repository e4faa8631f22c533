#!/bin/bash
# round 4: where a process's first HIP costs go (tools/init_probe.hip), default env and variants
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-init}
mkdir -p $out
for i in 1 2; do
  timeout -k 10 60 ./tools/init_probe > $out/default_$i.txt 2>&1 || { echo "probe failed"; cat $out/default_$i.txt; exit 1; }
done
GPU_MAX_HW_QUEUES=1 timeout -k 10 60 ./tools/init_probe > $out/hwq1.txt 2>&1 || { echo "probe hwq1 failed"; exit 1; }
HIP_ENABLE_DEFERRED_LOADING=0 timeout -k 10 60 ./tools/init_probe > $out/nodefer.txt 2>&1 || { echo "probe nodefer failed"; exit 1; }
for f in $out/*.txt; do echo "== $f"; cat $f; done
