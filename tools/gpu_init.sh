#!/bin/bash
# round 4: where a process's first HIP costs go (tools/init_probe.hip): serial vs threaded stream creation
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-init}
mkdir -p $out
for i in 1 2 3; do
  timeout -k 10 60 ./tools/init_probe > $out/serial_$i.txt 2>&1 || { echo "probe failed"; cat $out/serial_$i.txt; exit 1; }
  timeout -k 10 60 ./tools/init_probe par > $out/par_$i.txt 2>&1 || { echo "probe par failed"; cat $out/par_$i.txt; exit 1; }
done
for f in $out/*.txt; do echo "== $f"; head -8 $f; tail -1 $f; done
