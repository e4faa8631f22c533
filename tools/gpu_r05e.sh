#!/bin/bash
# Round 5: C4 XCD kernel timing diagnostics
cd "$(dirname "$0")/.."
O=gpurun_out/r05e; mkdir -p $O
SRG_DEBUG_SPARSE=1 timeout -k 10 300 python -u bench.py --config c4 --steps 1 --warmup 0 --no-cpu --no-verify > $O/c4_xcd.json 2> $O/c4_xcd.err; echo "c4 xcd rc=$?" >> $O/rc.txt
grep "sparse:" $O/c4_xcd.err
