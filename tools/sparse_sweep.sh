#!/bin/bash
# Sparse (C4) launch-variant sweep: rows in flight per wave x workgroups per CU, after the
# parity tests of every variant.  usage: tools/sparse_sweep.sh OUTDIR
set -o pipefail
out=$1
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_sparse_gpu.py -x -v --timeout 120 --timeout-method thread \
    > "$out/pytest_sparse.log" 2>&1 || { echo "sparse tests failed"; tail -30 "$out/pytest_sparse.log"; exit 1; }
tail -2 "$out/pytest_sparse.log"
for g in 4 8; do for w in 1 2; do
  timeout -k 10 120 python -u bench.py --graph ba --steps 2 --warmup 1 --no-cpu --sparse-group $g --sparse-wgs $w \
      > "$out/c4_g${g}_w${w}.json" 2> "$out/c4_g${g}_w${w}.err" || { echo "bench g$g w$w failed"; tail -20 "$out/c4_g${g}_w${w}.err"; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['roofline']['avg_launch_ms'])" "$out/c4_g${g}_w${w}.json"
done; done
