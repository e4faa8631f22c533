#!/bin/bash
# Sparse (C4) delta-stepping bucket-width sweep after the sparse parity tests.
# usage: tools/sparse_delta_sweep.sh OUTDIR
set -o pipefail
out=$1
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests/test_sparse_gpu.py -x -v --timeout 120 --timeout-method thread \
    > "$out/pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$out/pytest_gpu.log"; exit 1; }
tail -2 "$out/pytest_gpu.log"
for al in 0 1; do for d in ${DIVS:-0 1 2 4}; do
  timeout -k 10 120 python -u bench.py --graph ba --steps 2 --warmup 1 --no-cpu --sparse-delta-div $d --sparse-delta-all $al \
      > "$out/c4_all${al}_div${d}.json" 2> "$out/c4_all${al}_div${d}.err" || { echo "bench div $d failed"; tail -20 "$out/c4_all${al}_div${d}.err"; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['loss_rounds'])" "$out/c4_all${al}_div${d}.json"
done; done
