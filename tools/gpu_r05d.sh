#!/bin/bash
# Round 5: the XCD-cooperative sparse kernel -- sparse parity tests, then C4 timing (new vs old kernel).
cd "$(dirname "$0")/.."
O=gpurun_out/r05d; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -v -x --timeout 120 --timeout-method thread -m gpu tests/test_sparse_gpu.py -k "not c4_full" > $O/sparse_tests.log 2>&1; echo "tests rc=$?" >> $O/rc.txt
tail -3 $O/sparse_tests.log
if grep -q "passed" $O/sparse_tests.log && ! grep -q "failed" $O/sparse_tests.log; then
  SRG_DEBUG_SPARSE=1 timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu --no-verify > $O/c4_xcd.json 2> $O/c4_xcd.err; echo "c4 xcd rc=$?" >> $O/rc.txt
  SRG_DEBUG_SPARSE=1 SRG_SPARSE_KERNEL=bf timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu --no-verify > $O/c4_bf.json 2> $O/c4_bf.err; echo "c4 bf rc=$?" >> $O/rc.txt
fi
cat $O/rc.txt
