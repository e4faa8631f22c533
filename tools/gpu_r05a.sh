#!/bin/bash
# Round 5: the value-hop race fix -- the FW-overlap tests and the recorded failing
# sequence on the fixed library, then the regression test on a library without the fix.
cd "$(dirname "$0")/.."
O=gpurun_out/r05a; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_fw_overlap.py > $O/overlap.log 2>&1; echo "overlap rc=$?" >> $O/rc.txt
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_events.py tests/test_fw_overlap.py tests/test_fw_exchange.py tools/dbg/test_ov_after.py > $O/sequence.log 2>&1; echo "sequence rc=$?" >> $O/rc.txt
SRG_LIB_PATH=tools/dbg/libshadow_routing_noorder.so timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_fw_overlap.py -k "stale" > $O/noorder.log 2>&1; echo "noorder rc=$?" >> $O/rc.txt
cat $O/rc.txt
