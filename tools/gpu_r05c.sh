#!/bin/bash
# Round 5: the recorded failing sequence (r04 gpurun_out/dbg) on the library WITHOUT the reset-order fix
# and on the fixed one, three processes each.
cd "$(dirname "$0")/.."
O=gpurun_out/r05c; mkdir -p $O
export PYTHONUNBUFFERED=1
for i in 1 2 3; do
  for L in noorder fixed; do
    if [ $L = noorder ]; then LP=tools/dbg/libshadow_routing_noorder.so; else LP=shadow_amd/libshadow_routing.so; fi
    SRG_LIB_PATH=$LP timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_events.py tests/test_fw_overlap.py tests/test_fw_exchange.py tools/dbg/test_ov_after.py > $O/seq_${L}_$i.log 2>&1; echo "seq_${L}_$i rc=$?" >> $O/rc.txt
  done
done
cat $O/rc.txt
