#!/bin/bash
# Round 5: hardware-queue sharing of a context's streams, and the value-hop race A/B with the main and
# chain streams forced onto separate hardware queues.
cd "$(dirname "$0")/.."
O=gpurun_out/r05b; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 60 ./tools/queue_probe 3 > $O/queues.txt 2>&1; echo "queues rc=$?" >> $O/rc.txt
GPU_MAX_HW_QUEUES=16 timeout -k 10 60 ./tools/queue_probe 3 > $O/queues16.txt 2>&1; echo "queues16 rc=$?" >> $O/rc.txt
for L in noorder fixed; do
  if [ $L = noorder ]; then LP=tools/dbg/libshadow_routing_noorder.so; else LP=shadow_amd/libshadow_routing.so; fi
  GPU_MAX_HW_QUEUES=16 SRG_LIB_PATH=$LP timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_fw_overlap.py -k "stale" > $O/stale16_$L.log 2>&1; echo "stale16_$L rc=$?" >> $O/rc.txt
  SRG_LIB_PATH=$LP timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_events.py tests/test_fw_overlap.py -k "stale or events" > $O/stale_seq_$L.log 2>&1; echo "stale_seq_$L rc=$?" >> $O/rc.txt
done
cat $O/rc.txt $O/queues*.txt
