#!/bin/bash
# Round 5: where srg_create's library part goes (SRG_DEBUG_CREATE), fresh process each time;
# streams created one after another vs from four threads at once
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05c}; mkdir -p $O
for i in 1 2 3 4; do
  if [ $((i % 2)) = 0 ]; then export SRG_PAR_STREAMS=1; else unset SRG_PAR_STREAMS; fi
  SRG_DEBUG_CREATE=1 timeout -k 10 120 python3 -u -c "
import time, ctypes
from shadow_amd import Router
from shadow_amd import _native as N
t=time.perf_counter(); r=Router(0); t1=time.perf_counter()
print('create %.1f ms runtime %.1f lib %.1f' % ((t1-t)*1e3, r.get_option(N.SRG_OPT_CREATE_MS_RUNTIME), r.get_option(N.SRG_OPT_CREATE_MS_LIBRARY)))
" > $O/create_$i.log 2>&1 || { cat $O/create_$i.log; exit 1; }
  grep -v amdgpu.ids $O/create_$i.log
done
