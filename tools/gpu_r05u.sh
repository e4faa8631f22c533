#!/bin/bash
# Round 5: pipelined codec (encode chunk ch+1 while shipping ch) -- codec / overlap / parity tests,
# the FW-overlap timeline, C3 bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05u}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_fw_overlap.py tests/test_gpu_parity.py tests/test_multi_gpu.py -x -q --timeout 250 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
SRG_DEBUG_OVERLAP=1 SRG_DEBUG_CODEC=1 timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-ri --no-verify > $O/dbg.json 2> $O/dbg.err || { tail $O/dbg.err; exit 1; }
grep -E "fw-overlap: chunk (0|5|11|17|23) |codec: 24" $O/dbg.err | tail -7
grep -E "fw-overlap: last" $O/dbg.err | tail -1 | cut -c1-60
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-ri > $O/c3_$i.json 2> $O/c3_$i.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/c3_$i.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('c3', d['ms_per_step'], 'h2d', b['ms_h2d'], 'scan', b['ms_scan'], d['verified_rows'])"
done
