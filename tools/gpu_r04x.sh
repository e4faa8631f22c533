#!/bin/bash
# round 4 pass x: tight_v5 pipelined one group deep (SRG_SCAN_PIPE=1: LDS-DMA staging, 145 VGPRs,
# one workgroup per CU; =2: 128 VGPRs, two) vs the default; C3 device + host entry, then the parity suite on PIPE
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${1:-r04x}
mkdir -p $out
for i in 1 2; do
for v in 0 1 2; do
  SRG_SCAN_PIPE=$v timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu --no-ri --entry device > $out/dev_${v}_$i.json 2> $out/dev_${v}_$i.err || { echo "dev $v failed"; tail -5 $out/dev_${v}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/dev_${v}_$i.json')); print('pipe $v', 'device', d['ms_per_step'], 'fw', d['breakdown_ms']['ms_fw'], 'scan', d['breakdown_ms']['ms_scan'], 'verified', d.get('verified_rows',{}).get('bit_exact'))"
done
done
SRG_SCAN_PIPE=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread > $out/parity_pipe.log 2>&1 || { echo "parity failed"; tail -30 $out/parity_pipe.log; exit 1; }
tail -3 $out/parity_pipe.log
