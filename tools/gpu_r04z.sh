#!/bin/bash
# round 4 pass z: H2D ring copies on the copy engine (SRG_H2D_NOCU=1, device-to-device no-CU kind
# from the mapped ring) vs hipMemcpyAsync host-to-device (a blit kernel beside the FW); C3 host
# entry alternating, then the overlap + codec parity tests and a kernel trace under NOCU
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04z}
mkdir -p $out
for i in 1 2 3; do
for v in 0 1; do
  SRG_H2D_NOCU=$v timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu --no-ri > $out/host_${v}_$i.json 2> $out/host_${v}_$i.err || { echo "host $v failed"; tail -8 $out/host_${v}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/host_${v}_$i.json')); print('nocu $v', 'host', d['ms_per_step'], 'h2d', d['ms_h2d'], 'bulk', d['roofline']['avg_launch_ms'], 'verified', d['verified_rows']['bit_exact'])"
done
done
SRG_H2D_NOCU=1 timeout -k 10 600 python -u -m pytest tests/test_fw_overlap.py tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread > $out/parity_nocu.log 2>&1 || { echo "parity failed"; tail -30 $out/parity_nocu.log; exit 1; }
tail -2 $out/parity_nocu.log
(cd /tmp && SRG_H2D_NOCU=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o c3 -- python3 -u $GRAFT_REPO_ROOT/bench.py --no-cpu --no-ri --steps 3 > $out/bench_nocu_rocprof.json 2> $out/stats.err) || { echo "stats failed"; tail -10 $out/stats.err; exit 1; }
grep -c copyBuffer $out/stats/c3_kernel_stats.csv || true
