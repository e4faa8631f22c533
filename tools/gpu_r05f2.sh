#!/bin/bash
# Round 5: k_v5_fill with eight rows' loads in flight -- dense parity tests, C3 lines, rocprof kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05f2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_routing_info_keys.py -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-ri > $O/c3_$i.json 2> $O/c3_$i.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/c3_$i.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('c3', d['ms_per_step'], 'h2d', b['ms_h2d'], 'scan', b['ms_scan'], 'dev', d.get('device_entry_ms'), d['verified_rows']['bit_exact'])"
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/stats -o c3 -- python3 -u $GRAFT_REPO_ROOT/bench.py --steps 3 --no-cpu --no-ri --no-verify > $GRAFT_REPO_ROOT/$O/c3_prof.json 2> $GRAFT_REPO_ROOT/$O/c3_prof.err) || exit 1
python3 tools/kstats.py $O/stats/c3_kernel_stats.csv tight_v5 k_loss_rows k_v5_fill k_ess_mask k_build_dst k_v5_count k_pred_pack
