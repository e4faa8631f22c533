#!/bin/bash
# Round 5: loss rows of each scan group on the high-priority stream beside the next group's scan
# (SRG_LOSS_AUX=1) vs in line -- C3 host-entry lines alternating, parity tests with it on
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05l2}; mkdir -p $O
SRG_LOSS_AUX=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for i in 1 2 3; do
  for v in 0 1; do
    if [ $v = 1 ]; then export SRG_LOSS_AUX=1; else unset SRG_LOSS_AUX; fi
    timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-ri > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/c3_${v}_$i.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('aux=$v', d['ms_per_step'], 'h2d', b['ms_h2d'], 'scan', b['ms_scan'], 'd2h', b['ms_d2h'], d['verified_rows']['bit_exact'])"
  done
done
export SRG_LOSS_AUX=1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/stats -o c3 -- python3 -u $GRAFT_REPO_ROOT/bench.py --steps 3 --no-cpu --no-ri --no-verify > $GRAFT_REPO_ROOT/$O/c3_prof.json 2> $GRAFT_REPO_ROOT/$O/c3_prof.err) || exit 1
python3 tools/kstats.py $O/stats/c3_kernel_stats.csv tight_v5 k_loss_rows k_pred_pack
