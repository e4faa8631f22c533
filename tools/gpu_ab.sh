#!/bin/bash
# A/B launcher for the kernel experiments of round 5 (replaces the round's one-off gpu_r05*.sh):
# the GPU parity tests on the tree, then C3 host-entry bench lines alternating between variants
# (REPS rounds), then rocprof kernel stats of the last variant.
#   usage: tools/gpu_ab.sh TAG 'name|ENV=1 ENV2=x|--bench-flags' ['name2|...|...' ...]
#   e.g.   tools/gpu_ab.sh r05x 'base||' 'groups4||--scan-groups 4'
#          tools/gpu_ab.sh r05y 'sim8||--simulate-rank 8:0' 'sim8_split2||--simulate-rank 8:0 --fw-line-split 2'
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:?tag}; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for i in $(seq 1 ${REPS:-3}); do
  for v in "$@"; do
    IFS='|' read -r name envs flags <<< "$v"
    timeout -k 10 200 env $envs python -u bench.py --steps 10 --no-cpu --no-ri $flags > $O/${name}_$i.json 2> $O/${name}_$i.err || { tail -10 $O/${name}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${name}_$i.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; print('$name', d['ms_per_step'], {k: round(x, 2) for k, x in b.items() if x})"
  done
done
IFS='|' read -r name envs flags <<< "${@: -1}"
(cd /tmp && timeout -k 10 300 env $envs rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/stats -o c3 -- python3 -u $GRAFT_REPO_ROOT/bench.py --steps 3 --no-cpu --no-ri --no-verify $flags > $GRAFT_REPO_ROOT/$O/prof.json 2> $GRAFT_REPO_ROOT/$O/prof.err) || exit 1
python3 tools/kstats.py $O/stats/c3_kernel_stats.csv fw_bulk tight_v5 k_loss_rows k_pred_pack k_v5_fill k_ess_mask
