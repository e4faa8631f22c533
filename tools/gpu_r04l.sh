#!/bin/bash
# round 4 pass l: C4 old/new A/B (round-start tree in _old/), FW PMC + rocprof stats with the
# overlap off (full bulk launches only, matching bench.py's timed launches)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04l}
mkdir -p $out
for i in 1 2; do
  (cd _old && timeout -k 10 200 python3 -u bench.py --graph ba --vertices 50000 --entry device --steps 3 --no-cpu --no-verify > $out/c4_old_$i.json 2> $out/c4_old_$i.err) || { echo "old failed"; tail -5 $out/c4_old_$i.err; exit 1; }
  timeout -k 10 200 python3 -u bench.py --graph ba --vertices 50000 --entry device --steps 3 --no-cpu --no-verify --no-ri > $out/c4_new_$i.json 2> $out/c4_new_$i.err || { echo "new failed"; tail -5 $out/c4_new_$i.err; exit 1; }
  python3 -c "import json; a=json.load(open('$out/c4_old_$i.json')); b=json.load(open('$out/c4_new_$i.json')); print('c4 old', a['ms_per_step'], 'new', b['ms_per_step'])"
done
timeout -k 10 900 bash tools/pmc_fw.sh $out/pmc_fw --fw-overlap 0 > $out/pmc_fw.log 2>&1 || { echo "pmc_fw failed"; tail -20 $out/pmc_fw.log; exit 1; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats_ov0 -o c3 -- python3 -u $GRAFT_REPO_ROOT/bench.py --no-cpu --no-ri --fw-overlap 0 > $out/bench_c3_ov0_under_rocprof.json 2> $out/stats_ov0.err) || { echo "stats failed"; exit 1; }
grep fw_bulk_lb $out/stats_ov0/c3_kernel_stats.csv | cut -c1-40,150-260
