#!/bin/bash
# Round-5 closing pass, part B: the default bench line (C3 host entry, CPU baseline), its rocprof
# kernel stats, every config's line, the device entry and the simulated ranks
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05close}; mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step bench
for i in 1 2; do
  timeout -k 10 400 python3 -u bench.py > $O/bench_c3_$i.json 2> $O/bench_c3_$i.err || { tail -20 $O/bench_c3_$i.err; exit 1; }
done
step stats
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/stats -o c3 -- python3 -u $GRAFT_REPO_ROOT/bench.py --no-cpu > $GRAFT_REPO_ROOT/$O/bench_c3_under_rocprof.json 2> $GRAFT_REPO_ROOT/$O/stats.err) || { tail -20 $O/stats.err; exit 1; }
step configs
for cfg in c1 c2 c4 c5; do
  timeout -k 10 400 python3 -u bench.py --config $cfg --no-cpu > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { tail -10 $O/bench_$cfg.err; exit 1; }
done
timeout -k 10 400 python3 -u bench.py --entry device --no-cpu --no-ri > $O/bench_c3_device.json 2> $O/bench_c3_device.err || exit 1
step sims
for sr in 2:0 4:0 8:0 8:7; do
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-verify --no-ri --simulate-rank $sr > $O/sim_${sr/:/_}.json 2> $O/sim_${sr/:/_}.err || { tail -10 $O/sim_${sr/:/_}.err; exit 1; }
done
step done
python3 - <<PY
import json, glob, os
for f in sorted(glob.glob("$O/*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(os.path.basename(f), "unreadable", e); continue
    if not isinstance(d, dict) or "ms_per_step" not in d: continue
    r = d.get("roofline") or {}
    print(os.path.basename(f), d["ms_per_step"], d.get("value"), "frac", r.get("frac"), {k: round(v, 2) for k, v in (d.get("breakdown_ms") or {}).items()})
PY
