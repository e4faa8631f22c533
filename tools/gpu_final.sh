#!/bin/bash
# final pass (round 5, reused in round 6): rocprof stats of the default C3 bench command, FW + sparse PMC passes, every
# config's bench line, simulated ranks, device entry, u64 keys.  usage: tools/gpu_final.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=${1:-r05final}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
step() { echo "[$(date +%T)] $*"; }
step stats
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o c3 -- python3 -u $GRAFT_REPO_ROOT/bench.py --no-cpu > $out/bench_c3_under_rocprof.json 2> $out/stats.err) || { echo "stats failed"; tail -20 $out/stats.err; exit 1; }
step pmc_fw
timeout -k 10 900 bash tools/pmc_fw.sh $out/pmc_fw > $out/pmc_fw.log 2>&1 || { echo "pmc_fw failed"; tail -20 $out/pmc_fw.log; exit 1; }
python3 tools/pmc_extract.py $out/pmc_fw/ "rocprofv3 --pmc, $tag (tools/pmc_fw.sh, C3 atlas_like(10000) host entry, 1 step, fw_bulk_lb bulk launches)" "atlas:10000:10000:lb:packed2:tile128:div1:g8:w2" > $out/pmc_fw_extract.log 2>&1 || { echo "extract fw failed"; tail -5 $out/pmc_fw_extract.log; exit 1; }
step pmc_sparse
timeout -k 10 900 bash tools/pmc_sparse.sh $out/pmc_sparse > $out/pmc_sparse.log 2>&1 || { echo "pmc_sparse failed"; tail -20 $out/pmc_sparse.log; exit 1; }
python3 tools/pmc_extract_sparse.py $out/pmc_sparse "rocprofv3 --pmc, $tag (tools/pmc_sparse.sh, C4 barabasi_albert(50000, 4), 1 step, k_sparse_ds two-phase)" "ba:50000:50000:packed2:tile128:div1:g8:w2:ds2" > $out/pmc_sparse_extract.log 2>&1 || { echo "extract sparse failed"; tail -5 $out/pmc_sparse_extract.log; exit 1; }
cp profiles/sparse_pmc_latest.json profiles/fw_pmc_latest.json $out/
step configs
for cfg in c1 c2 c4 c5; do
  timeout -k 10 400 python3 -u bench.py --config $cfg --no-cpu > $out/bench_$cfg.json 2> $out/bench_$cfg.err || { echo "bench $cfg failed"; tail -10 $out/bench_$cfg.err; exit 1; }
done
timeout -k 10 400 python3 -u bench.py --entry device --no-cpu --no-ri > $out/bench_c3_device.json 2> $out/bench_c3_device.err || { echo "device failed"; exit 1; }
SRG_LATENCY_UNIT=1 timeout -k 10 400 python3 -u bench.py --lat-scale 1000 --no-cpu --no-ri --steps 3 > $out/bench_c3_u64.json 2> $out/bench_c3_u64.err || { echo "u64 failed"; exit 1; }
step sims
for sr in 2:0 2:1 4:0 4:3 8:0 8:7; do
  timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-verify --no-ri --simulate-rank $sr > $out/sim_${sr/:/_}.json 2> $out/sim_${sr/:/_}.err || { echo "sim $sr failed"; tail -10 $out/sim_${sr/:/_}.err; exit 1; }
done
step done
python3 - <<PY
import json, glob, os
for f in sorted(glob.glob("$out/*.json")):
    try:
        d = json.load(open(f))
    except Exception as e:
        print(os.path.basename(f), "unreadable", e); continue
    if not isinstance(d, dict) or "ms_per_step" not in d: continue
    r = d.get("roofline") or {}
    print(os.path.basename(f), d["ms_per_step"], d.get("value"), "frac", r.get("frac"), "traffic", r.get("traffic"), {k: round(v, 2) for k, v in (d.get("breakdown_ms") or {}).items()})
PY
