set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/prio
mkdir -p $out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fw_symmetric or golden" --timeout 100 --timeout-method thread > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
for p in 0 1 0 1; do timeout -k 10 120 python -u bench.py --entry device --steps 5 --no-cpu --chain-prio $p > $out/b$p.json 2>$out/b$p.err && python -c "
import json;d=json.load(open('$out/b$p.json'));r=d['roofline'];print('prio $p', d['ms_per_step'], d['breakdown_ms']['ms_fw'], r['frac'], r['avg_launch_ms'])" || exit 1; done
