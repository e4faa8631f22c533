# scan-variant check: parity of the u32 scan kernels, then C3 device-entry timing per variant
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/scanv
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "scan_variants or golden or scan_v5" --timeout 200 --timeout-method thread > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -2 $out/t.log
for v in ${VARIANTS:-2 5}; do timeout -k 10 120 python -u bench.py --entry device --steps 5 --no-cpu --scan-variant $v > $out/b$v.json 2>$out/b$v.err && python -c "
import json;d=json.load(open('$out/b$v.json'));r=d['roofline'];print('scan v$v', d['ms_per_step'], d['breakdown_ms'], r['frac'])" || exit 1; done
