set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fwv
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fw_kernels" --timeout 100 --timeout-method thread > gpurun_out/fwv/t.log 2>&1 && tail -2 gpurun_out/fwv/t.log && \
for v in 2 4 2 4; do timeout -k 10 120 python -u bench.py --entry device --steps 5 --no-cpu --fw-packed $v > gpurun_out/fwv/b$v.json 2>/dev/null && python -c "
import json;d=json.load(open('gpurun_out/fwv/b$v.json'));r=d['roofline'];print('v$v', d['ms_per_step'], d['breakdown_ms']['ms_fw'], r['avg_launch_ms'], r['frac'])" || exit 1; done
