set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "scan_variants or golden or random_vs" > gpurun_out/t30.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/b30.json 2> gpurun_out/b30.err
echo done
