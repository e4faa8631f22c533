set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sparse_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t23.log 2>&1 && \
timeout -k 10 300 python -u bench.py --graph ba --steps 2 --warmup 1 --no-cpu > gpurun_out/b23ba.json 2> gpurun_out/b23ba.err && \
timeout -k 10 300 python -u bench.py --graph ba --steps 2 --warmup 1 --no-cpu --no-locality > gpurun_out/b23ban.json 2> gpurun_out/b23ban.err
echo done
