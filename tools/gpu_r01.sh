set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_multi_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t18.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --fw-packed 0 > gpurun_out/b18c.json 2> gpurun_out/b18c.err && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --fw-packed 1 > gpurun_out/b18p.json 2> gpurun_out/b18p.err && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --fw-packed 0 --simulate-rank 8:3 > gpurun_out/b18s.json 2> gpurun_out/b18s.err && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --fw-packed 0 --fw-tile 64 --simulate-rank 8:3 >> gpurun_out/b18s.json 2>> gpurun_out/b18s.err
echo done
