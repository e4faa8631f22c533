set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t25.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/b25.json 2> gpurun_out/b25.err && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --simulate-rank 8:3 > gpurun_out/b25s.json 2> gpurun_out/b25s.err && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --simulate-rank 4:1 >> gpurun_out/b25s.json 2>> gpurun_out/b25s.err && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --simulate-rank 2:0 >> gpurun_out/b25s.json 2>> gpurun_out/b25s.err
echo done
