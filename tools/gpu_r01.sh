set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t22.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > gpurun_out/b22.json 2> gpurun_out/b22.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof22 -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/p22.log 2>&1
echo done
