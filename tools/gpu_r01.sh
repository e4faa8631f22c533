set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t20.log 2>&1 && \
timeout -k 10 300 python -u bench.py --graph events --steps 5 --warmup 1 > gpurun_out/b20e.json 2> gpurun_out/b20e.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof20e -o run -- python -u bench.py --graph events --steps 2 --warmup 1 --no-cpu > gpurun_out/p20e.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke20.log 2>&1
echo done
