set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_multi_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not c2_sampled and not c1_full" > gpurun_out/t29.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/b29.json 2> gpurun_out/b29.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc29f -o run -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --no-profile > gpurun_out/pmc29.log 2>&1
echo done
