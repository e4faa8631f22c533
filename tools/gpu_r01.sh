set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_multi_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not c3_bench and not c2_sampled and not c1_full" > gpurun_out/t27.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/b27.json 2> gpurun_out/b27.err
echo done
