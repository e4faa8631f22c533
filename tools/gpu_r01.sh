set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_multi_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not c2_sampled and not c1_full and not c3_bench" > gpurun_out/t31.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/b31.json 2> gpurun_out/b31.err && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --simulate-rank 8:3 > gpurun_out/b31s.json 2> gpurun_out/b31s.err && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --simulate-rank 4:1 >> gpurun_out/b31s.json 2>> gpurun_out/b31s.err
echo done
