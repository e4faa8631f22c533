#!/bin/bash
# Round 5: host codec throughput on the GPU box (no GPU use): ISA x thread count
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05n}; mkdir -p $O
for v in base avx2 avx512; do
  case $v in base) F="";; avx2) F="-mavx2";; avx512) F="-mavx512f -mavx512bw -mavx512vl";; esac
  /opt/rocm/lib/llvm/bin/clang++ -O3 -std=c++17 $F -pthread -o /tmp/codec_probe_$v tools/codec_probe.cpp || exit 1
  timeout -k 10 300 /tmp/codec_probe_$v > $O/codec_$v.txt || exit 1
  echo "== $v"; cat $O/codec_$v.txt
done
