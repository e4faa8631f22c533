#!/bin/bash
# PMC passes for the dominant C3 kernel (fw_product_sym bulk) and for C4's k_sparse_bf at the
# default options, summaries with the bench workload keys
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-pmc_r02c}
mkdir -p $out
bash tools/pmc_fw.sh $out/fw && python tools/pmc_extract.py $out/fw "rocprofv3 --pmc, r02c (tools/pmc_fw.sh, C3 atlas_like(10000) host entry, 1 step, symmetric FW bulk launches)" "atlas:10000:10000:packed2:tile128:div1:g8:w2" "fw_product_sym<" > $out/fw_pmc.txt || { echo fw pmc failed; tail -20 $out/fw/*.log; exit 1; }
tail -30 $out/fw_pmc.txt
bash tools/pmc_sparse.sh $out/sp --vertices 50000 && python tools/pmc_extract_sparse.py $out/sp "rocprofv3 --pmc, r02c (tools/pmc_sparse.sh, C4 barabasi_albert(50000, m=4), 1 step, defaults)" "ba:50000:50000:packed2:tile128:div1:g8:w2" > $out/sp_pmc.txt || { echo sp pmc failed; tail -20 $out/sp/*.log; exit 1; }
tail -30 $out/sp_pmc.txt
