#!/bin/bash
# Diagnostic build for the value-hop race A/B: the product source with the event that
# orders the chain stream after the FW sync-word reset (SymFw::begin) removed, into
# tools/dbg/libshadow_routing_noorder.so.  Load it with SRG_LIB_PATH to see the round-4 failure come
# back under tests/test_fw_overlap.py::test_stale_sync_words_do_not_release_the_chain.
set -euo pipefail
cd "$(dirname "$0")/../.."
T=$(mktemp -d)
mkdir -p "$T/shadow_amd" && cp -r shadow_amd/csrc "$T/shadow_amd/csrc" && cp -r include "$T/include"
python3 - "$T/shadow_amd/csrc/routing.hip" <<'PY'
import sys
p = sys.argv[1]
s = open(p).read()
a = "        HIP_CHECK(hipStreamWaitEvent(c.aux_stream, c.ev_fwreset, 0));\n"
assert a in s
open(p, "w").write(s.replace(a, "", 1))
PY
O="$T/o"; mkdir -p "$O"
for f in routing.hip comm.hip; do
  /opt/rocm/bin/hipcc -c -fPIC -O3 -std=c++17 -ffp-contract=off -I include -x hip --offload-arch=gfx950 "$T/shadow_amd/csrc/$f" -o "$O/$f.o"
done
for f in gml.cpp routing_info.cpp; do
  /opt/rocm/bin/hipcc -c -fPIC -O3 -std=c++17 -ffp-contract=off -I include "$T/shadow_amd/csrc/$f" -o "$O/$f.o"
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tools/dbg/libshadow_routing_noorder.so "$O"/*.o -ldl -lpthread -lhsa-runtime64
rm -rf "$T"
echo built tools/dbg/libshadow_routing_noorder.so
