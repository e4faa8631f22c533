// internal.h -- entry points shared by routing.hip and routing_info.cpp inside the library (not part
// of the C ABI in include/shadow_routing.h).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/shadow_routing.h"

// srg_internal_compute_keys could not keep the table on u32 keys (the build needed u64 keys): the
// caller builds the u64 table with srg_compute_shortest_paths instead
#define SRG_INTERNAL_NEED_U64 100

extern "C" {
// The host entry (srg_compute_shortest_paths) with the latency table kept in the build's certified
// u32 keys: out_key[i * n + j] = latency / *unit_ns for i != j (0xFFFFFFFF on the diagonal), and
// out_diag[i] = the raw self-loop latency of nodes[i] (mod.rs:211-217).  latency = key * unit_ns,
// exactly.  One rank only.  0.4 GB instead of 0.8 GB of latencies cross PCIe at C3.
int srg_internal_compute_keys(srg_ctx* ctx, const srg_edge_list* graph, const uint32_t* nodes, uint32_t num_nodes,
                              uint32_t* out_key, uint64_t* out_diag, float* out_loss, uint64_t* unit_ns,
                              srg_stats* stats, char* errbuf, size_t errlen);
}
