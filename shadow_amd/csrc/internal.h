// internal.h -- entry points shared by routing.hip and routing_info.cpp inside the library (not part
// of the C ABI in include/shadow_routing.h).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/shadow_routing.h"

// srg_internal_compute_table could not keep the table on u32 keys (the build needed u64 keys): the
// caller builds the u64 table with srg_compute_shortest_paths instead
#define SRG_INTERNAL_NEED_U64 100

// a host table from a context's pinned-table pool (routing.hip, TablePool)
struct srg_table;

extern "C" {
// The host entry (srg_compute_shortest_paths / srg_get_direct_paths by `shortest`) into tables
// from the context's pool (tab_lat, tab_loss: srg_internal_table_get; their page-locking is kept
// for the next build into them).  out_key non-null (shortest paths, one rank): the latency table is
// kept in the build's certified u32 keys: out_key[i * n + j] = latency / *unit_ns for i != j
// (0xFFFFFFFF on the diagonal), and out_diag[i] = the raw self-loop latency of nodes[i]
// (mod.rs:211-217); latency = key * unit_ns, exactly; 0.4 GB instead of 0.8 GB of latencies cross
// PCIe at C3.  Returns SRG_INTERNAL_NEED_U64 when the build needed u64 keys.
int srg_internal_compute_table(srg_ctx* ctx, const srg_edge_list* graph, const uint32_t* nodes, uint32_t num_nodes,
                               int shortest, uint64_t* out_lat, uint32_t* out_key, uint64_t* out_diag, float* out_loss,
                               uint64_t* unit_ns, srg_table* tab_lat, srg_table* tab_loss, srg_stats* stats,
                               char* errbuf, size_t errlen);
// a table of at least `bytes` (*host: its address, 2 MB aligned): a recycled one from the pool, or
// a fresh mapping (null: out of memory)
srg_table* srg_internal_table_get(srg_ctx* ctx, size_t bytes, void** host);
// back to its pool (still page-locked), or freed when the pool is closed or full
void srg_internal_table_put(srg_table* t);
}
