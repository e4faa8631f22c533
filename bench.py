"""Benchmark: Shadow routing-table build (all-pairs RoutingInfo) on MI355X.

Workload (BASELINE.json metric, config C3): 10,000-vertex Atlas-like complete GML graph
(shadow_amd.synth.atlas_like(10000, seed=10000); 49,995,000 undirected edges + 10,000
self-loops), all 10,000 nodes used.  One step = srg_compute_shortest_paths_device on the
edge list already resident in HBM -> every (latency_ns, packet_loss) of the 10^8 used pairs
written to HBM (dense W build, blocked FW, tight-DAG loss pass, extraction).

value = source-SSSPs/s over the whole job (sources routed per second, all ranks).
N > 1: ONE 10k-vertex RoutingInfo per step built by all N GPUs together ("scaling":
"strong"): FW row blocks split across ranks with a per-pivot-block RCCL broadcast of the
pivot row panel, each rank routes the sources whose rows it owns, and the output rows are
exchanged point to point so that every rank ends with the whole table.
--graph ba selects config C4 (50,000-vertex Barabasi-Albert, m=4; sparse batched
Bellman-Ford with sources sharded across ranks + output row exchange).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "APSP wall time + source-SSSPs/sec, 10k-vertex GML graph, 1/2/4/8 MI355X"
# VALU peak: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz (MI355X_MICROARCH.md chip table: wave64
# issues over 2 cycles on a SIMD-32) = 78.6 T int32 lane-ops/s.
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
# algorithmic int32 ops per min-plus relaxation c = min(c, a + b): one add + one min (u32 keys);
# u64 keys: 64-bit add (2) + 64-bit compare (1) + 2 selects.  Issued on gfx950 as
# v_lshl_add_u64 (two packed u32 adds) + v_min3_u32 per two relaxations (kernels.hip.h fw_tile_pk).
OPS_PER_RELAX = {0: 2.0, 1: 5.0}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(edges, target_s, threads):
    """Reference-equivalent CPU pipeline (oracle, 'port') on a bounded sample of sources."""
    import numpy as np
    import oracle
    g = edges.as_tuple()
    nodes = np.arange(edges.num_vertices, dtype=np.uint32)
    rng = np.random.default_rng(12345)
    done, spent = 0, 0.0
    k = threads
    while spent < target_s:
        sample = rng.choice(edges.num_vertices, size=k, replace=False).astype(np.uint32)
        spent += oracle.time_sources(g, nodes, sample, nthreads=threads)
        done += k
        log(f"cpu baseline: {done} sources in {spent:.1f}s")
        if spent > 0:
            k = max(threads, min(4 * k, int(threads * max(1.0, (target_s - spent) / max(spent / done * threads, 1e-3)))))
            k = min(k, edges.num_vertices)
    return done / spent, done, spent


def load_traffic(kernel_substr):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary
    (profiles/fw_pmc_latest.json for the FW tile, profiles/sparse_pmc_latest.json for k_sparse_bf)."""
    name = "sparse_pmc_latest.json" if "sparse" in kernel_substr else "fw_pmc_latest.json"
    p = os.path.join(ROOT, "profiles", name)
    try:
        with open(p) as f:
            d = json.load(f)
        return d.get("hbm_bytes_per_launch"), d.get("source")
    except Exception:
        return None, None


def bench_events(args, n=10**7, hosts=10000):
    """C5 stretch: one round's 10^7 cross-host packet events -> deliver times via the
    dense routing table (10k x 10k latencies resident in HBM), per-destination-host queue order,
    min next event / min used latency.  value = events ordered per second (1 GPU)."""
    import numpy as np
    import torch
    from shadow_amd import Router
    from shadow_amd import events as ev
    dev = torch.device("cuda", 0)
    b, round_end = ev.synthetic_round(n, hosts, hosts, seed=7)
    table = torch.randint(1_000_000, 100_000_000, (hosts, hosts), dtype=torch.int64, device=dev)
    db = ev.DeviceEventBatch(b, hosts, round_end, dev)
    deliver = torch.empty(n, dtype=torch.int64, device=dev)
    order = torch.empty(n, dtype=torch.int32, device=dev)
    off = torch.empty(hosts + 1, dtype=torch.int64, device=dev)
    router = Router(0)
    for _ in range(args.warmup):
        res = ev.order_packet_events_device(router, db, table, deliver, order, off)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = ev.order_packet_events_device(router, db, table, deliver, order, off)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    ms = el * 1e3 / args.steps
    cpu = None
    if not args.no_cpu:
        import oracle
        k = 2_000_000
        sub = {kk: v[:k] for kk, v in b.items()}
        tab = table.cpu().numpy().view(np.uint64)
        t1 = time.perf_counter()
        oracle.order_packet_events(sub, tab, hosts, round_end)
        cs = time.perf_counter() - t1
        cpu = {"value": round(k / cs, 1), "unit": "events/s", "cores": 1, "kind": "port",
               "sample": f"first {k} events of the batch, oracle restatement (per-host std::sort), {cs:.1f}s"}
    # HBM bytes per event: inputs 4*4 + 2*8, deliver write + table read 8 + 8, per radix pass
    # key+index read twice (hist + scatter) and written once: 3*12 (one-word key)
    per_ev = 16 + 16 + 16 + res["radix_passes"] * 36
    print(json.dumps({"metric": "packet events ordered/s (C5 stretch: deliver times + per-host queue order + "
                                "min next event, 10^7 events, 10k hosts)", "value": round(n / (ms * 1e-3), 1),
                      "unit": "events/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
                      "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                      "dtype": "u64", "data": "synthetic",
                      "config": {"workload": "C5 synthetic_round(1e7 events, 10000 hosts, seed 7)", "events": n,
                                 "hosts": hosts, "key_bits": res["key_bits"], "radix_passes": res["radix_passes"]},
                      "roofline": {"bound": "hbm", "achieved": round(per_ev * n / (ms * 1e-3) / 1e9, 1),
                                   "peak": 8000.0, "unit": "GB/s",
                                   "frac": round(per_ev * n / (ms * 1e-3) / 1e9 / 8000.0, 4), "traffic": None,
                                   "bytes_per_event": per_ev, "note": "whole-call time, all kernels"},
                      "cpu_baseline": cpu}), flush=True)


def init_strong_router(local, dev):
    """RCCL-backed router for the multi-GPU build, with an agreed go/no-go on every rank: librccl
    must load everywhere before the collective init, and a small multi-rank build must equal the
    single-GPU build bit for bit.  (None, reason) -> the caller runs independent replicas."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from shadow_amd import Router, synth
    from shadow_amd import dist as sd

    def agree(ok):
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    try:
        Router.comm_unique_id()  # loads librccl (no collective)
        ok = True
    except Exception as e:  # noqa: BLE001
        log(f"librccl: {e}")
        ok = False
    if not agree(ok):
        return None, "librccl unavailable"
    try:
        router = sd.init_router(local)
    except Exception as e:  # noqa: BLE001
        log(f"RCCL communicator: {e}")
        router = None
    if not agree(router is not None):
        return None, "RCCL communicator init failed"
    g = synth.random_graph(300, 0.05, 1234, lat_hi=1000)
    nodes = list(range(300))
    try:
        got = router.compute_shortest_paths(g, nodes)
        ref = Router(local).compute_shortest_paths(g, nodes)
        ok = np.array_equal(got.latency_ns, ref.latency_ns) and np.array_equal(
            got.packet_loss.view(np.uint32), ref.packet_loss.view(np.uint32))
    except Exception as e:  # noqa: BLE001
        log(f"multi-rank sanity build: {e}")
        ok = False
    if not agree(ok):
        return None, "multi-rank sanity check failed"
    return router, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--vertices", type=int, default=10000)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--graph", choices=["atlas", "ba", "events"], default="atlas",
                    help="atlas = C3 (headline), ba = C4, events = C5 stretch (10^7 packet events)")
    ap.add_argument("--entry", choices=["host", "device"], default="device",
                    help="host = srg_compute_shortest_paths (host edge list in, host table out: H2D + D2H "
                         "included); device = srg_compute_shortest_paths_device (inputs/outputs in HBM)")
    ap.add_argument("--replicas", action="store_true", help="N>1: independent full builds per rank (weak)")
    ap.add_argument("--no-gather", action="store_true", help="N>1: skip the output-row exchange")
    ap.add_argument("--sparse-group", type=int, default=None, help="sparse: label rows in flight per wave (4/8)")
    ap.add_argument("--sparse-wgs", type=int, default=None, help="sparse: resident batches per CU (1/2)")
    ap.add_argument("--sparse-delta-div", type=int, default=None,
                    help="sparse: bucket width = max edge latency / this (0 = plain Bellman-Ford)")
    ap.add_argument("--sparse-delta-all", type=int, default=None, help="sparse: 1 = bucket test over every dropped lane")
    ap.add_argument("--no-locality", action="store_true", help="sparse: batch sources in node order")
    ap.add_argument("--fw-tile", type=int, default=0, help="dense FW tile (0 = auto)")
    ap.add_argument("--fw-packed", type=int, default=1, help="u32 FW tiles: 1 = packed-pair adds, 0 = add + min3")
    ap.add_argument("--scan-variant", type=int, default=None, help="u32 tight scan kernel (0 readlane, 1 scalar)")
    ap.add_argument("--simulate-rank", type=str, default=None,
                    help="TIMING AID 'G:r': run rank r's share of a G-rank build alone, collectives elided "
                         "(outputs invalid; prints a diagnostic line, never the bench result)")
    args = ap.parse_args()
    if args.graph == "ba" and args.vertices == 10000 and "--vertices" not in sys.argv:
        args.vertices = 50000

    import torch
    import torch.distributed as dist

    if args.graph == "events":
        return bench_events(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from shadow_amd import Router, synth
    from shadow_amd import _native as N
    from shadow_amd.device import DeviceGraph, compute_shortest_paths_device, set_profiling

    V = args.vertices
    seed = args.seed if args.seed is not None else V
    t0 = time.time()
    if args.graph == "atlas":
        edges = synth.atlas_like(V, seed=seed)
        gdesc = f"C3 atlas_like({V}, seed={seed}): complete undirected GML-equivalent graph"
    else:
        edges = synth.barabasi_albert(V, 4, seed=seed)
        gdesc = f"C4 barabasi_albert({V}, m=4, seed={seed}): sparse undirected graph"
    log(f"[rank {rank}] generated {gdesc}: {edges.num_edges} edges in {time.time()-t0:.1f}s")
    dg = DeviceGraph(edges, dev)
    nodes = torch.arange(V, dtype=torch.int32, device=dev)
    out_lat = torch.empty((V, V), dtype=torch.int64, device=dev)
    out_loss = torch.empty((V, V), dtype=torch.float32, device=dev)
    strong = world > 1 and not args.replicas
    fallback = None
    if strong:
        router, fallback = init_strong_router(local, dev)
        if router is None:
            log(f"[rank {rank}] multi-rank build unavailable ({fallback}): running independent replicas")
            strong = False
        elif args.no_gather:
            router.set_option(N.SRG_OPT_GATHER_OUTPUT, 0)
    if not strong:
        router = Router(local)
    if args.no_locality:
        router.set_option(N.SRG_OPT_SPARSE_LOCALITY, 0)
    if args.fw_tile:
        router.set_option(N.SRG_OPT_FW_TILE, args.fw_tile)
    router.set_option(N.SRG_OPT_FW_PACKED, args.fw_packed)
    if args.sparse_group is not None:
        router.set_option(N.SRG_OPT_SPARSE_GROUP, args.sparse_group)
    if args.sparse_delta_all is not None:
        router.set_option(N.SRG_OPT_SPARSE_DELTA_ALL, args.sparse_delta_all)
    if args.sparse_delta_div is not None:
        router.set_option(N.SRG_OPT_SPARSE_DELTA_DIV, args.sparse_delta_div)
    if args.sparse_wgs is not None:
        router.set_option(N.SRG_OPT_SPARSE_WGS_PER_CU, args.sparse_wgs)
    if args.scan_variant is not None:
        router.set_option(N.SRG_OPT_SCAN_VARIANT, args.scan_variant)
    if args.simulate_rank:
        sg, sr = (int(x) for x in args.simulate_rank.split(":"))
        router.set_option(N.SRG_OPT_SIMULATE_RANK, sg * 1000 + sr)

    if args.entry == "host":
        import numpy as np
        h_nodes = np.arange(V, dtype=np.uint32)
        h_lat = np.empty((V, V), dtype=np.uint64)
        h_loss = np.empty((V, V), dtype=np.float32)
        h_lat.fill(0)  # fault the pages in once: the caller's Vecs are already allocated
        h_loss.fill(0)

        def step():
            return router.compute_shortest_paths(edges, h_nodes, h_lat, h_loss).stats
    else:
        def step():
            return compute_shortest_paths_device(router, dg, nodes, out_lat, out_loss)

    for i in range(args.warmup):
        s = step()
        log(f"[rank {rank}] warmup {i}: {s['ms_total']:.2f} ms (build {s['ms_build']:.2f}, fw/bf {s['ms_fw']:.2f}, "
            f"scan {s['ms_scan']:.2f}, loss {s['ms_loss']:.2f}, extract {s['ms_extract']:.2f}, "
            f"exchange {s['ms_exchange']:.2f}; rounds {s['loss_rounds']}, multi {s['multi_pred_pairs']}, "
            f"kind {s['path_kind']}, ess {s['essential_edges']} ({s['essential_edges'] / V / V:.3f} of V^2), "
            f"scan_kind {s['scan_kind']}, relax {s['relaxations']}, local {s['local_sources']})")
    set_profiling(router, not args.no_profile)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    agg = {}
    t_start = time.perf_counter()
    for i in range(args.steps):
        s = step()
        for k, v in s.items():
            if isinstance(v, (int, float)):
                agg[k] = agg.get(k, 0) + v
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1e3 / args.steps
    value = (1 if strong else world) * V * args.steps / elapsed

    kind = s["path_kind"]
    roofline = None
    if agg.get("prof_launches") and kind == 3:
        # sparse: HBM-bound; algorithmic bytes per source = one CSR sweep + one result row
        # (SURVEY §8d): arcs*16 + (V+1)*4 + V*12
        arcs = int(((edges.src != edges.dst).sum()) * (1 if edges.directed else 2))
        per_src = arcs * 16 + (V + 1) * 4 + V * 12
        avg_ms = agg["prof_kernel_ms"] / agg["prof_launches"]
        srcs = agg["prof_relaxations"] / agg["prof_launches"]
        achieved = per_src * srcs / (avg_ms * 1e-3) / 1e9
        traffic, tsrc = load_traffic("k_sparse_bf")
        roofline = {"bound": "hbm", "kernel": "k_sparse_bf (batched lexicographic Bellman-Ford, delta-stepping buckets)",
                    "achieved": round(achieved, 1), "peak": 8000.0, "unit": "GB/s",
                    "frac": round(achieved / 8000.0, 4), "traffic": traffic, "avg_launch_ms": round(avg_ms, 3),
                    "bytes_per_source": per_src, "sources_per_launch": int(srcs), "traffic_source": tsrc,
                    # measured HBM bytes per launch over this run's launch time: the real HBM rate
                    "traffic_GBps": round(traffic / (avg_ms * 1e-3) / 1e9, 1) if traffic else None}
    elif agg.get("prof_launches"):
        avg_ms = agg["prof_kernel_ms"] / agg["prof_launches"]
        relax = agg["prof_relaxations"] / agg["prof_launches"]
        achieved = relax * OPS_PER_RELAX.get(kind, 2.0) / (avg_ms * 1e-3) / 1e12
        traffic, tsrc = load_traffic("fw_product")
        roofline = {"bound": "valu", "kernel": ("fw_product<u32,128,32,packed> (FW phase 3, non-lookahead tiles)" if args.fw_packed else "fw_product<u32,128,32> (FW phase 3, non-lookahead tiles)") if kind == 0 else "fw_product<u64,64,32> (FW phase 3)", "achieved": round(achieved, 3),
                    "peak": round(VALU_PEAK_TOPS, 3), "unit": "TOP/s (int32 VALU lane-ops)",
                    "frac": round(achieved / VALU_PEAK_TOPS, 4), "traffic": traffic,
                    "avg_launch_ms": round(avg_ms, 4), "relaxations_per_launch": int(relax),
                    "ops_per_relaxation": OPS_PER_RELAX.get(kind, 2.0), "relax_per_s": round(relax / (avg_ms * 1e-3), 1),
                    "traffic_source": tsrc}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            aff = len(os.sched_getaffinity(0))
        except Exception:
            aff = os.cpu_count() or 1
        threads = max(1, min(16, aff))
        v, k, sec = cpu_baseline(edges, args.cpu_seconds, threads)
        cpu = {"value": round(v, 3), "unit": "source-SSSPs/s", "cores": threads, "kind": "port",
               "sample": f"{k} random sources of the same 10k-vertex graph, reference-equivalent pipeline "
                         f"(HashMap-score Dijkstra + linear nodes.contains + HashMap merge), {sec:.1f}s"}

    if args.simulate_rank:
        n = args.steps
        print(json.dumps({"diagnostic": "simulated rank (collectives elided, outputs invalid)",
                          "simulate_rank": args.simulate_rank, "ms_per_step": round(ms_per_step, 3),
                          "breakdown_ms": {k: round(agg.get(k, 0) / n, 3) for k in
                                           ("ms_h2d", "ms_build", "ms_fw", "ms_scan", "ms_loss", "ms_extract", "ms_exchange", "ms_d2h", "ms_total")},
                          "roofline": roofline}), flush=True)
        return
    if rank == 0:
        n = args.steps
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "source-SSSPs/s", "n_gpus": world, "steps": n,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None,
            "dtype": "u64+f32" if kind == 1 else "u32+f32",
            "data": "synthetic",
            "config": {"workload": f"{gdesc}, all {V} nodes used, edge list resident in HBM",
                       "vertices": V, "edges": int(edges.num_edges), "global_batch": V,
                       "parallelism": (f"rowblock{world}+rccl" if strong else f"replicas{world}") if world > 1 else "single",
                       **({"fallback": fallback} if fallback else {}),
                       "path": {0: "dense-u32", 1: "dense-u64", 3: "sparse-bf-u32"}.get(kind, str(kind))},
            "apsp_wall_ms": round(ms_per_step, 3),
            "breakdown_ms": {k: round(agg.get(k, 0) / n, 3) for k in ("ms_h2d", "ms_build", "ms_fw", "ms_scan", "ms_loss", "ms_extract", "ms_exchange", "ms_d2h", "ms_total")},
            "loss_rounds": s["loss_rounds"], "multi_pred_pairs": s["multi_pred_pairs"],
            "essential_edges": s["essential_edges"], "scan_kind": s["scan_kind"],
            "roofline": roofline, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
