"""Benchmark: Shadow routing-table build (all-pairs RoutingInfo) on MI355X.

Workload (BASELINE.json metric, config C3): 10,000-vertex Atlas-like complete GML graph
(shadow_amd.synth.atlas_like(10000, seed=10000); 49,995,000 undirected edges + 10,000
self-loops), all 10,000 nodes used.  One step = the host entry srg_compute_shortest_paths, the
"APSP wall time" SURVEY §8(d) defines: the host edge list (1.0 GB) in, H2D, dense W build,
blocked FW, tight-DAG loss pass, extraction, and every (latency_ns, packet_loss) of the 10^8
used pairs back in host memory (1.2 GB D2H, overlapped with the scan).  --entry device times
srg_compute_shortest_paths_device (inputs and outputs resident in HBM); the host-entry run also
reports that time as device_entry_ms.

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


def cpu_info():
    """Host CPU model, machine CPU count, and the CPU share this job is given."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count() or 1
    # the GPU pool grants each GPU job a CPU share (OMP_NUM_THREADS, 16 per GPU on the MI355X
    # boxes); the affinity mask shows the whole machine there, so the share sets the threads
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or aff
    return {"cpu_model": model, "machine_cpus": os.cpu_count(), "affinity_cpus": aff,
            "threads": max(1, min(share, aff))}


def cpu_rate(edges, target_s, threads, mode, seed=12345):
    """Sources/s of an oracle pipeline on growing random samples of the graph's sources until
    about target_s seconds of CPU work (oracle.time_sources_mode; setup excluded)."""
    import numpy as np
    import oracle
    g = edges.as_tuple()
    V = edges.num_vertices
    nodes = np.arange(V, dtype=np.uint32)
    rng = np.random.default_rng(seed)
    done, spent, setup = 0, 0.0, 0.0
    k = threads
    while spent < target_s and done < V:
        k = min(k, V - done) if done < V else k
        sample = rng.choice(V, size=k, replace=False).astype(np.uint32)
        t, setup = oracle.time_sources_mode(g, nodes, sample, nthreads=threads, mode=mode)
        spent += t
        done += k
        log(f"cpu baseline mode {mode}: {done} sources in {spent:.1f}s (setup {setup:.1f}s)")
        k = max(threads, min(4 * k, int(k * max(1.0, (target_s - spent) / max(t, 1e-3)))))
    return done / spent, done, spent, setup


def cpu_fixed(edges, k, threads, mode, seed=12345, step=32):
    """Sources/s of an oracle pipeline over a FIXED seeded sample of k sources (256),
    timed in slices of `step` sources so that progress is logged; setup excluded."""
    import numpy as np
    import oracle
    g = edges.as_tuple()
    V = edges.num_vertices
    nodes = np.arange(V, dtype=np.uint32)
    sample = np.random.default_rng(seed).choice(V, size=min(k, V), replace=False).astype(np.uint32)
    spent = 0.0
    for i in range(0, len(sample), step):
        t, _ = oracle.time_sources_mode(g, nodes, sample[i:i + step], nthreads=threads, mode=mode)
        spent += t
        log(f"cpu baseline mode {mode}: {min(i + step, len(sample))}/{len(sample)} sources in {spent:.1f}s")
    return len(sample) / spent, len(sample), spent


def cpu_baselines(edges, target_s, desc, sources=256):
    """SURVEY §8(d) CPU baseline on the box's host cores: the reference-equivalent pipeline
    (HashMap-score petgraph Dijkstra + linear nodes.contains + HashMap merge, like rayon x
    petgraph, mod.rs:190-208) on a fixed seeded sample of `sources` sources (256, as §8(d) asks),
    and a CPU-best variant (dense scores, O(1) membership, dense rows; the dense-matrix Dijkstra
    on dense graphs) on a bounded sample; both extrapolated to all sources at the measured
    per-source rate."""
    info = cpu_info()
    th = info["threads"]
    V = edges.num_vertices
    dense = edges.num_edges * 8 > V * V
    ref, k0, s0 = cpu_fixed(edges, sources, th, 0)
    best, k1, s1, setup1 = cpu_rate(edges, max(3.0, target_s / 2), th, 2 if dense else 1)
    return {"value": round(ref, 3), "unit": "source-SSSPs/s", "cores": th, "kind": "port",
            "sample": f"fixed seeded sample of {k0} sources of {desc} (SURVEY §8d), reference-equivalent pipeline "
                      f"(HashMap-score petgraph Dijkstra + linear nodes.contains + HashMap merge, mod.rs:190-208) on "
                      f"{th} threads, {s0:.1f}s",
            "extrapolated": True, "full_run_estimate_s": round(V / ref, 1),
            # rayon's default pool is every core (mod.rs:190-191); the box grants this job a CPU share,
            # so the all-core figure is the measured per-thread rate x the affinity core count (the
            # per-source runs are independent: linear in cores, an upper estimate, not a measurement)
            "all_cores_estimate": {"value": round(ref * info["affinity_cpus"] / th, 3), "cores": info["affinity_cpus"],
                                   "basis": f"measured {th}-thread rate x {info['affinity_cpus']}/{th} (linear scaling assumed)"},
            **info,
            "best": {"value": round(best, 3), "unit": "source-SSSPs/s", "cores": th,
                     "algorithm": ("dense-matrix Dijkstra, O(V^2) per source" if dense else
                                   "heap Dijkstra with dense scores") + ", O(1) membership, dense output rows",
                     "sample": f"{k1} random sources, {s1:.1f}s (+{setup1:.1f}s one-time setup)",
                     "extrapolated": True, "full_run_estimate_s": round(V / best + setup1, 1)}}


def load_traffic(kernel_substr, workload_key):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary
    (profiles/fw_pmc_latest.json for the FW tile, profiles/sparse_pmc_latest.json for k_sparse_bf),
    only when that summary was collected on this run's workload and options (else None)."""
    name = "sparse_pmc_latest.json" if "sparse" in kernel_substr else "fw_pmc_latest.json"
    p = os.path.join(ROOT, "profiles", name)
    try:
        with open(p) as f:
            d = json.load(f)
    except Exception:
        return None, None
    if d.get("workload_key") != workload_key:
        return None, f"{d.get('source')} (workload {d.get('workload_key')!r} != this run's {workload_key!r})"
    return d.get("hbm_bytes_per_launch"), d.get("source")


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
    import torch
    import torch.distributed as dist
    from shadow_amd import Router, gate
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
    # the same gate as the one-process rank group (shadow_amd.gate): dense, symmetric-FW and sparse
    # builds through the communicator equal to this GPU alone, bit for bit, on every rank
    single = Router(local)
    try:
        ok, why = gate.compare_builds(router.compute_shortest_paths, single.compute_shortest_paths, gate.gate_cases())
    finally:
        single.close()
    if not ok:
        log(f"multi-rank sanity build: {why}")
    if not agree(ok):
        return None, "multi-rank sanity check failed" + (f" ({why})" if why else "")
    return router, None


def make_edges(args):
    """The synthetic graph of the selected config (BASELINE.json configs; SURVEY §8d generators)."""
    from shadow_amd import synth
    V = args.vertices
    seed = args.seed if args.seed is not None else V
    if args.graph == "atlas":
        edges = synth.atlas_like(V, seed=seed)
        cname = {10000: "C3", 4096: "C2"}.get(V, "atlas")
        gdesc = f"{cname} atlas_like({V}, seed={seed}): complete undirected GML-equivalent graph"
    elif args.graph == "complete":
        seed = args.seed if args.seed is not None else 1001
        edges = synth.complete_random(V, seed=seed)
        gdesc = f"C1 complete_random({V}, seed={seed}): complete undirected graph, random latency/loss"
    else:
        edges = synth.barabasi_albert(V, 4, seed=seed)
        gdesc = f"C4 barabasi_albert({V}, m=4, seed={seed}): sparse undirected graph"
    if args.lat_scale != 1:
        import numpy as np
        edges.latency_ns = edges.latency_ns * np.uint64(args.lat_scale)
        gdesc += f", latencies x{args.lat_scale}"
    return edges, gdesc, seed


def apply_options(router, args):
    """Bench flags -> srg_set_option (Router and MultiRouter alike)."""
    from shadow_amd import _native as N
    if args.no_locality:
        router.set_option(N.SRG_OPT_SPARSE_LOCALITY, 0)
    if args.fw_tile:
        router.set_option(N.SRG_OPT_FW_TILE, args.fw_tile)
    for flag, opt in (("sparse_delta_div", "SPARSE_DELTA_DIV"), ("fw_symmetric", "FW_SYMMETRIC"),
                      ("h2d_codec", "H2D_CODEC"),
                      ("late_loss", "LATE_LOSS"), ("edge_shard", "EDGE_SHARD"), ("scan_groups", "SCAN_GROUPS"),
                      ("loss_chunks", "LOSS_CHUNKS"), ("d2h_mode", "D2H_MODE"), ("fw_line_split", "FW_LINE_SPLIT"),
                      ("fw_step", "FW_STEP"), ("fw_overlap", "FW_OVERLAP"), ("fw_xcd_order", "FW_XCD_ORDER")):
        v = getattr(args, flag)
        if v is not None:
            router.set_option(getattr(N, "SRG_OPT_" + opt), v)


def workload_key(args, V, seed, world):
    # "lb": the dense FW runs the line-buffer bulk kernel (fw_bulk_lb, round 3): PMC traffic
    # collected on an earlier kernel (fw_product_sym) is not attached to it
    return (f"{args.graph}:{V}:{seed}:" + (f"x{args.lat_scale}:" if args.lat_scale != 1 else "")
            + ("lb:" if args.graph != "ba" else "")
            + f"packed2:tile{args.fw_tile or 128}:"
            f"div{args.sparse_delta_div if args.sparse_delta_div is not None else 1}:g8:w2"
            + (":ds2" if args.graph == "ba" else "")  # the two-phase sparse kernel (round 6)
            + (f":sym{args.fw_symmetric}" if args.fw_symmetric is not None else "")
            + (f":n{world}" if world > 1 else "") + (f":sim{args.simulate_rank}" if args.simulate_rank else ""))


def roofline_for(agg, kind, args, edges, V, wkey, sym):
    """The dominant kernel's roofline from the HIP-event launch times the library recorded:
    dense = the FW bulk tile kernel (VALU), sparse = the k_sparse_ds build (HBM; its launches between two events)."""
    if not agg.get("prof_launches"):
        return None
    avg_ms = agg["prof_kernel_ms"] / agg["prof_launches"]
    if kind == 3:
        # sparse: HBM-bound; algorithmic bytes per source = one CSR sweep + one result row
        # (SURVEY §8d): arcs*16 + (V+1)*4 + V*12
        arcs = int(((edges.src != edges.dst).sum()) * (1 if edges.directed else 2))
        per_src = arcs * 16 + (V + 1) * 4 + V * 12
        srcs = agg["prof_relaxations"] / agg["prof_launches"]
        achieved = per_src * srcs / (avg_ms * 1e-3) / 1e9
        traffic, tsrc = load_traffic("k_sparse", wkey)
        return {"bound": "hbm", "kernel": "k_sparse_ds (two-phase: latency-only batched delta-stepping with "
                                          "wavefront-aggregated window pushes, tight records, per-lane Kahn loss fold)",
                "achieved": round(achieved, 1), "peak": 8000.0, "unit": "GB/s",
                "frac": round(achieved / 8000.0, 4), "traffic": traffic, "avg_launch_ms": round(avg_ms, 3),
                "bytes_per_source": per_src, "sources_per_launch": int(srcs), "traffic_source": tsrc,
                # measured HBM bytes per launch over this run's launch time: the real HBM rate
                "traffic_GBps": round(traffic / (avg_ms * 1e-3) / 1e9, 1) if traffic else None,
                "workload_key": wkey}
    relax = agg["prof_relaxations"] / agg["prof_launches"]
    achieved = relax * OPS_PER_RELAX.get(kind, 2.0) / (avg_ms * 1e-3) / 1e12
    traffic, tsrc = load_traffic("fw_product", wkey)
    if sym and kind == 1:
        kname = "fw_bulk_lb<u64,64,16> (FW phase 3 over the stored tiles I <= J, operands from the pivot's line buffer, u64 keys)"
    elif sym:
        kname = "fw_bulk_lb<128,16> (FW phase 3 over the stored tiles I <= J, operands from the pivot's line buffer, pair-packed)"
    elif kind == 0:
        kname = "fw_product<u32,128,16,2> (FW phase 3, pair-packed, non-lookahead tiles)"
    else:
        kname = "fw_product<u64,64,32,0> (FW phase 3)"
    r = {"bound": "valu", "kernel": kname, "achieved": round(achieved, 3),
         "peak": round(VALU_PEAK_TOPS, 3), "unit": "TOP/s (int32 VALU lane-ops)",
         "frac": round(achieved / VALU_PEAK_TOPS, 4), "traffic": traffic,
         "avg_launch_ms": round(avg_ms, 4), "relaxations_per_launch": int(relax),
         "ops_per_relaxation": OPS_PER_RELAX.get(kind, 2.0), "relax_per_s": round(relax / (avg_ms * 1e-3), 1),
         "traffic_source": tsrc, "workload_key": wkey}
    if kind == 0:
        # v_min* issue at half rate on gfx950: the pair-packed relaxation pair (v_lshl_add_u64 +
        # v_min3_u32) measured 0.187 wave-instr/SIMD/cycle = 2 relaxations per 10.7 cycles per
        # wave = 0.748 of the 2-op lane peak (profiles/r01_valu_rate_microbench.txt)
        r["instruction_mix_ceiling_frac"] = 0.748
        r["frac_of_mix_ceiling"] = round(achieved / VALU_PEAK_TOPS / 0.748, 4)
    return r


def verify_rows(edges, table_lat, table_loss, V, k=4, seed=4242):
    """k seeded rows of the benchmarked table against the oracle (outside the timed region)."""
    import numpy as np
    import oracle
    rows = np.random.default_rng(seed).choice(V, size=k, replace=False).tolist()
    dense = edges.num_edges * 8 > V * V
    lat, loss = oracle.compute_shortest_paths(edges.as_tuple(), list(range(V)), rows=rows, mode=2 if dense else 1,
                                              nthreads=cpu_info()["threads"])
    ok = np.array_equal(table_lat[rows], lat) and np.array_equal(table_loss[rows].view(np.uint32), loss.view(np.uint32))
    return {"rows": rows, "bit_exact": bool(ok)}


COLD_BREAKDOWN = {}  # cold_call: srg_create vs the first call, and that call's own stage times


def cold_call(make, args, edges, V):
    """srg_create (or srg_multi_create) + the first srg_compute_shortest_paths on freshly
    allocated, never-touched output arrays -- what Shadow's one call per simulation pays
    (sim_config.rs:137-141; the Rust binding's vec![0u64; n*n] is lazily zeroed memory)."""
    import numpy as np
    from shadow_amd import _native as N
    t0 = time.perf_counter()
    router = make()
    apply_options(router, args)
    t1 = time.perf_counter()
    lat = np.empty((V, V), dtype=np.uint64)   # not pre-faulted
    loss = np.empty((V, V), dtype=np.float32)
    t = router.compute_shortest_paths(edges, np.arange(V, dtype=np.uint32), lat, loss)
    t2 = time.perf_counter()
    ms = (t2 - t0) * 1e3
    del lat, loss
    st = t.stats
    if hasattr(router, "get_option"):  # srg_create: the HIP runtime's part vs the library's own
        COLD_BREAKDOWN.update({"create_hip_runtime_ms": round(router.get_option(N.SRG_OPT_CREATE_MS_RUNTIME), 1),
                               "create_library_ms": round(router.get_option(N.SRG_OPT_CREATE_MS_LIBRARY), 1)})
    COLD_BREAKDOWN.update({"create_ms": round((t1 - t0) * 1e3, 1), "first_call_ms": round((t2 - t1) * 1e3, 1),
                           **{k: round(st[k], 2) for k in ("ms_h2d", "ms_fw", "ms_scan", "ms_d2h", "ms_host_register")
                              if k in st}})
    return router, ms


def routing_info_times(edges, V, args, steps=3):
    """What Shadow's call site runs (sim_config.rs:425-462 -> RoutingInfo, mod.rs:428-477): one
    srg_routing_info_build per simulation.  cold = srg_create + the first build (fresh context, fresh
    host tables); steady = further builds on the same context (a RoutingInfo owns its tables, from the
    context's pinned-table pool: a freed RoutingInfo's tables are recycled still page-locked).  One
    rank: the table keeps the build's u32 keys (stats.table_keys)."""
    import numpy as np
    from shadow_amd import Router, generate_routing_info
    from shadow_amd import _native as N
    ids = list(range(V))
    t0 = time.perf_counter()
    r = Router(0)
    apply_options(r, args)
    ri = generate_routing_info(edges, ids, True, r)
    cold = (time.perf_counter() - t0) * 1e3
    keys = ri.stats.get("table_keys")
    cold_reg = ri.stats.get("ms_host_register")
    create = {"create_hip_runtime_ms": round(r.get_option(N.SRG_OPT_CREATE_MS_RUNTIME), 1),
              "create_library_ms": round(r.get_option(N.SRG_OPT_CREATE_MS_LIBRARY), 1)}
    ri.close()
    ts = []
    for _ in range(steps):
        t1 = time.perf_counter()
        ri = generate_routing_info(edges, ids, True, r)
        ts.append((time.perf_counter() - t1) * 1e3)
        st = ri.stats
        ri.close()
    r.close()
    return {"cold_ms": round(cold, 1), "steady_ms": round(float(np.median(ts)), 2),
            "steady_ms_all": [round(x, 2) for x in ts], "table_keys": keys,
            "h2d_ms": round(st["ms_h2d"], 2), "d2h_tail_ms": round(st["ms_d2h"], 2),
            "host_register_ms": {"cold": round(cold_reg, 2), "steady": round(st["ms_host_register"], 2)}, **create}


def emit(args, V, gdesc, edges, kind, world, value, ms_per_step, agg, s, roofline, cpu, extra_cfg, extra, scaling=None,
         steps_ms=None):
    n = args.steps
    brk = ("ms_h2d", "ms_build", "ms_fw", "ms_scan", "ms_loss", "ms_extract", "ms_exchange", "ms_d2h", "ms_total")
    entry_desc = ("host entry srg_compute_shortest_paths: host edge list in, host n x n table out "
                  "(H2D + kernels + D2H in the step)" if args.entry == "host" else
                  "device entry srg_compute_shortest_paths_device: edge list resident in HBM, table left in HBM")
    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "source-SSSPs/s", "n_gpus": world, "steps": n,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": scaling or ("strong" if world > 1 else "weak"), "vs_baseline": None,
        "dtype": "u64+f32" if kind == 1 else "u32+f32", "data": "synthetic",
        "config": {"workload": f"{gdesc}, all {V} nodes used, {entry_desc}", "entry": args.entry, "vertices": V,
                   "edges": int(edges.num_edges), "global_batch": V,
                   "path": {0: "dense-u32", 1: "dense-u64", 3: "sparse-ds-u32", 4: "sparse-bf-u64"}.get(kind, str(kind)), **extra_cfg},
        "apsp_wall_ms": round(ms_per_step, 3),
        # per-step wall times of the timed loop (this rank's clock; value uses the whole loop's max over ranks)
        "step_ms": steps_ms,
        "ms_h2d": round(agg.get("ms_h2d", 0) / n, 3), "ms_d2h": round(agg.get("ms_d2h", 0) / n, 3),
        "d2h_overlapped_GB": round(agg.get("d2h_overlapped_bytes", 0) / n / 1e9, 3),
        # page-locking of the caller's output rows on a helper thread (hidden unless it outlasts
        # H2D + FW; -1 = not used)
        "ms_host_register": round(agg.get("ms_host_register", 0) / n, 3),
        "breakdown_ms": {k: round(agg.get(k, 0) / n, 3) for k in brk},
        "loss_rounds": s["loss_rounds"], "multi_pred_pairs": s["multi_pred_pairs"],
        "essential_edges": s["essential_edges"], "scan_kind": s["scan_kind"],
        "latency_unit_ns": s["latency_unit_ns"],
        "roofline": roofline, "cpu_baseline": cpu, **extra,
    }
    print(json.dumps(line), flush=True)


def step_stats(ts):
    """median of the timed steps (>= 5 after 1 warm-up by default) plus min / max, ms."""
    import numpy as np
    a = np.asarray(ts, dtype=np.float64) * 1e3
    return {"median": round(float(np.median(a)), 3), "min": round(float(a.min()), 3), "max": round(float(a.max()), 3),
            "all": [round(float(x), 3) for x in a]}


def run_steps(step, args, label):
    s = None
    for i in range(args.warmup):
        s = step()
        log(f"[{label}] warmup {i}: {s['ms_total']:.2f} ms (h2d {s['ms_h2d']:.2f}, build {s['ms_build']:.2f}, "
            f"fw/bf {s['ms_fw']:.2f}, scan {s['ms_scan']:.2f}, loss {s['ms_loss']:.2f}, exchange {s['ms_exchange']:.2f}, "
            f"d2h {s['ms_d2h']:.2f}; kind {s['path_kind']}, ess {s['essential_edges']}, local {s['local_sources']})")
    return s


def bench_multi(args):
    """--gpus N without a launcher: ONE process drives N GPUs through srg_multi (Shadow's one-process
    model, manager.rs:301-324): one RoutingInfo per step, the whole n x n table in one host array,
    every GPU shipping its own sources' rows over its own PCIe link."""
    import numpy as np
    import torch
    from shadow_amd import MultiRouter
    from shadow_amd import _native as N
    G = args.gpus
    have = torch.cuda.device_count()
    if have < G:
        print(f"bench.py --gpus {G}: only {have} HIP device(s) visible; refusing to run {G} ranks on fewer GPUs",
              file=sys.stderr, flush=True)
        sys.exit(2)
    if args.entry != "host":
        print("bench.py --gpus N (one process): only the host entry is supported", file=sys.stderr, flush=True)
        sys.exit(2)
    edges, gdesc, seed = make_edges(args)
    V = args.vertices
    log(f"[multi{G}] generated {gdesc}: {edges.num_edges} edges")
    # go/no-go before anything is timed: small builds through the rank group must equal one GPU's
    # bit for bit (mod.rs:219: a table is whole or an error); otherwise independent replicas, labelled
    ok, reason = multi_gate(G, args)
    if not ok:
        log(f"[multi{G}] multi-device build refused by the gate ({reason}): running {G} independent replicas")
        return bench_replicas_inproc(args, G, edges, gdesc, seed, reason)
    router, cold_ms = cold_call(lambda: MultiRouter(list(range(G))), args, edges, V)
    log(f"[multi{G}] cold call (srg_multi_create + first call, unfaulted outputs): {cold_ms:.1f} ms")
    h_nodes = np.arange(V, dtype=np.uint32)
    h_lat = np.zeros((V, V), dtype=np.uint64)
    h_loss = np.zeros((V, V), dtype=np.float32)
    h_lat.fill(0)  # fault the pages in once: the caller's Vecs are already allocated
    h_loss.fill(0)

    def step():
        return router.compute_shortest_paths(edges, h_nodes, h_lat, h_loss).stats

    s = run_steps(step, args, f"multi{G}")
    router.set_option(N.SRG_OPT_PROFILING, 0 if args.no_profile else 1)
    for d in range(G):
        torch.cuda.synchronize(d)
    agg = {}
    ts = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        t1 = time.perf_counter()
        s = step()
        ts.append(time.perf_counter() - t1)
        for k, v in s.items():
            if isinstance(v, (int, float)):
                agg[k] = agg.get(k, 0) + v
    elapsed = time.perf_counter() - t0
    ms = elapsed * 1e3 / args.steps
    kind = s["path_kind"]
    ver = verify_rows(edges, h_lat, h_loss, V) if not args.no_verify else None
    roof = roofline_for(agg, kind, args, edges, V, workload_key(args, V, seed, G), kind == 0
                        and args.fw_symmetric != 0 and not edges.directed)
    emit(args, V, gdesc, edges, kind, G, G and V * args.steps / elapsed, ms, agg, s, roof, None,
         {"parallelism": f"multi{G} (one process, srg_multi: in-process group, pull collectives over xGMI)",
          "output": "full table in one host array (each GPU writes its sources' rows over its own PCIe link)",
          "cold_call_ms": round(cold_ms, 1)},
         {"verified_rows": ver}, steps_ms=step_stats(ts))


def multi_gate(G, args):
    """(ok, reason): the in-process rank group over G devices against device 0 alone
    (shadow_amd.gate: dense, symmetric-FW and sparse cases, latency and loss bit for bit)."""
    from shadow_amd import MultiRouter, Router, gate
    multi = single = None
    try:
        multi = MultiRouter(list(range(G)))
        single = Router(0)
        for r in (multi, single):
            apply_options(r, args)
        return gate.compare_builds(multi.compute_shortest_paths, single.compute_shortest_paths, gate.gate_cases())
    except Exception as e:  # noqa: BLE001
        return False, f"rank group setup: {type(e).__name__}: {e}"
    finally:
        for r in (multi, single):
            if r is not None:
                r.close()


def bench_replicas_inproc(args, G, edges, gdesc, seed, reason):
    """Fallback of bench_multi: G independent full builds per step, one per device, each on a host
    thread of its own (the C ABI releases the GIL), each into its own host table: weak scaling."""
    import threading

    import numpy as np
    from shadow_amd import Router
    from shadow_amd import _native as N
    V = args.vertices
    routers = [Router(d) for d in range(G)]
    for r in routers:
        apply_options(r, args)
    h_nodes = np.arange(V, dtype=np.uint32)
    tabs = [(np.zeros((V, V), dtype=np.uint64), np.zeros((V, V), dtype=np.float32)) for _ in range(G)]
    stats = [None] * G

    def one(d):
        stats[d] = routers[d].compute_shortest_paths(edges, h_nodes, tabs[d][0], tabs[d][1]).stats

    def step():
        th = [threading.Thread(target=one, args=(d,)) for d in range(G)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if any(x is None for x in stats):
            raise RuntimeError("a replica build failed")
        return stats[0]

    s = run_steps(step, args, f"replicas{G}")
    routers[0].set_option(N.SRG_OPT_PROFILING, 0 if args.no_profile else 1)
    agg = {}
    ts = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        t1 = time.perf_counter()
        s = step()
        ts.append(time.perf_counter() - t1)
        for k, v in s.items():
            if isinstance(v, (int, float)):
                agg[k] = agg.get(k, 0) + v
    elapsed = time.perf_counter() - t0
    ms = elapsed * 1e3 / args.steps
    kind = s["path_kind"]
    ver = verify_rows(edges, tabs[0][0], tabs[0][1], V) if not args.no_verify else None
    roof = roofline_for(agg, kind, args, edges, V, workload_key(args, V, seed, 1), kind == 0
                        and args.fw_symmetric != 0 and not edges.directed)
    emit(args, V, gdesc, edges, kind, G, G * V * args.steps / elapsed, ms, agg, s, roof, None,
         {"parallelism": f"replicas{G} (one process, one full build per GPU per step)", "fallback": reason},
         {"verified_rows": ver}, scaling="weak", steps_ms=step_stats(ts))
    for r in routers:
        r.close()


def shared_table(V, rank, tag):
    """The n x n output as ONE host table shared by every rank's process (POSIX shm): each GPU
    writes its own sources' rows into it over its own PCIe link, so rank 0 ends with the whole
    RoutingInfo in its address space."""
    import mmap
    import numpy as np
    import torch.distributed as dist
    path = f"/dev/shm/srg_bench_{tag}"
    nbytes = V * V * 12
    if rank == 0:
        with open(path, "wb") as f:
            f.truncate(nbytes)
    dist.barrier()
    fd = os.open(path, os.O_RDWR)
    mm = mmap.mmap(fd, nbytes)
    os.close(fd)
    lat = np.frombuffer(mm, dtype=np.uint64, count=V * V).reshape(V, V)
    loss = np.frombuffer(mm, dtype=np.float32, count=V * V, offset=V * V * 8).reshape(V, V)
    return path, mm, lat, loss


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--vertices", type=int, default=10000)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--lat-scale", type=int, default=1,
                    help="multiply every edge latency by this factor (e.g. 1000 puts C3's used paths past "
                         "2^31 ns; the latency unit then keeps u32 keys in units of the latencies' gcd, and "
                         "SRG_LATENCY_UNIT=1 in the environment forces nanosecond keys: the u64 path benchmark)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-best baseline: time budget of its sample")
    ap.add_argument("--cpu-sources", type=int, default=256,
                    help="reference-equivalent CPU baseline: fixed seeded sample of sources (SURVEY §8d: 256)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-verify", action="store_true", help="skip the 4 oracle rows checked after the timed steps")
    ap.add_argument("--no-ri", action="store_true", help="skip the RoutingInfo build times (cold / steady)")
    ap.add_argument("--graph", choices=["atlas", "complete", "ba", "events"], default="atlas",
                    help="atlas = C3 (headline; C2 with --vertices 4096), complete = C1, ba = C4, "
                         "events = C5 stretch (10^7 packet events)")
    ap.add_argument("--config", choices=["c1", "c2", "c3", "c4", "c5"], default=None,
                    help="BASELINE.json config preset (sets --graph / --vertices)")
    ap.add_argument("--entry", choices=["host", "device"], default=None,
                    help="host = srg_compute_shortest_paths (host edge list in, host table out: H2D + D2H "
                         "included); device = srg_compute_shortest_paths_device (inputs/outputs in HBM)")
    ap.add_argument("--replicas", action="store_true", help="N>1: independent full builds per rank (weak)")
    ap.add_argument("--gather", action="store_true",
                    help="N>1: every rank ends with the whole table (RCCL row exchange; host entry: all rows D2H)")
    ap.add_argument("--sparse-delta-div", type=int, default=None,
                    help="sparse: bucket width = max edge latency / this (0 = plain Bellman-Ford)")
    ap.add_argument("--fw-symmetric", type=int, default=None, help="dense u32: 0 = general FW on undirected graphs too")
    ap.add_argument("--fw-xcd-order", type=int, default=None, help="symmetric FW bulk: 1 = Z-order runs per XCD")
    ap.add_argument("--d2h-mode", type=int, default=None, help="host entry D2H engine: 1 = SDMA (default), 0 = hipMemcpyAsync")
    ap.add_argument("--h2d-codec", type=int, default=None, help="host entry: 1 = narrowed edge list over PCIe (default), 0 = plain")
    ap.add_argument("--late-loss", type=int, default=None,
                    help="host entry: 1 = edge losses shipped beside the W build and FW (default), 0 = with the edges")
    ap.add_argument("--edge-shard", type=int, default=None,
                    help="host entry, N > 1: 1 = each rank ships 1/N of the edges and the ranks exchange them, "
                         "0 = every rank ships all, -1 = auto (default: on from 4 ranks)")
    ap.add_argument("--scan-groups", type=int, default=None, help="host entry: scan launches interleaved with the loss (0 = auto)")
    ap.add_argument("--loss-chunks", type=int, default=None, help="dense: k_loss_rows launches (0 = auto)")
    ap.add_argument("--fw-line-split", type=int, default=None,
                    help="symmetric FW: sub-tiles per dimension of the chain's line launches (1/2/4; 0 = auto)")
    ap.add_argument("--fw-step", type=int, default=None,
                    help="symmetric FW line exchange between ranks: 2 = device-side stores (in-process ranks), "
                         "0 = the collective, -1 = auto")
    ap.add_argument("--fw-overlap", type=int, default=None,
                    help="host entry, one rank: 1 = FW starts while the edge list arrives (default), 0 = after it")
    ap.add_argument("--no-locality", action="store_true", help="sparse: batch sources in node order")
    ap.add_argument("--fw-tile", type=int, default=0, help="dense FW tile (0 = auto)")
    ap.add_argument("--simulate-rank", type=str, default=None,
                    help="TIMING AID 'G:r': run rank r's share of a G-rank build alone, collectives elided "
                         "(outputs invalid; prints a diagnostic line, never the bench result)")
    args = ap.parse_args()
    if args.config:
        args.graph, args.vertices = {"c1": ("complete", 1000), "c2": ("atlas", 4096), "c3": ("atlas", 10000),
                                     "c4": ("ba", 50000), "c5": ("events", 10000)}[args.config]
    if args.graph == "ba" and args.vertices == 10000 and "--vertices" not in sys.argv:
        args.vertices = 50000
    if args.graph == "complete" and args.vertices == 10000 and "--vertices" not in sys.argv:
        args.vertices = 1000
    if args.entry is None:
        # the headline: host edge list in, host table out.  C4's 30 GB table is
        # benchmarked device-resident by default (a host copy of it is 0.5 s of PCIe alone).
        args.entry = "device" if args.graph == "ba" else "host"

    import numpy as np
    import torch
    import torch.distributed as dist

    if args.graph == "events":
        return bench_events(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and args.gpus > 1:
        return bench_multi(args)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from shadow_amd import Router
    from shadow_amd import _native as N
    from shadow_amd.device import DeviceGraph, compute_shortest_paths_device, set_profiling

    V = args.vertices
    t0 = time.time()
    edges, gdesc, seed = make_edges(args)
    log(f"[rank {rank}] generated {gdesc}: {edges.num_edges} edges in {time.time()-t0:.1f}s")
    cold_ms = None
    strong = world > 1 and not args.replicas
    fallback = None
    if strong:
        router, fallback = init_strong_router(local, dev)
        if router is None:
            log(f"[rank {rank}] multi-rank build unavailable ({fallback}): running independent replicas")
            strong = False
        else:
            apply_options(router, args)
            if not args.gather:
                # each rank routes the sources at positions [n r/N, n (r+1)/N) and writes those rows
                # into the ONE host table all ranks share (shared_table); --gather instead runs the
                # RCCL row exchange so that every rank's own array holds the whole table
                router.set_option(N.SRG_OPT_GATHER_OUTPUT, 0)
    if not strong:
        if args.entry == "host" and not args.simulate_rank:
            router, cold_ms = cold_call(lambda: Router(local), args, edges, V)
            log(f"[rank {rank}] cold call (srg_create + first call, unfaulted outputs): {cold_ms:.1f} ms")
        else:
            router = Router(local)
            apply_options(router, args)
    if args.simulate_rank:
        sg, sr = (int(x) for x in args.simulate_rank.split(":"))
        router.set_option(N.SRG_OPT_SIMULATE_RANK, sg * 1000 + sr)
        if not args.gather:  # as the N > 1 default: this rank's rows only
            router.set_option(N.SRG_OPT_GATHER_OUTPUT, 0)
    dg = DeviceGraph(edges, dev)
    nodes = torch.arange(V, dtype=torch.int32, device=dev)
    shm = None
    if args.entry == "host":
        h_nodes = np.arange(V, dtype=np.uint32)
        if strong and not args.gather:
            shm = shared_table(V, rank, os.environ.get("MASTER_PORT", "0"))
            h_lat, h_loss = shm[2], shm[3]
        else:
            h_lat = np.empty((V, V), dtype=np.uint64)
            h_loss = np.empty((V, V), dtype=np.float32)
        h_lat.fill(0)  # fault the pages in once: the caller's Vecs are already allocated
        h_loss.fill(0)

        def step():
            return router.compute_shortest_paths(edges, h_nodes, h_lat, h_loss).stats
    else:
        out_lat = torch.empty((V, V), dtype=torch.int64, device=dev)
        out_loss = torch.empty((V, V), dtype=torch.float32, device=dev)

        def step():
            return compute_shortest_paths_device(router, dg, nodes, out_lat, out_loss)

    s = run_steps(step, args, f"rank {rank}")
    set_profiling(router, not args.no_profile)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    agg = {}
    ts = []
    t_start = time.perf_counter()
    for i in range(args.steps):
        t1 = time.perf_counter()
        s = step()
        if args.entry != "host":
            torch.cuda.synchronize(dev)
        ts.append(time.perf_counter() - t1)
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
        for k in ("prof_launches", "prof_kernel_ms", "prof_relaxations"):  # the dominant kernel over all ranks
            t = torch.tensor([float(agg.get(k, 0))], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            agg[k] = float(t.item())
    ms_per_step = elapsed * 1e3 / args.steps
    value = (1 if strong else world) * V * args.steps / elapsed

    kind = s["path_kind"]
    # the device-resident time of the same build (inputs and outputs in HBM): the kernel pipeline
    # alone, reported beside the host-entry headline
    dev_ms = None
    if args.entry == "host" and world == 1 and not args.simulate_rank:
        ol = torch.empty((V, V), dtype=torch.int64, device=dev)
        os_ = torch.empty((V, V), dtype=torch.float32, device=dev)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(2):
            compute_shortest_paths_device(router, dg, nodes, ol, os_)
        torch.cuda.synchronize(dev)
        dev_ms = (time.perf_counter() - t1) * 1e3 / 2
        del ol, os_
    wkey = workload_key(args, V, seed, world)
    sym = kind in (0, 1) and args.fw_symmetric != 0 and not edges.directed
    roofline = roofline_for(agg, kind, args, edges, V, wkey, sym)

    if args.simulate_rank:
        n = args.steps
        brk = ("ms_h2d", "ms_build", "ms_fw", "ms_scan", "ms_loss", "ms_extract", "ms_exchange", "ms_d2h", "ms_total")
        print(json.dumps({"diagnostic": "simulated rank (no data exchanged, outputs invalid; every collective costs "
                                        "the modelled xGMI time, comm.hip ModelComm)",
                          "simulate_rank": args.simulate_rank, "ms_per_step": round(ms_per_step, 3),
                          "model": {"coll_us": float(os.environ.get("SRG_SIM_COLL_US", 15)),
                                    "link_GBps": float(os.environ.get("SRG_SIM_LINK_GBPS", 64))},
                          "breakdown_ms": {k: round(agg.get(k, 0) / n, 3) for k in brk},
                          "roofline": roofline}), flush=True)
        return
    # RoutingInfo builds (Shadow's call site) beside the host-entry headline, one rank
    ri_times = None
    if args.entry == "host" and world == 1 and not args.simulate_rank and not args.no_ri:
        ri_times = routing_info_times(edges, V, args)
        log(f"[rank {rank}] routing info: {ri_times}")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baselines(edges, args.cpu_seconds, gdesc.split(":")[0], args.cpu_sources)
    ver = None
    if world > 1:
        dist.barrier()  # every rank's rows are in the shared table
    if rank == 0 and args.entry == "host" and not args.no_verify:
        ver = verify_rows(edges, h_lat, h_loss, V)
    if rank == 0:
        extra_cfg = {"parallelism": (f"rowblock{world}+rccl" if strong else f"replicas{world}") if world > 1 else "single"}
        if strong:
            extra_cfg["output"] = ("full table in one host array: POSIX shm shared by the N processes, each GPU "
                                   "writing its sources' rows over its own PCIe link" if not args.gather
                                   else "gathered (every rank's own array holds the whole table)")
            if args.entry == "host":
                extra_cfg["edge_list"] = ("sharded (1/N over each PCIe link, exchanged between GPUs)"
                                          if (args.edge_shard == 1 or (args.edge_shard in (None, -1) and world >= 4))
                                          else "whole list over each PCIe link")
        if fallback:
            extra_cfg["fallback"] = fallback
        if cold_ms is not None:
            extra_cfg["cold_call_ms"] = round(cold_ms, 1)
            if COLD_BREAKDOWN:
                extra_cfg["cold_call_breakdown_ms"] = dict(COLD_BREAKDOWN)
        emit(args, V, gdesc, edges, kind, world, value, ms_per_step, agg, s, roofline, cpu, extra_cfg,
             {"device_entry_ms": round(dev_ms, 3) if dev_ms is not None else None, "verified_rows": ver,
              "routing_info": ri_times}, steps_ms=step_stats(ts))
    if world > 1:
        dist.barrier()
        if shm is not None and rank == 0:
            try:
                os.unlink(shm[0])
            except OSError:
                pass
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
