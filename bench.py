#!/usr/bin/env python3
"""Benchmark: sequenced ops applied per second, conflict-farm replay (BASELINE.json metric).

One step = one replay of a whole resident batch (inputs already in HBM) through the C ABI
(fmt_mt_run / fmt_map_run). Default workload = T1: merge-tree conflict farm, 100k documents ×
8 writer clients × 2000 ops per GPU (weak scaling: every rank replays its own 100k-doc shard).
`--workload map` runs M2: SharedMap LWW, 1M documents × 8 clients × 1000 ops per GPU.

Synthetic data: every document is distinct by default (generated with the reference's XSadd PRNG and
conflict-farm shape on the host's cores, ≈20 s for T1 on 16 threads). `--unique-docs U` generates U
distinct documents and lays them out `docs / U` times as independent copies (own ops and text in
HBM, nothing shared) for quick experiments. See DESIGN.md.

Launch: `python bench.py` (N=1) or `python -m torch.distributed.run --nproc-per-node N ... bench.py
--gpus N`. Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "sequenced ops applied/sec (whole node) + achieved HBM GB/s, conflict-farm replay"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def host_cpus():
    """The host cores this process may actually run on, and the CPU model (the CPU
    baseline's pool is sized to the host's cores, stated with the model). os.cpu_count() counts the
    whole machine; the affinity mask and the cgroup CPU quota bound what this process gets."""
    n = os.cpu_count() or 1
    try:
        n_aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n_aff = n
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    usable = n_aff if quota is None else max(1, min(n_aff, int(quota + 0.999)))
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"model": model, "cpu_count": n, "affinity": n_aff, "cgroup_quota_cpus": quota, "usable": usable}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=["mt", "t2", "t3", "map", "ob", "local"], default="mt",
                    help="mt: T1 (per-GPU shard of 100k docs); t2: one 1M-doc batch partitioned over the ranks "
                         "(the default for mt when --gpus > 1); t3: one SharedString of 10M segments; map: M2; "
                         "ob: the reference's 30 obliterate conflict farms replicated to --docs documents")
    ap.add_argument("--segments", type=int, default=10_000_000, help="t3: segments of the loaded document")
    ap.add_argument("--t3-ops", type=int, default=10_000_000, help="t3: sequenced ops replayed")
    ap.add_argument("--t3-summary", choices=["legacy", "header"], default="legacy",
                    help="t3: the loaded summary's shape: legacy = SnapshotLegacy.emit's header chunk (~10,000 "
                         "units) + body chunk; header = every segment in one header chunk")
    ap.add_argument("--t3-range", type=int, default=8, help="t3: max range length of removes/annotates")
    ap.add_argument("--t3-check", action="store_true",
                    help="t3: replay the whole document through the oracle too (one core, minutes at full size) "
                         "and compare its state digest with the GPU's")
    ap.add_argument("--cpu-ops", type=int, default=200_000, help="t3: ops of the CPU baseline sample")
    ap.add_argument("--docs", type=int, default=None,
                    help="documents per GPU (mt, map) or in the whole batch (t2)")
    ap.add_argument("--gather-docs", type=int, default=256,
                    help="t2: legacy summaries per shard gathered to rank 0 by the gatherv (0 = none)")
    ap.add_argument("--ops-per-doc", type=int, default=None)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--min-length", type=int, default=0,
                    help="mt: keep every document at least this many UTF-16 units long (0 = T1's cycling "
                         "minLength); above 2048 the documents replay in the large tier")
    ap.add_argument("--unique-docs", type=int, default=0, help="0 = all documents distinct")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--key-pool", type=int, default=20, help="map: key ids per document (> 2560 takes the HBM-table path)")
    ap.add_argument("--no-summaries", action="store_true",
                    help="mt: skip the bulk legacy summaries of every document after the timed steps")
    ap.add_argument("--catchup-sample", type=int, default=200,
                    help="T1 summaries: build the catchupOps blob for this many documents (0: skip)")
    ap.add_argument("--sparse", action="store_true",
                    help="map: the sparse path (LDS hash reduce-by-key, one entry per live key; any key pool)")
    ap.add_argument("--cpu-sample-docs", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=25.0,
                    help="CPU baseline sample length (the sample stops early once every document was replayed)")
    ap.add_argument("--t2-check-docs", type=int, default=1024,
                    help="t2: documents of every shard replayed by the oracle and compared by state digest")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist", action="store_true",
                    help="initialise torch.distributed (nccl = RCCL) even at one rank, so the gathers go over RCCL")
    ap.add_argument("--no-js-baseline", action="store_true", help="skip the JS worker_threads baseline")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline pool (0 = every usable host core)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import numpy as np
    import torch

    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1 or args.dist:  # (--dist: the RCCL path at one rank too, e.g. on a one-GPU box)
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    from fluidframework_amd import native, shard, workloads

    if args.workload == "t3":
        return bench_t3(args, rank, world, local_rank, dist)
    ob = args.workload == "ob"
    loc = args.workload == "local"
    mt = args.workload in ("mt", "t2", "ob", "local")
    t2 = args.workload == "t2" or (args.workload == "mt" and world > 1)
    opd = 2040 if ob else args.ops_per_doc or (2000 if mt else 1000)
    if t2:
        # T2: ONE batch of total_docs documents (every document has opd ops), partitioned over the
        # ranks by shard.plan_shards; each rank generates exactly its shard's streams (doc_base).
        total_docs = args.docs or 1_000_000
        lo, hi = shard.plan_shards(np.arange(total_docs + 1, dtype=np.uint64) * np.uint64(opd), world)[rank]
        docs, doc_base = hi - lo, lo
    else:
        docs = args.docs or (100_000 if mt else 1_000_000)  # (local: pass --docs for a shorter run)
        total_docs, doc_base = docs * world, rank * docs  # weak scaling: every rank its own docs
    seed = args.seed if mt else args.seed + 1000 * rank

    t = time.time()
    uniq = docs
    if ob:
        # the reference's obliterate farms (2.3.0 fixtures, 30 documents of 2040 ops with the
        # sequenced messages the reference recorded), cycled to `docs` documents
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from golden_data import replay_fixtures

        fixtures = list(replay_fixtures("replay_obliterate_2.3.0.npz"))
        uniq = len(fixtures)
        batch = workloads.replicate_batches([f[1] for f in fixtures], docs)
    elif loc:
        # f4 local client: each writing client's own view of the reference's 0.40 conflict
        # farms (its ops of a round submitted locally, then the round's messages, its own acking them;
        # tests/local_farm.py), 28 (fixture, writer) streams cycled to `docs` documents
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from local_farm import fixture_local_docs

        fixtures = fixture_local_docs()
        uniq = len(fixtures)
        batch = workloads.replicate_batches([f[1] for f in fixtures], docs)
        opd = int(round(len(batch.ops) / docs))
    elif mt:
        uniq = min(args.unique_docs or docs, docs)
        if docs % uniq:
            raise SystemExit("--docs must be a multiple of --unique-docs")
        if t2 and uniq != docs:
            raise SystemExit("t2 generates every document of its shard (no --unique-docs)")
        batch = workloads.conflict_farm(uniq, n_clients=args.clients, ops_per_doc=opd, seed=seed,
                                        replicas=docs // uniq, doc_base=doc_base, min_length=args.min_length)
    else:
        batch = workloads.map_stream(docs, opd, key_pool=args.key_pool, seed=seed)
    n_ops = len(batch.ops)
    log(rank, f"[bench] generated {docs} docs / {n_ops} ops in {time.time() - t:.1f}s")

    eng = native.Engine(local_rank)
    t = time.time()
    if mt:
        eng.mt_load(batch)
    elif args.sparse:
        eng.map_load_sparse(batch)
    else:
        eng.map_load(batch)
    h2d_s = time.time() - t
    in_bytes = batch.ops.nbytes + (batch.text.nbytes if mt else 0)
    log(rank, f"[bench] host->HBM {in_bytes / 1e9:.2f} GB in {h2d_s:.2f}s ({eng.device_info()})")

    run = eng.mt_run if mt else (eng.map_run_sparse if args.sparse else eng.map_run)
    for _ in range(args.warmup):
        run()
        eng.sync()
    # algorithmic bytes of one launch (result sizes are known after the first run)
    if mt:
        hdrs = eng.mt_headers()
        bad = int((hdrs["status"] != 0).sum())
        if bad:
            raise SystemExit(f"{bad} documents failed: statuses {np.unique(hdrs['status'])}")
    elif args.sparse:
        eng.map_fetch_sparse()
    else:
        eng.map_fetch()
    st = eng.stats()
    bytes_per_launch = int(st.bytes_read + st.bytes_written)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        eng.sync()

    kernel_ms = []
    barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        run()
        kernel_ms.append(eng.stats().kernel_ms)  # waits for this launch's end event
        log(rank, f"[bench] step {k}: kernel {kernel_ms[-1]:.1f} ms")
    barrier()
    elapsed = time.perf_counter() - t0
    # the run's exchange step: a 64-byte stats record per rank, all-gathered, and for
    # T2 the shards' legacy summaries gathered to rank 0 (gatherv)
    rec = np.zeros(1, dtype=shard.STATS_DTYPE)
    rec["rank"], rec["doc_lo"], rec["doc_hi"] = rank, doc_base, doc_base + docs
    rec["ops"], rec["elapsed_s"], rec["bytes"] = n_ops, elapsed, bytes_per_launch
    rec["kernel_ms"] = sum(kernel_ms) / len(kernel_ms)
    digests = None
    t2_check = None
    if mt:
        hdrs = eng.mt_headers()
        rec["status_bad"] = int((hdrs["status"] != 0).sum())
        rec["checksum"] = shard.state_checksum(hdrs, doc_base)
        # every document's content digest (fmt_mt_state_digest: leaves, props by value, text, header)
        t = time.perf_counter()
        digests = eng.mt_digests()
        digest_ms = (time.perf_counter() - t) * 1e3
        if ob:
            _check_obliterate_farms(eng, hdrs, fixtures, docs)
        if loc:
            _check_local_farms(eng, hdrs, fixtures, docs)
        if t2 and args.t2_check_docs > 0:
            t2_check = _t2_oracle_check(batch, digests, docs, doc_base, args.t2_check_docs, world)
    elif args.sparse:
        rec["checksum"] = shard.map_sparse_checksum(*eng.map_fetch_sparse(), doc_base)
    else:
        rec["checksum"] = shard.map_checksum(eng.map_fetch(), doc_base)
    stats = shard.gather_stats(rec, dist, device="cuda") if dist is not None else rec
    content = None
    if digests is not None:  # whole-job content digest: Σ over ranks of Σ_d mix(global d, digest_d)
        part = shard.digest_checksum(digests, doc_base)
        content = shard.gather_u64(part, dist, device="cuda") if dist is not None else [part]
        if t2_check is not None:  # every rank checked a sample of its own shard
            n_chk = shard.gather_u64(t2_check["docs"], dist, device="cuda") if dist is not None else [t2_check["docs"]]
            n_bad = shard.gather_u64(t2_check["mismatches"], dist, device="cuda") if dist is not None else [t2_check["mismatches"]]
            t2_check = {**t2_check, "docs_all_ranks": sum(n_chk), "mismatches_all_ranks": sum(n_bad)}
    gathered = None
    if t2 and args.gather_docs > 0:
        from fluidframework_amd.summary import legacy_summary

        t = time.perf_counter()
        blobs = []
        for d in range(min(args.gather_docs, docs)):
            lv, ch, pr = eng.mt_doc(d, hdrs[d])
            head, body = legacy_summary(hdrs[d], lv, ch, pr, batch.keys, batch.doc_values(d))
            blobs.append(head.encode("utf-8", "surrogatepass") + b"\0" + (body or "").encode("utf-8", "surrogatepass"))
        build_s = time.perf_counter() - t
        t = time.perf_counter()
        allb = shard.gather_blobs(blobs, dist, device="cuda") if dist is not None else blobs
        gather_s = time.perf_counter() - t
        if rank == 0:
            gathered = {"docs": len(allb), "bytes": int(sum(len(b) for b in allb)), "gather_ms": gather_s * 1e3,
                        "build_ms_rank0": build_s * 1e3,
                        "what": f"legacy summaries (header, body) of the first {args.gather_docs} documents of every "
                                "shard, gathered to rank 0 (all-gather of byte counts + grouped send/recv)"}
    summaries = None
    if mt and not t2 and not ob and not loc and not args.no_summaries:
        # every document's legacy summary from the converged state (device merge + host JSON on the
        # usable cores), timed apart from the replay; a sample checked against the Python host
        from fluidframework_amd.summary import legacy_summary

        st_threads = host_cpus()["usable"]
        tm = eng.mt_summarize_legacy(batch.keys, batch.values, threads=st_threads)
        total_ms = tm["kernel_ms"] + tm["fetch_ms"] + tm["format_ms"]
        checked = 0
        for d in range(0, docs, max(1, docs // 16)):
            lv, ch, pr = eng.mt_doc(d, hdrs[d])
            if eng.mt_summary(d) != legacy_summary(hdrs[d], lv, ch, pr, batch.keys, batch.doc_values(d)):
                raise SystemExit(f"bulk summary of document {d} differs from the Python host's")
            checked += 1
        summaries = {"docs": docs, "summaries_per_s": docs / (total_ms / 1e3), **tm, "total_ms": total_ms,
                     "checked_vs_python": checked,
                     "what": "legacy SharedString summary (header + body chunk) of every document: extractSync "
                             "merge on the GPU (summaryRunsKernel), JSON on host threads; the catchupOps blob is "
                             "the 'catchup' record"}
        if args.catchup_sample > 0:
            summaries["catchup"] = _bench_catchup(eng, batch, hdrs, docs, args.catchup_sample)
        log(rank, f"[bench] summaries: {summaries['summaries_per_s']:.3g}/s ({total_ms:.1f} ms: kernel "
                  f"{tm['kernel_ms']:.1f}, fetch {tm['fetch_ms']:.1f}, format {tm['format_ms']:.1f} on {tm['threads']} threads)")
    elapsed = float(stats["elapsed_s"].max())
    total_ops = int(stats["ops"].sum()) * args.steps
    value = total_ops / elapsed
    avg_kernel_ms = sum(kernel_ms) / len(kernel_ms)
    achieved = bytes_per_launch / (avg_kernel_ms / 1e3) / 1e9

    cpu = cpu_js = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not t2:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle  # CPU baseline only ("port" of the reference path)

        hc = host_cpus()
        threads = args.cpu_threads or hc["usable"]
        # bounded sample: consecutive chunks of the same batch until >= --cpu-seconds of CPU work or
        # every document replayed once. The oracle's result of every sampled document is compared
        # with the GPU's (merge-tree: state digests; map: the result slots / entries), untimed.
        chunk = args.cpu_sample_docs or (min(docs, 4 * threads * 80) if mt else min(docs, 50_000 if args.sparse else 200_000))
        secs, sample_ops, sample_docs, lo = 0.0, 0, 0, 0
        checked = mismatched = 0
        first_bad = None
        gpu_map = None
        if not mt:
            gpu_map = eng.map_fetch_sparse() if args.sparse else eng.map_fetch()
            if args.sparse:
                gpu_first = np.concatenate([[0], np.cumsum(gpu_map[0].astype(np.int64))])
        while secs < args.cpu_seconds and sample_docs < docs:
            hi = min(lo + chunk, docs)
            if mt:
                rc_, dig_, _, s_ = oracle.mt_replay_digest(batch, lo, hi, threads=threads)
                bad = np.nonzero(dig_ != digests[lo:hi])[0]
            else:
                o0, o1 = int(batch.doc_op_offsets[lo]), int(batch.doc_op_offsets[hi])
                sub = batch.__class__(batch.ops[o0:o1], batch.doc_op_offsets[lo : hi + 1] - o0,
                                      batch.key_bound, batch.keys, batch.values)
                if args.sparse:  # hash map per document (the dense table would be key_bound x 8 B per doc)
                    cnt_, ent_, s_ = oracle.map_replay_sparse(sub, threads=threads)
                    g_cnt = gpu_map[0][lo:hi]
                    g_ent = gpu_map[1][int(gpu_first[lo]):int(gpu_first[hi])]
                    bad = np.zeros(0, dtype=np.int64) if np.array_equal(cnt_, g_cnt) and np.array_equal(ent_, g_ent) else \
                        np.nonzero(cnt_ != g_cnt)[0] if not np.array_equal(cnt_, g_cnt) else np.array([0])
                else:
                    slots_, s_ = oracle.map_replay(sub, threads=threads)
                    bad = np.nonzero((slots_ != gpu_map[lo:hi]).any(axis=1))[0]
            if len(bad) and first_bad is None:
                first_bad = lo + int(bad[0])
            mismatched += len(bad)
            checked += hi - lo
            secs += s_
            sample_ops += int(batch.doc_op_offsets[hi] - batch.doc_op_offsets[lo])
            sample_docs += hi - lo
            lo = hi % docs
        if mismatched:
            raise SystemExit(f"{mismatched} of {checked} documents differ from the oracle (first: document {first_bad})")
        cpu = {
            "value": sample_ops / secs,
            "unit": "ops/s",
            "cores": threads,
            "kind": "port",
            "seconds": secs,
            "sample": f"{sample_docs} documents ({sample_ops} ops) of the same workload in chunks of {chunk}, "
                      f"C++ oracle -O3{' (sparse: std::unordered_map key index per document)' if args.sparse else ''}, "
                      f"one document per task on {threads} std::threads",
            "cpu_model": hc["model"],
            "host_cpus": {k: hc[k] for k in ("cpu_count", "affinity", "cgroup_quota_cpus")},
            "checked_vs_oracle_docs": checked,
            "checked_how": ("per-document state digest (fmt_mt_state_digest vs the oracle's digest of its own replay: "
                            "every leaf field, props by value, text, header)" if mt else
                            "result entries equal" if args.sparse else "result slots equal"),
        }
        log(rank, f"[bench] cpu baseline {cpu['value']:.3g} ops/s on {threads} threads ({secs:.1f}s); "
                  f"{checked} documents equal to the oracle's")
        if not args.no_js_baseline and not ob and not loc and not args.sparse:
            cpu_js = (_js_mt_baseline if mt else _js_map_baseline)(oracle, batch, docs, threads, args.cpu_seconds / 2)
            if cpu_js is not None:
                log(rank, f"[bench] JS baseline {cpu_js['value']:.3g} ops/s on {threads} worker_threads")

    # HBM bytes per launch from the committed rocprofv3 PMC passes of this same workload
    # (tools/pmc_traffic.py; gfx950 FETCH_SIZE correction applied there), or null.
    traffic = None
    tkey = (f"{args.workload}:{docs}x{opd}" + ("" if mt or args.key_pool == 20 else f"k{args.key_pool}")
            + ("s" if args.sparse else "")
            + (f"m{args.min_length}" if mt and args.min_length else ""))
    tpath = os.path.join(REPO, "profiles", "traffic.json")
    if os.path.exists(tpath):
        traffic = json.load(open(tpath)).get(tkey)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "ops/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if t2 else "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": (f"reference fixtures: the 30 obliterate conflict farms (merge-tree 2.3.0 results), cycled to "
                     f"{docs} docs per GPU" if ob else
                     f"reference fixtures: each writing client's local view of the 0.40 conflict farms ({uniq} streams: "
                     f"local submissions, acks), cycled to {docs} docs per GPU" if loc else
                     f"synthetic ({'conflict-farm' if mt else 'map fuzz'} shape, reference XSadd PRNG; "
                     + (f"one {total_docs}-doc batch partitioned by shard.plan_shards)" if t2
                        else f"{docs} distinct docs per GPU)" if not mt or uniq == docs
                        else f"{uniq} distinct docs per GPU replicated to {docs})")),
            "config": {
                "workload": ("merge-tree conflict farms with obliterate (reference fixtures) replay" if ob
                             else "f4 local-client replay (writer views of the reference conflict farms)" if loc
                             else f"T2 merge-tree conflict-farm replay, {total_docs} docs doc-sharded over {world} GPU(s)" if t2
                             else (f"merge-tree conflict-farm replay, documents kept >= {args.min_length} UTF-16 units"
                                   if args.min_length else "T1 merge-tree conflict-farm replay") if mt
                             else "M2 SharedMap LWW replay" + (", sparse output" if args.sparse else "")),
                "docs_per_gpu": docs,
                "docs_total": total_docs,
                "clients": args.clients,
                "ops_per_doc": opd,
                **({} if mt or args.key_pool == 20 else {"key_pool": args.key_pool}),
                "ops_per_step": n_ops * world,
                "parallelism": f"doc-shard x{world}",
            },
            "hbm_gbps": bytes_per_launch * world / (elapsed / args.steps) / 1e9,
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": traffic["bytes"] if traffic else None,
                "traffic_fetch_write": [traffic["fetch_bytes"], traffic["write_bytes"]] if traffic else None,
                "traffic_source": traffic["source"][0].rsplit("/", 2)[0] if traffic else None,
                "kernel": "mergeTreeKernel" if mt else ("mapSparseKernel" if args.sparse else "mapLwwKernel"
                                                         if args.key_pool <= 2560 else "mapLwwHbmKernel+mapLwwFinishKernel"),
                "limiter": ("per-document dependent op chain: VALU issue + LDS/readlane latency of one wave per "
                            "document (HBM fraction is reported for the contract; see DESIGN.md)") if mt
                           else ("per-document LDS hash reduce-by-key (ds_cmpswap claims, dependent LDS "
                                 "round trips) at the occupancy the 16 KiB table allows; HBM streaming of 16-byte op "
                                 "records is the bound it is measured against") if args.sparse
                           else "HBM streaming of 16-byte op records",
                "bytes_per_launch": bytes_per_launch,
                "avg_kernel_ms": avg_kernel_ms,
                "lds_bank_conflict_rate": traffic.get("lds_bank_conflict_rate") if traffic else None,
                # what does bound the merge-tree kernel: instruction issue of the per-document op
                # chains (SQ/GRBM PMC passes of this workload, tools/pmc_issue.py)
                "issue": _issue_record(traffic) if mt else None,
            },
            "cpu_baseline": cpu,
            # secondary: the plain-JS observer restatement on worker_threads
            **({"cpu_baseline_js": cpu_js} if cpu_js is not None else {}),
            "state_checksum": f"{shard.combine_checksums(stats):016x}",
            "content_digest": f"{sum(content) & 0xFFFFFFFFFFFFFFFF:016x}" if content is not None else None,
            "checked_vs_oracle_docs": (cpu or {}).get("checked_vs_oracle_docs", 0) + (
                t2_check["docs_all_ranks"] if t2_check else 0),
            **({"t2_oracle_check": t2_check} if t2_check else {}),
            **({"digest_ms": digest_ms} if digests is not None else {}),
            "summary_gather": gathered,
            "summaries": summaries,
            "failed_docs": int(stats["status_bad"].sum()),
            "h2d_gbps": in_bytes / h2d_s / 1e9,
        }
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def _t2_oracle_check(batch, digests, docs, doc_base, n_check, world):
    """T2: this rank's shard checked against the oracle — n_check of its documents spread over the
    shard, replayed by the oracle and compared by state digest. Raises on a mismatch."""
    import numpy as np

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # parity checker only

    threads = max(1, host_cpus()["usable"] // max(1, int(os.environ.get("LOCAL_WORLD_SIZE", world))))
    n = min(n_check, docs)
    step = max(1, docs // n)
    t = time.perf_counter()
    checked = bad = 0
    first = None
    for lo in range(0, docs, step * 64):  # runs of 64 consecutive documents, spread over the shard
        hi = min(lo + 64, docs)
        rc, dig, _, _ = oracle.mt_replay_digest(batch, lo, hi, threads=threads)
        diff = np.nonzero(dig != digests[lo:hi])[0]
        if len(diff) and first is None:
            first = doc_base + lo + int(diff[0])
        bad += len(diff)
        checked += hi - lo
        if checked >= n:
            break
    if bad:
        raise SystemExit(f"t2: {bad} of {checked} documents of shard [{doc_base}, {doc_base + docs}) differ from the "
                         f"oracle (first: document {first})")
    return {"docs": checked, "mismatches": bad, "seconds": time.perf_counter() - t, "threads": threads,
            "what": "per rank: runs of 64 documents spread over its shard replayed by the C++ oracle, compared by "
                    "per-document state digest (fmt_mt_state_digest)"}


def _js_map_baseline(oracle, batch, docs, workers, seconds):
    """The JS restatement (oracle/js/map_observer.js) on `workers` worker_threads over the first
    documents of the batch, passes repeated to about `seconds` of work; checked against the C++
    oracle's entries on that sample. None when node is absent."""
    import shutil
    import subprocess

    import numpy as np

    if shutil.which("node") is None:
        return None
    n = min(docs, 20_000)
    o1 = int(batch.doc_op_offsets[n])
    sub = batch.__class__(batch.ops[:o1], batch.doc_op_offsets[: n + 1], batch.key_bound, batch.keys, batch.values)
    hashes, st = oracle.js_map_replay(sub, workers)
    slots, _ = oracle.map_replay(sub, threads=workers)
    if not np.array_equal(hashes, oracle.map_entry_hashes(slots)):
        raise SystemExit("JS baseline: final maps differ from the C++ oracle's")
    reps = max(1, int(seconds / max(st["seconds"], 1e-3)))
    _, st = oracle.js_map_replay(sub, workers, reps=reps)
    node_v = subprocess.run(["node", "--version"], capture_output=True, text=True).stdout.strip()
    return {"value": st["ops_per_s"], "unit": "ops/s", "cores": workers, "kind": "JS restatement, not the reference",
            "seconds": st["seconds"],
            "sample": f"{n} documents ({o1} ops) of the same workload, {st['reps']} passes, plain-JS Map per document "
                      f"(oracle/js/map_observer.js) on {workers} worker_threads, Node {node_v}; final maps checked "
                      "equal to the C++ oracle's"}


def _js_mt_baseline(oracle, batch, docs, workers, seconds):
    """The JS restatement (oracle/js/mt_observer.js: flat segment list, no B+tree) on `workers`
    worker_threads over the first documents of the batch, passes repeated to about `seconds`; the
    first 256 documents' final texts checked against the C++ oracle's. None when node is absent."""
    import shutil
    import subprocess

    if shutil.which("node") is None:
        return None
    n = min(docs, 4 * workers * 64)
    o1 = int(batch.doc_op_offsets[n])
    sub = _mt_prefix(batch, n)
    hashes, st = oracle.js_mt_replay(sub, workers)
    k = min(n, 256)
    rc, oh, ol, oc, _, _ = oracle.mt_replay_batch(sub, 0, k, threads=workers, cap_leaves=8192, cap_chars=1 << 17,
                                                  cap_props=1024)
    for d in range(k):
        if oh[d]["status"] == 0 and oracle.text_hash(oracle.visible_units(oh[d], ol[d], oc[d])) != hashes[d]:
            raise SystemExit(f"JS baseline: document {d} ends with a different text than the C++ oracle's")
    reps = max(1, int(seconds / max(st["seconds"], 1e-3)))
    if reps > 1:
        _, st = oracle.js_mt_replay(sub, workers, reps=reps)
    node_v = subprocess.run(["node", "--version"], capture_output=True, text=True).stdout.strip()
    return {"value": st["ops_per_s"], "unit": "ops/s", "cores": workers, "kind": "JS restatement, not the reference",
            "seconds": st["seconds"],
            "sample": f"{n} documents ({o1} ops) of the same workload, {st['reps']} pass(es), plain-JS flat segment "
                      f"list per document (oracle/js/mt_observer.js; no B+tree) on {workers} worker_threads, Node "
                      f"{node_v}; final texts of the first {k} checked equal to the C++ oracle's"}


def _mt_prefix(batch, n):
    """The first n documents of a merge-tree batch (shared text and props tables)."""
    from dataclasses import replace

    o1 = int(batch.doc_op_offsets[n])
    return replace(batch, ops=batch.ops[:o1], doc_op_offsets=batch.doc_op_offsets[: n + 1],
                   doc_init=batch.doc_init[:n] if batch.doc_init is not None else None, clients=[], messages=[])


def _check_obliterate_farms(eng, hdrs, fixtures, docs):
    """Every copy of a fixture ends in the same state, and the first copies hold the text the
    reference recorded as the farm's final result."""
    import numpy as np

    from fluidframework_amd.shard import _HDR_FIELDS

    n = len(fixtures)
    for f in _HDR_FIELDS:
        col = hdrs[f]
        if not (col == col[np.arange(docs) % n]).all():
            raise SystemExit(f"obliterate farm copies disagree on {f}")
    for d in range(min(n, docs)):
        lv, ch, _ = eng.mt_doc(d, hdrs[d])
        text = "".join(ch[int(L["char_off"]):int(L["char_off"]) + int(L["len"])].tobytes().decode("utf-16-le", "surrogatepass")
                       for L in lv[:int(hdrs[d]["n_leaves"])]
                       if int(L["rm_seq"]) == 0x7FFFFFFF and not int(L["pad"]) & 0x8000)
        if text != fixtures[d][4][-1]:
            raise SystemExit(f"obliterate farm {fixtures[d][0]}: final text differs from the reference's")


def _check_local_farms(eng, hdrs, fixtures, docs):
    """The first copy of every writer-view stream reaches the fixture's final resultText (the
    reference's own recorded result); the oracle digest check covers every sampled copy."""
    for d in range(min(len(fixtures), docs)):
        lv, ch, _ = eng.mt_doc(d, hdrs[d])
        text = "".join(ch[int(L["char_off"]):int(L["char_off"]) + int(L["len"])].tobytes().decode("utf-16-le", "surrogatepass")
                       for L in lv[:int(hdrs[d]["n_leaves"])]
                       if int(L["rm_seq"]) == 0x7FFFFFFF and not int(L["pad"]) & 0x8000)
        if text != fixtures[d][2]:
            raise SystemExit(f"local document {d} ({fixtures[d][0]}) does not reach the fixture's resultText")


def _bench_catchup(eng, batch, hdrs, docs, sample):
    """The legacy summary's catchupOps blob (sequence.ts:949-964, snapshotlegacy.ts:178-190) for the
    T1 documents: one more replay of the same batch with the catch-up window's ops flagged
    (FMT_MT_F_CATCHUP: the kernel records their delta ranges; the state must equal the timed
    replay's), every document's ranges in one copy (fmt_mt_fetch_catchup_all), and the messages
    rebuilt on the Python host for a sample of documents (their generated streams carry op records,
    so each message is the single-op ISequencedDocumentMessage streams.op_messages renders)."""
    from dataclasses import replace

    import numpy as np

    from fluidframework_amd import shard, streams, summary, workloads

    cb = replace(batch, ops=batch.ops.copy())
    streams.flag_catchup(cb.ops, cb.doc_op_offsets)
    eng.mt_load(cb)
    t = time.perf_counter()
    eng.mt_run()
    eng.sync()
    replay_ms = (time.perf_counter() - t) * 1e3
    h2 = eng.mt_headers()
    if shard.state_checksum(h2, 0) != shard.state_checksum(hdrs, 0):
        raise SystemExit("catch-up recording changed the replayed state")
    t = time.perf_counter()
    offs, ranges = eng.mt_catchup_all()
    fetch_ms = (time.perf_counter() - t) * 1e3
    step = max(1, docs // sample)
    t = time.perf_counter()
    n_docs = n_msgs = n_bytes = 0
    for d in range(0, docs, step):
        ms = int(h2[d]["min_seq"])
        msgs = streams.op_messages(batch, d, ms, workloads.CLIENT_NAMES)
        blob = summary.catchup_blob(summary.catchup_messages(msgs, ranges[int(offs[d]):int(offs[d + 1])], ms))
        n_docs += 1
        n_msgs += len(msgs)
        n_bytes += len(blob.encode("utf-8")) if blob else 0
    fmt_ms = (time.perf_counter() - t) * 1e3
    return {"ranges": int(offs[-1]), "ranges_per_doc": float(offs[-1]) / docs, "replay_ms": replay_ms, "fetch_ms": fetch_ms,
            "sample_docs": n_docs, "sample_messages": n_msgs, "sample_bytes": n_bytes,
            "python_ms_per_doc": fmt_ms / max(n_docs, 1),
            "what": "catchupOps of the same documents: the replay again with the catch-up window's ops flagged (the "
                    "kernel records their delta ranges; state equal to the timed replay), every document's ranges in "
                    "one fmt_mt_fetch_catchup_all copy, messages rebuilt on the Python host for a sample of documents"}


def _issue_record(traffic):
    """roofline.issue from the committed instruction-issue PMC passes (profiles/traffic.json)."""
    rec = traffic.get("issue") if traffic else None
    if not rec:
        return None
    split = rec.get("wave_cycle_split", {})
    counters = rec.get("counters", {})
    cycles, simds = rec.get("kernel_cycles"), 1024

    def busy(pipe, name):  # per-pipe fraction of SIMD issue slots (tools/pmc_issue.py), each <= 1
        if rec.get(f"{pipe}_busy") is not None:
            return rec[f"{pipe}_busy"]
        return 4.0 * counters[name] / (cycles * simds) if cycles and name in counters else None

    return {
        "insts_per_op": rec.get("insts_per_op"),
        "valu_busy": busy("valu", "SQ_ACTIVE_INST_VALU"),
        "salu_busy": busy("salu", "SQ_ACTIVE_INST_SCA"),
        "lds_busy": busy("lds", "SQ_ACTIVE_INST_LDS"),
        "wave_cycles_active": split.get("active_inst_any"),
        "wave_cycles_waitcnt": split.get("wait_any"),
        "wave_cycles_issue_stall": split.get("wait_inst_any"),
        "source": rec["source"][0].rsplit("/", 2)[0],
        "note": "<pipe>_busy = 4*SQ_ACTIVE_INST_<pipe> / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs), per pipe (they issue "
                "in parallel, so they do not sum to one); wave-cycle split from "
                "SQ_WAVE_CYCLES = ACTIVE_INST_ANY + WAIT_ANY (waitcnt) + WAIT_INST_ANY (issue stall)",
    }


def _wait(eng, rank, what, every=30.0, run=None):
    """run() (if given) then eng.sync() on a helper thread, printing progress while a long launch
    runs (a silent minute looks like a hang to the job runner; ctypes calls release the GIL)."""
    import threading

    def work():
        if run is not None:
            run()
        eng.sync()

    t0 = time.time()
    th = threading.Thread(target=work)
    th.start()
    while th.is_alive():
        th.join(every)
        if th.is_alive():
            log(rank, f"[bench] {what}: still running after {time.time() - t0:.0f}s")


def bench_t3(args, rank, world, local_rank, dist):
    """T3 (BASELINE config 5): one SharedString loaded from a 10M-segment summary, then 1e7 messages
    from 63 writers with refSeq lag U[0, 4096). Its ops are one dependency chain: a document is
    replayed by one wave (huge_engine.h); with N GPUs every rank replays its own replica (SURVEY §8e:
    replicas only). A step = load + replay + converged-state output of the whole document, all in
    the timed launch; ops/s counts the replayed messages only."""
    import numpy as np
    import torch

    from fluidframework_amd import native, shard, workloads

    t = time.time()
    batch = workloads.t3_stream(args.segments, args.t3_ops, n_clients=63, max_lag=4096, max_range=args.t3_range,
                                seed=args.seed)
    if args.t3_summary == "legacy":
        batch = workloads.as_legacy_load(batch)
    from fluidframework_amd.streams import MT_F_CATCHUP, flag_catchup

    # the summary's catchupOps blob: the engine records the delta ranges of the ops above the final
    # minSeq whose refSeq trails (sequence.ts:949-1018); only the last window's ops are flagged
    flag_catchup(batch.ops, batch.doc_op_offsets)
    n_ops = len(batch.ops)
    log(rank, f"[bench] t3: generated {args.segments} segments + {n_ops} ops in {time.time() - t:.1f}s")
    eng = native.Engine(local_rank)
    t = time.time()
    eng.mt_load(batch)
    h2d_s = time.time() - t
    in_bytes = batch.ops.nbytes + batch.text.nbytes + batch.snapshot_segs.nbytes
    log(rank, f"[bench] host->HBM {in_bytes / 1e9:.2f} GB in {h2d_s:.2f}s ({eng.device_info()})")
    for k in range(args.warmup):
        _wait(eng, rank, f"warmup {k}", run=eng.mt_run)
    hdrs = eng.mt_headers()
    if args.warmup and int(hdrs[0]["status"]) != 0:
        raise SystemExit(f"t3 replay failed: status {int(hdrs[0]['status'])} at seq {int(hdrs[0]['fail_seq'])}")
    st = eng.stats()
    bytes_per_launch = int(st.bytes_read + st.bytes_written)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        eng.sync()

    kernel_ms = []
    barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        _wait(eng, rank, f"step {k}", run=eng.mt_run)
        kernel_ms.append(eng.stats().kernel_ms)
        log(rank, f"[bench] t3 step {k}: kernel {kernel_ms[-1]:.1f} ms ({n_ops / kernel_ms[-1] * 1e3:.3g} ops/s)")
    barrier()
    elapsed = time.perf_counter() - t0
    rec = np.zeros(1, dtype=shard.STATS_DTYPE)
    rec["rank"], rec["doc_lo"], rec["doc_hi"], rec["ops"], rec["elapsed_s"] = rank, 0, 1, n_ops, elapsed
    rec["kernel_ms"] = sum(kernel_ms) / len(kernel_ms)
    hdrs = eng.mt_headers()
    if int(hdrs[0]["status"]) != 0:
        raise SystemExit(f"t3 replay failed: status {int(hdrs[0]['status'])} at seq {int(hdrs[0]['fail_seq'])}")
    st = eng.stats()
    bytes_per_launch = int(st.bytes_read + st.bytes_written)
    rec["status_bad"] = int((hdrs["status"] != 0).sum())
    rec["checksum"] = shard.state_checksum(hdrs, 0)
    stats = shard.gather_stats(rec, dist, device="cuda") if dist is not None else rec
    elapsed = float(stats["elapsed_s"].max())
    value = n_ops * world * args.steps / elapsed
    avg_kernel_ms = sum(kernel_ms) / len(kernel_ms)
    prof = eng.huge_profile(0)
    log(rank, f"[bench] t3 phase clocks per op: " + ", ".join(f"{k} {v / n_ops:.0f}" for k, v in prof.items()))
    # Summary emission of the replayed document (SharedString.summarizeCore, legacy format:
    # snapshotlegacy.ts:126-193 + the catchupOps blob, sequence.ts:949-964), timed on its own:
    # the device merge of the segment runs, host JSON, the catch-up ranges' fetch and their messages.
    import hashlib

    from fluidframework_amd import summary as fsum
    from fluidframework_amd.streams import op_messages

    names = batch.clients[0] if batch.clients else [f"client-{k}" for k in range(64)]
    min_seq = int(hdrs[0]["min_seq"])
    t = time.perf_counter()
    stiming = eng.mt_summarize_legacy(batch.keys, batch.values)
    head, body = eng.mt_summary(0)
    cu = eng.mt_catchup(0, hdrs[0])
    msgs = op_messages(batch, 0, min_seq, names)
    cblob = fsum.catchup_blob(fsum.catchup_messages(msgs, cu, min_seq))
    sum_s = time.perf_counter() - t
    blob_hash = hashlib.sha256("\x00".join([head, body or "", cblob or ""]).encode("utf-8")).hexdigest()[:16]
    t3_summary = {"seconds": sum_s, "kernel_ms": stiming["kernel_ms"], "fetch_ms": stiming["fetch_ms"],
                  "format_ms": stiming["format_ms"], "header_bytes": len(head), "body_bytes": len(body or ""),
                  "catchup_bytes": len(cblob or ""), "catchup_ops": int(((batch.ops["flags"] & MT_F_CATCHUP) != 0).sum()),
                  "catchup_ranges": int(len(cu)), "sha16": blob_hash,
                  "what": "legacy summary (header + body at minSeq, snapshotlegacy.ts:126-193) + catchupOps "
                          "(sequence.ts:949-1018) of the 10M-segment document, after the timed replay"}
    log(rank, f"[bench] t3 summary: {sum_s:.2f}s, header {len(head)} B, body {len(body or '')} B, "
              f"catchup {len(cblob or '')} B ({len(cu)} ranges), sha {blob_hash}")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle  # CPU baseline only ("port" of the reference path, with its length index)

        oracle.set_index(True)
        rc, oh, *_, load_s, ops_s, done = oracle.mt_replay_timed(batch, 0, min(args.cpu_ops, n_ops))
        hc = host_cpus()
        cpu = {"value": done / ops_s, "unit": "ops/s", "cores": 1, "kind": "port", "seconds": ops_s,
               "sample": f"the first {done} ops of the same document after loading its {args.segments} segments "
                         f"({load_s:.1f}s, untimed): C++ oracle -O3 with its per-block remote-length index "
                         f"(BlockIdx), one thread (a single document's ops are one dependency chain)",
               "cpu_model": hc["model"]}
        log(rank, f"[bench] t3 cpu baseline {cpu['value']:.3g} ops/s ({done} ops in {ops_s:.1f}s)")
    t3_check = None
    if rank == 0 and args.t3_check:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle  # parity at full size (test infrastructure; after the timed region)

        gpu_dig = eng.mt_digests()
        oracle.set_index(True)
        t = time.time()
        import threading

        res = {}

        def full():
            try:
                res["r"] = oracle.mt_replay_full(batch, 0, batch.keys, batch.values)
            except Exception as e:  # (reported below)
                res["e"] = e
        th = threading.Thread(target=full)
        th.start()
        while th.is_alive():  # (ctypes releases the GIL; progress lines keep the job runner from calling it hung)
            th.join(30.0)
            if th.is_alive():
                log(rank, f"[bench] t3 oracle check: still running after {time.time() - t:.0f}s")
        oracle.set_index(False)
        if "e" in res:
            raise SystemExit(f"t3: oracle replay failed: {res['e']}")
        odig, ohead, obody, ocu = res["r"]
        oblob = fsum.catchup_blob(fsum.catchup_messages(msgs, ocu, min_seq))
        t3_check = {"equal": bool(int(odig) == int(gpu_dig[0])), "oracle_rc": 0,
                    "gpu_digest": f"{int(gpu_dig[0]):016x}", "oracle_digest": f"{int(odig):016x}",
                    "summary_equal": bool(ohead == head and obody == body and oblob == cblob),
                    "catchup_ranges_equal": bool(len(ocu) == len(cu) and (len(cu) == 0 or bool((ocu == cu).all()))),
                    "oracle_s": time.time() - t,
                    "what": "state digest (every leaf field, props by value, text, header; DESIGN.md §2) of the whole "
                            "replayed document and its legacy summary + catchupOps blobs, GPU vs the oracle's own "
                            "full replay (one replay) and its SnapshotLegacy restatement"}
        t3_check["equal"] = t3_check["equal"] and t3_check["summary_equal"] and t3_check["catchup_ranges_equal"]
        log(rank, f"[bench] t3 oracle check: {t3_check}")
        if not t3_check["equal"]:
            raise SystemExit(f"t3: GPU state differs from the oracle's: {t3_check}")
    if rank == 0:
        h = hdrs[0]
        out = {
            "metric": METRIC, "value": value, "unit": "ops/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int32",
            "data": "synthetic (one SharedString loaded from a summary of U[1,8]-char segments, then conflict-farm "
                    "op kinds from 63 writers with refSeq lag U[0,4096) and local edit ranges, reference XSadd PRNG)",
            "config": {"workload": "T3 single huge SharedString replay (load + replay + output in the timed launch)",
                       "segments": args.segments, "ops": n_ops, "clients": 63, "max_lag": 4096, "max_range": args.t3_range,
                       "summary": {"shape": args.t3_summary, "header_segments": int(batch.snapshots[0]["n_header"]),
                                   "body_segments": int(batch.snapshots[0]["n_body"])},
                       "parallelism": f"replicas x{world} (one dependency chain per document)"},
            "roofline": {"bound": "hbm", "achieved": bytes_per_launch / (avg_kernel_ms / 1e3) / 1e9,
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": bytes_per_launch / (avg_kernel_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, "traffic": None,
                         "kernel": "hugeDocKernel",
                         "limiter": "one wave replays one dependent op chain: per op, a pass over the window table, "
                                    "a group scan, one slot list and one leaf block (HBM/L2 round trips), plus "
                                    "block/heap updates; bandwidth is idle by construction",
                         "bytes_per_launch": bytes_per_launch, "avg_kernel_ms": avg_kernel_ms},
            "cpu_baseline": cpu,
            "t3_oracle_check": t3_check,
            "t3_summary": t3_summary,
            "state_checksum": f"{shard.combine_checksums(stats):016x}",
            "phase_clocks_per_op": {k: v / n_ops for k, v in prof.items() if k not in ("text_compactions", "merge_units_in_use", "resumed_at")},
            "merge_area": {"compactions": prof.get("text_compactions"), "units_in_use": prof.get("merge_units_in_use")},
            "final_state": {"leaves": int(h["n_leaves"]), "chars": int(h["n_chars"]), "visible": int(h["visible_len"]),
                            "blocks": int(h["n_blocks"]), "depth": int(h["depth"]), "min_seq": int(h["min_seq"])},
            "h2d_gbps": in_bytes / h2d_s / 1e9,
        }
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
