"""Benchmark: requests inspected/s + GB/s scanned on MI355X (BASELINE.json metric).

One "step" = one pass of the inspection pipeline (gi_run_staged: collect ->
phase A -> phase 1 -> body -> phase 2 -> verdicts + tallies) over one batch
of synthetic requests already resident in HBM, plus (N > 1) the RCCL
all-gather of the per-GPU tally (7 counters + score histogram + per-rule
match counts).  Requests are sharded with no data-path collective: the N
ranks inspect one seeded request set (chunk k = the generator's batch for
seed SEED + k), cut into byte-balanced contiguous slices before timing
(shard.rebalance; weak scaling: the set grows with N).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c1|c3|c4|c5] [--n-req R]

N > 1 is launched by torch.distributed.run (RANK/LOCAL_RANK/WORLD_SIZE env).
Prints ONE JSON line on rank 0.

Self-checks: the verdicts of the timed batch are compared with the CPU oracle
on a sample (`parity_sample`) and with the C++ CPU baseline on its sample
(`cpu_baseline.agrees_with_gpu`); a mismatch is reported, never hidden.  `e2e` times one more pass including host staging (layout + H2D of
pageable buffers) and the verdict D2H.
"""

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "coraza-kubernetes-operator_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

import gpuinspect  # noqa: E402
import shard  # noqa: E402
import traffic  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
# ds_read_b32 lanes/s with every CU streaming (MI355X_MICROARCH.md: ~75 TB/s
# aggregate for ds_read_b32, 4 B per lane): one automaton transition of k_scan
# is one such LDS lane read, so k_scan's transitions/s over this is its LDS
# (secondary) roofline fraction
LDS_B32_LANES_PER_S = 75e12 / 4

# launch name (gi_stats) -> kernel name as rocprofv3 reports it
ROCPROF_NAMES = {
    "k_stream0": "k_stream<16u, 20u, 4u>", "k_stream1": "k_stream<32u, 36u, 3u>", "k_stream2": "k_stream<64u, 68u, 1u>",
    "k_stream3": "k_stream<128u, 132u, 0u>", "k_stream4": "k_stream<0u, 0u, 0u>", "k_scan": "k_scan<true, false>",
    "k_scan_big": "k_scan<true, true>", "k_scan_hbm": "k_scan<false, false>",
}

CONFIGS = {
    # name: (ruleset file, default n_req, post_frac, description)
    "c2": ("rulesets/crs_pl1.conf", 1_000_000, 0.0,
           "CRS-shaped v4 PL1 ruleset (rulesets/crs_pl1.conf) x 1M synthetic GET with query args"),
    "c1": ("tests/golden/samples_ruleset.conf", 10_000, 0.0,
           "config/samples RuleSet x 10k synthetic GET"),
    "c3": ("rulesets/crs_pl1.conf", 200_000, 0.5,
           "CRS-shaped v4 PL1 x mixed GET/POST (50% POST, 4-64 KB bodies: 60% urlencoded, 40% JSON), "
           "200k requests per batch (run as request chunks)"),
    "c4": ("rulesets/crs_pl4.conf", 200_000, 0.5,
           "CRS-shaped v4 PL4 (blocking paranoia 4: +35 PL2-4 rules, @detectSQLi/@detectXSS) x C3 mix "
           "(50% POST 4-64 KB urlencoded/JSON), 200k requests per GPU per batch; SURVEY C4 = 10M across 8 GPUs "
           "= this batch per GPU, repeated"),
    "c2x": ("rulesets/crs_pl1_rxstress.conf", 1_000_000, 0.0,
            "C2 traffic x the PL1 stand-in + 20 CRS-scale assembled regexes of 2-6 KB (tools/gen_rxstress.py; "
            "two past the DFA state cap, run as NFA position tables): the regex-stress line"),
    "c5": (None, 32, 1.0,
           "generated 10k @rx rules + 100k-phrase @pmFromFile (traffic.c5_ruleset) x ~1 MB multipart bodies "
           "(traffic.c5_batch)"),
}


def _oracle_worker(args):
    text, blob, idx, exports, files = args
    from oracle import compare, coraza
    cfg = coraza.parse_seclang(text, files)
    data, reqs, headers = blob
    b = gpuinspect.PackedBatch(data, reqs, headers)
    out = {}
    t0 = time.perf_counter()
    for i in idx:
        t = b.request(i)
        out[i] = coraza.inspect(cfg, compare.oracle_request(t), exports)
    return time.perf_counter() - t0, out


def oracle_sample(text, batch, exports, budget_s=15.0, procs=16, n_max=4000, files=None, calib=100, min_n=200):
    """The CPU oracle over a bounded sample of the batch: (verdicts by request
    index, wall seconds, processes).  Sized from a `calib`-request calibration
    to about budget_s of wall time, at least min(min_n, 2 x procs) requests."""
    blob = (batch.data, batch.reqs, batch.headers)
    calib = min(calib, batch.n_req)
    dt, _ = _oracle_worker((text, blob, range(calib), exports, files))
    per = dt / calib
    log("oracle calibration: %.2f s per request" % per)
    procs = max(1, min(procs, os.cpu_count() or 1))
    n_sample = int(min(n_max * procs, max(min(min_n, 2 * procs), budget_s * procs / max(per, 1e-6)), batch.n_req))
    log("oracle sample: %d requests in %d processes" % (n_sample, procs))
    chunks = [range(k, n_sample, procs) for k in range(procs)]
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(procs) as pool:
        outs = pool.map(_oracle_worker, [(text, blob, c, exports, files) for c in chunks])
    wall = time.perf_counter() - t0
    verdicts = {}
    for _, o in outs:
        verdicts.update(o)
    return verdicts, wall, procs


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cpu_share():
    """The host cores this process may use, and why that many: the CPU
    affinity mask (os.sched_getaffinity), the cgroup CPU quota (cpu.max), and
    OMP_NUM_THREADS (the GPU box sets it to the job's CPU share, 16, while
    os.cpu_count() reports the whole machine)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    omp_n = int(omp) if omp and omp.isdigit() else None
    cands = [("affinity", aff)]
    if quota:
        cands.append(("cgroup cpu.max", max(1, int(quota))))
    if omp_n:
        cands.append(("OMP_NUM_THREADS", omp_n))
    why, n = min(cands, key=lambda c: c[1])
    return {"threads": max(1, n), "limited_by": why, "affinity": aff, "cpu_count": os.cpu_count(),
            "cgroup_quota": quota, "omp_num_threads": omp_n}


def cpu_baseline(rs, batch, res, budget_s=10.0, threads=None):
    """SURVEY §8(d)'s CPU baseline when Coraza Go is absent: the engine's own
    C++ interpreter (gi_cpu_baseline_inspect: kernels.hip compiled for the
    host, every rule link evaluated, no phase A) on `threads` host cores, over
    a prefix of the benchmark batch sized from a calibration to ~budget_s.
    Its verdicts are also compared with the GPU's for the same requests (the
    same interpreter source: they must agree bit for bit)."""
    share = host_cpu_share()
    threads = threads or share["threads"]
    # calibration sample: one request per thread when requests are large (C5's
    # 1 MB bodies take seconds each on a core), else 64 per thread
    big = len(batch.data) > 65536 * max(batch.n_req, 1)
    n_cal = min(batch.n_req, threads if big else 64 * threads)
    log("cpu baseline calibration: %d requests, %d threads" % (n_cal, threads))
    cres, dt = gpuinspect.cpu_baseline_inspect(rs, batch.take(0, n_cal), threads=threads,
                                               matched_cap=res.matched.shape[1])
    n, secs = n_cal, dt
    if dt < budget_s / 2 and n_cal < batch.n_req:  # else the calibration is the sample
        n = int(min(batch.n_req, max(n_cal, budget_s * n_cal / max(dt, 1e-6))))
        log("cpu baseline: %d requests" % n)
        cres, secs = gpuinspect.cpu_baseline_inspect(rs, batch.take(0, n), threads=threads,
                                                     matched_cap=res.matched.shape[1])
    agree = int(((cres.verdicts[:n]["rule_id"] == res.verdicts[:n]["rule_id"]) &
                 (cres.verdicts[:n]["status"] == res.verdicts[:n]["status"]) &
                 (cres.verdicts[:n]["match_cnt"] == res.verdicts[:n]["match_cnt"]) &
                 (cres.verdicts[:n]["tx_export"] == res.verdicts[:n]["tx_export"]).all(axis=1) &
                 (cres.matched[:n] == res.matched[:n]).all(axis=1)).sum())
    return {"value": round(n / secs, 1), "unit": "requests/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": "first %d requests of the benchmark batch through gi_cpu_baseline_inspect: this engine's "
                      "own interpreter (kernels.hip) compiled for the host, %d threads, every rule link evaluated "
                      "(no phase A) -- a C++ restatement, not Coraza (no Go toolchain on the box)" % (n, threads),
            "seconds": round(secs, 3), "agrees_with_gpu": agree, "agree_of": n, "host_cpu_share": share}


def parity(res, verdicts):
    from oracle import compare
    bad = compare.compare(res, verdicts, max_report=10 ** 9)
    return {"n": len(verdicts), "mismatches": len({b[0] for b in bad}),
            "first": [str(b)[:300] for b in bad[:3]],
            "def": "timed batch's GPU verdicts vs oracle/coraza.py on the same requests: interruption, "
                   "ordered matched ids, exported TX values, unsupported flag (oracle/compare.py)"}


def e2e_pipelined(rs, eng, batch, device, matched_cap, iters, raw):
    """Steady-state host-inclusive throughput: two contexts on one GPU take
    turns; while context A runs batch k, the host fetches batch k-1 from B and
    stages batch k+1 into B (layout on the host cores, H2D from page-locked
    memory on B's stream).  The same request set is inspected every time."""
    eng2 = gpuinspect.Engine(rs, device=device, matched_cap=matched_cap)
    engines = [eng, eng2]
    pinned = eng.pin(batch.data, batch.reqs, batch.headers)
    for e in engines:
        e.stage(batch)  # allocations happen here, outside the timed loop
        e.pin(*[a for a in e.result_buffers(batch.n_req)])
    stage_s = fetch_s = 0.0
    t0 = time.perf_counter()
    engines[0].stage(batch)
    for k in range(iters):
        cur, other = engines[k % 2], engines[(k + 1) % 2]
        cur.run()  # asynchronous on cur's stream
        if k > 0:
            ta = time.perf_counter()
            other.fetch(reuse=True)  # batch k-1 (its kernels finished at the last sync)
            fetch_s += time.perf_counter() - ta
        if k + 1 < iters:
            ta = time.perf_counter()
            other.stage(batch)  # batch k+1
            stage_s += time.perf_counter() - ta
        cur.sync()
    engines[(iters - 1) % 2].fetch(reuse=True)
    dt = time.perf_counter() - t0
    eng2.close()
    eng.unpin()
    return {"requests_per_s": round(iters * batch.n_req / dt, 1), "GB/s": round(iters * raw / dt / 1e9, 3),
            "iters": iters, "ms_per_batch": round(dt / iters * 1e3, 2),
            "host_stage_ms_per_batch": round(stage_s / max(iters - 1, 1) * 1e3, 2),
            "host_fetch_ms_per_batch": round(fetch_s / max(iters - 1, 1) * 1e3, 2), "pinned_arrays": pinned,
            "def": "two contexts alternating: H2D of batch k+1 (page-locked) and D2H of batch k-1 overlap batch k's "
                   "kernels; includes every stage, run and fetch"}


def log(msg):
    """Progress on stderr (a long compile or batch must not look hung to a watchdog)."""
    sys.stderr.write("[bench %s] %s\n" % (time.strftime("%H:%M:%S"), msg))
    sys.stderr.flush()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--n-req", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--matched-cap", type=int, default=64)
    ap.add_argument("--no-balance", action="store_true", help="N > 1: keep each rank's own chunk (no byte balancing)")
    ap.add_argument("--e2e-iters", type=int, default=4, help="batches in the pipelined host-inclusive leg (0: skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    rs_file, n_default, post_frac, desc = CONFIGS[args.config]
    files = None
    if rs_file is None:  # c5: generated ruleset + phrase file
        text, files = traffic.c5_ruleset()
    else:
        text = open(os.path.join(ROOT, rs_file)).read()
    n_req = args.n_req or n_default
    t_compile = time.perf_counter()
    log("compiling %s (%d bytes of SecLang)" % (args.config, len(text)))
    rs = gpuinspect.Ruleset(text, data_files=files)
    t_compile = time.perf_counter() - t_compile
    log("compiled in %.1f s: %s" % (t_compile, rs.info))
    eng = gpuinspect.Engine(rs, device=local, matched_cap=args.matched_cap)
    t_gen = time.perf_counter()
    if args.config == "c5":
        batch = traffic.c5_batch(n_req, seed=shard.shard_seed(traffic.SEED, rank))
    else:
        # GI_BENCH_JSON_FRAC: a diagnostic A/B of the body mix (the configs' lines use the default 0.4)
        jf = float(os.environ.get("GI_BENCH_JSON_FRAC", "0.4"))
        batch = traffic.TrafficGen(shard.shard_seed(traffic.SEED, rank)).batch(n_req, post_frac=post_frac,
                                                                                json_frac=jf)
        if jf != 0.4:
            log("DIAGNOSTIC body mix: json_frac %.2f (not the config's)" % jf)
    split = None
    if dist is not None and not args.no_balance:
        log("rebalancing the request set by bytes across %d ranks" % world)
        batch, rng, totals = shard.rebalance(dist, world, rank, batch, "cuda")
        split = {"kind": "byte-balanced contiguous slices of one seeded request set (shard.rebalance)",
                 "bytes_per_rank": totals,
                 "max_over_mean": round(max(totals) / (sum(totals) / len(totals)), 4) if sum(totals) else 1.0}
    t_gen = time.perf_counter() - t_gen
    raw = batch.raw_bytes()
    log("generated %d requests (%d bytes) in %.1f s; staging" % (batch.n_req, raw, t_gen))
    eng.stage(batch)

    gather = shard.TallyGather(dist, world, "cuda", n_rules=eng.tally_rule_count()) if dist is not None else None

    def step():
        eng.run()
        eng.sync()
        if gather is not None:
            gather.push(eng.tally(), eng.tally_detail())

    for w in range(args.warmup):
        step()
        log("warmup %d done" % w)
    if dist is not None:
        dist.barrier()
        torch.cuda.synchronize()
    eng.sync()
    kern_ms = []
    launch_ms, launch_bytes, launch_steps = {}, {}, {}
    t0 = time.perf_counter()
    for k in range(args.steps):
        step()
        log("step %d done" % k)
        st = eng.stats()
        kern_ms.append(st["last_kernel_ms"])
        for ln in st["launches"]:
            launch_ms.setdefault(ln["name"], []).append(ln["ms"])
            launch_bytes[ln["name"]] = ln["alg_bytes"]
            launch_steps[ln["name"]] = ln["steps"]
    eng.sync()
    if dist is not None:
        torch.cuda.synchronize()
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tally = eng.tally()
    detail = eng.tally_detail()
    if dist is not None:
        elapsed = shard.max_over_ranks(dist, elapsed, "cuda")
        tot = gather.total()
        total_req = tot["n_req"]
        total_bytes = tot["bytes_scanned"]
        node_tally = tot
    else:
        total_req, total_bytes = int(tally["n_req"]), int(tally["bytes_scanned"])
        node_tally = dict(tally, **detail)
    ms_per_step = elapsed / args.steps * 1e3
    value = total_req * args.steps / elapsed
    gbs = total_bytes * args.steps / elapsed / 1e9

    # Roofline of the dominant launch (HIP events recorded on the context
    # stream around every launch).  achieved = SURVEY.md §8(d) algorithmic
    # bytes of the batch (raw request bytes once + 16 B verdict + 4 B per
    # matched id) / the dominant launch's average time.
    avg_launch = {k: float(np.mean(v)) for k, v in launch_ms.items()}
    dom = max(avg_launch, key=lambda k: avg_launch[k])
    req_bytes = raw + 16 * batch.n_req + 4 * int(tally["matched_total"])
    achieved = req_bytes / (avg_launch[dom] * 1e-3) / 1e9
    avg_kern_ms = float(np.mean(kern_ms))
    hbm_traffic = None
    tpath = os.path.join(ROOT, "profiles", "traffic_%s.json" % args.config)
    traffic_all = None
    if os.path.exists(tpath):  # rocprofv3 FETCH_SIZE/WRITE_SIZE passes (tools/pmc_traffic.py)
        tj = json.load(open(tpath))
        if tj.get("requests") == batch.n_req:
            kt = tj.get("kernels", {})
            rk = ROCPROF_NAMES.get(dom, dom)
            for name in (rk, "gi::" + rk):  # rocprofv3 may report the namespace
                if name in kt:
                    hbm_traffic = kt[name]["hbm_bytes_per_launch"]
            traffic_all = {"source": "profiles/traffic_%s.json (%s)" % (args.config, tj.get("tag", "")),
                           "hbm_bytes_per_launch": {k: v["hbm_bytes_per_launch"] for k, v in kt.items()}}
    steps_s = launch_steps.get(dom, 0) / (avg_launch[dom] * 1e-3)
    metric_set = {"c1": "config/samples RuleSet", "c2": "CRS-shaped v4 PL1 stand-in", "c3": "CRS-shaped v4 PL1 stand-in",
                  "c4": "CRS-shaped v4 PL4 stand-in", "c5": "generated 10k-rule set",
                  "c2x": "CRS-shaped v4 PL1 stand-in + 20 CRS-scale regexes"}[args.config]
    out = {
        "metric": "requests inspected/sec (node), " + metric_set,
        "value": round(value, 1),
        "unit": "requests/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded generator coraza-kubernetes-operator_amd/traffic.py, seed 0xC0A2A+rank)",
        "config": {"workload": desc, "config": args.config, "requests_per_gpu": batch.n_req,
                   "bytes_per_request": round(raw / batch.n_req, 1), "parallelism": "dp%d" % world,
                   "rules": rs.info["n_rules"], "dfas": rs.info["n_dfas"],
                   **({"diagnostic_json_frac": float(os.environ["GI_BENCH_JSON_FRAC"])}
                      if os.environ.get("GI_BENCH_JSON_FRAC", "0.4") not in ("0.4", "") else {})},
        "gb_per_s_scanned": round(gbs, 3),
        "interrupted_frac": round(tally["n_interrupted"] / max(tally["n_req"], 1), 4),
        "pa_void_requests": int(tally["n_pa_void"]),
        # the phase gate: requests with a body it evaluated in its
        # first stage, and of those the ones its body stage scanned and evaluated again
        "gate": {"body_requests": int(st.get("gate_requests", 0)), "pending": int(st.get("gate_pending", 0))},
        "error_requests": int(tally["n_error"]),
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": hbm_traffic, "traffic_by_kernel": traffic_all,
            "kernel": dom, "rocprof_kernel": ROCPROF_NAMES.get(dom, dom), "kernel_ms": round(avg_launch[dom], 4),
            "alg_bytes_per_launch": int(req_bytes),
            "alg_bytes_def": "SURVEY.md 8(d): sum of raw request bytes (method+uri+proto+headers+body, each "
                             "once) + 16 B verdict + 4 B x matched ids, for the whole batch the launch processes",
            "pipeline": {"ms": round(avg_kern_ms, 4), "GB/s": round(req_bytes / (avg_kern_ms * 1e-3) / 1e9, 3),
                         "frac": round(req_bytes / (avg_kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6)},
            "secondary": {
                "bound": "lds/valu (automaton steps, transformation chains)",
                "byte_steps_per_launch": int(launch_steps.get(dom, 0)), "byte_steps_per_s": round(steps_s, 1),
                "queue_bytes_def": "bytes the launch itself must move once (DESIGN.md §4): item bytes + records "
                                   "in, transformed queue words out (k_stream); queue words in (k_scan)",
                "byte_steps_def": "k_scan*: automaton transitions; k_stream*: value bytes fed into a stream's "
                                  "transformation chain (value x streams reading it); k_detect: value bytes "
                                  "through libinjection",
                "launches": {k: {"ms": round(v, 4), "queue_bytes": int(launch_bytes[k]),
                                 "GB/s": round(launch_bytes[k] / (v * 1e-3) / 1e9, 2) if v > 0 else None,
                                 "byte_steps": int(launch_steps.get(k, 0)),
                                 "byte_steps_per_s": round(launch_steps.get(k, 0) / (v * 1e-3), 1) if v > 0 else None,
                                 **({"lds_frac": round(launch_steps.get(k, 0) / (v * 1e-3) / LDS_B32_LANES_PER_S, 5)}
                                    if k.startswith("k_scan") and v > 0 else {})}
                             for k, v in avg_launch.items()},
                "lds_peak_lanes_per_s": LDS_B32_LANES_PER_S,
                "lds_frac_def": "k_scan*: automaton transitions/s (one ds_read_b32 lane each) / the chip's "
                                "ds_read_b32 lane rate (MI355X_MICROARCH.md: ~75 TB/s)"},
        },
        "tally": {"n_req": int(node_tally["n_req"]), "n_interrupted": int(node_tally["n_interrupted"]),
                  "matched_total": int(node_tally["matched_total"]),
                  "score_hist_nonzero": {str(b): int(x) for b, x in enumerate(node_tally["score_hist"]) if x},
                  "top_rules": sorted(([int(i), int(h)] for i, h in zip(detail["rule_ids"], node_tally["rule_hits"]) if h),
                                      key=lambda x: -x[1])[:8]},
        "gen_s": round(t_gen, 1),
        "compile_s": round(t_compile, 1),
        # what the parity sample can not vouch for: the oracle
        # restates third-party code absent from /root/reference
        "parity_unpinned": [
            "@detectSQLi fingerprint grammar + 304-word keyword table (authored, not libinjection's tables)",
            "CRS-shaped stand-in ruleset (CRS v4.23.0 rules are a download; rulesets/crs/*.conf are authored)",
            "Go regexp / Coraza v3.3.3 semantics beyond the reference KATs (oracle restatement, no Go toolchain)",
            "body-limit (413 / ProcessPartial), FULL_REQUEST_LENGTH / URLENCODED_ERROR semantics (restated from memory)",
        ],
    }
    if split is not None:
        out["split"] = dict(split, set_requests=int(total_req))
    # Host-inclusive passes (never `value`).  serial: one stage (host layout +
    # H2D of pageable numpy buffers) + pipeline + D2H of verdicts and matched
    # ids.  pipelined: the batch's buffers page-locked (gi_host_register) and
    # two contexts alternating, so batch k+1's staging and batch k-1's fetch
    # overlap batch k's kernels (steady-state requests/s over e2e_iters batches).
    t1 = time.perf_counter()
    eng.stage(batch)
    t2 = time.perf_counter()
    eng.run()
    eng.sync()
    t3 = time.perf_counter()
    res = eng.fetch()
    t4 = time.perf_counter()
    # which rules decide the verdicts: the interrupting rule of every
    # interrupted request (0: the 413 of SecRequestBodyLimitAction Reject), and
    # the most-matched ids without the request-independent ones (the folded
    # initialisation SecActions match every request)
    iv = res.verdicts[res.verdicts["status"] != 0]["rule_id"]
    ids_i, cnt_i = np.unique(iv, return_counts=True)
    out["tally"]["interrupting_rules"] = [[int(i), int(c)] for c, i in sorted(zip(cnt_i, ids_i), reverse=True)[:8]]
    out["tally"]["top_rules_request_dependent"] = sorted(
        ([int(i), int(h)] for i, h in zip(detail["rule_ids"], node_tally["rule_hits"]) if 0 < h < node_tally["n_req"]),
        key=lambda x: -x[1])[:8]
    out["e2e"] = {"requests_per_s": round(batch.n_req / (t4 - t1), 1), "ms": round((t4 - t1) * 1e3, 2),
                  "stage_ms": round((t2 - t1) * 1e3, 2), "run_ms": round((t3 - t2) * 1e3, 2),
                  "fetch_ms": round((t4 - t3) * 1e3, 2),
                  "GB/s": round(raw / (t4 - t1) / 1e9, 3),
                  "def": "one pass incl. gi_stage_batch (host layout + H2D, pageable) and gi_fetch_results (D2H), per GPU"}
    if args.e2e_iters > 0:
        try:
            out["e2e"]["pipelined"] = e2e_pipelined(rs, eng, batch, local, args.matched_cap, args.e2e_iters, raw)
        except gpuinspect.EngineError as ex:  # e.g. not enough HBM for a second context: reported, not fatal
            out["e2e"]["pipelined"] = {"error": str(ex)[:200]}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if args.config == "c5":
            # every one of the 10k rule links over every ~1 MB value, exactly: more
            # than 3 minutes per request on one core, beyond this leg's budget
            out["cpu_baseline"] = {"skipped": "C5: the C++ interpreter evaluates all 10k links over each ~1 MB "
                                              "body exactly (> 3 min per request per core)"}
        else:
            log("cpu baseline (C++ interpreter on the host cores)")
            out["cpu_baseline"] = cpu_baseline(rs, batch, res, budget_s=10.0)
        log("parity sample (oracle)")
        verdicts, wall, procs = oracle_sample(text, batch, rs.exports, files=files,
                                              calib=1 if args.config == "c5" else 100,
                                              min_n=16 if args.config == "c5" else 200,
                                              budget_s=30.0 if args.config == "c5" else 15.0)
        out["parity_sample"] = parity(res, verdicts)
        out["parity_sample"]["oracle_requests_per_s"] = round(len(verdicts) / wall, 1)
        out["parity_sample"]["oracle_procs"] = procs
    elif world > 1:
        # every rank checks a small sample of its own batch against the oracle
        from oracle import compare, coraza
        cfg = coraza.parse_seclang(text, files)
        idx = range(0, batch.n_req, max(1, batch.n_req // (8 if args.config == "c5" else 128)))
        ps = parity(res, compare.oracle_verdicts(cfg, batch, rs.exports, idx))
        import torch
        t = torch.tensor([ps["n"], ps["mismatches"]], dtype=torch.int64, device="cuda")
        dist.all_reduce(t)
        out["parity_sample"] = dict(ps, n=int(t[0]), mismatches=int(t[1]), first=ps["first"] if rank == 0 else [])
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
