"""Benchmark: requests inspected/s + GB/s scanned on MI355X (BASELINE.json metric).

One "step" = one pass of the inspection pipeline (gi_run_staged: collect ->
phase 1 -> body -> phase 2 -> verdicts + tallies) over one batch of synthetic
requests already resident in HBM, plus (N > 1) the RCCL all-gather of the
per-GPU tally.  Requests are sharded with no data-path collective: each rank
inspects its own batch (weak scaling).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c1|c3] [--n-req R]

N > 1 is launched by torch.distributed.run (RANK/LOCAL_RANK/WORLD_SIZE env).
Prints ONE JSON line on rank 0.
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

# launch name (gi_stats) -> kernel name as rocprofv3 reports it
ROCPROF_NAMES = {
    "k_stream0": "k_stream<16u, 20u>", "k_stream1": "k_stream<32u, 36u>", "k_stream2": "k_stream<64u, 68u>",
    "k_stream3": "k_stream<128u, 132u>", "k_stream4": "k_stream<0u, 0u>", "k_scan": "k_scan<true, false>",
    "k_scan_big": "k_scan<true, true>", "k_scan_hbm": "k_scan<false, false>",
}

CONFIGS = {
    # name: (ruleset file, default n_req, post_frac, description)
    "c2": ("rulesets/crs_pl1.conf", 1_000_000, 0.0,
           "CRS-shaped v4 PL1 ruleset (rulesets/crs_pl1.conf) x 1M synthetic GET with query args"),
    "c1": ("tests/golden/samples_ruleset.conf", 10_000, 0.0,
           "config/samples RuleSet x 10k synthetic GET"),
    "c3": ("rulesets/crs_pl1.conf", 50_000, 0.5,
           "CRS-shaped v4 PL1 x mixed GET/POST (50% POST, 4-64 KB bodies: 60% urlencoded, 40% JSON)"),
}


def _oracle_worker(args):
    text, blob, idx = args
    from oracle import coraza
    cfg = coraza.parse_seclang(text)
    data, reqs, headers = blob
    b = gpuinspect.PackedBatch(data, reqs, headers)
    t0 = time.perf_counter()
    for i in idx:
        t = b.request(i)
        coraza.inspect(cfg, coraza.Request(t.method, t.uri, t.proto, list(t.headers), t.body))
    return time.perf_counter() - t0, len(idx)


def cpu_baseline(text, batch, budget_s=15.0, procs=16):
    """The CPU oracle (port) on a bounded sample of the same workload."""
    n_sample = min(batch.n_req, 4000)
    blob = (batch.data, batch.reqs, batch.headers)
    # calibrate on 100 requests, then size the sample for ~budget_s wall
    dt, n = _oracle_worker((text, blob, range(100)))
    per = dt / max(n, 1)
    procs = max(1, min(procs, os.cpu_count() or 1))
    n_sample = int(min(n_sample * procs, max(200, budget_s * procs / max(per, 1e-6))))
    n_sample = min(n_sample, batch.n_req)
    chunks = [range(k, n_sample, procs) for k in range(procs)]
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(procs) as pool:
        outs = pool.map(_oracle_worker, [(text, blob, c) for c in chunks])
    wall = time.perf_counter() - t0
    done = sum(o[1] for o in outs)
    return {"value": round(done / wall, 1), "unit": "requests/s", "cores": procs, "kind": "port",
            "sample": "%d requests of the benchmark batch, oracle/coraza.py (pure-Python Coraza "
                      "restatement, CPython re for @rx) in %d processes" % (done, procs)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--n-req", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--matched-cap", type=int, default=64)
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
    text = open(os.path.join(ROOT, rs_file)).read()
    n_req = args.n_req or n_default
    rs = gpuinspect.Ruleset(text)
    eng = gpuinspect.Engine(rs, device=local, matched_cap=args.matched_cap)
    t_gen = time.perf_counter()
    batch = traffic.TrafficGen(shard.shard_seed(traffic.SEED, rank)).batch(n_req, post_frac=post_frac)
    t_gen = time.perf_counter() - t_gen
    raw = batch.raw_bytes()
    eng.stage(batch)

    gather = shard.TallyGather(dist, world, "cuda") if dist is not None else None

    def step():
        eng.run()
        eng.sync()
        if gather is not None:
            gather.push(eng.tally())

    for _ in range(args.warmup):
        step()
    if dist is not None:
        dist.barrier()
        torch.cuda.synchronize()
    eng.sync()
    kern_ms, stage_ms = [], {"k_collect": [], "k_stream": [], "k_scan": [], "k_eval": []}
    launch_ms, launch_bytes, launch_steps = {}, {}, {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        st = eng.stats()
        kern_ms.append(st["last_kernel_ms"])
        stage_ms["k_collect"].append(st["last_collect_ms"])
        stage_ms["k_stream"].append(st["last_stream_ms"])
        stage_ms["k_scan"].append(st["last_scan_ms"])
        stage_ms["k_eval"].append(st["last_eval_ms"])
        for ln in st["launches"]:
            launch_ms.setdefault(ln["name"], []).append(ln["ms"])
            launch_bytes[ln["name"]] = ln["alg_bytes"]
            launch_steps[ln["name"]] = ln["steps"]
    eng.sync()
    if dist is not None:
        torch.cuda.synchronize()
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        elapsed = shard.max_over_ranks(dist, elapsed, "cuda")
        tot = gather.total()
        total_req = tot["n_req"]
        total_bytes = tot["bytes_scanned"]
    else:
        t = eng.tally()
        total_req, total_bytes = int(t["n_req"]), int(t["bytes_scanned"])
    tally = eng.tally()
    ms_per_step = elapsed / args.steps * 1e3
    value = total_req * args.steps / elapsed
    gbs = total_bytes * args.steps / elapsed / 1e9

    # Roofline of the dominant single kernel launch (HIP events recorded on the
    # context stream around every launch; DESIGN.md §4 defines each kernel's
    # algorithmic bytes per launch, counted on the device).
    avg_kern_ms = float(np.mean(kern_ms))
    avg_stage = {k: float(np.mean(v)) for k, v in stage_ms.items()}
    avg_launch = {k: float(np.mean(v)) for k, v in launch_ms.items()}
    dom = max(avg_launch, key=lambda k: avg_launch[k])
    alg_bytes = launch_bytes[dom]
    achieved = alg_bytes / (avg_launch[dom] * 1e-3) / 1e9
    # SURVEY.md §8(d) figure: raw request bytes once + verdict record + 4 B per
    # matched id, over the whole pipeline
    req_bytes = raw + 16 * batch.n_req + 4 * int(tally["matched_total"])
    req_gbs = req_bytes / (avg_kern_ms * 1e-3) / 1e9
    steps_s = launch_steps.get(dom, 0) / (avg_launch[dom] * 1e-3)
    hbm_traffic = None
    tpath = os.path.join(ROOT, "profiles", "traffic_%s.json" % args.config)
    if os.path.exists(tpath):  # rocprofv3 FETCH_SIZE/WRITE_SIZE passes (tools/pmc_traffic.py)
        tj = json.load(open(tpath))
        if tj.get("kernel") == dom and tj.get("requests") == batch.n_req:
            hbm_traffic = tj["hbm_bytes_per_launch"]
    out = {
        "metric": "requests inspected/sec (node), CRS v4 PL1",
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
                   "rules": rs.info["n_rules"], "dfas": rs.info["n_dfas"]},
        "gb_per_s_scanned": round(gbs, 3),
        "interrupted_frac": round(tally["n_interrupted"] / max(tally["n_req"], 1), 4),
        "pa_void_requests": int(tally["n_pa_void"]),
        "error_requests": int(tally["n_error"]),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": hbm_traffic,
                     "kernel": dom, "rocprof_kernel": ROCPROF_NAMES.get(dom, dom),
                     "kernel_ms": round(avg_launch[dom], 4), "alg_bytes_per_launch": int(alg_bytes),
                     "alg_bytes_def": "bytes the launch must move once: for k_scan, every queue word "
                                      "(transformed value + 16 B lane header) of its streams read once",
                     "secondary": {"bound": "valu/lds (automaton steps)", "byte_steps_per_launch": int(launch_steps.get(dom, 0)),
                                   "byte_steps_per_s": round(steps_s, 1)},
                     "pipeline_request_bytes": {"def": "SURVEY.md 8(d): raw request bytes + 16 B verdict + 4 B x matched ids",
                                                "bytes": int(req_bytes), "GB/s": round(req_gbs, 3),
                                                "frac": round(req_gbs / HBM_PEAK_GBS, 6)},
                     "launches": {k: {"ms": round(v, 4), "alg_bytes": int(launch_bytes[k]),
                                      "GB/s": round(launch_bytes[k] / (v * 1e-3) / 1e9, 2) if v > 0 else None}
                                  for k, v in avg_launch.items()},
                     "stages_ms": {k: round(v, 4) for k, v in avg_stage.items()},
                     "pipeline_kernel_ms": round(avg_kern_ms, 4)},
        "gen_s": round(t_gen, 1),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(text, batch)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
