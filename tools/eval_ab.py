"""k_eval time vs request mix (diagnostic, GPU): C2's ruleset over 1M GET
requests at several attack rates; prints each launch's time."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "coraza-kubernetes-operator_amd")):
    sys.path.insert(0, p)
import gpuinspect  # noqa: E402
import traffic  # noqa: E402

rs = gpuinspect.Ruleset(open(os.path.join(ROOT, "rulesets/crs_pl1.conf")).read())
eng = gpuinspect.Engine(rs)
for rate in [float(x) for x in (sys.argv[1:] or ["0", "0.05", "0.3"])]:
    b = traffic.TrafficGen(traffic.SEED).batch(1_000_000, attack_rate=rate)
    eng.stage(b)
    for _ in range(2):
        eng.run()
        eng.sync()
    st = eng.stats()
    t = eng.tally()
    ms = {ln["name"]: round(ln["ms"], 2) for ln in st["launches"]}
    print("attack_rate", rate, "total_ms", round(st["last_kernel_ms"], 2), "interrupted", t["n_interrupted"],
          "k_eval", ms.get("k_eval"), "k_detect", ms.get("k_detect"), "k_scan", ms.get("k_scan"), flush=True)
