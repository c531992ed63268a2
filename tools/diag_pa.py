"""Phase-A diagnostics on one batch (GPU): items per length bucket, queue
pool use, slow values, stage times.  GI_DIAG=1 enables the device counters."""
import os
import sys

os.environ.setdefault("GI_DIAG", "1")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "coraza-kubernetes-operator_amd"))
import gpuinspect as g  # noqa: E402
import traffic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
conf = sys.argv[2] if len(sys.argv) > 2 else "rulesets/crs_pl1.conf"
post = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
rs = g.Ruleset(open(os.path.join(os.path.dirname(__file__), "..", conf)).read())
eng = g.Engine(rs, device=0)
b = traffic.TrafficGen(traffic.SEED).batch(n, post_frac=post)
eng.stage(b)
for it in range(3):
    eng.run()
    eng.sync()
st = eng.stats()
t = eng.tally()
d = st["diag"]
print("n_req", n, "raw_bytes/req %.1f" % (b.raw_bytes() / n))
print("pool words/req %.1f (cap %.1f MB)  slow entries %d  slow bytes %d  items/bucket %s" %
      (d[0] / n, st["last_pa_bytes"] / 1e6, d[2], d[1], d[3:8]))
print("pa_void", t["n_pa_void"], "interrupted", t["n_interrupted"], "matched_total", t["matched_total"])
print({k: round(st[k], 3) for k in ("last_collect_ms", "last_stream_ms", "last_scan_ms", "last_eval_ms",
                                     "last_kernel_ms")})
