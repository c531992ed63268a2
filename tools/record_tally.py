"""Record the engine's per-rank tallies of one seeded request set cut into
byte-balanced slices (the multi-GPU bench's split, shard.balanced_slices) as a
fixture for tests/test_dist_cpu.py (GPU run; the test itself needs no GPU).

  python tools/record_tally.py [--world 2] [--n-req 600] [--out tests/golden/tally_crs_pl1_world2.json]

Every slice is inspected on device 0 in turn (the ranks of a node run the same
engine on their own GPU); the fixture holds each slice's gi_tally counters and
gi_tally_detail_get histogram / per-rule counts.  test_dist_cpu checks the
fixture against the CPU oracle and all-gathers it over gloo."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "coraza-kubernetes-operator_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import gpuinspect  # noqa: E402
import shard  # noqa: E402
import traffic  # noqa: E402

RULESET = "rulesets/crs_pl1.conf"
SEED = traffic.SEED + 77
ATTACK_RATE = 0.3
POST_FRAC = 0.2


def request_set(n_req):
    """The seeded set and its byte-balanced slices (shared with the test)."""
    batch = traffic.TrafficGen(SEED).batch(n_req, attack_rate=ATTACK_RATE, post_frac=POST_FRAC)
    return batch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--n-req", type=int, default=600)
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "tally_crs_pl1_world2.json"))
    a = ap.parse_args()
    text = open(os.path.join(ROOT, RULESET)).read()
    rs = gpuinspect.Ruleset(text)
    eng = gpuinspect.Engine(rs, device=0)
    batch = request_set(a.n_req)
    slices = shard.balanced_slices(batch.request_bytes(), a.world)
    rows = []
    for lo, hi in slices:
        part = batch.take(lo, hi)
        eng.stage(part)
        eng.run()
        eng.sync()
        t = eng.tally()
        d = eng.tally_detail()
        rows.append({"slice": [lo, hi], "tally": {k: int(t[k]) for k in shard.TALLY_KEYS},
                     "score_hist": [int(x) for x in d["score_hist"]],
                     "rule_ids": [int(x) for x in d["rule_ids"]], "rule_hits": [int(x) for x in d["rule_hits"]]})
    out = {"ruleset": RULESET, "seed": SEED, "n_req": a.n_req, "attack_rate": ATTACK_RATE, "post_frac": POST_FRAC,
           "world": a.world, "exports": list(rs.exports), "ranks": rows,
           "made_by": "tools/record_tally.py on one MI355X (gi_tally_get / gi_tally_detail_get per slice)"}
    json.dump(out, open(a.out, "w"), indent=0)
    print("wrote %s: %d ranks, %d rule ids" % (a.out, len(rows), len(rows[0]["rule_ids"])))


if __name__ == "__main__":
    main()
