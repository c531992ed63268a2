"""Print the phase-A scan plan of a ruleset (streams, filters, jobs, automata)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "coraza-kubernetes-operator_amd"))
import gpuinspect as g  # noqa: E402

path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "rulesets", "crs_pl1.conf")
rs = g.Ruleset(open(path).read())
d = rs.describe()
print(rs.info)
print("jobs", d["jobs"], "hit_slots", d["hit_slots"], "image_bytes", d["image_bytes"])
for s in d["streams"]:
    print("chain", s["chain"], "kinds", s["kinds"], "filters", len(s["filters"]), "vals", s["vals"])
    for j in s["jobs"]:
        print("   job", [(x["states"], x["classes"], x["pats"], "lds" if x["lds"] else "GLOBAL") for x in j])
