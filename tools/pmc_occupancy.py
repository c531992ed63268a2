"""Per-kernel occupancy / stall / LDS counters from rocprofv3 PMC passes.

Runs a short bench.py under rocprofv3 once per counter pass (gfx950 slot
limits: <= 8 SQ and <= 2 GRBM counters per pass, each pass its own run, under
`timeout -s KILL`) and writes, per kernel, the per-dispatch medians and the
derived figures:

  waves_per_simd   = 4 * SQ_WAVE_CYCLES / (1024 SIMDs * GRBM_GUI_ACTIVE / 8)
                     (SQ_* count quad-cycles summed over waves; GRBM_GUI_ACTIVE
                     is summed over the 8 XCDs: /8 = kernel cycles;
                     MI355X_MICROARCH.md, rocprofv3 PMC and DVFS sections)
  valu_busy        = 4 * SQ_ACTIVE_INST_VALU / (1024 * GRBM_GUI_ACTIVE / 8)
  wait_any_frac    = SQ_WAIT_ANY / SQ_WAVE_CYCLES        (wave parked on s_waitcnt / barrier)
  issue_stall_frac = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (issue stalls)
  active_frac      = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  lds_conflict_frac= SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  eff_clock_ghz    = GRBM_GUI_ACTIVE / 8 / kernel duration

  python tools/pmc_occupancy.py --config c2 --n-req 1000000 --out profiles/pmc_c2_r02.json
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = [
    "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE",
    "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR",
]


def run_pass(i, counters, args, base):
    out = os.path.join(base, "p%d" % i)
    os.makedirs(out, exist_ok=True)
    cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc"] + counters.split() + [
        "--kernel-trace", "--output-format", "csv", "-d", out, "-o", "run", "--",
        sys.executable, os.path.join(ROOT, "bench.py"), "--config", args.config, "--n-req", str(args.n_req),
        "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    env = dict(os.environ, TMPDIR="/tmp")
    with open(out + ".log", "w") as log:
        subprocess.run(cmd, check=True, cwd="/tmp", env=env, stdout=log, stderr=subprocess.STDOUT)
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("gi::", "")
            vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    durs = defaultdict(list)
    for f in glob.glob(os.path.join(out, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("gi::", "")
            durs[k].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return vals, durs


def med(x):
    x = sorted(x)
    return x[len(x) // 2] if x else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--n-req", type=int, default=1000000)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    base = os.path.join(ROOT, "gpurun_out", "pmc_occ")
    merged = defaultdict(dict)
    durs = defaultdict(list)
    for i, p in enumerate(PASSES):
        vals, d = run_pass(i, p, args, base)
        for k, cs in vals.items():
            for c, v in cs.items():
                merged[k][c] = med(v)
        for k, v in d.items():
            durs[k] += v
        print("pass %d ok (%s)" % (i, p), flush=True)
    res = {}
    for k, c in merged.items():
        if k.startswith("__amd"):
            continue
        g = c.get("GRBM_GUI_ACTIVE")
        cyc = g / 8 if g else None
        wc = c.get("SQ_WAVE_CYCLES")
        r = {"counters": c, "dispatch_ns": med(durs.get(k, []))}
        if cyc and wc:
            r["waves_per_simd"] = round(4 * wc / (1024 * cyc), 3)
            r["valu_busy"] = round(4 * c.get("SQ_ACTIVE_INST_VALU", 0) / (1024 * cyc), 4)
            r["wait_any_frac"] = round(c.get("SQ_WAIT_ANY", 0) / wc, 4)
            r["issue_stall_frac"] = round(c.get("SQ_WAIT_INST_ANY", 0) / wc, 4)
            r["active_frac"] = round(c.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4)
            if r["dispatch_ns"]:
                r["eff_clock_ghz"] = round(cyc / r["dispatch_ns"], 3)
        if c.get("SQ_LDS_IDX_ACTIVE"):
            r["lds_conflict_frac"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"], 4)
        res[k] = r
    out = {"config": args.config, "requests": args.n_req, "passes": PASSES,
           "derived": __doc__.split("\n\n")[1].strip(), "kernels": res}
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    json.dump(out, open(args.out, "w"), indent=1)
    for k in sorted(res, key=lambda k: -(res[k].get("dispatch_ns") or 0)):
        r = res[k]
        print("%-28s %8.2f ms waves/SIMD %s valu %s wait %s stall %s lds-conf %s" % (
            k, (r.get("dispatch_ns") or 0) / 1e6, r.get("waves_per_simd"), r.get("valu_busy"),
            r.get("wait_any_frac"), r.get("issue_stall_frac"), r.get("lds_conflict_frac")))


if __name__ == "__main__":
    main()
