"""HBM traffic per launch of every pipeline kernel from rocprofv3 PMC passes.

Runs bench.py twice under rocprofv3 (one pass FETCH_SIZE, one pass
WRITE_SIZE -- separate runs: TCC slot limits), groups the per-dispatch values
by kernel name, applies the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md ("FETCH_SIZE reports 1/2 of the bytes
of a wide coalesced streaming read": x2; WRITE_SIZE exact; both in KB), and
writes profiles/traffic_<config>.json, which bench.py reports as
roofline.traffic (the dominant launch) and roofline.traffic_by_kernel.

  python tools/pmc_traffic.py --config c2 --n-req 1000000 [--tag r03]
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short_name(k):
    """'void k_stream<16u, 20u>(DProgram, DBatch, unsigned int)' -> 'k_stream<16u, 20u>'."""
    k = k.strip()
    if k.startswith("void "):
        k = k[5:]
    depth = 0
    for i, ch in enumerate(k):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return k[:i]
    return k


def run_pass(counter, args, out):
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", out, "-o", "run", "--",
           sys.executable, os.path.join(ROOT, "bench.py"), "--config", args.config, "--n-req", str(args.n_req),
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    env = dict(os.environ, TMPDIR="/tmp")
    subprocess.run(["timeout", "-s", "KILL", "300"] + cmd, check=True, cwd="/tmp", env=env,
                   stdout=open(out + ".log", "w"), stderr=subprocess.STDOUT)
    vals = {}
    for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == counter:
                vals.setdefault(short_name(row["Kernel_Name"]), []).append(float(row["Counter_Value"]))
    return vals


def median(v):
    v = sorted(v)
    return v[len(v) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--n-req", type=int, default=1000000)
    ap.add_argument("--tag", default="")
    ap.add_argument("--out", default="", help="also write the JSON here (e.g. under gpurun_out/)")
    args = ap.parse_args()
    base = os.path.join(ROOT, "gpurun_out", "traffic")
    os.makedirs(base, exist_ok=True)
    fetch = run_pass("FETCH_SIZE", args, os.path.join(base, "fetch"))
    print("fetch pass: %d kernels" % len(fetch), flush=True)
    write = run_pass("WRITE_SIZE", args, os.path.join(base, "write"))
    print("write pass: %d kernels" % len(write), flush=True)
    if not fetch or not write:
        raise SystemExit("no counter rows")
    kernels = {}
    for k in sorted(set(fetch) & set(write)):
        # FETCH_SIZE / WRITE_SIZE are in KB; per dispatch = median over dispatches
        f_kb, w_kb = median(fetch[k]), median(write[k])
        kernels[k] = {"fetch_size_kb_raw": f_kb, "write_size_kb": w_kb,
                      "hbm_bytes_per_launch": int(2 * f_kb * 1024 + w_kb * 1024),
                      "dispatches": [len(fetch[k]), len(write[k])]}
    out = {"config": args.config, "requests": args.n_req, "tag": args.tag, "kernels": kernels,
           "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); WRITE_SIZE as reported"}
    json.dump(out, open(os.path.join(ROOT, "profiles", "traffic_%s.json" % args.config), "w"), indent=1)
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
