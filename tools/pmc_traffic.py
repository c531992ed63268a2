"""HBM traffic per launch of the roofline kernel from rocprofv3 PMC passes.

Runs bench.py twice under rocprofv3 (one pass FETCH_SIZE, one pass
WRITE_SIZE -- separate runs: TCC slot limits), takes the per-dispatch values
of the named kernel, applies the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md ("FETCH_SIZE reports 1/2 of the bytes
of a wide coalesced streaming read": x2; WRITE_SIZE exact; both in KB), and
writes profiles/traffic_<config>.json, which bench.py reports as
roofline.traffic.

  python tools/pmc_traffic.py --config c2 --n-req 1000000 [--kernel k_eval]
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_pass(counter, args, out):
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", out, "-o", "run", "--",
           sys.executable, os.path.join(ROOT, "bench.py"), "--config", args.config, "--n-req", str(args.n_req),
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    env = dict(os.environ, TMPDIR="/tmp")
    subprocess.run(["timeout", "-s", "KILL", "300"] + cmd, check=True, cwd="/tmp", env=env,
                   stdout=open(out + ".log", "w"), stderr=subprocess.STDOUT)
    vals = []
    for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if args.kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--n-req", type=int, default=1000000)
    ap.add_argument("--kernel", default="", help="launch name (default: the dominant launch of a bench run)")
    ap.add_argument("--out", default="", help="also write the JSON here (e.g. under gpurun_out/)")
    args = ap.parse_args()
    base = os.path.join(ROOT, "gpurun_out", "traffic")
    os.makedirs(base, exist_ok=True)
    sys.path.insert(0, ROOT)
    import bench  # noqa: E402  (launch-name -> rocprof kernel-name map)
    if not args.kernel:  # the dominant launch of a short bench run
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", args.config, "--n-req",
                            str(args.n_req), "--steps", "2", "--warmup", "1", "--no-cpu-baseline"],
                           check=True, capture_output=True, text=True)
        args.kernel = json.loads(r.stdout.strip().splitlines()[-1])["roofline"]["kernel"]
    launch = args.kernel
    args.kernel = bench.ROCPROF_NAMES.get(launch, launch)
    fetch = run_pass("FETCH_SIZE", args, os.path.join(base, "fetch"))
    write = run_pass("WRITE_SIZE", args, os.path.join(base, "write"))
    if not fetch or not write:
        raise SystemExit("no counter rows for kernel %s" % args.kernel)
    # FETCH_SIZE / WRITE_SIZE are in KB; per dispatch = median over dispatches
    fetch.sort()
    write.sort()
    f_kb = fetch[len(fetch) // 2]
    w_kb = write[len(write) // 2]
    out = {"kernel": launch, "rocprof_kernel": args.kernel, "config": args.config, "requests": args.n_req,
           "fetch_size_kb_raw": f_kb, "write_size_kb": w_kb,
           "hbm_bytes_per_launch": int(2 * f_kb * 1024 + w_kb * 1024),
           "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); WRITE_SIZE as reported",
           "dispatches": [len(fetch), len(write)]}
    json.dump(out, open(os.path.join(ROOT, "profiles", "traffic_%s.json" % args.config), "w"), indent=1)
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
