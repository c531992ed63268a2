"""Offline go-ftw replay through the GPU engine.

The reference runs the CRS regression suite with go-ftw against a live
gateway (`/root/reference/ftw/run.py:339-348`, `Makefile:235-247`), with the
override list of `ftw/ftw.yml:4-72` (`testoverride.ignore`: test id ->
reason) and the X-CRS-Test configuration appended to the base rules
(`hack/generate_coreruleset_configmaps.py:113-141`, our
`rulesets/crs_ftw.conf`).  This module replays go-ftw YAML test files
without a network: every stage's request becomes one transaction of a
single `gi_inspect_batch`, and the stage's `output` is checked against the
engine's verdict and matched-rule ids (the ids go-ftw greps out of the
audit log):

* `log.expect_ids` / `log.no_expect_ids` (go-ftw v2 / CRS v4 test format),
* `log_contains` / `no_log_contains` (v1: `id "942100"` patterns),
* `status` (an int or a list of ints; 200 when not interrupted).

Stages whose input cannot be expressed as a request here (`encoded_request`,
`raw_request`) are reported as skipped, not passed.
"""
from __future__ import annotations

import glob
import os
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import yaml

import gpuinspect

_ID_RX = re.compile(r'id[ "\\:]+(\d+)')


@dataclass
class Stage:
    test: str        # test_title (e.g. "942100-1")
    index: int       # stage number within the test
    tx: Optional[gpuinspect.Transaction]
    expect_ids: List[int] = field(default_factory=list)
    no_expect_ids: List[int] = field(default_factory=list)
    status: List[int] = field(default_factory=list)
    skip_reason: str = ""


def load_overrides(path: Optional[str]) -> Dict[str, str]:
    """testoverride.ignore of a go-ftw config (ftw.yml): {test id: reason}."""
    if not path:
        return {}
    with open(path) as f:
        cfg = yaml.safe_load(f) or {}
    ign = ((cfg.get("testoverride") or {}).get("ignore") or {})
    return {str(k): str(v) for k, v in ign.items()}


def _ids(v) -> List[int]:
    if v is None:
        return []
    if isinstance(v, (list, tuple)):
        return [int(x) for x in v]
    return [int(v)]


def _stage_tx(inp: dict) -> (Optional[gpuinspect.Transaction], str):
    if "encoded_request" in inp or "raw_request" in inp:
        return None, "raw/encoded request input"
    method = str(inp.get("method", "GET")).encode()
    uri = str(inp.get("uri", "/")).encode("latin-1")
    proto = str(inp.get("version", "HTTP/1.1")).encode()
    t = gpuinspect.Transaction(method=method, uri=uri, proto=proto)
    headers = inp.get("headers") or {}
    items = headers.items() if isinstance(headers, dict) else [(h.get("name"), h.get("value")) for h in headers]
    for k, v in items:
        t.add_request_header(str(k).encode("latin-1"), str(v).encode("latin-1"))
    data = inp.get("data")
    if data is not None:
        if isinstance(data, list):  # v1 allows a list of lines
            data = "\r\n".join(str(x) for x in data)
        t.write_request_body(str(data).encode("latin-1"))
    return t, ""


def load_tests(paths: Sequence[str]) -> List[Stage]:
    """Every stage of every go-ftw YAML file under `paths` (files or directories)."""
    files: List[str] = []
    for p in paths:
        files += sorted(glob.glob(os.path.join(p, "**", "*.yaml"), recursive=True)) if os.path.isdir(p) else [p]
    out: List[Stage] = []
    for fn in files:
        with open(fn) as f:
            doc = yaml.safe_load(f) or {}
        if (doc.get("meta") or {}).get("enabled") is False:
            continue
        for t in doc.get("tests") or []:
            title = str(t.get("test_title") or t.get("test_id"))
            for k, st in enumerate(t.get("stages") or []):
                st = st.get("stage", st)
                tx, why = _stage_tx(st.get("input") or {})
                o = st.get("output") or {}
                log = o.get("log") or {}
                s = Stage(title, k, tx, _ids(log.get("expect_ids")), _ids(log.get("no_expect_ids")),
                          _ids(o.get("status")), why)
                if o.get("log_contains"):
                    s.expect_ids += [int(m) for m in _ID_RX.findall(str(o["log_contains"]))]
                if o.get("no_log_contains"):
                    s.no_expect_ids += [int(m) for m in _ID_RX.findall(str(o["no_log_contains"]))]
                out.append(s)
    return out


def replay(ruleset: gpuinspect.Ruleset, stages: List[Stage], overrides: Dict[str, str], device: int = 0,
           engine: Optional[gpuinspect.Engine] = None) -> dict:
    """One batch through the engine; per test: pass / fail / ignored (override) / skipped."""
    run = [s for s in stages if s.tx is not None and s.test not in overrides]
    eng = engine or gpuinspect.Engine(ruleset, device=device, matched_cap=256)
    res = eng.inspect(gpuinspect.pack([s.tx for s in run])) if run else None
    results: Dict[str, str] = {}
    failures = []
    for s in stages:
        if s.test in overrides:
            results[s.test] = "ignored"
    for s in stages:
        if s.tx is None and s.test not in overrides:
            results.setdefault(s.test, "skipped")
    for i, s in enumerate(run):
        got = set(res.matched_rules(i))
        it = res.interruption(i)
        status = it["status"] if it else 200
        bad = []
        miss = [x for x in s.expect_ids if x not in got]
        extra = [x for x in s.no_expect_ids if x in got]
        if miss:
            bad.append("missing ids %s" % miss)
        if extra:
            bad.append("unexpected ids %s" % extra)
        if s.status and status not in s.status:
            bad.append("status %d not in %s" % (status, s.status))
        if bad:
            results[s.test] = "fail"
            failures.append({"test": s.test, "stage": s.index, "why": "; ".join(bad)})
        else:
            results.setdefault(s.test, "pass")
    counts = {k: sum(1 for v in results.values() if v == k) for k in ("pass", "fail", "ignored", "skipped")}
    return {"tests": len(results), **counts, "failures": failures, "results": results}


def main(argv=None):
    import argparse
    import json
    ap = argparse.ArgumentParser(description="offline go-ftw replay through gi_inspect_batch")
    ap.add_argument("tests", nargs="+", help="go-ftw YAML files or directories")
    ap.add_argument("--rules", required=True, help="SecLang ruleset (e.g. rulesets/crs_ftw.conf)")
    ap.add_argument("--config", default=None, help="go-ftw config with testoverride.ignore (ftw.yml)")
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args(argv)
    rs = gpuinspect.Ruleset(open(a.rules).read())
    out = replay(rs, load_tests(a.tests), load_overrides(a.config), a.device)
    out.pop("results")
    print(json.dumps(out))
    return 0 if out["fail"] == 0 else 1


if __name__ == "__main__":
    raise SystemExit(main())
