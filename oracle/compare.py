"""Parity checker: GPU results vs the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's parity spot-check.
Bar (exact, integer/byte work): for every request the interruption
(rule id, status, action, phase), the ordered matched-rule-id list and every
exported TX value must be identical; requests the oracle flags as
unsupported input must carry a GI_REQ_ERROR_MASK flag on the GPU and vice
versa.
"""

from __future__ import annotations

from . import coraza

ACTION_CODES = {"": 0, "deny": 1, "drop": 2, "redirect": 3}


def oracle_request(t):
    """gpuinspect.Transaction -> the oracle's Request (the same inputs)."""
    return coraza.Request(t.method, t.uri, t.proto, list(t.headers), t.body,
                          getattr(t, "remote_addr", b""), int(getattr(t, "remote_port", 0)),
                          getattr(t, "server_name", b""))


def oracle_verdicts(cfg, batch, exports, idx=None):
    idx = range(batch.n_req) if idx is None else idx
    out = {}
    for i in idx:
        t = batch.request(i)
        req = oracle_request(t)
        out[i] = coraza.inspect(cfg, req, exports)
    return out


def compare(res, oracle, error_mask=0x0F, max_report=10):
    """Returns list of mismatch descriptions (empty == parity)."""
    bad = []
    for i, ov in oracle.items():
        v = res.verdicts[i]
        gpu_err = bool(int(v["flags"]) & error_mask)
        if ov.unsupported or gpu_err:
            if ov.unsupported != gpu_err:
                bad.append((i, "unsupported flag", ov.unsupported, int(v["flags"])))
            continue
        exp = (ov.rule_id, ov.status, ACTION_CODES[ov.action], ov.phase)
        got = (int(v["rule_id"]), int(v["status"]), int(v["action"]), int(v["phase"]))
        if exp != got:
            bad.append((i, "interruption", exp, got))
        gm = res.matched_rules(i)
        if int(v["match_cnt"]) != len(ov.matched) or gm != ov.matched[:len(gm)]:
            bad.append((i, "matched", ov.matched, gm, int(v["match_cnt"])))
        for k, name in enumerate(res.exports):
            a, ok = coraza.go_atoi(ov.tx.get(name, b""))
            a = a if ok else 0
            if int(v["tx_export"][k]) != a:
                bad.append((i, "tx." + name, a, int(v["tx_export"][k])))
        # observable captures (rules the compiler lists in its plan's
        # capture_rules; the others change no output and are not recorded)
        crules = getattr(res, "capture_rules", None)
        if crules is not None and getattr(res, "capture_recs", None) is not None:
            exp_c = [c for c in ov.captures if c[0] in crules]
            got_c = res.captures(i)
            trunc = bool(int(v["flags"]) & 0x40)  # GI_REQ_CAPTURE_TRUNC: the records are a prefix
            if (got_c != exp_c[:len(got_c)]) if trunc else (got_c != exp_c):
                bad.append((i, "captures", exp_c[:6], got_c[:6]))
        if len(bad) >= max_report:
            break
    return bad
