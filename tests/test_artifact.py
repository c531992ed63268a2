"""GPU artifact (gi_ruleset_save / gi_ruleset_load) and hot swap.

CPU: round trips, corruption handling, the source digest, the poller's
reload logic.  GPU: an engine built from the
artifact is bit-exact with one built from the SecLang text, and hot swaps
follow the reference's reconcile KATs (test/integration/reconcile_test.go:
67-88).
"""
import json
import os

import pytest

import artifact
import gpuinspect
import traffic

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
KATS = {s["name"]: s for s in json.load(open(os.path.join(GOLDEN, "kats.json")))["scenarios"]}
TEXTS = {
    "samples": open(os.path.join(GOLDEN, "samples_ruleset.conf")).read(),
    "crs_pl1": open(os.path.join(ROOT, "rulesets", "crs_pl1.conf")).read(),
}


@pytest.mark.parametrize("name", sorted(TEXTS))
def test_artifact_round_trip(name):
    rs = gpuinspect.Ruleset(TEXTS[name])
    blob = rs.save()
    back = gpuinspect.Ruleset.load(blob)
    assert back.info == rs.info
    assert back.exports == rs.exports
    assert back.describe() == rs.describe()
    assert back.save() == blob  # deterministic, lossless
    assert rs.selftest_plan()[0] == 0 and back.selftest_plan()[0] == 0


def test_artifact_rejects_damage():
    blob = gpuinspect.Ruleset(TEXTS["samples"]).save()
    bad = [blob[:20], blob[:-8], b"XXXXXXXX" + blob[8:], blob + b"\0" * 8]
    flipped = bytearray(blob)
    flipped[len(blob) // 2] ^= 0x40
    bad.append(bytes(flipped))
    other = bytearray(blob)
    other[8] = 99  # version
    bad.append(bytes(other))
    for b in bad:
        with pytest.raises(gpuinspect.SecLangError, match="invalid GPU artifact"):
            gpuinspect.Ruleset.load(b)


def _sections(blob):
    """{tag: (payload offset of the records, elem size, count)} of an artifact
    (csrc/artifact.cpp layout: 40-byte header, then tag/esz/count sections)."""
    import struct
    out, off = {}, 40
    nsec = struct.unpack_from("<I", blob, 12)[0]
    for _ in range(nsec):
        tag, esz, cnt = struct.unpack_from("<IIQ", blob, off)
        off += 16
        out[tag] = (off, esz, cnt)
        off += (esz * cnt + 7) & ~7
    return out


def _reseal(buf):
    import struct
    struct.pack_into("<Q", buf, 24, artifact.fnv64(bytes(buf[40:])))
    return bytes(buf)


_BLOBS = {}


def _crs_blob():
    if "crs" not in _BLOBS:
        _BLOBS["crs"] = gpuinspect.Ruleset(TEXTS["crs_pl1"]).save()
    return _BLOBS["crs"]


# (section tag, record index, byte offset in the record, u32 value) -> an index
# or offset some kernel dereferences, pushed outside its table
_CORRUPT = [
    (1, 0, 24, 0xFFFF0000),   # DRule.var_begin
    (1, 0, 32, 0x7FFF0000),   # DRule.op
    (1, 0, 56, 0x7FFF0000),   # DRule.hit_slot
    (1, 0, 12, 0x7FFF0000),   # DRule.chain_next
    (2, 0, 0, 0x7FFF0000),    # top-level rule index
    (5, 0, 4, 0x7FFF0000),    # DOp.dfa
    (10, 0, 16, 0xFFFF0000),  # DDfa.trans_off
    (10, 0, 0, 0x00FFFFFF),   # DDfa.n_states
    (11, 0, 0, 0x7FFF7FFF),   # transition targets
    (22, 0, 4, 0xFFFF0000),   # DJob.img_off
    (22, 0, 0, 0x7FFF0000),   # DJob.stream
    (23, 0, 0, 0x7FFF0000),   # DJobDfa.dfa
    (24, 0, 0, 0x7FFF0000),   # DPat.slot
    (17, 0, 16, 0x7FFF0000),  # DStream.job_begin
    (19, 0, 0, 0x000000FF),   # stream filter id (u8 section: whole first word)
    (27, 0, 0, 0x7FFF0000),   # export slot
]


@pytest.mark.parametrize("case", _CORRUPT, ids=["%d.%d+%d" % c[:3] for c in _CORRUPT])
def test_artifact_rejects_out_of_range_records(case):
    """A checksummed but malformed artifact is rejected before any kernel sees
    it: every index / offset a kernel dereferences is bounds-checked
    (csrc/artifact.cpp validate_program)."""
    import struct
    blob = _crs_blob()
    tag, rec, at, val = case
    off, esz, cnt = _sections(blob)[tag]
    assert cnt > rec
    buf = bytearray(blob)
    if esz == 1:
        buf[off + rec] = val & 0xFF
    else:
        struct.pack_into("<I", buf, off + rec * esz + at, val)
    with pytest.raises(gpuinspect.SecLangError, match="invalid GPU artifact"):
        gpuinspect.Ruleset.load(_reseal(buf))


def test_artifact_rejects_capture_flag_without_program():
    """RF_CAPTURE on a link without a capture program would make k_eval read
    P.pikes[-1]: the loader refuses it."""
    import struct
    blob = _crs_blob()
    off, esz, cnt = _sections(blob)[1]  # DRule records (64 B)
    assert esz == 64
    for i in range(cnt):
        op = struct.unpack_from("<i", blob, off + i * esz + 32)[0]
        flags = blob[off + i * esz + 54]
        if op >= 0 and not flags & 4:
            break
    else:
        pytest.fail("no operator rule without capture")
    buf = bytearray(blob)
    buf[off + i * esz + 54] |= 4  # RF_CAPTURE
    with pytest.raises(gpuinspect.SecLangError, match="invalid GPU artifact"):
        gpuinspect.Ruleset.load(_reseal(buf))


def test_artifact_other_compiler_revision():
    blob = gpuinspect.Ruleset(TEXTS["samples"]).save()
    off, esz, _ = _sections(blob)[100]  # scalars: compiler_rev is the last u64
    buf = bytearray(blob)
    buf[off + esz - 1] ^= 0x5A
    with pytest.raises(gpuinspect.SecLangError, match="compiler revision"):
        gpuinspect.Ruleset.load(_reseal(buf))
    assert gpuinspect.compiler_rev()


def test_source_digest():
    rs = gpuinspect.Ruleset(TEXTS["samples"])
    assert rs.info["source_digest"] == artifact.source_digest(TEXTS["samples"])
    assert artifact.source_digest(TEXTS["samples"] + "\n") != rs.info["source_digest"]
    e = artifact.entry("u1", "2026-01-01T00:00:00Z", TEXTS["samples"], rs)
    assert set(e) >= {"uuid", "timestamp", "rules", "gpu_artifact"}
    assert artifact.ruleset_from_entry(e).text is None  # loaded, not recompiled
    stale = dict(e, rules=TEXTS["samples"] + "\n")
    assert artifact.ruleset_from_entry(stale).text == stale["rules"]  # digest mismatch: recompiled
    broken = dict(e, gpu_artifact=e["gpu_artifact"][:-16] + "A" * 16)
    assert artifact.ruleset_from_entry(broken).text == e["rules"]


class _FakeEngine:
    def __init__(self):
        self.swaps = []

    def swap(self, rs):
        self.swaps.append(rs)


def test_poller_reloads_on_new_uuid():
    store = {}
    latest = {"uuid": None}

    def put(uuid, rules):
        store[uuid] = artifact.entry(uuid, "t", rules)
        latest["uuid"] = uuid

    eng = _FakeEngine()
    p = artifact.RulesetPoller(eng, lambda: dict(latest, timestamp="t"), lambda u: store[u])
    put("a", "\n".join(KATS["reconcile_initial"]["configmaps"]))
    assert p.poll() and p.loaded_from_artifact and len(eng.swaps) == 1
    assert not p.poll() and len(eng.swaps) == 1  # same UUID: nothing to do
    put("b", "\n".join(KATS["reconcile_add_sinister"]["configmaps"]))
    assert p.poll() and p.uuid == "b" and len(eng.swaps) == 2
    assert eng.swaps[0].info["n_rules"] == 1 and eng.swaps[-1].info["n_rules"] == 2


PMF = 'SecRule ARGS "@pmFromFile bad.data" "id:7,phase:2,deny,status:403"'


def test_poller_pmfromfile_entry():
    """A ruleset with @pmFromFile: the data files are part of the digest, so the
    artifact is used when the poller holds the same files and a recompile with
    those files happens otherwise (never a SecLangError inside poll)."""
    files = {"bad.data": b"evilmonkey\nsinister\n"}
    e = artifact.entry("u1", "t", PMF, data_files=files)
    assert artifact.ruleset_from_entry(e, data_files=files).text is None
    other = {"bad.data": b"maniacal\n"}
    assert artifact.ruleset_from_entry(e, data_files=other).text == PMF
    eng = _FakeEngine()
    p = artifact.RulesetPoller(eng, lambda: {"uuid": "u1", "timestamp": "t"}, lambda u: e, data_files=files)
    assert p.poll() and p.loaded_from_artifact
    assert eng.swaps[0].info["source_digest"] == artifact.source_digest(PMF, data_files=files)


def _tx(uri):
    t = gpuinspect.Transaction(method=b"GET", uri=uri.encode())
    t.add_request_header("Host", "example.com")
    return t


@pytest.mark.gpu
def test_gpu_artifact_bit_exact():
    text = TEXTS["crs_pl1"]
    a = gpuinspect.Ruleset(text)
    b = gpuinspect.Ruleset.load(a.save())
    batch = traffic.TrafficGen(traffic.SEED + 5).batch(600, post_frac=0.3, attack_rate=0.3)
    ra = gpuinspect.Engine(a, matched_cap=128).inspect(batch)
    rb = gpuinspect.Engine(b, matched_cap=128).inspect(batch)
    assert (ra.verdicts == rb.verdicts).all()
    assert all(ra.matched_rules(i) == rb.matched_rules(i) for i in range(batch.n_req))
    assert int((ra.verdicts["action"] != 0).sum()) > 20


@pytest.mark.gpu
def test_gpu_hot_swap_reconcile_kats():
    """reconcile_test.go:67-88 through one engine, swapped per RuleSet update."""
    store, latest = {}, {"uuid": None}
    steps = ["reconcile_initial", "reconcile_add_sinister", "reconcile_replace_maniacal"]
    first = gpuinspect.Ruleset("\n".join(KATS[steps[0]]["configmaps"]))
    eng = gpuinspect.Engine(first)
    poller = artifact.RulesetPoller(eng, lambda: dict(latest, timestamp="t"), lambda u: store[u])
    for i, name in enumerate(steps):
        sc = KATS[name]
        uuid = "uuid-%d" % i
        store[uuid] = artifact.entry(uuid, "t", "\n".join(sc["configmaps"]))
        latest["uuid"] = uuid
        assert poller.poll() and poller.loaded_from_artifact
        res = eng.inspect(gpuinspect.pack([_tx(r["uri"]) for r in sc["requests"]]))
        for k, r in enumerate(sc["requests"]):
            it = res.interruption(k)
            assert (it["status"] if it else 200) == r["expect_status"], (name, r["uri"], it)
