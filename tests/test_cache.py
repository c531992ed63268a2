"""RuleSet cache store + HTTP wire binding.

Each test replays the assertions of the reference's own Go tests:
internal/rulesets/cache/cache_test.go:29-241 and server_test.go:73-336.
The last tests run the GPU engine's poller against the real HTTP server
(the engine is a stand-in that records swaps: no GPU is needed to check the
wire path; tests/test_artifact.py swaps a real engine on the GPU).
"""
import json
import threading
import time
import urllib.error
import urllib.request

import pytest

import artifact
import cache as C
import gpuinspect

HOUR = 3600e9


def test_put_and_get():  # cache_test.go:29-70
    c = C.RuleSetCache()
    for inst, rules in [("test-instance", 'SecRule REQUEST_URI "@contains /admin" "id:1,deny"'),
                        ("empty-instance", ""),
                        ("multi-instance", 'SecRule REQUEST_URI "@contains /admin" "id:1,deny"\n'
                                           'SecRule REQUEST_URI "@contains /api" "id:2,deny"')]:
        c.put(inst, rules)
        e = c.get(inst)
        assert e is not None
        assert e.rules == rules
        assert e.uuid
        assert e.timestamp_ns > 0


def _now():
    return time.time_ns()


PRUNE_CASES = [
    # name, setup, max_age (s) or None, max_size or None, expected count or None, verify
    ("prune old entries by age",
     lambda c: (c.put("instance1", "old-rules"), c.put("instance1", "new-rules"), c.put("instance2", "rules2"),
                c.set_entry_timestamp("instance1", 0, _now() - int(25 * HOUR))),
     24 * 3600, None, 1, lambda c: c.get("instance1").rules == "new-rules"),
    ("prune nothing when all entries are recent",
     lambda c: (c.put("instance1", "rules1"), c.put("instance2", "rules2")), 48 * 3600, None, 0, None),
    ("prune by size",
     lambda c: (c.put("instance1", "rules1"), c.put("instance1", "new1"), c.put("instance2", "rules2"),
                c.put("instance2", "new2"), c.put("instance3", "rules3"),
                c.set_entry_timestamp("instance1", 0, _now() - int(2 * HOUR)),
                c.set_entry_timestamp("instance2", 0, _now() - int(1 * HOUR))),
     None, 20, None,
     lambda c: c.total_size() <= 20 and all(c.get("instance%d" % i) for i in (1, 2, 3))),
    ("prune by size under limit does nothing",
     lambda c: (c.put("instance1", "rules1"), c.put("instance2", "rules2")), None, 1000, 0, None),
    ("never prune latest entry by age",
     lambda c: (c.put("instance1", "v1"), c.put("instance1", "v2"), c.put("instance1", "v3"),
                [c.set_entry_timestamp("instance1", i, _now() - int(48 * HOUR)) for i in range(3)]),
     24 * 3600, None, 2, lambda c: c.get("instance1").rules == "v3"),
    ("never prune latest entry by size",
     lambda c: (c.put("instance1", "small"), c.put("instance1", "medium-size"),
                c.put("instance1", "this-is-a-much-larger-entry")),
     None, 1, 2, lambda c: c.get("instance1").rules == "this-is-a-much-larger-entry"),
]


@pytest.mark.parametrize("case", PRUNE_CASES, ids=[c[0] for c in PRUNE_CASES])
def test_pruning(case):  # cache_test.go:72-205
    _, setup, max_age, max_size, want, verify = case
    c = C.RuleSetCache()
    setup(c)
    pruned = c.prune_by_size(max_size) if max_size else c.prune(max_age)
    if want is not None:
        assert pruned == want
    if verify is not None:
        assert verify(c)


def test_list_keys_total_size_count():  # cache_test.go:207-229
    c = C.RuleSetCache()
    assert c.list_keys() == []
    for i in (1, 2, 3):
        c.put("instance%d" % i, "rules%d" % i)
    assert sorted(c.list_keys()) == ["instance1", "instance2", "instance3"]
    c = C.RuleSetCache()
    assert c.total_size() == 0
    c.put("instance1", "12345")
    c.put("instance2", "1234567890")
    assert c.total_size() == 15
    c.put("instance1", "123")
    assert c.total_size() == 18
    assert c.count_entries("instance1") == 2 and c.count_entries("nope") == 0


def test_put_updates_uuid_and_get_missing():  # cache_test.go:231-256
    c = C.RuleSetCache()
    c.put("test-instance", "rules v1")
    e1 = c.get("test-instance")
    c.put("test-instance", "rules v2")
    e2 = c.get("test-instance")
    assert e1.uuid != e2.uuid
    assert e1.timestamp_ns != e2.timestamp_ns
    assert e2.rules == "rules v2"
    assert c.get("non-existent") is None


def test_timestamp_format_rfc3339nano():
    assert C.format_timestamp(0) == "1970-01-01T00:00:00Z"
    assert C.format_timestamp(1_500_000_000_120_000_000) == "2017-07-14T02:40:00.12Z"
    assert C.format_timestamp(1_500_000_000_000_000_001) == "2017-07-14T02:40:00.000000001Z"
    for ns in (0, 1, 1_700_000_000_123_456_789, 1_700_000_000_100_000_000):
        assert C.parse_timestamp(C.format_timestamp(ns)) == ns


# ------------------------------------------------------------- handlers
def test_handle_get_rules_and_latest():  # server_test.go:73-156
    c = C.RuleSetCache()
    rules = 'SecRule REQUEST_URI "@contains /admin" "id:1,deny"'
    c.put("test-instance", rules)
    st, hdrs, body = C.handle(c, "GET", "/rules/test-instance")
    assert st == 200 and hdrs["Content-Type"] == "application/json"
    e = json.loads(body)
    assert e["uuid"] and e["timestamp"] and e["rules"] == rules
    st, hdrs, body = C.handle(c, "GET", "/rules/test-instance/latest")
    assert st == 200 and hdrs["Content-Type"] == "application/json"
    lt = json.loads(body)
    assert set(lt) == {"uuid", "timestamp"}
    C.parse_timestamp(lt["timestamp"])  # RFC3339Nano
    assert lt["uuid"] == e["uuid"] and lt["timestamp"] == e["timestamp"]


def test_handle_errors():  # server_test.go:293-336
    c = C.RuleSetCache()
    assert C.handle(c, "GET", "/rules/non-existent")[0] == 404
    assert C.handle(c, "GET", "/rules/")[0] == 400
    assert C.handle(c, "GET", "/rules/non-existent/latest")[0] == 404
    for m in ("POST", "PUT", "DELETE", "PATCH"):
        assert C.handle(c, m, "/rules/test-instance")[0] == 405


def _wait(pred, timeout=5.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return True
        time.sleep(0.02)
    return pred()


def test_server_gc_by_age():  # server_test.go:158-207
    c = C.RuleSetCache()
    srv = C.RuleSetCacheServer(c, gc=C.GarbageCollectionConfig(0.05, 0.1, 1 << 30))
    srv.start()
    try:
        c.put("instance1", "instance1 old")
        c.put("instance1", "instance1 new")
        c.put("instance2", "instance2 old")
        c.put("instance2", "instance2 new")
        c.put("instance3", "only version")
        c.set_entry_timestamp("instance1", 0, _now() - 200_000_000)
        c.set_entry_timestamp("instance2", 0, _now() - 200_000_000)
        c.set_entry_timestamp("instance3", 0, _now() - 50_000_000)
        assert _wait(lambda: c.count_entries("instance1") == 1 and c.count_entries("instance2") == 1)
        assert c.get("instance1").rules == "instance1 new"
        assert c.get("instance2").rules == "instance2 new"
        assert c.get("instance3").rules == "only version"
        assert c.count_entries("instance3") == 1
    finally:
        srv.stop()


def test_server_gc_by_size():  # server_test.go:209-269
    c = C.RuleSetCache()
    srv = C.RuleSetCacheServer(c, gc=C.GarbageCollectionConfig(0.05, 24 * 3600, 50))
    c.put("instance1", "instance1 old - 27 chars...")
    c.put("instance1", "instance1 new - 27 chars...")
    c.put("instance2", "instance2 old - 27 chars...")
    c.put("instance2", "instance2 new - 27 chars...")
    c.put("instance3", "instance3 - 25 characters..")
    large = "This is a large ruleset that exceeds the max size limit by itself"
    c.put("instance4", large)
    size0 = c.total_size()
    count = lambda: sum(c.count_entries("instance%d" % i) for i in (1, 2, 3, 4))  # noqa: E731
    assert size0 > 50 and count() == 6
    srv.start()
    try:
        assert _wait(lambda: count() == 4)
        assert c.get("instance1").rules == "instance1 new - 27 chars..."
        assert c.get("instance2").rules == "instance2 new - 27 chars..."
        assert c.get("instance3").rules == "instance3 - 25 characters.."
        assert c.get("instance4").rules == large
        assert c.total_size() < size0
        assert c.total_size() > 50  # the latest entries alone exceed the limit
    finally:
        srv.stop()


def test_server_gc_empty_cache():  # server_test.go:271-291
    c = C.RuleSetCache()
    srv = C.RuleSetCacheServer(c, gc=C.GarbageCollectionConfig(0.02, 0.1, 10))
    srv.start()
    time.sleep(0.1)
    srv.stop()
    assert c.total_size() == 0 and c.list_keys() == []


def _http(url, method="GET"):
    req = urllib.request.Request(url, method=method)
    try:
        with urllib.request.urlopen(req, timeout=5) as r:
            return r.status, r.headers.get("Content-Type"), r.read()
    except urllib.error.HTTPError as e:
        return e.code, e.headers.get("Content-Type"), e.read()


def test_server_over_http():
    c = C.RuleSetCache()
    srv = C.RuleSetCacheServer(c)
    srv.start()
    try:
        base = srv.base_url
        assert _http(base + "/rules/x")[0] == 404
        assert _http(base + "/rules/")[0] == 400
        assert _http(base + "/rules/x", "POST")[0] == 405
        c.put("ns/name", "SecRule ARGS \"@contains evil\" \"id:1,phase:2,deny,status:403\"")
        st, ct, body = _http(base + "/rules/ns/name")
        assert st == 200 and ct == "application/json" and body.endswith(b"\n")
        e = json.loads(body)
        st, _, body = _http(base + "/rules/ns/name/latest")
        assert st == 200 and json.loads(body) == {"uuid": e["uuid"], "timestamp": e["timestamp"]}
    finally:
        srv.stop()


class _RecordingEngine:
    def __init__(self):
        self.swaps = []

    def swap(self, rs):
        self.swaps.append(rs)


def test_poller_against_server_with_artifact_emitter():
    """The operator's Put emits the GPU artifact beside `rules`; the data
    plane's poller fetches /latest and the entry over HTTP, loads the artifact
    (no recompile) and swaps it in; a new Put is picked up on the next poll
    (reconcile_test.go:72-88 shape)."""
    gpuinspect.load_library()
    c = C.RuleSetCache(emitter=artifact.artifact_fields)
    srv = C.RuleSetCacheServer(c)
    srv.start()
    try:
        rule = 'SecRule ARGS|REQUEST_URI|REQUEST_HEADERS "@contains %s" "id:%d,phase:2,deny,status:403"'
        c.put("default/ruleset", rule % ("evilmonkey", 3001))
        e = json.loads(_http(srv.base_url + "/rules/default/ruleset")[2])
        assert e["gpu_artifact_version"] == artifact.ARTIFACT_VERSION and e["gpu_artifact"]
        eng = _RecordingEngine()
        p = artifact.RulesetPoller(eng, *C.http_fetchers(srv.base_url, "default/ruleset"))
        assert p.poll() and p.loaded_from_artifact and p.uuid == e["uuid"]
        assert not p.poll()  # same UUID: no reload
        c.put("default/ruleset", rule % ("evilmonkey", 3001) + "\n" + rule % ("sinistermonkey", 3002))
        assert p.poll() and p.loaded_from_artifact and len(eng.swaps) == 2
        assert p.ruleset.info["n_rules"] == 2
        # an entry whose emitter failed carries no artifact: the poller recompiles
        bad = C.RuleSetCache(emitter=lambda rules: 1 / 0)
        bad.put("k", rule % ("x", 1))
        assert "gpu_artifact" not in bad.get("k").to_json()
    finally:
        srv.stop()


def test_cache_concurrent_put_get():
    c = C.RuleSetCache()
    errs = []

    def worker(k):
        try:
            for i in range(200):
                c.put("i%d" % k, "r%d" % i)
                assert c.get("i%d" % k) is not None
                c.prune_by_size(1000)
        except Exception as ex:  # noqa: BLE001
            errs.append(ex)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs
    assert all(c.get("i%d" % k).rules == "r199" for k in range(4))


def test_artifact_reused_for_unchanged_rules_and_counted_apart():
    """A reconcile with unchanged rules (ruleset_controller.go:181 Puts every
    time) reuses the stored artifact instead of recompiling.  Sizes follow the
    reference: total_size / prune_by_size count len(Rules) only
    (cache.go:113-124, 188-220); the artifacts' memory is tracked apart, a
    shared artifact once."""
    calls = []

    def emitter(rules):
        calls.append(rules)
        return {"gpu_artifact": rules.ljust(100, "A"), "gpu_artifact_version": 1}

    c = C.RuleSetCache(emitter=emitter)
    a = c.put("ns/r", "rules-v1")
    b = c.put("ns/r", "rules-v1")
    assert a.uuid != b.uuid and b.artifact == a.artifact and calls == ["rules-v1"]
    c.put("ns/r", "rules-v2")
    assert calls == ["rules-v1", "rules-v2"]
    assert c.total_size() == 3 * 8
    assert c.artifact_bytes() == 2 * 100  # v1's artifact is shared by two entries
    # the reference's SizeLimit semantics: 24 bytes of rules fit 24, 8 prunes the two old entries
    assert c.prune_by_size(24) == 0
    assert c.prune_by_size(8) == 2 and c.count_entries("ns/r") == 1
    assert c.artifact_bytes() == 100
    # another instance with the same text compiles its own (no cross-instance sharing)
    c.put("ns/other", "rules-v2")
    assert calls[-1] == "rules-v2" and len(calls) == 3
