"""RuleSet cache store and its HTTP wire binding.

The operator aggregates a RuleSet's ConfigMaps, validates them and stores the
text in an in-memory, versioned cache that the data plane polls over HTTP.
This module restates that store and server so the GPU engine's poller
(`artifact.RulesetPoller`) can run against the same wire format, and so the
compiled GPU artifact (`artifact.entry`) is served beside `rules`, keyed by the
entry's UUID:

* `RuleSetCache` follows internal/rulesets/cache/cache.go:
  * `put` appends a new entry with a fresh UUID and timestamp and moves
    `latest` to it (cache.go:81-100);
  * `get` returns the entry whose UUID is `latest` (:63-78);
  * `prune(max_age)` drops entries older than `max_age` (:155-184) and
    `prune_by_size(max_size)` drops the oldest entries until the total
    `len(rules)` is under `max_size` (:186-231). Neither ever drops an
    instance's latest entry.
* `RuleSetCacheServer` follows server.go:
  * `GET /rules/<key>` returns the entry as JSON (:183-198);
  * `GET /rules/<key>/latest` returns `{uuid, timestamp}` (:163-181);
  * an empty key gives 400, an unknown key 404, and any method but GET 405
    (:143-161);
  * a GC thread runs age pruning, then size pruning, every `gc_interval`
    (:236-266).
* The artifact emitter hook: `RuleSetCache(emitter=...)` calls
  `emitter(rules) -> dict` on every `put` and stores the returned fields
  (`gpu_artifact`, `gpu_artifact_version`, `gpu_source_digest`, see
  `artifact.artifact_fields`) in the entry. This is the "compile once per
  RuleSet UUID" step of SURVEY §8f row 1 (ruleset_controller.go:158-181). An
  emitter that raises leaves the entry without an artifact, and the poller
  then recompiles `rules`.
"""

from __future__ import annotations

import datetime as _dt
import json
import threading
import time
import urllib.error
import urllib.request
import uuid as _uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable, Dict, List, Optional, Tuple

# server.go:29-50
CACHE_GC_INTERVAL = 5 * 60.0
CACHE_MAX_AGE = 24 * 3600.0
CACHE_MAX_SIZE = 100 * 1024 * 1024
MAX_HEADER_SIZE = 64 * 1024


def format_timestamp(ns: int) -> str:
    """Go `time.Time.Format(time.RFC3339Nano)` of a UTC instant given in
    nanoseconds since the epoch: trailing zeros of the fraction are dropped,
    and so is the fraction itself when it is zero; the zone is "Z"."""
    sec, frac = divmod(ns, 1_000_000_000)
    base = _dt.datetime.fromtimestamp(sec, _dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%S")
    if frac:
        base += "." + ("%09d" % frac).rstrip("0")
    return base + "Z"


def parse_timestamp(s: str) -> int:
    """Inverse of format_timestamp (RFC3339Nano in UTC) -> nanoseconds."""
    if not s.endswith("Z"):
        raise ValueError("timestamp not in UTC: %r" % s)
    body = s[:-1]
    frac = 0
    if "." in body:
        body, f = body.split(".", 1)
        if not f.isdigit() or len(f) > 9:
            raise ValueError("bad fraction in %r" % s)
        frac = int(f.ljust(9, "0"))
    t = _dt.datetime.strptime(body, "%Y-%m-%dT%H:%M:%S").replace(tzinfo=_dt.timezone.utc)
    return int(t.timestamp()) * 1_000_000_000 + frac


class RuleSetEntry:
    """cache.go:32-36 (`uuid`, `timestamp`, `rules`) plus the GPU artifact
    fields the emitter adds."""

    __slots__ = ("uuid", "timestamp_ns", "rules", "artifact")

    def __init__(self, uuid: str, timestamp_ns: int, rules: str, artifact: Optional[Dict] = None):
        self.uuid = uuid
        self.timestamp_ns = timestamp_ns
        self.rules = rules
        self.artifact = dict(artifact or {})

    @property
    def timestamp(self) -> str:
        return format_timestamp(self.timestamp_ns)

    def to_json(self) -> Dict:
        d = {"uuid": self.uuid, "timestamp": self.timestamp, "rules": self.rules}
        d.update(self.artifact)
        return d

    def size(self) -> int:
        """len(Rules), exactly as cache.go:113-124 (TotalSize) and
        cache.go:188-220 (PruneBySize) count an entry: the same SizeLimit
        prunes the same entries as the reference does."""
        return len(self.rules)

    def artifact_size(self) -> int:
        """Bytes of the GPU artifact's string fields stored beside the entry
        (not part of the reference's accounting: RuleSetCache.artifact_bytes)."""
        return sum(len(v) for v in self.artifact.values() if isinstance(v, (str, bytes)))


class RuleSetCache:
    """Thread-safe versioned RuleSet store (cache.go:46-231)."""

    def __init__(self, emitter: Optional[Callable[[str], Dict]] = None,
                 clock_ns: Callable[[], int] = time.time_ns):
        self._mu = threading.RLock()
        self._entries: Dict[str, Tuple[str, List[RuleSetEntry]]] = {}  # instance -> (latest uuid, oldest..newest)
        self._emitter = emitter
        self._clock = clock_ns
        self._last_ns = 0

    def _now(self) -> int:
        # strictly increasing: two Puts never share a timestamp (PutUpdatesUUID)
        t = max(self._clock(), self._last_ns + 1)
        self._last_ns = t
        return t

    def get(self, instance: str) -> Optional[RuleSetEntry]:
        with self._mu:
            got = self._entries.get(instance)
            if not got or not got[1]:
                return None
            latest, ents = got
            for e in ents:
                if e.uuid == latest:
                    return e
            return None

    def _artifact_of(self, instance: str, rules: str) -> Optional[Dict]:
        """The artifact of an entry of `instance` with the same rules text:
        the reconciler Puts on every reconcile (ruleset_controller.go:181),
        mostly with unchanged rules -- reused instead of recompiled."""
        with self._mu:
            got = self._entries.get(instance)
            for e in reversed(got[1] if got else []):
                if e.rules == rules and e.artifact:
                    return e.artifact
        return None

    def put(self, instance: str, rules: str) -> RuleSetEntry:
        art: Dict = {}
        if self._emitter is not None:
            prev = self._artifact_of(instance, rules)
            if prev is not None:
                art = prev
            else:
                try:
                    art = self._emitter(rules) or {}
                except Exception:  # noqa: BLE001 -- the entry is stored without an artifact
                    art = {}
        with self._mu:
            e = RuleSetEntry(str(_uuid.uuid4()), self._now(), rules, art)
            if instance not in self._entries:
                self._entries[instance] = (e.uuid, [e])
            else:
                self._entries[instance][1].append(e)
                self._entries[instance] = (e.uuid, self._entries[instance][1])
            return e

    def list_keys(self) -> List[str]:
        with self._mu:
            return list(self._entries)

    def total_size(self) -> int:
        """cache.go:113-124: the sum of len(Rules) over every stored entry."""
        with self._mu:
            return sum(e.size() for _, ents in self._entries.values() for e in ents)

    def artifact_bytes(self) -> int:
        """Memory the GPU artifacts hold, tracked apart from total_size (the
        reference has no artifact).  An artifact reused by several entries
        (unchanged rules, _artifact_of) is one object and counts once."""
        with self._mu:
            seen = {}  # the reused artifact's fields are the same string objects
            for _, ents in self._entries.values():
                for e in ents:
                    for v in e.artifact.values():
                        if isinstance(v, (str, bytes)):
                            seen[id(v)] = len(v)
            return sum(seen.values())

    def set_entry_timestamp(self, instance: str, index: int, timestamp_ns: int) -> None:
        with self._mu:
            got = self._entries.get(instance)
            if got and 0 <= index < len(got[1]):
                got[1][index].timestamp_ns = timestamp_ns

    def count_entries(self, instance: str) -> int:
        with self._mu:
            got = self._entries.get(instance)
            return len(got[1]) if got else 0

    def prune(self, max_age_s: float) -> int:
        """Drop entries older than max_age_s, never an instance's latest."""
        with self._mu:
            now = self._clock()
            max_ns = int(max_age_s * 1e9)
            pruned = 0
            for inst, (latest, ents) in list(self._entries.items()):
                keep = []
                for e in ents:
                    if e.uuid == latest or now - e.timestamp_ns <= max_ns:
                        keep.append(e)
                    else:
                        pruned += 1
                self._entries[inst] = (latest, keep)
            return pruned

    def prune_by_size(self, max_size: int) -> int:
        """cache.go:188-220: drop the oldest entries (instance by instance)
        until the total len(Rules) is at most max_size, never an instance's
        latest."""
        with self._mu:
            cur = sum(e.size() for _, ents in self._entries.values() for e in ents)
            if cur <= max_size:
                return 0
            pruned = 0
            for inst, (latest, ents) in list(self._entries.items()):
                if cur <= max_size:
                    break
                keep = []
                for e in ents:
                    if e.uuid == latest:
                        keep.append(e)
                    elif cur > max_size:
                        cur -= e.size()
                        pruned += 1
                    else:
                        keep.append(e)
                self._entries[inst] = (latest, keep)
            return pruned


class GarbageCollectionConfig:
    """server.go:205-226 (seconds instead of time.Duration)."""

    def __init__(self, gc_interval: float = CACHE_GC_INTERVAL, max_age: float = CACHE_MAX_AGE,
                 max_size: int = CACHE_MAX_SIZE):
        self.gc_interval = gc_interval
        self.max_age = max_age
        self.max_size = max_size


def handle(cache: RuleSetCache, method: str, path: str) -> Tuple[int, Dict[str, str], bytes]:
    """The `/rules/` handler as a pure function: (status, headers, body).
    server.go handleRules / handleLatest / handleGetRules."""
    if method != "GET":
        return 405, {"Content-Type": "text/plain; charset=utf-8"}, b"Method not allowed\n"
    if not path.startswith("/rules/"):
        return 404, {"Content-Type": "text/plain; charset=utf-8"}, b"404 page not found\n"
    key = path[len("/rules/"):]
    if key == "":
        return 400, {"Content-Type": "text/plain; charset=utf-8"}, b"RuleSet key required\n"
    latest = key.endswith("/latest")
    if latest:
        key = key[:-len("/latest")]
    e = cache.get(key)
    if e is None:
        return 404, {"Content-Type": "text/plain; charset=utf-8"}, b"RuleSet not found\n"
    body = {"uuid": e.uuid, "timestamp": e.timestamp} if latest else e.to_json()
    # json.NewEncoder(w).Encode appends a newline
    return 200, {"Content-Type": "application/json"}, (json.dumps(body) + "\n").encode()


class RuleSetCacheServer:
    """HTTP server over a RuleSetCache (server.go NewServer / Start / rungc)."""

    def __init__(self, cache: RuleSetCache, addr: Tuple[str, int] = ("127.0.0.1", 0),
                 gc: Optional[GarbageCollectionConfig] = None):
        self.cache = cache
        self.gc = gc or GarbageCollectionConfig()
        self._stop = threading.Event()
        outer = self

        class _H(BaseHTTPRequestHandler):
            def _serve(self):
                if sum(len(k) + len(v) for k, v in self.headers.items()) > MAX_HEADER_SIZE:
                    self.send_error(431)
                    return
                path = self.path.split("?", 1)[0]
                st, hdrs, body = handle(outer.cache, self.command, path)
                self.send_response(st)
                for k, v in hdrs.items():
                    self.send_header(k, v)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                if self.command != "HEAD":
                    self.wfile.write(body)

            do_GET = do_POST = do_PUT = do_DELETE = do_PATCH = do_HEAD = _serve

            def log_message(self, *a):  # quiet
                pass

        self._httpd = ThreadingHTTPServer(addr, _H)
        self._threads: List[threading.Thread] = []

    @property
    def address(self) -> Tuple[str, int]:
        return self._httpd.server_address[:2]

    @property
    def base_url(self) -> str:
        h, p = self.address
        return "http://%s:%d" % (h, p)

    def run_gc_once(self) -> Tuple[int, int]:
        """One GC tick (server.go rungc): age pruning, then size pruning when
        the cache is over max_size. Returns (pruned by age, pruned by size)."""
        by_age = self.cache.prune(self.gc.max_age)
        by_size = 0
        if self.cache.total_size() > self.gc.max_size:
            by_size = self.cache.prune_by_size(self.gc.max_size)
        return by_age, by_size

    def _gc_loop(self):
        while not self._stop.wait(self.gc.gc_interval):
            self.run_gc_once()

    def start(self) -> None:
        for fn in (self._httpd.serve_forever, self._gc_loop):
            th = threading.Thread(target=fn, daemon=True)
            th.start()
            self._threads.append(th)

    def stop(self) -> None:
        self._stop.set()
        self._httpd.shutdown()
        self._httpd.server_close()
        for th in self._threads:
            th.join(timeout=5)


def http_fetchers(base_url: str, key: str, timeout: float = 5.0):
    """(fetch_latest, fetch_entry) for artifact.RulesetPoller over the wire:
    GET <base>/rules/<key>/latest and GET <base>/rules/<key>. The entry must
    carry the UUID `/latest` named, else the cache moved on in between and the
    fetch raises (the poller retries on its next tick)."""

    def _get(path):
        with urllib.request.urlopen(base_url + path, timeout=timeout) as r:
            return json.loads(r.read().decode())

    def fetch_latest():
        return _get("/rules/%s/latest" % key)

    def fetch_entry(uuid: str):
        e = _get("/rules/%s" % key)
        if e["uuid"] != uuid:
            raise urllib.error.URLError("latest moved from %s to %s" % (uuid, e["uuid"]))
        return e

    return fetch_latest, fetch_entry
