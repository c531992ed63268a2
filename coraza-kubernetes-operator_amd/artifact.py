"""GPU artifact next to the RuleSet cache entry, and the data plane's hot swap.

SURVEY §8f rows 1 and 4.

* Artifact emitter.  The operator compiles a RuleSet once per cache entry
  (next to `r.Cache.Put(cacheKey, aggregatedRules.String())`,
  internal/controller/ruleset_controller.go:179-181).  It serves the compiled
  program (gi_ruleset_save) beside the entry's `rules`.
  * `entry()` builds that JSON object: RuleSetEntry's fields `uuid`,
    `timestamp`, `rules` (internal/rulesets/cache/cache.go:32-36; JSON names
    from server.go:35) plus `gpu_artifact` (base64), `gpu_artifact_version`
    and `gpu_source_digest`.
* Hot swap.  The data plane polls `GET /rules/<key>/latest` and reloads when
  the UUID changes (server.go:163-181; pollIntervalSeconds,
  config/samples/engine.yaml:18; KATs reconcile_test.go:72-88).
  * `RulesetPoller.poll()` does the same against any fetch functions.
  * It loads the artifact when it matches the entry's rules (source digest +
    version), recompiles `rules` otherwise, and swaps the engine's program
    with gi_ctx_swap_ruleset.
"""

from __future__ import annotations

import base64
from typing import Callable, Dict, Optional, Sequence

import gpuinspect

ARTIFACT_VERSION = 5  # csrc/artifact.h kArtifactVersion


def fnv64(data: bytes, h: int = 1469598103934665603) -> int:
    for c in data:
        h = ((h ^ c) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def source_digest(rules: str, exports: Sequence[str] = gpuinspect.DEFAULT_EXPORTS,
                  data_files: Optional[Dict[str, bytes]] = None) -> int:
    """The digest gi_compile stores in the artifact (runtime.cpp gi_compile):
    the rules text, the export list, the compiler revision and the
    @pmFromFile data files (by name, in the order Ruleset passes them)."""
    data = rules.encode() + b"".join(b"\0export:" + e.encode() for e in exports)
    data += b"\0compiler:" + gpuinspect.compiler_rev().encode()
    for name, body in sorted((data_files or {}).items()):
        data += b"\0file:" + name.encode() + b"\0" + bytes(body)
    return fnv64(data)


def artifact_fields(rules: str, ruleset: Optional[gpuinspect.Ruleset] = None,
                    data_files: Optional[Dict[str, bytes]] = None) -> Dict:
    """The GPU artifact of `rules` as the fields an entry carries beside
    `rules` (the emitter cache.RuleSetCache calls on every Put)."""
    rs = ruleset if ruleset is not None else gpuinspect.Ruleset(rules, data_files=data_files)
    return {"gpu_artifact": base64.b64encode(rs.save()).decode(),
            "gpu_artifact_version": ARTIFACT_VERSION,
            "gpu_source_digest": "%016x" % rs.info["source_digest"]}


def entry(uuid: str, timestamp: str, rules: str, ruleset: Optional[gpuinspect.Ruleset] = None,
          data_files: Optional[Dict[str, bytes]] = None) -> Dict:
    """RuleSetEntry JSON plus the GPU artifact of `rules`."""
    e = {"uuid": uuid, "timestamp": timestamp, "rules": rules}
    e.update(artifact_fields(rules, ruleset, data_files))
    return e


def ruleset_from_entry(e: Dict, exports: Sequence[str] = gpuinspect.DEFAULT_EXPORTS,
                       data_files: Optional[Dict[str, bytes]] = None) -> gpuinspect.Ruleset:
    """The entry's program: its artifact if it belongs to `rules` (and to the
    data files the poller holds), else a compile of `rules`."""
    art = e.get("gpu_artifact")
    want = source_digest(e["rules"], exports, data_files)
    if art and e.get("gpu_artifact_version") == ARTIFACT_VERSION and \
            e.get("gpu_source_digest") == "%016x" % want:
        try:
            rs = gpuinspect.Ruleset.load(base64.b64decode(art))
            if rs.info["source_digest"] == want:
                return rs
        except gpuinspect.SecLangError:
            pass  # corrupted / other build: recompile below
    return gpuinspect.Ruleset(e["rules"], tx_exports=exports, data_files=data_files)


class RulesetPoller:
    """Reloads an engine's ruleset when the cache's latest UUID changes."""

    def __init__(self, engine, fetch_latest: Callable[[], Dict], fetch_entry: Callable[[str], Dict],
                 exports: Sequence[str] = gpuinspect.DEFAULT_EXPORTS,
                 data_files: Optional[Dict[str, bytes]] = None):
        """data_files: the @pmFromFile files the rules name ({name: bytes});
        they are part of the artifact's source digest and of a recompile."""
        self.engine = engine
        self.fetch_latest = fetch_latest  # -> {"uuid", "timestamp"} (handleLatest)
        self.fetch_entry = fetch_entry    # uuid -> entry() (handleGetRules)
        self.exports = tuple(exports)
        self.data_files = dict(data_files or {})
        self.uuid: Optional[str] = None
        self.ruleset: Optional[gpuinspect.Ruleset] = None
        self.loaded_from_artifact = False

    def poll(self) -> bool:
        """True when a new ruleset was swapped in."""
        latest = self.fetch_latest()
        if latest["uuid"] == self.uuid:
            return False
        e = self.fetch_entry(latest["uuid"])
        rs = ruleset_from_entry(e, self.exports, self.data_files)
        self.loaded_from_artifact = rs.text is None
        self.engine.swap(rs)
        self.ruleset = rs  # the engine borrows it: keep it alive
        self.uuid = latest["uuid"]
        return True
