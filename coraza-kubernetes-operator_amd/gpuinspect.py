"""Python host binding of the gpuinspect C ABI (include/gpuinspect.h).

Mirrors the shape of the reference's interfaces for this path:

* `Ruleset(text)`  <->  `coraza.NewWAF(coraza.NewWAFConfig().WithDirectives(text))`
  (/root/reference/internal/controller/ruleset_controller.go:159-160).  A
  SecLang error raises `SecLangError` carrying the compiler message, the way
  the controller surfaces it in the RuleSet status (:161-170).
* `Transaction`    <->  coraza's `types.Transaction` as driven by
  coraza-proxy-wasm: `process_uri`, `add_request_header`,
  `write_request_body`; the whole batch is evaluated by `Engine.inspect`,
  which runs ProcessRequestHeaders (phase 1) + ProcessRequestBody (phase 2)
  on the GPU and returns per-request `interruption` / `matched_rules`.
* `aggregate_configmaps(texts)` <-> the RuleSet controller's join of the
  ConfigMap `rules` strings with "\\n" (ruleset_controller.go:173-176).

There is deliberately no CPU fallback: without the HIP library or a GPU
every inspection call raises.
"""

from __future__ import annotations

import ctypes
import json
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GI_LIB") or os.path.join(HERE, "libgpuinspect.so")  # GI_LIB: A/B builds

GI_OK = 0
GI_EPARSE = -1
GI_EUNSUPPORTED = -2
GI_EINVAL = -3
GI_ENODEV = -4
GI_ENOMEM = -5
GI_ETRUNC = -6
GI_ESTATE = -7

GI_REQ_UNSUPPORTED_URI = 0x1
GI_REQ_UNSUPPORTED_BODY = 0x2
GI_REQ_BODY_LIMIT = 0x4
GI_REQ_OVERFLOW = 0x8
GI_REQ_MATCH_TRUNC = 0x10
GI_REQ_BODY_ERROR = 0x20
GI_REQ_CAPTURE_TRUNC = 0x40
GI_REQ_ERROR_MASK = 0x0F

ACTIONS = {0: "", 1: "deny", 2: "drop", 3: "redirect"}
MAX_EXPORTS = 8
STATS_LAUNCHES = 48  # include/gpuinspect.h GI_STATS_LAUNCHES

SPAN_DT = np.dtype([("off", "<u8"), ("len", "<u4"), ("_pad", "<u4")])
REQUEST_DT = np.dtype([("method", SPAN_DT), ("uri", SPAN_DT), ("proto", SPAN_DT), ("body", SPAN_DT),
                       ("hdr_begin", "<u4"), ("hdr_count", "<u4"), ("remote_addr", SPAN_DT),
                       ("remote_port", "<u4"), ("_pad", "<u4"), ("server_name", SPAN_DT)])
HEADER_DT = np.dtype([("name", SPAN_DT), ("value", SPAN_DT)])
VERDICT_DT = np.dtype([("rule_id", "<i4"), ("status", "<i4"), ("action", "u1"), ("phase", "u1"),
                       ("flags", "<u2"), ("match_cnt", "<u4"), ("tx_export", "<i8", (MAX_EXPORTS,)),
                       ("capture_cnt", "<u4"), ("_pad", "<u4")])
CAPTURE_DT = np.dtype([("rule_id", "<i4"), ("group", "<u4"), ("off", "<u4"), ("len", "<u4")])
assert REQUEST_DT.itemsize == 112 and HEADER_DT.itemsize == 32 and VERDICT_DT.itemsize == 88

EXPORTED_SYMBOLS = (
    "gi_abi_version", "gi_cpu_baseline_inspect", "gi_compile", "gi_ruleset_free", "gi_ruleset_info_get", "gi_ruleset_export_name", "gi_ruleset_describe",
    "gi_ctx_create", "gi_ctx_free", "gi_last_error", "gi_inspect_batch", "gi_stage_batch",
    "gi_run_staged", "gi_sync", "gi_fetch_results", "gi_tally_get", "gi_stats_get",
    "gi_ctx_stream", "gi_selftest_regex", "gi_selftest_plan", "gi_selftest_triggers",
    "gi_ruleset_save", "gi_ruleset_load", "gi_ctx_swap_ruleset", "gi_compiler_rev", "gi_tally_detail_get", "gi_selftest_regex_many",
    "gi_ctx_set_capture_cap", "gi_selftest_capture", "gi_host_register", "gi_host_unregister",
)
SCORE_BINS = 64  # GI_SCORE_BINS


class SecLangError(ValueError):
    """Rule text the engine rejects (code GI_EPARSE or GI_EUNSUPPORTED)."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


class EngineError(RuntimeError):
    pass


class _CompileOpts(ctypes.Structure):
    _fields_ = [("tx_exports", ctypes.POINTER(ctypes.c_char_p)), ("dfa_state_cap", ctypes.c_uint32),
                ("n_data_files", ctypes.c_uint32), ("data_file_names", ctypes.POINTER(ctypes.c_char_p)),
                ("data_file_data", ctypes.POINTER(ctypes.c_char_p)), ("data_file_lens", ctypes.POINTER(ctypes.c_size_t))]


class _Info(ctypes.Structure):
    _fields_ = [("n_rules", ctypes.c_uint32), ("n_links", ctypes.c_uint32), ("n_dfas", ctypes.c_uint32),
                ("n_tx_slots", ctypes.c_uint32), ("program_bytes", ctypes.c_uint64),
                ("n_scan_jobs", ctypes.c_uint32), ("n_hit_slots", ctypes.c_uint32),
                ("n_union_dfas", ctypes.c_uint32), ("n_scan_streams", ctypes.c_uint32), ("n_nfas", ctypes.c_uint32),
                ("source_digest", ctypes.c_uint64)]


class _Batch(ctypes.Structure):
    _fields_ = [("n_req", ctypes.c_uint32), ("data", ctypes.c_void_p), ("data_len", ctypes.c_uint64),
                ("reqs", ctypes.c_void_p), ("headers", ctypes.c_void_p), ("n_headers", ctypes.c_uint32)]


class _Results(ctypes.Structure):
    _fields_ = [("verdicts", ctypes.c_void_p), ("matched_ids", ctypes.c_void_p), ("matched_cap", ctypes.c_uint32),
                ("captures", ctypes.c_void_p), ("capture_bytes", ctypes.c_void_p), ("capture_cap", ctypes.c_uint32),
                ("capture_bytes_cap", ctypes.c_uint32)]


class _Tally(ctypes.Structure):
    _fields_ = [("n_req", ctypes.c_uint64), ("n_interrupted", ctypes.c_uint64),
                ("n_matched_any", ctypes.c_uint64), ("n_error", ctypes.c_uint64),
                ("bytes_scanned", ctypes.c_uint64), ("matched_total", ctypes.c_uint64),
                ("n_pa_void", ctypes.c_uint64)]


class _Stats(ctypes.Structure):
    _fields_ = [("batches", ctypes.c_uint64), ("last_kernel_ms", ctypes.c_double),
                ("last_stage_ms", ctypes.c_double), ("last_scratch_bytes", ctypes.c_uint64),
                ("last_collect_ms", ctypes.c_double), ("last_scan_ms", ctypes.c_double),
                ("last_eval_ms", ctypes.c_double), ("last_stream_ms", ctypes.c_double),
                ("last_pa_bytes", ctypes.c_uint64), ("diag", ctypes.c_uint64 * 8),
                ("n_launches", ctypes.c_uint32), ("_pad", ctypes.c_uint32),
                ("launch_ms", ctypes.c_double * STATS_LAUNCHES), ("launch_alg_bytes", ctypes.c_uint64 * STATS_LAUNCHES),
                ("launch_name", (ctypes.c_char * 16) * STATS_LAUNCHES), ("launch_steps", ctypes.c_uint64 * STATS_LAUNCHES),
                ("gate_requests", ctypes.c_uint64), ("gate_pending", ctypes.c_uint64)]


_LIB = None


ABI_VERSION = 6  # include/gpuinspect.h GI_ABI_VERSION: the ctypes structs below mirror that layout


def load_library(path: str = LIB_PATH):
    """Load libgpuinspect.so (raises if it has not been built)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise EngineError("libgpuinspect.so not built (run __graft_entry__.build() or make -C "
                          "coraza-kubernetes-operator_amd)")
    lib = ctypes.CDLL(path)
    lib.gi_abi_version.restype = ctypes.c_uint32
    if lib.gi_abi_version() != ABI_VERSION:
        raise EngineError("libgpuinspect.so has ABI %d, this binding expects %d (rebuild the library)"
                          % (lib.gi_abi_version(), ABI_VERSION))
    vp, u32, u64, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t
    lib.gi_compile.argtypes = [ctypes.c_char_p, sz, ctypes.POINTER(_CompileOpts), ctypes.POINTER(vp),
                               ctypes.c_char_p, sz]
    lib.gi_ruleset_free.argtypes = [vp]
    lib.gi_ruleset_info_get.argtypes = [vp, ctypes.POINTER(_Info)]
    lib.gi_ruleset_export_name.argtypes = [vp, u32, ctypes.c_char_p, sz]
    lib.gi_ruleset_describe.argtypes = [vp, ctypes.c_char_p, sz]
    lib.gi_ruleset_describe.restype = ctypes.c_int64
    lib.gi_ctx_create.argtypes = [vp, ctypes.c_int, u32, ctypes.POINTER(vp)]
    lib.gi_ctx_swap_ruleset.argtypes = [vp, vp]
    lib.gi_ruleset_save.argtypes = [vp, ctypes.c_void_p, sz]
    lib.gi_ruleset_save.restype = ctypes.c_int64
    lib.gi_ruleset_load.argtypes = [ctypes.c_void_p, sz, ctypes.POINTER(vp), ctypes.c_char_p, sz]
    lib.gi_compiler_rev.argtypes = []
    lib.gi_compiler_rev.restype = ctypes.c_char_p
    lib.gi_ctx_free.argtypes = [vp]
    lib.gi_last_error.argtypes = [vp]
    lib.gi_last_error.restype = ctypes.c_char_p
    for fn in ("gi_inspect_batch",):
        getattr(lib, fn).argtypes = [vp, ctypes.POINTER(_Batch), ctypes.POINTER(_Results)]
    lib.gi_stage_batch.argtypes = [vp, ctypes.POINTER(_Batch)]
    lib.gi_run_staged.argtypes = [vp]
    lib.gi_sync.argtypes = [vp]
    lib.gi_fetch_results.argtypes = [vp, ctypes.POINTER(_Results)]
    lib.gi_tally_get.argtypes = [vp, ctypes.POINTER(_Tally)]
    lib.gi_stats_get.argtypes = [vp, ctypes.POINTER(_Stats)]
    lib.gi_tally_detail_get.argtypes = [vp, ctypes.POINTER(u64), ctypes.POINTER(u32), ctypes.POINTER(u64), u32,
                                        ctypes.POINTER(u32)]
    lib.gi_ctx_stream.argtypes = [vp]
    lib.gi_ctx_stream.restype = vp
    lib.gi_cpu_baseline_inspect.argtypes = [vp, ctypes.POINTER(_Batch), ctypes.POINTER(_Results), u32,
                                            ctypes.POINTER(ctypes.c_double)]
    lib.gi_host_register.argtypes = [vp, ctypes.c_void_p, sz]
    lib.gi_host_unregister.argtypes = [vp, ctypes.c_void_p]
    lib.gi_selftest_regex.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, sz, ctypes.POINTER(u32)]
    lib.gi_selftest_plan.argtypes = [vp, ctypes.c_char_p, sz]
    lib.gi_selftest_regex_many.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, ctypes.POINTER(u64), u32,
                                           ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(u32)]
    lib.gi_selftest_triggers.argtypes = [ctypes.POINTER(u32), u32, ctypes.POINTER(u32)]
    lib.gi_ctx_set_capture_cap.argtypes = [vp, u32, u32]
    lib.gi_selftest_capture.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, sz, ctypes.POINTER(ctypes.c_int32),
                                        ctypes.POINTER(u32)]
    _LIB = lib
    return lib


def compiler_rev() -> str:
    """The compiler revision folded into every source digest and artifact."""
    return load_library().gi_compiler_rev().decode()


def aggregate_configmaps(texts: Sequence[str]) -> str:
    """ruleset_controller.go:173-176: ConfigMap rules joined with "\\n"."""
    return "\n".join(texts)


def score_hist_value(tx_export_values, exports):
    """The score gi_tally_detail_get's histogram bins for one request (k_tally):
    the sum of the exported inbound_anomaly_score_pl1..pl4 (each clamped to
    +-2^50), or the first export when none is exported; then clamped to
    [0, 63]."""
    idx = [i for i, e in enumerate(exports[:8]) if len(e) == 25 and e.startswith("inbound_anomaly_score_pl")
           and e[24] in "1234"] or [0]
    s = sum(min(max(int(tx_export_values[i]), -(1 << 50)), 1 << 50) for i in idx)
    return min(max(s, 0), 63)


DEFAULT_EXPORTS = (
    "blocking_inbound_anomaly_score", "inbound_anomaly_score_pl1", "inbound_anomaly_score_pl2",
    "inbound_anomaly_score_pl3", "inbound_anomaly_score_pl4", "detection_inbound_anomaly_score",
    "anomaly_score",
)


class Ruleset:
    """A compiled RuleSet (immutable; share across Engines like a coraza WAF)."""

    def __init__(self, text: str, tx_exports: Optional[Sequence[str]] = None, dfa_state_cap: int = 0,
                 data_files: Optional[dict] = None):
        """data_files: {name: bytes} for @pmFromFile (Coraza reads them from the
        rules' directory, internal/operators/pm_from_file.go)."""
        lib = load_library()
        self._lib = lib
        self.text = text
        self.exports = tuple(tx_exports) if tx_exports is not None else DEFAULT_EXPORTS
        arr = (ctypes.c_char_p * (len(self.exports) + 1))(*[e.encode() for e in self.exports], None)
        files = sorted((data_files or {}).items())
        nf = len(files)
        names = (ctypes.c_char_p * max(nf, 1))(*[k.encode() for k, _ in files])
        blobs = (ctypes.c_char_p * max(nf, 1))(*[bytes(v) for _, v in files])
        lens = (ctypes.c_size_t * max(nf, 1))(*[len(v) for _, v in files])
        opts = _CompileOpts(ctypes.cast(arr, ctypes.POINTER(ctypes.c_char_p)), dfa_state_cap, nf,
                            ctypes.cast(names, ctypes.POINTER(ctypes.c_char_p)),
                            ctypes.cast(blobs, ctypes.POINTER(ctypes.c_char_p)),
                            ctypes.cast(lens, ctypes.POINTER(ctypes.c_size_t)))
        h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(4096)
        raw = text.encode()
        rc = lib.gi_compile(raw, len(raw), ctypes.byref(opts), ctypes.byref(h), err, 4096)
        if rc != GI_OK:
            raise SecLangError(rc, err.value.decode(errors="replace"))
        self._h = h
        self._load_info()

    def _load_info(self):
        info = _Info()
        self._lib.gi_ruleset_info_get(self._h, ctypes.byref(info))
        self.info = {k: getattr(info, k) for k, _ in _Info._fields_ if not k.startswith("_")}
        self.capture_rules = frozenset(self.describe().get("capture_rules", []))

    def save(self) -> bytes:
        """The GPU artifact (gi_ruleset_save): the compiled program as one blob."""
        n = self._lib.gi_ruleset_save(self._h, None, 0)
        if n < 0:
            raise EngineError("gi_ruleset_save failed (%d)" % n)
        buf = ctypes.create_string_buffer(int(n))
        self._lib.gi_ruleset_save(self._h, buf, int(n))
        return buf.raw

    @classmethod
    def load(cls, artifact: bytes) -> "Ruleset":
        """A ruleset from a GPU artifact (gi_ruleset_load), without recompiling."""
        lib = load_library()
        h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(512)
        rc = lib.gi_ruleset_load(artifact, len(artifact), ctypes.byref(h), err, 512)
        if rc != GI_OK:
            raise SecLangError(rc, err.value.decode(errors="replace"))
        self = cls.__new__(cls)
        self._lib = lib
        self.text = None
        self._h = h
        self._load_info()
        names = []
        buf = ctypes.create_string_buffer(256)
        for i in range(MAX_EXPORTS):
            if lib.gi_ruleset_export_name(h, i, buf, 256) != GI_OK:
                break
            names.append(buf.value.decode())
        self.exports = tuple(names)
        return self

    def selftest_plan(self):
        """Host emulation of the phase-A scan images (compiler self-test)."""
        err = ctypes.create_string_buffer(256)
        rc = self._lib.gi_selftest_plan(self._h, err, 256)
        return rc, err.value.decode()

    def describe(self):
        """The phase-A scan plan as a dict (streams, jobs, automata sizes)."""
        lib = self._lib
        n = lib.gi_ruleset_describe(self._h, None, 0)
        buf = ctypes.create_string_buffer(int(n) + 1)
        lib.gi_ruleset_describe(self._h, buf, len(buf))
        return json.loads(buf.value.decode())

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._lib.gi_ruleset_free(h)
            self._h = None


@dataclass
class Transaction:
    """Request accumulator with coraza's Transaction method names."""
    method: bytes = b"GET"
    uri: bytes = b"/"
    proto: bytes = b"HTTP/1.1"
    headers: List[Tuple[bytes, bytes]] = field(default_factory=list)
    body: bytes = b""
    remote_addr: bytes = b""
    remote_port: int = 0
    server_name: bytes = b""

    def process_connection(self, client, cport, server=b"", sport=0):
        """ProcessConnection: REMOTE_ADDR / REMOTE_PORT (the server side is not
        a variable this engine evaluates)."""
        self.remote_addr, self.remote_port = _b(client), int(cport)

    def set_server_name(self, name):
        """SetServerName: SERVER_NAME (coraza-proxy-wasm passes :authority
        without its port)."""
        self.server_name = _b(name)

    def process_uri(self, uri, method, proto):
        self.uri, self.method, self.proto = _b(uri), _b(method), _b(proto)

    def add_request_header(self, key, value):
        self.headers.append((_b(key), _b(value)))

    def write_request_body(self, chunk):
        self.body += _b(chunk)


def _b(x) -> bytes:
    return x if isinstance(x, (bytes, bytearray)) else str(x).encode()


@dataclass
class PackedBatch:
    """SoA batch in the gi_batch layout (host memory)."""
    data: np.ndarray      # uint8 arena
    reqs: np.ndarray      # REQUEST_DT
    headers: np.ndarray   # HEADER_DT

    @property
    def n_req(self):
        return len(self.reqs)

    def raw_bytes(self) -> int:
        r = self.reqs
        return int(r["method"]["len"].sum() + r["uri"]["len"].sum() + r["proto"]["len"].sum()
                   + r["body"]["len"].sum() + self.headers["name"]["len"].sum()
                   + self.headers["value"]["len"].sum())

    def request_bytes(self) -> np.ndarray:
        """Raw bytes of each request (SURVEY §8(d) B_req)."""
        r = self.reqs
        per = (r["method"]["len"].astype(np.int64) + r["uri"]["len"] + r["proto"]["len"] + r["body"]["len"])
        hl = self.headers["name"]["len"].astype(np.int64) + self.headers["value"]["len"]
        hs = np.concatenate([[0], np.cumsum(hl)])
        b = r["hdr_begin"].astype(np.int64)
        return per + hs[b + r["hdr_count"]] - hs[b]

    def take(self, lo: int, hi: int) -> "PackedBatch":
        """Requests [lo, hi) as their own batch (a shard of this one): the
        records are sliced and the byte arena is cut to the range they span."""
        reqs = self.reqs[lo:hi].copy()
        if hi <= lo:
            return PackedBatch(np.zeros(1, np.uint8), reqs, np.zeros(0, HEADER_DT))
        h0 = int(self.reqs[lo]["hdr_begin"])
        h1 = int(self.reqs[hi - 1]["hdr_begin"] + self.reqs[hi - 1]["hdr_count"])
        headers = self.headers[h0:h1].copy()
        starts = [reqs[n]["off"] for n in ("method", "uri", "proto", "body", "remote_addr")]
        ends = [reqs[n]["off"] + reqs[n]["len"] for n in ("method", "uri", "proto", "body", "remote_addr")]
        sn = reqs["server_name"]["len"] > 0
        if sn.any():
            starts.append(reqs["server_name"]["off"][sn])
            ends.append(reqs["server_name"]["off"][sn] + reqs["server_name"]["len"][sn])
        if len(headers):
            starts += [headers["name"]["off"], headers["value"]["off"]]
            ends += [headers["name"]["off"] + headers["name"]["len"], headers["value"]["off"] + headers["value"]["len"]]
        d0 = int(min(int(x.min()) for x in starts))
        d1 = int(max(int(x.max()) for x in ends))
        for n in ("method", "uri", "proto", "body", "remote_addr"):
            reqs[n]["off"] -= d0
        reqs["server_name"]["off"] = np.where(sn, reqs["server_name"]["off"] - d0, 0)
        if len(headers):
            headers["name"]["off"] -= d0
            headers["value"]["off"] -= d0
        reqs["hdr_begin"] -= h0
        data = self.data[d0:max(d1, d0 + 1)].copy()
        return PackedBatch(data, reqs, headers)

    def to_ctypes(self) -> _Batch:
        return _Batch(self.n_req, self.data.ctypes.data, len(self.data), self.reqs.ctypes.data,
                      self.headers.ctypes.data, len(self.headers))

    def request(self, i: int) -> Transaction:
        q = self.reqs[i]
        d = self.data

        def sp(s):
            return bytes(d[int(s["off"]):int(s["off"]) + int(s["len"])])
        hs = [(sp(h["name"]), sp(h["value"])) for h in
              self.headers[int(q["hdr_begin"]):int(q["hdr_begin"]) + int(q["hdr_count"])]]
        return Transaction(sp(q["method"]), sp(q["uri"]), sp(q["proto"]), hs, sp(q["body"]),
                           sp(q["remote_addr"]), int(q["remote_port"]), sp(q["server_name"]))


def concat(batches: Sequence[PackedBatch]) -> PackedBatch:
    """One batch of the requests of `batches`, in order (arenas appended)."""
    datas, reqs, hdrs = [], [], []
    doff = hoff = 0
    for b in batches:
        r = b.reqs.copy()
        h = b.headers.copy()
        for n in ("method", "uri", "proto", "body", "remote_addr"):
            r[n]["off"] += doff
        r["server_name"]["off"] = np.where(r["server_name"]["len"] > 0, r["server_name"]["off"] + doff, 0)
        h["name"]["off"] += doff
        h["value"]["off"] += doff
        r["hdr_begin"] += hoff
        datas.append(b.data)
        reqs.append(r)
        hdrs.append(h)
        doff += len(b.data)
        hoff += len(b.headers)
    if not batches:
        return PackedBatch(np.zeros(1, np.uint8), np.zeros(0, REQUEST_DT), np.zeros(0, HEADER_DT))
    return PackedBatch(np.concatenate(datas), np.concatenate(reqs), np.concatenate(hdrs))


def pack(txs: Sequence) -> PackedBatch:
    """Pack transactions (objects with method/uri/proto/headers/body and
    optionally remote_addr/remote_port) into the gi_batch arena: per request
    [method, uri, proto, body, remote_addr, h0.name, h0.value, ...]."""
    parts = []
    nh = np.empty(len(txs), np.int64)
    ports = np.zeros(len(txs), np.int64)
    for i, t in enumerate(txs):
        parts.append(t.method)
        parts.append(t.uri)
        parts.append(t.proto)
        parts.append(t.body)
        parts.append(getattr(t, "remote_addr", b""))
        ports[i] = getattr(t, "remote_port", 0)
        for k, v in t.headers:
            parts.append(k)
            parts.append(v)
        nh[i] = len(t.headers)
    pb = pack_parts(parts, nh, ports)
    names = [getattr(t, "server_name", b"") for t in txs]
    if any(names):  # SERVER_NAME values after the request parts
        base = sum(map(len, parts))
        extra = np.frombuffer(b"".join(names), dtype=np.uint8)
        pb.data = np.concatenate([pb.data[:base], extra])
        lens = np.array([len(x) for x in names], np.int64)
        offs = base + np.concatenate([[0], np.cumsum(lens)[:-1]])
        pb.reqs["server_name"]["off"] = np.where(lens > 0, offs, 0)
        pb.reqs["server_name"]["len"] = lens
    return pb


NFIXED = 5  # fixed parts per request in pack_parts: method, uri, proto, body, remote_addr


def pack_parts(parts: List[bytes], nh: np.ndarray, ports=None) -> PackedBatch:
    lens = np.fromiter(map(len, parts), dtype=np.int64, count=len(parts))
    offs = np.zeros(len(parts), np.int64)
    if len(parts):
        np.cumsum(lens[:-1], out=offs[1:])
    data = np.frombuffer(b"".join(parts), dtype=np.uint8) if parts else np.zeros(0, np.uint8)
    if len(data) == 0:
        data = np.zeros(1, np.uint8)
    n = len(nh)
    per = NFIXED + 2 * nh
    start = np.zeros(n, np.int64)
    if n:
        np.cumsum(per[:-1], out=start[1:])
    reqs = np.zeros(n, REQUEST_DT)
    for j, name in enumerate(("method", "uri", "proto", "body", "remote_addr")):
        reqs[name]["off"] = offs[start + j]
        reqs[name]["len"] = lens[start + j]
    if ports is not None:
        reqs["remote_port"] = ports
    hb = np.zeros(n, np.int64)
    if n:
        np.cumsum(nh[:-1], out=hb[1:])
    reqs["hdr_begin"] = hb
    reqs["hdr_count"] = nh
    H = int(nh.sum())
    headers = np.zeros(H, HEADER_DT)
    if H:
        # index of each header's name part
        req_of_h = np.repeat(np.arange(n), nh)
        k_in_req = np.arange(H) - hb[req_of_h]
        name_idx = start[req_of_h] + NFIXED + 2 * k_in_req
        headers["name"]["off"] = offs[name_idx]
        headers["name"]["len"] = lens[name_idx]
        headers["value"]["off"] = offs[name_idx + 1]
        headers["value"]["len"] = lens[name_idx + 1]
    return PackedBatch(data, reqs, headers)


@dataclass
class Results:
    verdicts: np.ndarray     # VERDICT_DT
    matched: np.ndarray      # uint32 [n_req, matched_cap]
    exports: Tuple[str, ...]
    capture_recs: Optional[np.ndarray] = None   # CAPTURE_DT [n_req, capture_cap]
    capture_bytes: Optional[np.ndarray] = None  # uint8 [n_req, capture_bytes_cap]
    capture_rules: Optional[frozenset] = None   # rule ids with observable captures (the plan's capture_rules)

    def captures(self, i: int) -> List[Tuple[int, int, bytes]]:
        """The observable captures of request i in evaluation order:
        (top-level rule id, group, captured bytes)."""
        if self.capture_recs is None:
            return []
        n = min(int(self.verdicts[i]["capture_cnt"]), self.capture_recs.shape[1])
        row = self.capture_bytes[i]
        return [(int(c["rule_id"]), int(c["group"]), bytes(row[int(c["off"]):int(c["off"]) + int(c["len"])]))
                for c in self.capture_recs[i, :n]]

    def matched_rules(self, i: int) -> List[int]:
        n = min(int(self.verdicts[i]["match_cnt"]), self.matched.shape[1])
        return [int(x) for x in self.matched[i, :n]]

    def interruption(self, i: int):
        v = self.verdicts[i]
        if v["action"] == 0:
            return None
        return {"rule_id": int(v["rule_id"]), "status": int(v["status"]),
                "action": ACTIONS[int(v["action"])], "phase": int(v["phase"])}

    def tx(self, i: int, name: str) -> int:
        return int(self.verdicts[i]["tx_export"][self.exports.index(name)])


def cpu_baseline_inspect(ruleset: "Ruleset", batch, threads: int = 0, matched_cap: int = 64,
                         capture_cap: int = 0, capture_bytes_cap: int = 512):
    """The CPU baseline (gi_cpu_baseline_inspect): this engine's
    interpreter compiled for the host, `threads` host threads (0: all cores),
    every rule link evaluated without phase A.  Not Coraza, and never a
    fallback of Engine (which only runs on the GPU).  Returns (Results without
    captures, evaluation seconds)."""
    lib = load_library()
    if not isinstance(batch, PackedBatch):
        batch = pack(batch)
    n = batch.n_req
    verd = np.zeros(n, VERDICT_DT)
    matched = np.zeros((n, matched_cap), np.uint32)
    crec = cbytes = None
    if capture_cap:
        crec = np.zeros((n, capture_cap), CAPTURE_DT)
        cbytes = np.zeros((n, capture_bytes_cap), np.uint8)
    res = _Results(verd.ctypes.data, matched.ctypes.data, matched_cap,
                   crec.ctypes.data if capture_cap else None, cbytes.ctypes.data if capture_cap else None,
                   capture_cap, capture_bytes_cap if capture_cap else 0)
    cb = batch.to_ctypes()
    secs = ctypes.c_double(0.0)
    rc = lib.gi_cpu_baseline_inspect(ruleset._h, ctypes.byref(cb), ctypes.byref(res), threads, ctypes.byref(secs))
    if rc != GI_OK:
        raise EngineError("gi_cpu_baseline_inspect failed (%d)" % rc)
    if capture_cap:
        return Results(verd, matched, ruleset.exports, crec, cbytes, ruleset.capture_rules), secs.value
    return Results(verd, matched, ruleset.exports), secs.value


class Engine:
    """A device context (one HIP stream) evaluating batches on one GPU."""

    def __init__(self, ruleset: Ruleset, device: int = 0, matched_cap: int = 64, capture_cap: int = 8,
                 capture_bytes_cap: int = 512):
        lib = load_library()
        self._lib = lib
        self.ruleset = ruleset
        self.matched_cap = matched_cap
        h = ctypes.c_void_p()
        rc = lib.gi_ctx_create(ruleset._h, device, matched_cap, ctypes.byref(h))
        if rc != GI_OK:
            raise EngineError("gi_ctx_create failed (%d): no usable HIP device %d" % (rc, device))
        self._h = h
        self._staged = None
        self._pinned = []   # host arrays page-locked through this ctx (gi_host_register)
        self._rbuf = None   # reusable result arrays (fetch(reuse=True))
        self.capture_cap, self.capture_bytes_cap = capture_cap, capture_bytes_cap
        self._check(lib.gi_ctx_set_capture_cap(h, capture_cap, capture_bytes_cap), "gi_ctx_set_capture_cap")

    def swap(self, ruleset: Ruleset):
        """Hot swap (gi_ctx_swap_ruleset): later batches run `ruleset`; a staged
        batch is dropped."""
        self._check(self._lib.gi_ctx_swap_ruleset(self._h, ruleset._h), "gi_ctx_swap_ruleset")
        self.ruleset = ruleset
        self._staged = None

    def _check(self, rc, what):
        if rc != GI_OK:
            raise EngineError("%s failed (%d): %s" % (what, rc, self._lib.gi_last_error(self._h).decode()))

    def pin(self, *arrays) -> int:
        """Page-lock host arrays a later batch (or fetch) uses: gi_host_register,
        the C ABI's optional pinned-host fast path.  Returns how many were
        pinned (a refusal, e.g. an array sharing pages with one already pinned,
        leaves that array pageable: staging stays correct, only slower)."""
        k = 0
        for a in arrays:
            if a is None or a.nbytes == 0 or any(a is b for b in self._pinned):
                continue
            if self._lib.gi_host_register(self._h, ctypes.c_void_p(a.ctypes.data), ctypes.c_size_t(a.nbytes)) == GI_OK:
                self._pinned.append(a)
                k += 1
        return k

    def unpin(self):
        for a in self._pinned:
            self._lib.gi_host_unregister(self._h, ctypes.c_void_p(a.ctypes.data))
        self._pinned = []

    def stage(self, batch: PackedBatch):
        self._staged = batch
        cb = batch.to_ctypes()
        self._check(self._lib.gi_stage_batch(self._h, ctypes.byref(cb)), "gi_stage_batch")

    def run(self):
        self._check(self._lib.gi_run_staged(self._h), "gi_run_staged")

    def sync(self):
        self._check(self._lib.gi_sync(self._h), "gi_sync")

    def result_buffers(self, n: int):
        """The reusable result arrays for n requests (allocated once)."""
        if self._rbuf is None or self._rbuf[0] != n:
            self._rbuf = (n, np.empty(n, VERDICT_DT), np.empty((n, self.matched_cap), np.uint32),
                          np.empty((n, self.capture_cap), CAPTURE_DT), np.empty((n, self.capture_bytes_cap), np.uint8))
        return self._rbuf[1:]

    def fetch(self, reuse: bool = False) -> Results:
        """Verdicts, matched ids and captures of the staged batch (D2H).  reuse:
        write into this engine's reusable arrays (result_buffers; overwritten by
        the next fetch) instead of fresh ones."""
        n = self._staged.n_req
        if reuse:
            verd, matched, crec, cbytes = self.result_buffers(n)
        else:
            verd = np.zeros(n, VERDICT_DT)
            matched = np.zeros((n, self.matched_cap), np.uint32)
            crec = np.zeros((n, self.capture_cap), CAPTURE_DT)
            cbytes = np.zeros((n, self.capture_bytes_cap), np.uint8)
        res = _Results(verd.ctypes.data, matched.ctypes.data, self.matched_cap, crec.ctypes.data, cbytes.ctypes.data,
                       self.capture_cap, self.capture_bytes_cap)
        self._check(self._lib.gi_fetch_results(self._h, ctypes.byref(res)), "gi_fetch_results")
        return Results(verd, matched, self.ruleset.exports, crec, cbytes, self.ruleset.capture_rules)

    def inspect(self, batch) -> Results:
        if not isinstance(batch, PackedBatch):
            batch = pack(batch)
        self.stage(batch)
        self.run()
        return self.fetch()

    def tally(self) -> dict:
        t = _Tally()
        self._check(self._lib.gi_tally_get(self._h, ctypes.byref(t)), "gi_tally_get")
        return {k: getattr(t, k) for k, _ in _Tally._fields_}

    def tally_rule_count(self) -> int:
        """Distinct rule ids of the ruleset (width of the per-rule tally)."""
        n = ctypes.c_uint32(0)
        self._check(self._lib.gi_tally_detail_get(self._h, None, None, None, 0, ctypes.byref(n)), "gi_tally_detail_get")
        return n.value

    def tally_detail(self) -> dict:
        """Score histogram (first export, clamped to [0, 63]) and the match
        count of every distinct rule id of the last batch (gi_tally_detail_get)."""
        n = ctypes.c_uint32(0)
        self._check(self._lib.gi_tally_detail_get(self._h, None, None, None, 0, ctypes.byref(n)), "gi_tally_detail_get")
        hist = (ctypes.c_uint64 * SCORE_BINS)()
        ids = (ctypes.c_uint32 * max(n.value, 1))()
        hits = (ctypes.c_uint64 * max(n.value, 1))()
        self._check(self._lib.gi_tally_detail_get(self._h, hist, ids, hits, n.value, ctypes.byref(n)),
                    "gi_tally_detail_get")
        return {"score_hist": list(hist), "rule_ids": list(ids)[:n.value], "rule_hits": list(hits)[:n.value]}

    def stats(self) -> dict:
        s = _Stats()
        self._check(self._lib.gi_stats_get(self._h, ctypes.byref(s)), "gi_stats_get")
        out = {k: getattr(s, k) for k, _ in _Stats._fields_ if not k.startswith("launch") and k != "_pad"}
        out["diag"] = list(out["diag"])
        out["launches"] = [{"name": s.launch_name[k].value.decode(), "ms": s.launch_ms[k],
                            "alg_bytes": int(s.launch_alg_bytes[k]), "steps": int(s.launch_steps[k])}
                           for k in range(s.n_launches)]
        return out

    def stream(self) -> int:
        return int(self._lib.gi_ctx_stream(self._h) or 0)

    def close(self):
        if getattr(self, "_h", None):
            self.unpin()
            self._lib.gi_ctx_free(self._h)
            self._h = None

    def __del__(self):
        self.close()


def selftest_triggers(n_codes: int = 32):
    """(triggers[code], byte_summary[256]) as the kernels use them."""
    lib = load_library()
    t = (ctypes.c_uint32 * n_codes)()
    b = (ctypes.c_uint32 * 256)()
    lib.gi_selftest_triggers(t, n_codes, b)
    return list(t), list(b)


def selftest_regex(pattern: str, data: bytes):
    """Host walk of the compiled @rx DFA (compiler self-test only)."""
    lib = load_library()
    pb = pattern.encode()
    n = ctypes.c_uint32(0)
    rc = lib.gi_selftest_regex(pb, len(pb), data, len(data), ctypes.byref(n))
    return rc, n.value


def selftest_regex_many(pattern: str, strings):
    """Host walk of the compiled @rx automaton over many strings (one build):
    ([0/1 per string], DFA states or 0 when the NFA tables answered)."""
    lib = load_library()
    pb = pattern.encode()
    data = b"".join(strings)
    offs = (ctypes.c_uint64 * (len(strings) + 1))()
    o = 0
    for k, x in enumerate(strings):
        offs[k] = o
        o += len(x)
    offs[len(strings)] = o
    out = (ctypes.c_uint8 * max(len(strings), 1))()
    n = ctypes.c_uint32(0)
    rc = lib.gi_selftest_regex_many(pb, len(pb), data, offs, len(strings), out, ctypes.byref(n))
    if rc != GI_OK:
        raise SecLangError(rc, "selftest_regex_many failed")
    return [int(out[k]) for k in range(len(strings))], n.value



def selftest_capture(pattern: str, data: bytes):
    """The capture submatch program (pike.h, what k_eval runs) on the host:
    None without a match, else the group spans [(start, end) or None, ...]
    (FindStringSubmatchIndex restricted to groups 0..8)."""
    lib = load_library()
    pb = pattern.encode()
    caps = (ctypes.c_int32 * 18)()
    ns = ctypes.c_uint32(0)
    rc = lib.gi_selftest_capture(pb, len(pb), data, len(data), caps, ctypes.byref(ns))
    if rc < 0:
        raise SecLangError(rc, "selftest_capture failed")
    if rc == 0:
        return None
    return [(caps[2 * g], caps[2 * g + 1]) if caps[2 * g] >= 0 else None for g in range(ns.value // 2)]
