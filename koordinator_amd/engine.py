"""Python handle on the HIP engine (``libkoordgpu.so``), used by the plugin mirror, tests and bench."""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from . import _native as nat
from . import debug


class EngineError(RuntimeError):
    pass


def _check(st: int, eng: Optional["Engine"] = None, what: str = "") -> None:
    if st != 0:
        msg = nat.lib().kg_last_error(eng._h).decode() if eng is not None and eng._h else ""
        raise EngineError(f"{what} failed with status {st}: {msg}")


def build_pod_rows(cfg: np.ndarray, view, pod_index: Sequence[int]) -> np.ndarray:
    idx = np.ascontiguousarray(pod_index, dtype=np.int32)
    out = np.zeros(len(idx), dtype=nat.POD_ROW)
    _check(nat.lib().kg_build_pod_rows(nat.ptr(cfg), ctypes.byref(view.c_view), nat.ptr(idx), len(idx), nat.ptr(out)),
           what="kg_build_pod_rows")
    return out


def build_node_rows(cfg: np.ndarray, view, node_index: Optional[Sequence[int]] = None) -> np.ndarray:
    n = len(view.nodes)
    idx = np.arange(n, dtype=np.int32) if node_index is None else np.ascontiguousarray(node_index, dtype=np.int32)
    out = np.zeros(len(idx), dtype=nat.NODE_ROW)
    _check(nat.lib().kg_build_node_rows(nat.ptr(cfg), ctypes.byref(view.c_view), nat.ptr(idx), len(idx), nat.ptr(out)),
           what="kg_build_node_rows")
    return out


def row_commit(cfg: np.ndarray, node_row: np.ndarray, pod_row: np.ndarray) -> None:
    _check(nat.lib().kg_row_commit(nat.ptr(cfg), nat.ptr(node_row), nat.ptr(pod_row)), what="kg_row_commit")


def row_reserve(cfg: np.ndarray, node_row: np.ndarray, pod_row: np.ndarray, cpus: np.ndarray, max_ref_count: int = 1,
                numa_allocate_strategy: int = 0):
    """kg_row_reserve: the Reserve of one pair on a host row and the node's CPU_INFO array (both updated in
    place).  Returns the taken cpuset (bool per cpu), or None when the Reserve fails (KG_NOT_FOUND)."""
    taken = np.zeros(len(cpus), dtype=np.uint8)
    st = nat.lib().kg_row_reserve(nat.ptr(cfg), nat.ptr(node_row), nat.ptr(pod_row), nat.ptr(cpus) if len(cpus) else None,
                                  len(cpus), int(max_ref_count), int(numa_allocate_strategy),
                                  nat.ptr(taken) if len(cpus) else None)
    if st == nat.NOT_FOUND:
        return None
    _check(st, what="kg_row_reserve")
    return taken.astype(bool)


def row_eval(cfg: np.ndarray, node_row: np.ndarray, pod_row: np.ndarray, now_ns: int):
    """(feasible, fit, la, numa) of one pair on host rows (the kernels' per-pair code, run on the CPU)."""
    f, a, b, c = (ctypes.c_int32() for _ in range(4))
    _check(nat.lib().kg_row_eval(nat.ptr(cfg), nat.ptr(node_row), nat.ptr(pod_row), int(now_ns), ctypes.byref(f),
                                 ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), what="kg_row_eval")
    return bool(f.value), a.value, b.value, c.value


def row_eval_rsv(cfg: np.ndarray, node_row: np.ndarray, rsv: np.ndarray, pod_row: np.ndarray, now_ns: int):
    """(feasible, fit, la, numa, raw, order, nominated) of one pair with the node's reservation slots
    (host rows)."""
    rsv = np.ascontiguousarray(rsv, dtype=nat.RESERVATION)
    f, a, b, n, r, nm = (ctypes.c_int32() for _ in range(6))
    o = ctypes.c_int64()
    _check(nat.lib().kg_row_eval_rsv(nat.ptr(cfg), nat.ptr(node_row), nat.ptr(rsv) if len(rsv) else None, len(rsv),
                                     nat.ptr(pod_row), int(now_ns), ctypes.byref(f), ctypes.byref(a), ctypes.byref(b),
                                     ctypes.byref(n), ctypes.byref(r), ctypes.byref(o), ctypes.byref(nm)),
           what="kg_row_eval_rsv")
    return bool(f.value), a.value, b.value, n.value, r.value, o.value, nm.value


def row_rsv_restore(cfg: np.ndarray, node_row: np.ndarray, rsv: np.ndarray, pod_row: np.ndarray) -> np.ndarray:
    """The Reservation restore of one pair (kg_row_rsv_restore): a RSV_RESTORED record."""
    rsv = np.ascontiguousarray(rsv, dtype=nat.RESERVATION)
    out = np.zeros((), dtype=nat.RSV_RESTORED)
    _check(nat.lib().kg_row_rsv_restore(nat.ptr(cfg), nat.ptr(node_row), nat.ptr(rsv) if len(rsv) else None, len(rsv),
                                        nat.ptr(pod_row), nat.ptr(out)), what="kg_row_rsv_restore")
    return out


class Engine:
    """One engine = one GPU, one HIP stream, one HBM-resident node snapshot."""

    def __init__(self, cfg: np.ndarray):
        self.cfg = cfg.copy()
        self._h = ctypes.c_void_p()
        _check(nat.lib().kg_engine_create(nat.ptr(self.cfg), ctypes.byref(self._h)), what="kg_engine_create")
        self.n_nodes = 0
        self.n_pods = 0

    # lifecycle --------------------------------------------------------------------------
    def close(self) -> None:
        if self._h:
            nat.lib().kg_engine_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_stream(self, stream_ptr: int) -> None:
        _check(nat.lib().kg_set_stream(self._h, ctypes.c_void_p(stream_ptr)), self, "kg_set_stream")

    def sync(self) -> None:
        _check(nat.lib().kg_sync(self._h), self, "kg_sync")

    # snapshot ---------------------------------------------------------------------------
    def load_snapshot(self, rows: np.ndarray) -> None:
        rows = np.ascontiguousarray(rows, dtype=nat.NODE_ROW)
        _check(nat.lib().kg_snapshot_reset(self._h, len(rows)), self, "kg_snapshot_reset")
        self.n_nodes = len(rows)
        self.shard = (0, len(rows))
        self.upsert(np.arange(len(rows), dtype=np.int32), rows)

    def upsert(self, idx, rows: np.ndarray) -> None:
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        rows = np.ascontiguousarray(rows, dtype=nat.NODE_ROW)
        _check(nat.lib().kg_snapshot_upsert(self._h, nat.ptr(idx), nat.ptr(rows), len(idx)), self, "kg_snapshot_upsert")

    def set_cpus(self, view, view_index: Optional[Sequence[int]] = None,
                 snap_index: Optional[Sequence[int]] = None) -> None:
        """kg_cpus_set: snapshot node snap_index[k] takes the CPU detail of view node view_index[k] (both
        default to k over every view node); other nodes keep their tables."""
        n = len(view.nodes) if view_index is None else len(view_index)
        vi = None if view_index is None else np.ascontiguousarray(view_index, dtype=np.int32)
        si = None if snap_index is None else np.ascontiguousarray(snap_index, dtype=np.int32)
        _check(nat.lib().kg_cpus_set(self._h, ctypes.byref(view.c_view), nat.ptr(vi), nat.ptr(si), n), self,
               "kg_cpus_set")

    def download_cpus(self, node: int, n_cpus: int) -> np.ndarray:
        out = np.zeros(n_cpus, dtype=nat.CPU_INFO)
        _check(nat.lib().kg_cpus_download(self._h, int(node), nat.ptr(out), n_cpus), self, "kg_cpus_download")
        return out

    def remove(self, i: int) -> None:
        _check(nat.lib().kg_snapshot_remove(self._h, int(i)), self, "kg_snapshot_remove")

    def download(self, first: int = 0, n: Optional[int] = None) -> np.ndarray:
        n = self.n_nodes - first if n is None else n
        out = np.zeros(n, dtype=nat.NODE_ROW)
        _check(nat.lib().kg_snapshot_download(self._h, first, n, nat.ptr(out)), self, "kg_snapshot_download")
        return out

    def generation(self) -> int:
        """kg_snapshot_generation: successful snapshot mutations so far; raises once the state is stale."""
        g = ctypes.c_uint64(0)
        _check(nat.lib().kg_snapshot_generation(self._h, ctypes.byref(g)), self, "kg_snapshot_generation")
        return int(g.value)

    def set_shard(self, begin: int, end: int) -> None:
        _check(nat.lib().kg_set_shard(self._h, begin, end), self, "kg_set_shard")
        self.shard = (begin, end)

    def set_profiling(self, on: bool = True) -> None:
        _check(nat.lib().kg_set_profiling(self._h, int(on)), self, "kg_set_profiling")

    def eval_kernel_times(self, n: int = 256) -> np.ndarray:
        """Durations (ms) of the last ≤ n profiled k_eval launches, oldest first."""
        ms = np.zeros(n, dtype=np.float32)
        k = nat.lib().kg_eval_kernel_times(self._h, nat.ptr(ms), n)
        if k < 0:
            _check(k, self, "kg_eval_kernel_times")
        return ms[:k].astype(np.float64)

    @property
    def num_tiles(self) -> int:
        return nat.lib().kg_num_tiles(self._h)

    partial_slots = nat.PARTIAL_SLOTS   # uint32 per (pod, tile) of kg_place_chunk_eval's buffer

    # pods -------------------------------------------------------------------------------
    def set_pods(self, rows: np.ndarray) -> None:
        rows = np.ascontiguousarray(rows, dtype=nat.POD_ROW)
        _check(nat.lib().kg_pods_set(self._h, nat.ptr(rows), len(rows)), self, "kg_pods_set")
        self.n_pods = len(rows)

    # evaluation -------------------------------------------------------------------------
    @property
    def mask_words(self) -> int:
        return (self.shard[1] - self.shard[0] + 63) // 64

    @property
    def score_stride(self) -> int:
        return self.mask_words * 64

    def eval(self, now_ns: int, mask: bool = True, scores: bool = True, top1: bool = True,
             numa_scores: Optional[bool] = None, rsv_scores: Optional[bool] = None) -> dict:
        """Matrix mode into host arrays: mask [P][words] u64, scores [P][stride][2] u8, top1 [P] u64,
        numa_scores [P][stride] u8 (by default when NodeNUMAResource is enabled), rsv_scores [P][stride]
        u8 (normalized Reservation score, by default when Reservation is enabled)."""
        P = self.n_pods
        res = {}
        out = nat.EvalOut()
        if mask:
            res["mask"] = np.zeros((P, self.mask_words), dtype=np.uint64)
            out.mask = res["mask"].ctypes.data
        if scores:
            res["scores"] = np.zeros((P, self.score_stride, 2), dtype=np.uint8)
            out.scores = res["scores"].ctypes.data
        if top1:
            res["top1"] = np.zeros(P, dtype=np.uint64)
            out.top1 = res["top1"].ctypes.data
        if numa_scores is None:
            numa_scores = bool(int(self.cfg["enabled_plugins"]) & nat.PLUGIN_NUMA)
        if numa_scores:
            res["numa_scores"] = np.zeros((P, self.score_stride), dtype=np.uint8)
            out.numa_scores = res["numa_scores"].ctypes.data
        if rsv_scores is None:
            rsv_scores = bool(int(self.cfg["enabled_plugins"]) & nat.PLUGIN_RESERVATION)
        if rsv_scores:
            res["rsv_scores"] = np.zeros((P, self.score_stride), dtype=np.uint8)
            out.rsv_scores = res["rsv_scores"].ctypes.data
        out.out_on_device = 0
        _check(nat.lib().kg_eval(self._h, int(now_ns), ctypes.byref(out)), self, "kg_eval")
        top_n = debug.debug_top_n()   # --debug-scores (frameworkext/debug.go:32-48)
        if top_n:
            debug.dump_eval(self.cfg, res, min(self.n_nodes, self.score_stride), top_n)
        return res

    def eval_device(self, now_ns: int, mask_ptr: int = 0, scores_ptr: int = 0, top1_ptr: int = 0,
                    numa_ptr: int = 0) -> None:
        out = nat.EvalOut()
        out.mask, out.scores, out.top1, out.out_on_device = mask_ptr or None, scores_ptr or None, top1_ptr or None, 1
        out.numa_scores = numa_ptr or None
        _check(nat.lib().kg_eval(self._h, int(now_ns), ctypes.byref(out)), self, "kg_eval")

    @staticmethod
    def comm_unique_id() -> bytes:
        """An RCCL unique id for kg_comm_init (one rank makes it, every rank passes it)."""
        buf = ctypes.create_string_buffer(nat.COMM_ID_BYTES)
        st = nat.lib().kg_comm_unique_id(buf)
        if st != 0:
            raise EngineError(f"kg_comm_unique_id failed ({st})")
        return buf.raw

    def comm_init(self, rank: int, world: int, unique_id: bytes) -> None:
        buf = ctypes.create_string_buffer(bytes(unique_id), nat.COMM_ID_BYTES)
        _check(nat.lib().kg_comm_init(self._h, int(rank), int(world), buf), self, "kg_comm_init")

    def comm_init_loopback(self, rank: int, world: int, name: str) -> None:
        """kg_comm_init_loopback: the ranks merge partial keys through the host shared-memory segment `name`
        (the same "/…" on every rank) instead of RCCL — several ranks on one GPU run kg_place_sharded's own loop."""
        _check(nat.lib().kg_comm_init_loopback(self._h, int(rank), int(world), name.encode()), self,
               "kg_comm_init_loopback")

    def comm_kind(self) -> str:
        return {nat.COMM_NONE: "none", nat.COMM_RCCL: "rccl", nat.COMM_LOOPBACK: "loopback"}[nat.lib().kg_comm_kind(self._h)]

    def place_sharded(self, now_ns: int):
        """kg_place over the ranks' node shards (kg_place_sharded): per chunk one max-merge of the partial keys over
        the communicator (RCCL or loopback), the resolve and host Reserve steps replicated.  Same outputs as place()."""
        P = self.n_pods
        nodes = np.zeros(P, dtype=np.int32)
        scores = np.zeros(P, dtype=np.int64)
        _check(nat.lib().kg_place_sharded(self._h, int(now_ns), nat.ptr(nodes), nat.ptr(scores)), self,
               "kg_place_sharded")
        return nodes, scores

    def set_forms(self, forms: int) -> None:
        """Force size-chosen kernel forms (nat.FORM_*; 0 = by size), for parity tests on small clusters."""
        _check(nat.lib().kg_set_forms(self._h, int(forms)), self, "kg_set_forms")

    def eval_host(self, now_ns: int, mask_ptr: int = 0, scores_ptr: int = 0, top1_ptr: int = 0,
                  numa_ptr: int = 0, rsv_ptr: int = 0) -> None:
        """Matrix mode into caller-owned host buffers (e.g. pinned memory): the outputs the Go plugins read
        (INTEGRATION.md `Eval`), copied back over PCIe before the call returns."""
        out = nat.EvalOut()
        out.mask, out.scores, out.top1, out.out_on_device = mask_ptr or None, scores_ptr or None, top1_ptr or None, 0
        out.numa_scores, out.rsv_scores = numa_ptr or None, rsv_ptr or None
        _check(nat.lib().kg_eval(self._h, int(now_ns), ctypes.byref(out)), self, "kg_eval")

    def place(self, now_ns: int):
        P = self.n_pods
        nodes = np.zeros(P, dtype=np.int32)
        scores = np.zeros(P, dtype=np.int64)
        _check(nat.lib().kg_place(self._h, int(now_ns), nat.ptr(nodes), nat.ptr(scores)), self, "kg_place")
        return nodes, scores

    def chunk_eval(self, now_ns: int, pod_begin: int, n: int, partial_ptr: int) -> None:
        _check(nat.lib().kg_place_chunk_eval(self._h, int(now_ns), pod_begin, n, ctypes.c_void_p(partial_ptr)), self,
               "kg_place_chunk_eval")

    def chunk_resolve(self, now_ns: int, pod_begin: int, n: int, partial_ptr: int, node_ptr: int,
                      score_ptr: int, prev_ptr: int = 0, n_prev: int = 0) -> None:
        """kg_place_chunk_resolve; with prev_ptr / n_prev the pipelined form kg_place_chunk_resolve_prev (the
        previous chunk's placements, device int32, re-scored like touched nodes)."""
        if n_prev:
            _check(nat.lib().kg_place_chunk_resolve_prev(self._h, int(now_ns), pod_begin, n, ctypes.c_void_p(partial_ptr),
                                                         ctypes.c_void_p(node_ptr), ctypes.c_void_p(score_ptr),
                                                         ctypes.c_void_p(prev_ptr), n_prev), self,
                   "kg_place_chunk_resolve_prev")
            return
        _check(nat.lib().kg_place_chunk_resolve(self._h, int(now_ns), pod_begin, n, ctypes.c_void_p(partial_ptr),
                                                ctypes.c_void_p(node_ptr), ctypes.c_void_p(score_ptr)), self,
               "kg_place_chunk_resolve")

    def set_eval_stream(self, hip_stream: int) -> None:
        """kg_set_eval_stream: chunk evaluations launch on this stream (0 ⇒ the engine stream)."""
        _check(nat.lib().kg_set_eval_stream(self._h, ctypes.c_void_p(hip_stream or None)), self, "kg_set_eval_stream")

    def counters(self) -> dict:
        """kg_counters_get as a dict (evals, out_bytes, resolved, placed, h2d_bytes, kernel_ns, ...)."""
        out = np.zeros(1, dtype=nat.COUNTERS)
        _check(nat.lib().kg_counters_get(self._h, nat.ptr(out)), self, "kg_counters_get")
        return {k: int(out[k][0]) for k in nat.COUNTERS.names}

    def reset_counters(self) -> None:
        _check(nat.lib().kg_counters_reset(self._h), self, "kg_counters_reset")

    def commit(self, pod: int, node: int) -> bool:
        """kg_commit; False ⇔ the Reserve failed (a cpuset the accumulator cannot take; nothing changed)."""
        st = nat.lib().kg_commit(self._h, pod, node)
        if st == nat.NOT_FOUND:
            return False
        _check(st, self, "kg_commit")
        return True

    # Reservation / ElasticQuota -----------------------------------------------------------
    def set_reservations(self, rsv: np.ndarray) -> None:
        rsv = np.ascontiguousarray(rsv, dtype=nat.RESERVATION)
        _check(nat.lib().kg_rsv_set(self._h, nat.ptr(rsv), len(rsv)), self, "kg_rsv_set")
        self.n_rsv = len(rsv)

    def download_reservations(self) -> np.ndarray:
        out = np.zeros(getattr(self, "n_rsv", 0), dtype=nat.RESERVATION)
        _check(nat.lib().kg_rsv_download(self._h, nat.ptr(out), len(out)), self, "kg_rsv_download")
        return out

    def set_quotas(self, q: np.ndarray) -> None:
        q = np.ascontiguousarray(q, dtype=nat.QUOTA)
        _check(nat.lib().kg_quota_set(self._h, nat.ptr(q), len(q)), self, "kg_quota_set")
        self.n_quota = len(q)

    def download_quotas(self) -> np.ndarray:
        out = np.zeros(getattr(self, "n_quota", 0), dtype=nat.QUOTA)
        _check(nat.lib().kg_quota_download(self._h, nat.ptr(out), len(out)), self, "kg_quota_download")
        return out


def decode_top1(keys: np.ndarray):
    """(total+1) << 32 | (0xFFFFFFFF − node) → (node or −1, total or −1)."""
    keys = np.asarray(keys, dtype=np.uint64)
    ok = keys != 0
    node = np.where(ok, (np.uint64(0xFFFFFFFF) - (keys & np.uint64(0xFFFFFFFF))).astype(np.int64), -1)
    total = np.where(ok, (keys >> np.uint64(32)).astype(np.int64) - 1, -1)
    return node, total


def unpack_mask(mask: np.ndarray, n_nodes: int) -> np.ndarray:
    """[P][words] u64 → [P][n_nodes] bool."""
    b = np.unpackbits(mask.view(np.uint8), axis=1, bitorder="little")
    return b[:, :n_nodes].astype(bool)
