"""Informer-event feeders of the node snapshot (SURVEY §3.3 and §8b "Snapshot feeders").

koord-scheduler keeps per-plugin caches fed by informer events; the engine keeps one HBM row per node.
`SnapshotFeeder` mirrors those caches event by event, with the reference's semantics, and turns every
event into the set of node rows it changes; `flush()` rebuilds exactly those rows through the C-ABI row
builder (kg_build_node_rows) and hands them to `kg_snapshot_upsert` / `kg_snapshot_remove`:

* pod add / update / delete — the upstream scheduler cache's NodeInfo (bound, non-terminated pods:
  Requested, NonZeroRequested, pod count); LoadAware's podAssignCache (pod_assign_cache.go:53-117:
  OnAdd assigns a bound, non-terminated pod with timestamp timeNowFn(); OnUpdate unassigns a terminated
  pod and re-assigns any other bound pod with a NEW timestamp; OnDelete unassigns); NodeNUMAResource's
  NodeAllocation from the pod's resource-status (pod_eventhandler.go:94-144: a terminated pod releases
  it); and the pod lister that NodeMetric.PodsMetric entries are looked up in (helper.go:153-170), so a
  pod event also dirties every node whose NodeMetric names that pod;
* node add / update / delete (TransformNode at ingest, node_transformer.go:40-75);
* NodeMetric add / update / delete (read through the lister on every Filter / Score: load_aware.go:133,278);
* NodeResourceTopology add / update / delete (TopologyOptionsManager, topology_eventhandler.go:62-113).

Node indices are stable; a deleted node's index is reused by the next new node (free list).  A row is a
pure function of the node's objects, its bound pods, their assign timestamps, its NodeMetric and its NRT,
so "event stream → upserts" equals "fresh build of the final state" (tests/test_feeders_cpu.py).
"""
from __future__ import annotations

import time
from typing import Callable, Dict, List, Optional, Set, Tuple

import numpy as np

from . import _native as nat
from . import engine as _engine
from . import ingest


def _meta(obj: dict) -> dict:
    return obj.get("metadata") or {}


def _uid(pod: dict) -> str:
    uid = _meta(pod).get("uid")
    if not uid:
        raise ValueError("pod events need metadata.uid (the caches are keyed by UID)")
    return uid


def _key(pod: dict) -> str:
    m = _meta(pod)
    return f"{m.get('namespace', 'default')}/{m.get('name', '')}"


def _node_name(pod: dict) -> str:
    return (pod.get("spec") or {}).get("nodeName", "") or ""


def _terminated(pod: dict) -> bool:
    """util.IsPodTerminated: phase Succeeded or Failed."""
    return (pod.get("status") or {}).get("phase") in ("Succeeded", "Failed")


class SnapshotFeeder:
    """The scheduler-side caches behind the engine's node rows, fed by informer events."""

    def __init__(self, cfg: np.ndarray, now_fn: Optional[Callable[[], int]] = None):
        self.cfg = cfg
        self.now_fn = now_fn or time.time_ns          # podAssignCache's timeNowFn
        self.nodes: Dict[str, dict] = {}               # node informer
        self.index: Dict[str, int] = {}                # node name → engine row index (stable)
        self._free: List[int] = []
        self.n_index = 0                               # indices handed out so far (rows in use or freed)
        self.nrts: Dict[str, dict] = {}
        self.metrics: Dict[str, dict] = {}
        self.pods: Dict[str, dict] = {}                # pod informer / lister, by UID
        self.by_key: Dict[str, str] = {}               # namespace/name → UID (the lister's key)
        self.bound: Dict[str, Set[str]] = {}           # NodeInfo: node → UIDs of bound, non-terminated pods
        self.assign_cache: Dict[str, Dict[str, int]] = {}   # podAssignCache: node → UID → timestamp ns
        self.metric_refs: Dict[str, Set[str]] = {}     # namespace/name → nodes whose PodsMetric names it
        self._dirty: Set[str] = set()
        self._removed: List[int] = []

    # ---- podAssignCache (pod_assign_cache.go:53-80) -------------------------------------------
    def _assign(self, node: str, pod: dict) -> None:
        if node == "" or _terminated(pod):
            return
        self.assign_cache.setdefault(node, {})[_uid(pod)] = int(self.now_fn())

    def _unassign(self, node: str, pod: dict) -> None:
        if node == "":
            return
        items = self.assign_cache.get(node)
        if items is not None:
            items.pop(_uid(pod), None)
            if not items:
                del self.assign_cache[node]

    # ---- NodeInfo (bound pods) and the lister ----------------------------------------------------
    def _bind(self, pod: dict) -> None:
        node = _node_name(pod)
        if node and not _terminated(pod):
            self.bound.setdefault(node, set()).add(_uid(pod))

    def _unbind(self, pod: dict) -> None:
        node = _node_name(pod)
        s = self.bound.get(node)
        if s is not None:
            s.discard(_uid(pod))
            if not s:
                del self.bound[node]

    def _touch_pod(self, pod: dict) -> None:
        if _node_name(pod):
            self._dirty.add(_node_name(pod))
        self._dirty.update(self.metric_refs.get(_key(pod), ()))

    # ---- pod events -------------------------------------------------------------------------------
    def on_pod_add(self, pod: dict) -> None:
        uid = _uid(pod)
        self.pods[uid] = pod
        self.by_key[_key(pod)] = uid
        self._bind(pod)
        self._assign(_node_name(pod), pod)                       # podAssignCache.OnAdd
        self._touch_pod(pod)

    def on_pod_update(self, old: dict, new: dict) -> None:
        uid = _uid(new)
        prev = self.pods.get(uid, old)        # the cached object (the informer's old object when unseen)
        if prev is not None:
            self._unbind(prev)
            self._touch_pod(prev)
            if _key(prev) != _key(new):
                self.by_key.pop(_key(prev), None)
        self.pods[uid] = new
        self.by_key[_key(new)] = uid
        self._bind(new)
        if _terminated(new):                                    # podAssignCache.OnUpdate
            self._unassign(_node_name(new), new)
        else:
            self._assign(_node_name(new), new)
        self._touch_pod(new)

    def on_pod_delete(self, pod: dict) -> None:
        uid = _uid(pod)
        prev = self.pods.pop(uid, pod)
        if self.by_key.get(_key(prev)) == uid:
            del self.by_key[_key(prev)]
        self._unbind(prev)
        self._unassign(_node_name(prev), prev)                  # podAssignCache.OnDelete
        self._touch_pod(prev)

    # ---- node, NodeMetric, NodeResourceTopology events -------------------------------------------
    def on_node_add(self, node: dict) -> None:
        name = _meta(node)["name"]
        self.nodes[name] = node
        if name not in self.index:
            if self._free:
                self.index[name] = self._free.pop()
            else:
                self.index[name] = self.n_index
                self.n_index += 1
        self._dirty.add(name)

    on_node_update = on_node_add

    def on_node_delete(self, name: str) -> None:
        if name not in self.nodes:
            return
        del self.nodes[name]
        i = self.index.pop(name)
        self._free.append(i)
        self._removed.append(i)
        self._dirty.discard(name)

    def on_node_metric(self, nm: dict) -> None:
        name = _meta(nm)["name"]
        old = self.metrics.get(name)
        if old is not None:
            for pm in (old.get("status") or {}).get("podsMetric") or []:
                self.metric_refs.get(f"{pm.get('namespace', 'default')}/{pm.get('name', '')}", set()).discard(name)
        self.metrics[name] = nm
        for pm in (nm.get("status") or {}).get("podsMetric") or []:
            self.metric_refs.setdefault(f"{pm.get('namespace', 'default')}/{pm.get('name', '')}", set()).add(name)
        self._dirty.add(name)

    def on_node_metric_delete(self, name: str) -> None:
        old = self.metrics.pop(name, None)
        if old is not None:
            for pm in (old.get("status") or {}).get("podsMetric") or []:
                self.metric_refs.get(f"{pm.get('namespace', 'default')}/{pm.get('name', '')}", set()).discard(name)
        self._dirty.add(name)

    def on_nrt(self, nrt: dict) -> None:
        name = _meta(nrt)["name"]
        self.nrts[name] = nrt
        self._dirty.add(name)

    def on_nrt_delete(self, name: str) -> None:
        self.nrts.pop(name, None)
        self._dirty.add(name)

    # ---- rows ------------------------------------------------------------------------------------
    def _rows_for(self, names: List[str]) -> np.ndarray:
        """kg_node_row of each named node from the current cache state (the C-ABI row builder)."""
        rows, _ = self._rows_view_for(names)
        return rows

    def _rows_view_for(self, names: List[str]):
        """(rows, the flat view they were built from: view node k ⇔ names[k])."""
        if not names:
            return np.zeros(0, dtype=nat.NODE_ROW), None
        uids: Set[str] = set()
        for n in names:
            uids.update(self.bound.get(n, ()))
            uids.update(self.assign_cache.get(n, {}).keys())
            for pm in (self.metrics.get(n, {}).get("status") or {}).get("podsMetric") or []:
                u = self.by_key.get(f"{pm.get('namespace', 'default')}/{pm.get('name', '')}")
                if u is not None:
                    uids.add(u)
        cl = ingest.cluster_from_objects(
            [self.nodes[n] for n in names], [self.pods[u] for u in sorted(uids)],
            [self.metrics[n] for n in names if n in self.metrics], [self.nrts[n] for n in names if n in self.nrts],
            now_ns=int(self.now_fn()), assign_cache={n: self.assign_cache[n] for n in names if n in self.assign_cache})
        # cluster_from_objects binds every given non-terminated pod to its node: pods given only for the
        # lister are bound to nodes outside `names` (or terminated), so NodeInfo stays the bound set
        view = cl.view()
        return _engine.build_node_rows(self.cfg, view), view

    def take_deltas(self) -> Tuple[np.ndarray, np.ndarray, List[int]]:
        """(indices, rows) of every node changed since the last call, and the indices removed since."""
        idx, rows, removed, _ = self._take()
        return idx, rows, removed

    def _take(self):
        names = sorted(n for n in self._dirty if n in self.nodes)
        self._dirty.clear()
        removed, self._removed = self._removed, []
        idx = np.array([self.index[n] for n in names], dtype=np.int32)
        rows, view = self._rows_view_for(names)
        return idx, rows, removed, view

    def full_rows(self) -> Tuple[np.ndarray, np.ndarray]:
        """(indices, rows) of every live node, built from scratch (the reference point of the deltas)."""
        names = sorted(self.nodes, key=lambda n: self.index[n])
        return np.array([self.index[n] for n in names], dtype=np.int32), self._rows_for(names)

    def flush(self, eng: "_engine.Engine") -> int:
        """Apply the pending deltas to an engine whose snapshot holds ≥ n_index rows — the changed rows and,
        for a cpuset Reserve, the changed nodes' CPU tables (kg_cpus_set); returns rows written."""
        idx, rows, removed, view = self._take()
        for i in removed:
            if i not in set(idx.tolist()):
                eng.remove(i)
        if len(idx):
            eng.upsert(idx, rows)
            eng.set_cpus(view, np.arange(len(idx)), idx)
        return len(idx)

    def cluster(self) -> "ingest.ob.Cluster":
        """The whole cache state as an objects.Cluster, nodes in row-index order (indices must be dense:
        a deleted node's slot refilled), for evaluation by the host tools and the oracle."""
        names = sorted(self.nodes, key=lambda n: self.index[n])
        if [self.index[n] for n in names] != list(range(len(names))):
            raise ValueError("row indices have holes (a deleted node's slot not refilled)")
        return ingest.cluster_from_objects(
            [self.nodes[n] for n in names], list(self.pods.values()), [self.metrics[n] for n in names if n in self.metrics],
            [self.nrts[n] for n in names if n in self.nrts], now_ns=int(self.now_fn()),
            assign_cache={n: self.assign_cache[n] for n in names if n in self.assign_cache})
