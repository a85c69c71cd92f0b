"""Score-table debug dump: the engine's counterpart of koord-scheduler's ``--debug-scores`` top-N table.

Reference: ``pkg/scheduler/frameworkext/debug.go:61-108`` (``debugScores``: every plugin's weighted
NodeScore summed per feasible node, nodes sorted by total descending, plugin columns sorted by name,
rendered as a markdown table) and ``debug.go:32-48`` (the ``debugTopNScores`` switch, 0 = off).  Here
the switch is the ``KOORD_GPU_DEBUG_TOPN`` environment variable, read by ``Engine.eval``; the table is
built from the score planes the matrix mode already returns, so enabling it adds no device work.

Go's ``sort.Slice`` is not stable, so the reference leaves the order of equal totals unspecified; this
dump keeps node order among ties (lowest index first, the engine's own tie-break).
"""
from __future__ import annotations

import logging
import os
from typing import Mapping, Optional, Sequence

import numpy as np

from . import _native as nat

log = logging.getLogger("koordinator_amd.debug")


def debug_top_n() -> int:
    """The ``KOORD_GPU_DEBUG_TOPN`` switch (``debugTopNScores``): 0 or unset disables the dump."""
    try:
        return max(0, int(os.environ.get("KOORD_GPU_DEBUG_TOPN", "0")))
    except ValueError:
        return 0


def render_scores(top_n: int, pod_ref: str, plugin_scores: Mapping[str, Sequence[int]],
                  node_names: Sequence[str]) -> str:
    """``debugScores`` (debug.go:61-108): ``plugin_scores[name][i]`` is the weighted score of
    ``node_names[i]``; returns the markdown of the top ``top_n`` rows (prettytable's RenderMarkdown:
    string columns left-aligned, integer columns right-aligned)."""
    names = sorted(plugin_scores)
    totals = [sum(int(plugin_scores[p][i]) for p in names) for i in range(len(node_names))]
    order = sorted(range(len(node_names)), key=lambda i: -totals[i])  # stable: ties keep node order
    header = ["#", "Pod", "Node", "Score", *names]
    lines = ["| " + " | ".join(header) + " |",
             "| " + " | ".join(["---"] * 3) + " |" + "".join(" ---:|" for _ in header[3:])]
    for rank, i in enumerate(order[:top_n]):
        row = [str(rank), pod_ref, node_names[i], str(totals[i]), *(str(int(plugin_scores[p][i])) for p in names)]
        lines.append("| " + " | ".join(row) + " |")
    return "\n".join(lines)


def plane_scores(cfg: Mapping, res: Mapping[str, np.ndarray], pod: int, n_nodes: int):
    """Feasible nodes of one pod and every enabled engine plugin's weighted score on them, from the
    planes of ``Engine.eval`` (the framework multiplies each plugin's normalized score by its profile
    weight before the table is built)."""
    bits = np.unpackbits(res["mask"][pod].view(np.uint8), bitorder="little")[:n_nodes].astype(bool)
    nodes = np.flatnonzero(bits)
    plugins = int(cfg["enabled_plugins"])
    out = {}
    if plugins & nat.PLUGIN_FIT:
        out["NodeResourcesFit"] = res["scores"][pod, nodes, 0].astype(np.int64) * int(cfg["weight_fit"])
    if plugins & nat.PLUGIN_LOADAWARE:
        out["LoadAwareScheduling"] = res["scores"][pod, nodes, 1].astype(np.int64) * int(cfg["weight_loadaware"])
    if plugins & nat.PLUGIN_NUMA and "numa_scores" in res:
        out["NodeNUMAResource"] = res["numa_scores"][pod, nodes].astype(np.int64) * int(cfg["weight_numa"])
    if plugins & nat.PLUGIN_RESERVATION and "rsv_scores" in res:
        out["Reservation"] = res["rsv_scores"][pod, nodes].astype(np.int64) * int(cfg["weight_reservation"])
    return nodes, out


def dump_eval(cfg: Mapping, res: Mapping[str, np.ndarray], n_nodes: int, top_n: int,
              pod_refs: Optional[Sequence[str]] = None, node_names: Optional[Sequence[str]] = None) -> list:
    """One table per pod of a matrix-mode result (needs its mask and score planes); each is logged at
    INFO like ``klog.Infof`` in debug.go:107 and returned."""
    tables = []
    if top_n <= 0 or "mask" not in res or "scores" not in res:
        return tables
    for p in range(res["mask"].shape[0]):
        nodes, scores = plane_scores(cfg, res, p, n_nodes)
        names = [node_names[i] if node_names is not None else f"node-{i}" for i in nodes]
        ref = pod_refs[p] if pod_refs is not None else f"pod-{p}"
        t = render_scores(top_n, ref, scores, names)
        log.info("Top%d scores for Pod: %s, feasibleNodes: %d, plugins:%s\n%s", top_n, ref, len(nodes),
                 sorted(scores), t)
        tables.append(t)
    return tables
