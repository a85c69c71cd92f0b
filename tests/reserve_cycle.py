"""Host-side sequential cycle with cpuset Reserve, through the engine's own per-pair code on the CPU
(kg_row_eval for Filter + Score, kg_row_reserve for Reserve) — the same functions the device kernels and
kg_place's host Reserve run.  Used by the CPU suite against the oracle's literal cycle, and by the GPU tests to
replay the rows kg_place should end with."""
import numpy as np

from koordinator_amd import _native as nat
from koordinator_amd import engine


def cpu_tables(view):
    """{node: (first_cpu, n_cpus, max_ref_count, numa_allocate_strategy)} for nodes with CPU detail."""
    out = {}
    for j in range(len(view.nodes)):
        k = int(view.nodes[j]["numa"])
        if k < 0:
            continue
        nm = view.numa_arr[k]
        if int(nm["n_cpus"]) > 0:
            out[j] = (int(nm["first_cpu"]), int(nm["n_cpus"]), int(nm["max_ref_count"]),
                      int(nm["numa_allocate_strategy"]))
    return out


def host_cycle(cfg, view, pod_index, now_ns):
    """(nodes, scores, rows after, cpus after) of the sequential cycle over pod_index."""
    rows = engine.build_node_rows(cfg, view)
    pods = engine.build_pod_rows(cfg, view, pod_index)
    cpus = view.cpu_arr.copy()
    tabs = cpu_tables(view)
    w = (int(cfg["weight_fit"]), int(cfg["weight_loadaware"]), int(cfg["weight_numa"]))
    en = int(cfg["enabled_plugins"])
    N = len(rows)
    nodes = np.full(len(pods), -1, np.int32)
    scores = np.full(len(pods), -1, np.int64)
    for i in range(len(pods)):
        best, best_j = -1, -1
        for j in range(N):
            ok, f, la, nu = engine.row_eval(cfg, rows[j:j + 1], pods[i:i + 1], now_ns)
            if not ok:
                continue
            tot = (w[0] * f if en & nat.PLUGIN_FIT else 0) + (w[1] * la if en & nat.PLUGIN_LOADAWARE else 0) + \
                  (w[2] * nu if en & nat.PLUGIN_NUMA else 0)
            if tot > best:
                best, best_j = tot, j
        if best_j < 0:
            continue
        if best_j in tabs:
            first, n, max_ref, strat = tabs[best_j]
            tab = cpus[first:first + n].copy()
            row = rows[best_j:best_j + 1].copy()
            taken = engine.row_reserve(cfg, row, pods[i:i + 1], tab, max_ref, strat)
            if taken is None:   # the Reserve failed: nothing changed, the pod is not placed
                continue
            cpus[first:first + n] = tab
        else:
            row = rows[best_j:best_j + 1].copy()
            taken = engine.row_reserve(cfg, row, pods[i:i + 1], np.zeros(0, nat.CPU_INFO))
            if taken is None:
                continue
        rows[best_j] = row[0]
        nodes[i], scores[i] = best_j, best
    return nodes, scores, rows, cpus
