"""Exact int64 evaluation of (pod, node) pairs from engine rows alone, and a numpy mirror of the
engine's chunk API (partial keys per 1024-node tile + the sequential resolve of k_resolve).

TEST INFRASTRUCTURE: used to check the host row builders and the multi-rank placement protocol on
CPU against the oracle; the product path never uses it.
"""
import ctypes
import math

import numpy as np

from koordinator_amd import _native as nat
from koordinator_amd import engine

def _lr(req, cap):
    """LR(req, cap) = req > cap ? 0 : (cap - req) * 100 / cap, int64 (cap > 0)."""
    safe = np.where(cap > 0, cap, 1)
    q = ((safe - req) * 100) // safe
    return np.where((cap > 0) & (req <= cap), q, 0)


def _mr(req, cap):
    safe = np.where(cap > 0, cap, 1)
    return np.where(cap > 0, (np.minimum(req, safe) * 100) // safe, 0)


def rows_eval(cfg, nodes, pods, now_ns):
    """Exact evaluation of every (pod, node) pair from engine rows only (mirrors kg_pair_exact)."""
    N, P = len(nodes), len(pods)
    fit_on = bool(cfg["enabled_plugins"] & nat.PLUGIN_FIT)
    la_on = bool(cfg["enabled_plugins"] & nat.PLUGIN_LOADAWARE)
    most = int(cfg["fit_strategy"]) == nat.STRATEGY_MOST_ALLOCATED
    fw = cfg["fit_resource_weight"].astype(np.int64)
    lw = cfg["la_resource_weight"].astype(np.int64)
    valid = (nodes["flags"] & nat.NODE_VALID) != 0
    full = nodes["pod_count"].astype(np.int64) + 1 > nodes["allowed_pods"].astype(np.int64)
    has_metric = (nodes["flags"] & nat.NODE_HAS_METRIC) != 0
    has_upd = (nodes["flags"] & nat.NODE_HAS_UPDATE_TIME) != 0
    exp_ns = int(cfg["la_expiration_seconds"]) * 10**9 if cfg["la_has_expiration"] else 0
    expired = ~has_upd | ((exp_ns > 0) & (now_ns - nodes["metric_update_ns"] >= exp_ns))
    skip_filter = bool(cfg["la_filter_expired_node_metrics"]) and bool(cfg["la_has_expiration"])
    la_valid = has_metric & ~(bool(cfg["la_has_expiration"]) & expired)
    free = nodes["alloc"] - nodes["requested"]
    mask = np.zeros((P, N), bool)
    fit = np.zeros((P, N), np.int64)
    la = np.zeros((P, N), np.int64)
    for i, p in enumerate(pods):
        ok = valid.copy()
        if fit_on:
            ok &= ~full
            if p["flags"] & nat.POD_HAS_REQUEST:
                for r in range(nat.NUM_RES):
                    if r < 3 or (p["request_present"] >> r) & 1:
                        ok &= p["request"][r] <= free[:, r]
        if la_on and not (p["flags"] & nat.POD_DAEMONSET):
            bit = nat.NODE_LA_PASS_PROD if p["flags"] & nat.POD_PROD else nat.NODE_LA_PASS_NONPROD
            passes = ~has_metric | (skip_filter & expired) | ((nodes["flags"] & bit) != 0)
            ok &= passes
        mask[i] = ok
        if fit_on:
            s = np.zeros(N, np.int64)
            w = np.zeros(N, np.int64)
            for r in range(nat.NUM_RES):
                pr = int(p["fit_score_request"][r])
                if fw[r] <= 0 or (r >= 3 and pr == 0):
                    continue
                a = nodes["alloc"][:, r]
                present = np.ones(N, bool) if r < 3 else ((nodes["alloc_present"] >> r) & 1) == 1
                use = present & (a != 0)
                base = nodes["nonzero_requested"][:, r] if r < 2 else nodes["requested"][:, r]
                q = _mr(base + pr, a) if most else _lr(base + pr, a)
                s += np.where(use, q * fw[r], 0)
                w += np.where(use, fw[r], 0)
            fit[i] = np.where(w > 0, s // np.where(w > 0, w, 1), 0)
        if la_on:
            v = 1 if p["flags"] & nat.POD_LA_PROD_SCORE else 0
            s = np.zeros(N, np.int64)
            for r in range(2):
                if lw[r] == 0:
                    continue
                s += _lr(p["la_estimate"][r] + nodes["la_used"][:, v, r], nodes["la_alloc"][:, r]) * lw[r]
            la[i] = np.where(la_valid, s // max(int(lw[:2].sum()), 1), 0)
    return mask, fit, la


def pair_totals(cfg, nodes, pod_row, now_ns):
    """(feasible, total) of one pod against every node row."""
    m, f, l = rows_eval(cfg, nodes, pod_row[None], now_ns)
    tot = int(cfg["weight_fit"]) * f[0] + int(cfg["weight_loadaware"]) * l[0]
    return m[0], tot


class RowsBackend:
    """numpy mirror of kg_place_chunk_eval / kg_place_chunk_resolve over a replicated snapshot,
    evaluating only the node shard [begin, end) in chunk_eval."""

    def __init__(self, cfg, node_rows, pod_rows, shard):
        self.cfg = cfg
        self.nodes = node_rows.copy()
        self.pods = pod_rows
        self.n_pods = len(pod_rows)
        n = len(node_rows)
        self.num_tiles = max(1, math.ceil(n / nat.TILE))
        self.shard = shard

    @staticmethod
    def _view(ptr, count, ctype):
        return np.ctypeslib.as_array((ctype * count).from_address(ptr))

    def chunk_eval(self, now_ns, b, n, partial_ptr):
        T = self.num_tiles
        part = self._view(partial_ptr, n * T, ctypes.c_uint32).reshape(n, T)
        part[:] = 0
        lo, hi = self.shard
        if hi <= lo:
            return
        for j in range(n):
            ok, tot = pair_totals(self.cfg, self.nodes[lo:hi], self.pods[b + j], now_ns)
            for k in np.nonzero(ok)[0]:
                node = lo + int(k)
                t, local = divmod(node, nat.TILE)
                key = ((int(tot[k]) + 1) << 10) | (nat.TILE - 1 - local)
                part[j, t] = max(int(part[j, t]), key)

    def _key(self, pod, node, now_ns):
        ok, tot = pair_totals(self.cfg, self.nodes[node:node + 1], pod, now_ns)
        return ((int(tot[0]) + 1) << 32) | (0xFFFFFFFF - node) if ok[0] else 0

    def chunk_resolve(self, now_ns, b, n, partial_ptr, node_ptr, score_ptr, prev_ptr=0, n_prev=0):
        T = self.num_tiles
        part = self._view(partial_ptr, n * T, ctypes.c_uint32).reshape(n, T)
        out_node = self._view(node_ptr, n, ctypes.c_int32)
        out_score = self._view(score_ptr, n, ctypes.c_int64)
        N = len(self.nodes)
        # the previous chunk's placements (pipelined order): their keys may predate those commits, so re-score
        touched = [int(x) for x in self._view(prev_ptr, n_prev, ctypes.c_int32) if x >= 0] if n_prev else []
        for j in range(n):
            pod = self.pods[b + j]
            best, rescan = 0, []
            for t in range(T):
                k = int(part[j, t])
                if k == 0:
                    continue
                node = t * nat.TILE + (nat.TILE - 1) - (k & (nat.TILE - 1))
                key = ((k >> 10) << 32) | (0xFFFFFFFF - node)
                if node in touched:
                    rescan.append(t)
                else:
                    best = max(best, key)
            for node in touched:
                best = max(best, self._key(pod, node, now_ns))
            for t in rescan:
                lo, hi = t * nat.TILE, min(N, (t + 1) * nat.TILE)
                ok, tot = pair_totals(self.cfg, self.nodes[lo:hi], pod, now_ns)
                for k in np.nonzero(ok)[0]:
                    best = max(best, ((int(tot[k]) + 1) << 32) | (0xFFFFFFFF - (lo + int(k))))
            if best:
                node = 0xFFFFFFFF - (best & 0xFFFFFFFF)
                engine.row_commit(self.cfg, self.nodes[node:node + 1], self.pods[b + j:b + j + 1])
                if node not in touched:
                    touched.append(node)
                out_node[j] = node
                out_score[j] = (best >> 32) - 1
            else:
                out_node[j] = -1
                out_score[j] = -1
