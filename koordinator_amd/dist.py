"""Node-sharded scheduling across GPUs (one process per GPU, ``torch.distributed``; backend ``nccl``
is RCCL on ROCm).

SURVEY §8e: every per-pair quantity depends on one pod row and one node row, so the path shards over
nodes with no data-path collective. The only exchange is the per-pod best-node merge:

* matrix mode (``merge_top1``): each rank evaluates its own node shard and emits one u64 key per pod,
  ``(total+1) << 32 | (0xFFFFFFFF − global node)``; one ``all_reduce(MAX)`` (equivalently an
  all-gather of P × 8 B and a max over ranks) gives the highest total, then the lowest node index.
* placement mode (``place_sharded``): the node snapshot is replicated on every rank (1M nodes × 200 B
  is 0.2 GB of a 288 GB device). For each chunk of pods in queue order, every rank evaluates only its
  own tile range (``kg_place_chunk_eval`` on its shard), the per-(pod, 1024-node tile) partial keys are
  merged with one ``all_reduce(MAX)`` (chunk × tiles × 4 B: 250 KB at 1M nodes and 64 pods), and every
  rank runs the same deterministic resolve (``kg_place_chunk_resolve``) on identical inputs. The replicas
  therefore stay identical, and the placements equal the single-GPU ones (and the oracle's sequential
  cycle).

Keys are unsigned 32/64-bit; ``torch.distributed`` reduces signed integers, so the sign bit is flipped
before and after the max (an order-preserving map from unsigned to signed).
"""
from __future__ import annotations

import math
import os
import uuid
from typing import Optional, Protocol, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import _native as nat

SIGN32 = -(2**31)
SIGN64 = -(2**63)


def shard_range(n_nodes: int, rank: int, world: int, tile: int = nat.TILE) -> Tuple[int, int]:
    """Contiguous, tile-aligned node range [begin, end) of `rank` (possibly empty)."""
    tiles = max(1, math.ceil(n_nodes / tile))
    per = math.ceil(tiles / world)
    t0 = min(rank * per, tiles)
    t1 = min(tiles, t0 + per)
    if t0 >= t1 or t0 * tile >= n_nodes:
        return n_nodes, n_nodes          # empty shard (more ranks than tiles)
    return t0 * tile, min(n_nodes, t1 * tile)


def _max_unsigned_(t: torch.Tensor, sign: int, group=None) -> None:
    t.bitwise_xor_(sign)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    t.bitwise_xor_(sign)


def merge_partials_(partial: torch.Tensor, group=None) -> None:
    """In-place max over ranks of u32 per-(pod, tile) keys held in an int32 tensor."""
    _max_unsigned_(partial, SIGN32, group)


def merge_top1_(keys: torch.Tensor, group=None) -> None:
    """In-place max over ranks of u64 per-pod keys held in an int64 tensor."""
    _max_unsigned_(keys, SIGN64, group)


class ChunkBackend(Protocol):
    """What `place_sharded` needs from an engine (the HIP engine implements it through the C-ABI).

    Optional attributes: ``torch_stream`` (the torch stream the engine launches on; the merge runs on it) and
    ``eval_torch_stream`` (a second stream for ``chunk_eval``: its presence turns the pipelined order on, and
    ``chunk_resolve`` is then called with the previous chunk's placed nodes, ``prev_ptr`` / ``n_prev``, to
    re-score)."""

    n_pods: int
    num_tiles: int
    partial_slots: int     # uint32 keys per (pod, tile) in the partial buffer

    def chunk_eval(self, now_ns: int, pod_begin: int, n: int, partial_ptr: int) -> None: ...

    def chunk_resolve(self, now_ns: int, pod_begin: int, n: int, partial_ptr: int, node_ptr: int,
                      score_ptr: int, prev_ptr: int = 0, n_prev: int = 0) -> None: ...


def place_sharded(backend: ChunkBackend, now_ns: int, device: torch.device, chunk: int = 8,
                  group=None, pipeline: Optional[bool] = None,
                  collective: Optional[bool] = None) -> Tuple[np.ndarray, np.ndarray]:
    """Sequential-cycle placement of the backend's pod batch, node-sharded across the group.

    The backend must hold the full (replicated) snapshot with its evaluation restricted to this
    rank's `shard_range`. Returns (node or −1, total or −1) per pod, identical on every rank.

    pipeline (default: when the backend offers it, ``backend.eval_torch_stream``): chunk i + 1 is evaluated and
    its partials merged on the eval stream while chunk i is resolved on the backend's stream; the resolve of
    chunk i + 1 re-scores the nodes chunk i placed (``kg_place_chunk_resolve_prev``), as the one-GPU kg_place
    pipeline does.  collective (default: world size > 1) runs the partial-key merge even on one rank (the RCCL
    path exercised alone)."""
    if chunk < 1 or chunk > nat.PLACE_CHUNK_MAX:
        raise ValueError(f"chunk {chunk} outside 1..{nat.PLACE_CHUNK_MAX}")
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    merge = world > 1 if collective is None else collective
    P, tiles = backend.n_pods, backend.num_tiles
    stream = getattr(backend, "torch_stream", None)
    eval_stream = getattr(backend, "eval_torch_stream", None)
    if pipeline is None:
        pipeline = eval_stream is not None
    if pipeline and (eval_stream is None or stream is None):
        raise ValueError("the pipelined placement needs the backend's eval and resolve streams")
    slots = getattr(backend, "partial_slots", 1)
    if not pipeline:
        with torch.cuda.stream(stream) if stream is not None else _nullctx():
            partial = torch.zeros((max(chunk, 1), tiles, slots), dtype=torch.int32, device=device)
            nodes = torch.full((max(P, 1),), -1, dtype=torch.int32, device=device)
            scores = torch.full((max(P, 1),), -1, dtype=torch.int64, device=device)
            for b in range(0, P, chunk):
                n = min(chunk, P - b)
                if eval_stream is not None:   # the engine evaluates on its eval stream: order it in
                    eval_stream.wait_stream(stream)
                backend.chunk_eval(now_ns, b, n, partial.data_ptr())
                if eval_stream is not None:
                    stream.wait_stream(eval_stream)
                if merge:
                    merge_partials_(partial[:n], group)
                backend.chunk_resolve(now_ns, b, n, partial.data_ptr(), nodes.data_ptr() + 4 * b,
                                      scores.data_ptr() + 8 * b)
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            return nodes[:P].cpu().numpy(), scores[:P].cpu().numpy()
    # pipelined: eval(i) + merge(i) on eval_stream, resolve(i) on stream; eval(i) waits for resolve(i − 2) (its
    # partial buffer, and the snapshot older than one chunk), resolve(i) for eval(i) + merge(i)
    with torch.cuda.stream(stream):
        nodes = torch.full((max(P, 1),), -1, dtype=torch.int32, device=device)
        scores = torch.full((max(P, 1),), -1, dtype=torch.int64, device=device)
    eval_stream.wait_stream(stream)
    with torch.cuda.stream(eval_stream):
        partial = [torch.zeros((max(chunk, 1), tiles, slots), dtype=torch.int32, device=device) for _ in range(2)]
    stream.wait_stream(eval_stream)
    ev_eval = [torch.cuda.Event() for _ in range(2)]
    ev_res = [torch.cuda.Event() for _ in range(3)]
    prev_b = prev_n = 0
    for i, b in enumerate(range(0, P, chunk)):
        n = min(chunk, P - b)
        part = partial[i & 1]
        if i >= 2:
            eval_stream.wait_event(ev_res[(i - 2) % 3])
        with torch.cuda.stream(eval_stream):
            backend.chunk_eval(now_ns, b, n, part.data_ptr())
            if merge:
                merge_partials_(part[:n], group)
            ev_eval[i & 1].record(eval_stream)
        stream.wait_event(ev_eval[i & 1])
        with torch.cuda.stream(stream):
            backend.chunk_resolve(now_ns, b, n, part.data_ptr(), nodes.data_ptr() + 4 * b, scores.data_ptr() + 8 * b,
                                  nodes.data_ptr() + 4 * prev_b if i else 0, prev_n if i else 0)
            ev_res[i % 3].record(stream)
        prev_b, prev_n = b, n
    torch.cuda.synchronize(device)
    return nodes[:P].cpu().numpy(), scores[:P].cpu().numpy()


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def place_chunk_of(cfg: np.ndarray) -> int:
    """kg_place's rule for the chunk size: 0 ⇒ 16, capped at KG_PLACE_CHUNK_MAX (negative values are
    rejected by kg_config_validate).  The chunk is also the number of pods per partial-key all_reduce
    in `place_sharded`: 16 halves the collectives of 8 at the same one-GPU rate (profiles/r02_v4)."""
    chunk = int(cfg["place_chunk"])
    if chunk < 0:
        raise ValueError(f"place_chunk {chunk} < 0")
    return min(chunk if chunk > 0 else 16, nat.PLACE_CHUNK_MAX)


def sharded_engine(cfg: np.ndarray, node_rows: np.ndarray, pod_rows: np.ndarray, device: torch.device,
                   group=None, reservations: Optional[np.ndarray] = None, quotas: Optional[np.ndarray] = None):
    """A HIP engine on `device` holding the full snapshot, restricted to this rank's node shard.

    The engine is bound to a dedicated torch stream (``eng.torch_stream``); `place_sharded` runs the
    collectives and tensor ops on that same stream, so engine kernels and merges are ordered. (The
    legacy null stream cannot be shared: ``kg_set_stream(NULL)`` means an engine-owned stream.)
    Reservation slots and ElasticQuota groups are replicated like the snapshot: every rank evaluates
    all reservation nodes and applies the same quota gate in its (identical) resolve."""
    from .engine import Engine

    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    cfg = cfg.copy()
    cfg["device"] = device.index or 0
    eng = Engine(cfg)
    eng.torch_stream = torch.cuda.Stream(device)
    eng.set_stream(eng.torch_stream.cuda_stream)
    if reservations is None:   # the pipelined placement (reservation entries are written by chunk_eval)
        eng.eval_torch_stream = torch.cuda.Stream(device)
        eng.set_eval_stream(eng.eval_torch_stream.cuda_stream)
    eng.load_snapshot(node_rows)
    if reservations is not None:
        eng.set_reservations(reservations)
    if quotas is not None:
        eng.set_quotas(quotas)
    eng.set_pods(pod_rows)
    begin, end = shard_range(len(node_rows), rank, world)
    eng.set_shard(begin, end)
    return eng


def native_engine(cfg: np.ndarray, node_rows: np.ndarray, pod_rows: np.ndarray, device: torch.device, group=None,
                  reservations: Optional[np.ndarray] = None, quotas: Optional[np.ndarray] = None,
                  stream: Optional[torch.cuda.Stream] = None, comm: str = "rccl", rank: Optional[int] = None,
                  world: Optional[int] = None, shm_name: Optional[str] = None):
    """A HIP engine holding the full snapshot, restricted to this rank's shard, with its own communicator: the
    engine then runs the whole sharded placement natively (Engine.place_sharded = kg_place_sharded), the chunk loop,
    the partial-key merges and the replicated resolve / host Reserve steps in C++.

    comm="rccl": an RCCL communicator over the group (kg_comm_init; rank 0's unique id is broadcast through
    torch.distributed).  comm="loopback": the host shared-memory communicator (kg_comm_init_loopback) — several ranks
    on ONE GPU (RCCL refuses two ranks on a device) run the same C++ loop; its segment name is rank 0's, broadcast
    through torch.distributed, or `shm_name` when the caller starts the processes itself (rank / world given)."""
    from .engine import Engine

    if rank is None:
        rank = dist.get_rank(group) if dist.is_initialized() else 0
    if world is None:
        world = dist.get_world_size(group) if dist.is_initialized() else 1
    cfg = cfg.copy()
    cfg["device"] = device.index or 0
    eng = Engine(cfg)
    if stream is not None:
        eng.set_stream(stream.cuda_stream)
    eng.load_snapshot(node_rows)
    if reservations is not None:
        eng.set_reservations(reservations)
    if quotas is not None:
        eng.set_quotas(quotas)
    eng.set_pods(pod_rows)
    begin, end = shard_range(len(node_rows), rank, world)
    eng.set_shard(begin, end)
    if comm == "loopback":
        name = [shm_name or (f"/kg_loopback_{os.getpid()}_{uuid.uuid4().hex[:8]}" if rank == 0 else None)]
        if shm_name is None and world > 1:
            dist.broadcast_object_list(name, src=0, group=group)
        eng.comm_init_loopback(rank, world, name[0])
        return eng
    if comm != "rccl":
        raise ValueError(f"unknown communicator {comm!r}")
    uid = [Engine.comm_unique_id() if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(uid, src=0, group=group)
    eng.comm_init(rank, world, uid[0])
    return eng


def place(cfg: np.ndarray, node_rows: np.ndarray, pod_rows: np.ndarray, now_ns: int,
          device: Optional[torch.device] = None, group=None, reservations: Optional[np.ndarray] = None,
          quotas: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray]:
    """Convenience wrapper: build the sharded engine, place the batch, release the engine."""
    device = device or torch.device("cuda", torch.cuda.current_device())
    eng = sharded_engine(cfg, node_rows, pod_rows, device, group, reservations, quotas)
    try:
        return place_sharded(eng, now_ns, device, chunk=place_chunk_of(cfg), group=group)
    finally:
        eng.close()
