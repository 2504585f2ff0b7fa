"""Multi-GPU plumbing for the ICP path: one process per GPU.

* Independent pairs (config C4): rank r owns global pairs [r*n, (r+1)*n);
  no collective on the data path; the fp32 poses are all-gathered at the end
  (RCCL over xGMI under the "nccl" backend, gloo in the CPU tests).
* Streamed sequence (config C5): the F-1 frame pairs (k, k+1) are split into
  contiguous ranges; rank r also holds the frame after its last pair (a
  1-frame halo), so no data crosses ranks during tracking.  Rank 0 composes
  the world trajectory by an ordered fp64 prefix product.

Pure torch.distributed; no device code here.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist


def pair_shard(rank: int, pairs_per_rank: int) -> tuple[int, int]:
    """(first global pair index, count) of `rank` under weak scaling."""
    return rank * pairs_per_rank, pairs_per_rank


def pair_range(n_pairs: int, world: int, rank: int) -> tuple[int, int]:
    """(first global pair index, count) of `rank` when ONE batch of n_pairs is
    split into contiguous shards (strong scaling, SURVEY §8e: 512 pairs ->
    512/256/128/64 per GPU at N = 1/2/4/8); the first n_pairs % world ranks
    take one extra pair."""
    base, extra = divmod(n_pairs, world)
    return rank * base + min(rank, extra), base + (1 if rank < extra else 0)


def sequence_shard(n_frames: int, world: int, rank: int) -> tuple[int, int]:
    """Frames [f0, f1) held by `rank` so that its pairs (k, k+1), k in
    [f0, f1-1), tile the F-1 pairs exactly once across ranks; the last frame
    of each shard is the next shard's first (halo).  Ranks with no pairs get
    (f, f)."""
    n_pairs = n_frames - 1
    base, extra = divmod(n_pairs, world)
    p0 = rank * base + min(rank, extra)
    cnt = base + (1 if rank < extra else 0)
    if cnt == 0:
        return p0, p0
    return p0, p0 + cnt + 1


def gather_poses(local: torch.Tensor, world: int) -> torch.Tensor:
    """All-gather [n, 16] pose rows from every rank, rank-ordered.  World 1
    returns `local` unless a process group is up (then the collective runs:
    the one-GPU RCCL check of bench.py, YOUTH_BENCH_DIST=1)."""
    if world == 1 and not dist.is_initialized():
        return local
    out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    if dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(out, local.contiguous())
    else:  # gloo: host tensors (CPU tests; the one-GPU rehearsal of bench.py)
        host = local.detach().cpu().contiguous()
        parts = list(torch.empty((world,) + tuple(host.shape), dtype=host.dtype).unbind(0))
        dist.all_gather(parts, host)
        out.copy_(torch.cat(parts).to(out.device))
    return out


def gather_poses_async(local: torch.Tensor, out: torch.Tensor, world: int):
    """Start the all-gather of [n, 16] pose rows into `out` ([world * n, 16],
    rank-ordered) and return its work handle (RCCL: `handle.wait()` makes the
    current stream wait for it, the host does not block), or None when there
    is nothing to wait for (world 1: no gather, `out` untouched; gloo: host
    tensors, synchronous).
    Callers double-buffer `local` / `out` so the next align overlaps the
    gather of the previous one."""
    if world == 1 and not dist.is_initialized():
        return None   # nothing to gather: `out` is not written
    if dist.get_backend() == "nccl":
        return dist.all_gather_into_tensor(out, local.contiguous(), async_op=True)
    out.copy_(gather_poses(local, world))
    return None


def gather_poses_ragged_async(local: torch.Tensor, out: torch.Tensor, world: int,
                              counts: list[int]):
    """gather_poses_async for shards of rank-dependent size (counts[r] rows on
    rank r, pair_range): equal shards take the single RCCL all-gather, ragged
    ones are padded to the largest shard (synchronous).  Returns the work
    handle or None (world 1: nothing to gather, `out` untouched)."""
    if world == 1 and not dist.is_initialized():
        return None
    if all(c == counts[0] for c in counts):
        return gather_poses_async(local, out, world)
    out.copy_(gather_ragged(local, world, max(counts), counts))
    return None


def gather_ragged(local: torch.Tensor, world: int, max_rows: int,
                  counts: list[int] | None = None) -> torch.Tensor:
    """All-gather [m_r, 16] rows with different m_r per rank (sequence
    shards): pad to max_rows, gather the rows (and the counts, unless the
    caller knows them: sequence_shard gives every rank's), strip padding."""
    if world == 1 and not dist.is_initialized():
        return local
    pad = torch.zeros((max_rows,) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    pad[: local.shape[0]] = local
    if counts is None:
        cnt = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
        counts = [int(v) for v in gather_poses(cnt, world)]
    rows = gather_poses(pad, world).view(world, max_rows, *local.shape[1:])
    return torch.cat([rows[r, : counts[r]] for r in range(world)])


def rank_report(timings: dict, world: int, values: dict | None = None) -> dict:
    """Every rank's timings (ms) in rank order plus what the process group
    itself reports, for an N > 1 bench line that proves its own shape
    (VERDICT r2 item 7): `rccl_world_size` / `backend` from the group, and
    `per_rank_ms[name] = [rank 0, rank 1, ...]`; `values` (non-time figures,
    e.g. each rank's pose error against the CPU oracle) the same way under
    `per_rank`.  Collective: every rank calls it with the same keys.  No group
    (N = 1 without YOUTH_BENCH_DIST): world size 1, this rank's values."""
    values = values or {}
    keys = sorted(timings)
    vkeys = sorted(values)
    vals = [float(timings[k]) for k in keys] + [float(values[k]) for k in vkeys]
    if not dist.is_initialized():
        out = {"rccl_world_size": 1, "backend": None,
               "per_rank_ms": {k: [float(timings[k])] for k in keys}}
        if vkeys:
            out["per_rank"] = {k: [float(values[k])] for k in vkeys}
        return out
    backend = dist.get_backend()
    gw = dist.get_world_size()
    dev = "cuda" if backend == "nccl" else "cpu"
    t = torch.tensor(vals, dtype=torch.float64, device=dev)
    out = torch.zeros(gw * len(vals), dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(out, t)
    rows = out.view(gw, len(vals)).cpu().numpy()
    rep = {"rccl_world_size": int(gw), "backend": backend, "launch_world": int(world),
           "per_rank_ms": {k: [float(rows[r, i]) for r in range(gw)]
                           for i, k in enumerate(keys)}}
    if vkeys:
        rep["per_rank"] = {k: [float(rows[r, len(keys) + i]) for r in range(gw)]
                           for i, k in enumerate(vkeys)}
    return rep


def compose_trajectory(rel: np.ndarray) -> np.ndarray:
    """World poses of frames 0..F-1 from relative poses T_k (P_k = T_k P_{k+1}):
    T_w,0 = I, T_w,k+1 = T_w,k @ T_k (fp64, ordered)."""
    rel = np.asarray(rel, dtype=np.float64).reshape(-1, 4, 4)
    out = np.empty((rel.shape[0] + 1, 4, 4), np.float64)
    out[0] = np.eye(4)
    for k in range(rel.shape[0]):
        out[k + 1] = out[k] @ rel[k]
    return out


# ---- the C-ABI RCCL gather (include/youth_dist.h, libyouth_dist.so) --------
# For one-process-per-GPU hosts that do not use torch.distributed: the same
# contiguous shards, one ncclAllGather of the padded largest shard and a
# compaction kernel.  Python binding for the tests (tests/test_gpu_bench.py).
DIST_ID_BYTES = 128
_dist_lib = None


def _dist():
    global _dist_lib
    if _dist_lib is None:
        import ctypes
        from ctypes import POINTER, c_char_p, c_int, c_void_p
        import youth_icp
        youth_icp.load_library()  # libyouth_icp.so first (DT_NEEDED of libyouth_dist.so)
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libyouth_dist.so")
        if not os.path.exists(path):
            raise OSError(f"{path} not built: run `make -C {os.path.dirname(path)}`")
        lib = ctypes.CDLL(path)
        sig = {
            "youth_dist_unique_id": (c_int, [c_char_p]),
            "youth_dist_create": (c_void_p, [c_int, c_int, c_int, c_char_p]),
            "youth_dist_allgather_poses": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
            "youth_dist_allgather_poses_host": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
            "youth_dist_row_source": (c_int, [c_int, c_int, c_int, POINTER(c_int), POINTER(c_int)]),
            "youth_dist_nranks": (c_int, [c_void_p]),
            "youth_dist_rank": (c_int, [c_void_p]),
            "youth_dist_destroy": (None, [c_void_p]),
            "youth_dist_last_error": (c_char_p, []),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _dist_lib = lib
    return _dist_lib


def _dist_check(rc):
    import youth_icp
    if rc < 0:
        raise youth_icp.IcpError(rc, (_dist().youth_dist_last_error() or b"").decode())


def row_source(n_pairs, nranks, row):
    """youth_dist_row_source -> (rank, index in its shard)."""
    import ctypes
    q, i = ctypes.c_int(0), ctypes.c_int(0)
    _dist_check(_dist().youth_dist_row_source(n_pairs, nranks, row, ctypes.byref(q),
                                               ctypes.byref(i)))
    return q.value, i.value


def unique_id() -> bytes:
    import ctypes
    buf = ctypes.create_string_buffer(DIST_ID_BYTES)
    _dist_check(_dist().youth_dist_unique_id(buf))
    return buf.raw


class RcclPoseGather:
    """youth_dist_create / allgather_poses(_host) / destroy."""

    def __init__(self, nranks: int, rank: int, device: int, uid: bytes):
        import youth_icp
        lib = _dist()
        self._h = lib.youth_dist_create(nranks, rank, device, uid)
        if not self._h:
            msg = (lib.youth_dist_last_error() or b"").decode()
            code = youth_icp.YOUTH_ENODEV if "no HIP device" in msg else youth_icp.YOUTH_EHIP
            raise youth_icp.IcpError(code, msg)

    def allgather_device(self, d_local: int, n_pairs: int, d_all: int, stream: int = 0):
        _dist_check(_dist().youth_dist_allgather_poses(self._h, d_local or None, n_pairs, d_all,
                                                       stream or None))

    def allgather_host(self, local, n_pairs: int):
        import numpy as np
        loc = np.ascontiguousarray(local, np.float32).reshape(-1, 16)
        out = np.zeros((n_pairs, 16), np.float32)
        _dist_check(_dist().youth_dist_allgather_poses_host(
            self._h, loc.ctypes.data if loc.size else None, n_pairs, out.ctypes.data))
        return out

    def close(self):
        if self._h:
            _dist().youth_dist_destroy(self._h)
            self._h = None

    __del__ = close
