"""Multi-GPU plumbing for the dwarf: one process per GPU, columns sharded with
no data-path collective.

Rank r of W owns the global columns [r*ngptot, (r+1)*ngptot) (weak scaling:
ngptot columns per GPU).  Every rank expands its columns from the KLON-column
template with the GLOBAL index (g % klon), so a sharded run computes exactly
the columns an unsharded run of W*ngptot columns would.  torch.distributed is
used only for control: the barriers around the timed region and the
max-over-ranks of the wall time (gloo on the host; nothing touches the
kernels' data).  The reference has no multi-GPU path; the Fortran dwarf's MPI
variant combines validation partials with MPI_Reduce (validate_mod.F90:53-55),
which combine_stats mirrors.
"""
from __future__ import annotations

import os
import sys
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple


@dataclass
class Topology:
    rank: int
    world: int
    local_rank: int

    @property
    def is_root(self) -> bool:
        return self.rank == 0


def topology_from_env() -> Topology:
    """RANK / WORLD_SIZE / LOCAL_RANK as set by torch.distributed.run."""
    return Topology(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                    int(os.environ.get("LOCAL_RANK", "0")))


def shard(rank: int, ngptot_per_rank: int) -> Tuple[int, int]:
    """(col_offset, ncols) of a rank under weak scaling."""
    if rank < 0 or ngptot_per_rank <= 0:
        raise ValueError("bad shard request")
    return rank * ngptot_per_rank, ngptot_per_rank


def split_blocks(ngptot: int, nproma: int, nparts: int) -> List[Tuple[int, int]]:
    """Block-aligned contiguous (col_offset, ncols) ranges covering ngptot
    columns with nparts parts (strong scaling; the C driver's --gpus split)."""
    nblocks = -(-ngptot // nproma)
    per, extra = divmod(nblocks, nparts)
    out, col = [], 0
    for p in range(nparts):
        cols = min((per + (1 if p < extra else 0)) * nproma, ngptot - col)
        if cols <= 0:
            break
        out.append((col, cols))
        col += cols
    return out


def _without_stdout(fn):
    """Run fn() with file descriptor 1 on /dev/null: gloo's C++ side prints its
    "[Gloo] Rank r is connected to ..." lines to stdout while the group connects,
    which would land beside rank 0's one-line JSON result."""
    sys.stdout.flush()
    saved = os.dup(1)
    devnull = os.open(os.devnull, os.O_WRONLY)
    try:
        os.dup2(devnull, 1)
        return fn()
    finally:
        os.dup2(saved, 1)
        os.close(saved)
        os.close(devnull)


class Control:
    """Barrier + max-over-ranks on a host (gloo) process group; a no-op for W=1."""

    def __init__(self, topo: Topology, backend: str = "gloo"):
        self.topo = topo
        self.dist = None
        if topo.world > 1:
            import torch.distributed as dist
            if not dist.is_initialized():
                # connect (and settle) with stdout muted
                _without_stdout(lambda: (dist.init_process_group(backend), dist.barrier()))
            self.dist = dist

    def barrier(self) -> None:
        if self.dist is not None:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather_stats(self, stats: Sequence[Sequence[float]]) -> Optional[List[Tuple[float, ...]]]:
        """Combine per-field (min, max, maxerr, errsum, refsum) over ranks."""
        if self.dist is None:
            return [tuple(s) for s in stats]
        import torch
        t = torch.tensor(stats, dtype=torch.float64)
        parts = [torch.zeros_like(t) for _ in range(self.topo.world)]
        self.dist.all_gather(parts, t)
        return combine_stats([p.tolist() for p in parts])

    def gather_records(self, rec: dict) -> List[dict]:
        """Every rank's record (a small JSON-able dict), in rank order, on every
        rank -- the per-rank timing table the reference gathers to rank 0
        (src/common/module/timer_mod.F90:160-167)."""
        if self.dist is None:
            return [dict(rec)]
        out: List[dict] = [None] * self.topo.world   # type: ignore[list-item]
        self.dist.all_gather_object(out, dict(rec))
        return out

    def close(self) -> None:
        if self.dist is not None:
            self.dist.destroy_process_group()
            self.dist = None


def dd_add(a, b):
    """Double-double sum of (hi, lo) pairs: the arithmetic of cloudsc_stats_combine
    (cloudsc_state.hip) in IEEE doubles, so partial sums combine to the same
    double in any grouping."""
    s = a[0] + b[0]
    bb = s - a[0]
    e = (a[0] - (s - bb)) + (b[0] - bb)
    t = e + (a[1] + b[1])
    hi = s + t
    return hi, t - (hi - s)


def combine_stats(per_rank: Sequence[Sequence[Sequence[float]]]) -> List[Tuple[float, ...]]:
    """min of mins, max of maxes, max of max|d|, sums of sum|d| and sum|ref|.
    Rows are (min, max, maxerr, errsum, refsum[, errsum_lo, refsum_lo]); with the
    low parts the sums are combined as double-doubles (cloudsc_stats_t), so the
    result does not depend on how the columns were split over ranks."""
    out = []
    for f in range(len(per_rank[0])):
        rows = [r[f] for r in per_rank]
        if all(len(r) >= 7 for r in rows):
            es, rs = (0.0, 0.0), (0.0, 0.0)
            for r in rows:
                es = dd_add(es, (r[3], r[5]))
                rs = dd_add(rs, (r[4], r[6]))
            out.append((min(r[0] for r in rows), max(r[1] for r in rows), max(r[2] for r in rows),
                        es[0], rs[0], es[1], rs[1]))
        else:
            out.append((min(r[0] for r in rows), max(r[1] for r in rows), max(r[2] for r in rows),
                        sum(r[3] for r in rows), sum(r[4] for r in rows)))
    return out
