"""Multi-process control path of bench.py on the CPU (gloo, world size 2):
weak-scaling shards, barrier + max-over-ranks, combined validation statistics,
and the sharding semantics themselves -- rank r's columns, computed by the
oracle with the GLOBAL g % klon map, equal the matching slice of an unsharded
run bit for bit (no data-path collective exists to get this wrong later)."""
import os
import socket

import numpy as np
import pytest

import cloudsc_amd as ca
import cloudsc_dist as cd


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    try:
        topo = cd.topology_from_env()
        ctl = cd.Control(topo)
        ctl.barrier()
        wall = ctl.max(0.5 + rank)                       # the slowest rank defines the step time
        off, n = cd.shard(topo.rank, 1000)
        # per-rank validation partials: field 0 gets rank-dependent numbers
        stats = [[-1.0 - rank, 1.0 + rank, 0.1 * (rank + 1), 2.0, 10.0]] + [[0.0, 0.0, 0.0, 0.0, 1.0]] * 20
        comb = ctl.gather_stats(stats)
        # bench.py's per-rank record, gathered in rank order on every rank
        recs = ctl.gather_records({"rank": rank, "device": rank % 1, "kernel_ms": 1.5 + rank, "col_offset": off})
        ctl.barrier()
        ctl.close()
        q.put((rank, wall, off, n, comb[0], len(comb), recs))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, "error", repr(e)))


def test_gloo_world2_control_path():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] != "error", r
    assert [r[1] for r in res] == [1.5, 1.5]
    assert [(r[2], r[3]) for r in res] == [(0, 1000), (1000, 1000)]
    for r in res:
        assert r[4] == (-2.0, 2.0, 0.2, 4.0, 20.0) and r[5] == 21
        assert r[6] == [{"rank": 0, "device": 0, "kernel_ms": 1.5, "col_offset": 0},
                        {"rank": 1, "device": 0, "kernel_ms": 2.5, "col_offset": 1000}]


def test_gloo_connect_leaves_stdout_to_rank0():
    """Under torch.distributed.run (the driver's N>1 launch) gloo's connection
    messages go to stdout from C++; Control mutes them, so rank 0's one line
    is the whole of stdout."""
    import subprocess
    import sys
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_stdout_child.py")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()), child],
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines() == ['{"rank0": true}'], r.stdout


def test_single_rank_control_is_noop():
    ctl = cd.Control(cd.Topology(0, 1, 0))
    ctl.barrier()
    assert ctl.max(3.0) == 3.0
    st = [[1.0, 2.0, 3.0, 4.0, 5.0]]
    assert ctl.gather_stats(st) == [(1.0, 2.0, 3.0, 4.0, 5.0)]
    assert ctl.gather_records({"rank": 0, "kernel_ms": 1.0}) == [{"rank": 0, "kernel_ms": 1.0}]


def test_split_blocks_covers_columns():
    for ngptot, nproma, parts in [(163840, 128, 8), (1000, 128, 3), (100, 32, 8), (1310720, 128, 8)]:
        sp = cd.split_blocks(ngptot, nproma, parts)
        assert sp[0][0] == 0 and sum(n for _, n in sp) == ngptot
        for (o1, n1), (o2, _) in zip(sp, sp[1:]):
            assert o1 + n1 == o2 and o2 % nproma == 0


def test_sharded_oracle_equals_unsharded(ds, oracle_mod):
    """Weak-scaling semantics: two 256-column shards == one 512-column run."""
    full, _ = oracle_mod.run_oracle(ds, 512, 128)
    ref = ca.state_outputs_to_template(full.arrays, 512)
    for rank in range(2):
        off, n = cd.shard(rank, 256)
        part, _ = oracle_mod.run_oracle(ds, n, 128, col_offset=off)
        out = ca.state_outputs_to_template(part.arrays, n)
        for _, k in ca.VALIDATED:
            assert np.array_equal(out[k], ref[k][..., off:off + n]), (rank, k)


def test_combine_stats_matches_unsharded(ds):
    """Host-side combination of per-shard ERROR_PRINT partials equals the
    statistics of the whole field (sums up to rounding)."""
    rng = np.random.default_rng(7)
    for _, k in ca.VALIDATED[:5]:
        ref = ds.reference[k]
        out = ref * (1 + 1e-12 * rng.standard_normal(ref.shape))
        whole = ca.field_stats(out, ref)
        halves = [ca.field_stats(out[..., :50], ref[..., :50]), ca.field_stats(out[..., 50:], ref[..., 50:])]
        comb = cd.combine_stats([[h] for h in halves])[0]
        assert comb[:3] == whole[:3]
        assert comb[3] == pytest.approx(whole[3], rel=1e-12) and comb[4] == pytest.approx(whole[4], rel=1e-12)


def test_double_double_sums_are_partition_invariant():
    """The validation sums are double-doubles (cloudsc_stats_t), so per-block,
    per-shard and per-rank partials combine to the same double however the
    columns are split -- the property that makes a sharded dwarf print the
    unsharded run's table to the last digit.  Checked against math.fsum (the
    correctly rounded sum) for random splits of 10^5 non-negative terms."""
    import math
    rng = np.random.default_rng(3)
    x = np.abs(rng.standard_normal(100000)) * 10.0 ** rng.integers(-20, 5, 100000)
    exact = math.fsum(x)
    for nparts in (1, 2, 3, 8, 10240):
        cuts = np.sort(rng.choice(np.arange(1, x.size), nparts - 1, replace=False)) if nparts > 1 else []
        parts = np.split(x, cuts)
        partial = []
        for p in parts:                          # each part summed element by element
            acc = (0.0, 0.0)
            for v in p.tolist():
                acc = cd.dd_add(acc, (v, 0.0))
            partial.append(acc)
        order = rng.permutation(len(partial))    # and combined in any order
        tot = (0.0, 0.0)
        for i in order:
            tot = cd.dd_add(tot, partial[i])
        assert tot[0] == exact, nparts


def test_stats_combine_c_abi_matches_python():
    """cloudsc_stats_combine (libcloudsc_amd, host code: no GPU needed) is the
    same arithmetic as cloudsc_dist.combine_stats."""
    import ctypes as C
    lib = ca.gpu_lib()
    lib.cloudsc_stats_combine.argtypes = [C.POINTER(ca.Stats), C.POINTER(ca.Stats)]
    rng = np.random.default_rng(5)
    rows = [tuple(float(v) for v in (-rng.random(), rng.random(), rng.random(), rng.random() * 1e3,
                                      rng.random() * 1e6, rng.random() * 1e-14, rng.random() * 1e-11))
            for _ in range(17)]
    acc = ca.Stats(1.7976931348623157e308, -1.7976931348623157e308, 0.0, 0.0, 0.0, 0.0, 0.0)
    for r in rows:
        part = ca.Stats(*r)
        lib.cloudsc_stats_combine(C.byref(acc), C.byref(part))
    py = cd.combine_stats([[r] for r in rows])[0]
    assert (acc.minval, acc.maxval, acc.maxerr, acc.errsum, acc.refsum, acc.errsum_lo, acc.refsum_lo) == py
