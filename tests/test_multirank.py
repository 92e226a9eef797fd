"""World-size-2 run of the multi-GPU plumbing on CPU (gloo): shards of a device-generated
workload regenerated per rank, verdicts per rank, and the per-rule counter all-reduce
(vpp_amd.dist, what bench.py runs over RCCL) equal to the single-process histogram over the
whole index range."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

N_PER_RANK = 20000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _histogram(w, wd, base, n):
    from oracle import gen
    src, dst, sport, dport, proto = gen.gen_tuples(n, index_base=base, **w.gen)
    conn, slot = wd.conn(src, dst, sport, dport, proto, threads=2)
    return np.bincount(slot, minlength=w.engine.num_counter_slots()).astype(np.int64), conn


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.world import World
        from vpp_amd import dist as vd
        from vpp_amd import workloads as W
        w = W.config1(0, n_tuples=N_PER_RANK)
        wd = World(w.engine, w.local_ifs, w.node_if)
        base, n = vd.shard(rank, world, N_PER_RANK)
        h, _ = _histogram(w, wd, base, n)
        counters = torch.from_numpy(h.copy())
        vd.allreduce_counters(counters)
        ranges = [None] * world
        dist.all_gather_object(ranges, (base, n))
        if rank == 0:
            q.put((counters.numpy().tolist(), ranges))
    finally:
        dist.destroy_process_group()


def test_two_rank_shards_and_counter_allreduce():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        reduced, ranges = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    # shards are contiguous, disjoint and cover [0, world * N)
    assert sorted(ranges) == [(r * N_PER_RANK, N_PER_RANK) for r in range(world)]

    from oracle.world import World
    from vpp_amd import workloads as W
    w = W.config1(0, n_tuples=N_PER_RANK)
    wd = World(w.engine, w.local_ifs, w.node_if)
    full, conn = _histogram(w, wd, 0, world * N_PER_RANK)
    assert reduced == full.tolist()
    assert full.sum() == world * N_PER_RANK
    assert len(set(conn.tolist())) >= 2


def test_shard_helpers():
    from vpp_amd import dist as vd
    assert vd.shard(3, 8, 125) == (375, 125)
    parts = [vd.shard_strong(r, 3, 10) for r in range(3)]
    assert parts == [(0, 4), (4, 4), (8, 2)]
    with pytest.raises(ValueError):
        vd.shard(2, 2, 5)
