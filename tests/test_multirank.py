"""Multi-GPU plumbing of the path rehearsed on CPU (gloo, world size 2), with the PRODUCT
classifying every shard: each rank runs the library's per-tuple code (pg_debug_classify_host,
the same templates the kernels instantiate) over its contiguous global index range of a
device-generator-identical workload, and the per-rule hit counters are summed over the ranks
(vpp_amd.dist.allreduce_counters; on GPUs bench.py sums them with the library's own RCCL
communicator, pg_allreduce_counters). The all-reduced histogram must equal the C oracle's
histogram over the whole index range.

Also: bench.py's launcher (--gpus 2 without a torchrun environment re-launches itself under
torchrun, one rank per GPU) on its CPU dry-run path, weak and strong scaling."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

N_PER_RANK = 20000
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gen(w, base, n):
    """the shard's tuples as k_gen makes them (oracle.gen restatement)"""
    from oracle import gen
    e = w.engine
    rules = e.GetACLByName(e.ACLNames()[w.table_id])["rules"] if w.table_id >= 0 else None
    return gen.gen_tuples(n, index_base=base, rules=rules, **w.gen)


def _product_counters(w, base, n):
    """the shard's tuples classified by the product's per-tuple code on the host"""
    src, dst, sport, dport, proto = _gen(w, base, n)
    out, cnt = w.engine.debug_classify_host(w.mode, w.table_id, src, dst, sport, dport, proto, counters=True)
    return out, cnt.astype(np.int64)


def _worker(rank, world, port, q, config):
    import traceback

    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=__import__("datetime").timedelta(seconds=120))
    try:
        from vpp_amd import dist as vd
        from vpp_amd import workloads as W
        w = W.CONFIGS[config](0, n_tuples=N_PER_RANK)
        base, n = vd.shard(rank, world, N_PER_RANK)
        out, cnt = _product_counters(w, base, n)
        counters = torch.from_numpy(cnt.copy())
        vd.allreduce_counters(counters)
        ranges = [None] * world
        dist.all_gather_object(ranges, (base, n))
        verdicts = [None] * world
        dist.all_gather_object(verdicts, out.tolist())
        if rank == 0:
            q.put((counters.numpy().tolist(), ranges, verdicts))
    except Exception:
        q.put(("error", rank, traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("config", [1, 2])
def test_two_rank_product_shards_and_counter_allreduce(config):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, config)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert res[0] != "error", res[2]
    reduced, ranges, verdicts = res
    assert all(p.exitcode == 0 for p in procs)
    # shards are contiguous, disjoint and cover [0, world * N)
    assert sorted(ranges) == [(r * N_PER_RANK, N_PER_RANK) for r in range(world)]

    from oracle.world import World
    from vpp_amd import workloads as W
    w = W.CONFIGS[config](0, n_tuples=N_PER_RANK)
    src, dst, sport, dport, proto = _gen(w, 0, world * N_PER_RANK)
    if w.mode == 2:  # config 1: testConnection (CONN)
        wd = World(w.engine, w.local_ifs, w.node_if)
        # CONN counts every evalACL testConnection makes: the oracle's per-evaluation histogram
        act, slot, hist = wd.conn(src, dst, sport, dport, proto, threads=2, hist=True)
        assert reduced == hist.tolist()
        assert sum(reduced) > world * N_PER_RANK
    else:  # config 2: evalACL of the single table, one evaluation per tuple
        from oracle import fast
        e = w.engine
        rules = e.GetACLByName(e.ACLNames()[w.table_id])["rules"]
        act, idx = fast.eval_acl(fast.OraACL(rules), src, dst, dport, proto)
        slot = np.where(idx >= 0, e.slot_of_rule(w.table_id, 0) + idx.astype(np.int64),
                        e.slot_of_rule(w.table_id, -1)).astype(np.uint32)
        assert reduced == np.bincount(slot, minlength=len(reduced)).tolist()
    got = np.concatenate([np.asarray(v, np.uint32) for v in verdicts])
    assert np.array_equal(got >> 30, act.astype(np.uint32)) and np.array_equal(got & 0x3FFFFFFF, slot)
    assert len(set((got >> 30).tolist())) >= 2


def test_shard_helpers():
    from vpp_amd import dist as vd
    assert vd.shard(3, 8, 125) == (375, 125)
    parts = [vd.shard_strong(r, 3, 10) for r in range(3)]
    assert parts == [(0, 4), (4, 4), (8, 2)]
    with pytest.raises(ValueError):
        vd.shard(2, 2, 5)


def _bench(*args):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("scaling", ["weak", "strong"])
def test_bench_launcher_two_ranks_cpu_dry_run(scaling):
    """bench.py --gpus 2 started as one process re-launches itself under torchrun: two ranks,
    disjoint shards, one JSON line from rank 0 with n_gpus 2 and the all-reduced counters
    accounting for every tuple of both ranks."""
    args = ["--gpus", "2", "--cpu-dry-run", "--config", "2", "--steps", "2", "--warmup", "1", "--scaling", scaling]
    if scaling == "strong":
        args += ["--total-tuples", "20001"]
    d = _bench(*args)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["scaling"] == scaling
    assert d["counter_allreduce_check"] is True
    # every rank checked its own shard against the oracle: verdicts and hit counters
    assert [p["index_base"] for p in d["parity_per_rank"]] == [0, d["parity_per_rank"][0]["tuples"]]
    assert all(p["bit_exact_action_and_rule_index"] and p["counters_equal_oracle_histogram"]
               for p in d["parity_per_rank"])
    assert d["parity_sample"]["tuples"] == d["config"]["tuples_total"]
    if scaling == "strong":
        assert d["config"]["tuples_total"] == 20001
    else:
        assert d["config"]["tuples_total"] == 2 * d["config"]["tuples_per_gpu"]
    one = _bench("--gpus", "1", "--cpu-dry-run", "--config", "2", "--steps", "1", "--warmup", "0")
    assert one["n_gpus"] == 1 and one["parity_sample"]["bit_exact_action_and_rule_index"]


def test_bench_two_ranks_conn_counters_cpu_dry_run():
    """config 5 (testConnection with hit counters) over two ranks: each rank's counters equal
    the oracle's per-evaluation histogram of its shard, and the summed counters that of the
    whole job."""
    d = _bench("--gpus", "2", "--cpu-dry-run", "--config", "5", "--tuples", "6000", "--steps", "1", "--warmup", "0")
    assert d["counter_allreduce_check"] is True and d["parity_sample"]["counters_equal_oracle_histogram"]
    assert all(p["evaluations"] > p["tuples"] for p in d["parity_per_rank"])


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu-dry-run"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode != 0 and "--gpus 2" in (r.stderr + r.stdout)
