#!/usr/bin/env python3
"""Benchmark: classified 5-tuples/s of the policy classification path on MI355X.

One step = one pass of the classify kernel over one batch of synthetic 5-tuples already
resident in HBM (BASELINE.json configs[1] by default: 1k-rule gen-policy-shaped table,
64M tuples per GPU). Multi-GPU (torchrun, one process per GPU): every rank classifies its
own shard (tuple index range) against replicated tables -- no data-path collective, weak
scaling. After the timed region the per-rule hit counters are summed across ranks with one
RCCL all-reduce (the statscollector path) and its time is reported separately.

Prints ONE JSON line (rank 0). See DESIGN.md §Measurement for the byte accounting.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from vpp_amd import _capi  # noqa: E402
from vpp_amd import device as D  # noqa: E402
from vpp_amd import dist as VD  # noqa: E402
from vpp_amd import workloads as W  # noqa: E402

METRIC = "classified 5-tuples/sec (Mpps) at 1/2/4/8 GPUs vs rule count; % of HBM peak"
HBM_PEAK_GBS = 8000.0           # MI355X HBM3E spec (MI355X_MICROARCH.md)
MODE_NAME = {0: "single", 1: "perpod", 2: "conn"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1,
                   help="GPUs = ranks; > 1 without a torchrun environment re-launches under torchrun")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", type=int, default=2, choices=sorted(W.CONFIGS))
    p.add_argument("--tuples", type=int, default=0, help="tuples per GPU (weak scaling; default: the config's)")
    p.add_argument("--rules", type=int, default=0,
                   help="config 2 only: rules of the gen-policy-shaped table (rule-count sweep; default 1000)")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="budget of the multithreaded CPU baseline (the sample is sized by a calibration run)")
    p.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                   help="weak: --tuples per GPU; strong: --total-tuples split over the GPUs")
    p.add_argument("--total-tuples", type=int, default=0,
                   help="strong scaling: tuples of the whole job (default 8 x the config's per-GPU count)")
    p.add_argument("--counters", action="store_true", help="time with per-rule hit counters on")
    p.add_argument("--cpu-sample", type=int, default=16 << 20, help="tuples in the CPU-baseline sample")
    p.add_argument("--faithful-seconds", type=float, default=8.0,
                   help="budget of the single-thread reference-faithful CPU variant")
    p.add_argument("--side", default="auto",
                   help="configs timed after the main line in labelled side blocks, same launches and "
                        "self-check (comma list, 'none'; auto = 3,4,5 when the main config is 2 without "
                        "--rules / --counters: BASELINE.json configs[2..4] -- the 10k-rule per-pod config "
                        "north_star names, the 100k-rule table, testConnection with hit counters)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--check-tuples", type=int, default=1 << 20,
                   help="tuples of every rank's shard checked against the oracle after the timed region")
    p.add_argument("--no-check", action="store_true", help="skip the per-rank oracle self-check")
    p.add_argument("--per-table", action="store_true",
                   help="PERPOD/CONN through the per-table blobs + IP hash instead of the node classifier")
    p.add_argument("--cpu-dry-run", action="store_true",
                   help="no GPU: the launcher, sharding, timing and counter all-reduce over gloo, with the "
                        "product's per-tuple code run on the host (tests only; no throughput claim)")
    return p.parse_args()


def relaunch(a):
    """--gpus N > 1 started as a plain process: run this script under torchrun (one rank per GPU)
    as a child -- before anything touches the GPU -- and exit with its status."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % a.gpus,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def shard_of(a, w, rank, world):
    """global tuple-index range of this rank"""
    if a.scaling == "strong":
        total = a.total_tuples or 8 * w.n_tuples
        return VD.shard_strong(rank, world, total)
    return VD.shard(rank, world, a.tuples or w.n_tuples)


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch(a))
    rank, world, local = VD.env()
    if world != a.gpus:
        raise SystemExit("bench.py: --gpus %d but the launcher started %d ranks" % (a.gpus, world))
    if a.cpu_dry_run:
        return dry_run(a, rank, world)
    # under torchrun (the driver's N > 1 launch, or --nproc-per-node 1 to rehearse it on one
    # GPU) the process group, barriers, max-over-ranks timing and the library's RCCL counter
    # all-reduce all run, whatever the world size
    launched = "WORLD_SIZE" in os.environ
    # stdout carries the ONE JSON line: whatever native libraries print there (RCCL's version
    # banner at communicator init) goes to stderr instead
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    torch.cuda.set_device(local)
    if launched:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    kw = {"n_tuples": a.tuples} if a.tuples else {}
    if a.rules:
        if a.config != 2:
            raise SystemExit("--rules applies to config 2 (the gen-policy-shaped table)")
        kw["n_rules"] = a.rules
    w = W.CONFIGS[a.config](local, **kw)
    e = w.engine
    if a.per_table:
        e.set_tuning("node_path", 0)
    st = w.stats()
    base, n = shard_of(a, w, rank, world)  # disjoint global index ranges
    b = D.TupleBatch(n, with_sport=(w.mode == 2))
    D.gen_tuples(e, b, index_base=base, **w.gen)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    nslots = e.num_counter_slots()
    counters = torch.zeros(nslots, dtype=torch.int64, device="cuda")
    use_counters = a.counters or w.counters  # config 5 runs with per-rule hit counters
    cptr = counters if use_counters else None
    torch.cuda.synchronize()

    for _ in range(a.warmup):
        D.classify(e, w.mode, w.table_id, b, out, counters=cptr)
    # HIP events on the stream the kernel is launched on (torch's current stream, which
    # D.classify passes to pg_classify), bracketing the K back-to-back launches: the
    # per-launch average includes the inter-launch gaps, so it is an upper bound of the
    # kernel duration rocprofv3 reports.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    if launched:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(a.steps):
        D.classify(e, w.mode, w.table_id, b, out, counters=cptr)
    ev1.record()
    torch.cuda.synchronize()
    if launched:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / a.steps
    wall = VD.max_over_ranks(wall, "cuda")
    ms_per_step = wall * 1e3 / a.steps
    total_tuples = VD.sum_over_ranks(n, "cuda") * a.steps
    mpps = total_tuples / wall / 1e6

    # after the timed region (reported beside `value`, never as it): the same launches once the
    # core clock has settled -- the first ~40 launches of a burst run at a lower clock while the
    # chip's power management settles (profiles/r03_ramp_*: config 3 launches 4-10 at 1.8-1.95
    # GHz, 2.37 GHz from launch ~36), which the driver's 5-warm-up / 20-step window catches
    steady = steady_state(e, w, b, out, cptr, n, world)

    bpt, fields = bytes_per_tuple(w)
    achieved = n * bpt / (kern_ms * 1e-3) / 1e9
    label = "%d" % a.config + ("r%d" % a.rules if a.rules else "")
    traffic, traffic_src = pmc_traffic(label, n, a.counters and not w.counters)
    line = {
        "metric": METRIC, "value": round(mpps, 1), "unit": "Mpps", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": a.scaling,
        "vs_baseline": None, "dtype": "u32", "data": "synthetic (device-generated, counter-based splitmix64)",
        "config": {"workload": "config%d: %s" % (a.config, w.desc) + (" [rule-count sweep]" if a.rules else ""),
                   "mode": MODE_NAME[w.mode],
                   "tuples_per_gpu": n, "tuples_total": total_tuples // a.steps, "rules": st["rules"],
                   "tables": st["tables"], "parallelism": "dp%d" % world,
                   "counters": bool(use_counters), "classifier": classifier(w, a.per_table)},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "bytes_per_tuple": bpt, "fields": fields, "kernel_ms": round(kern_ms, 4),
                     "algorithmic_bytes_per_launch": n * bpt, "traffic_source": traffic_src},
    }
    line["steady_state"] = steady
    # the same fraction against what moving this launch's own bytes reaches on this GPU (after
    # the timed region): pg_stream_probe issues the classify launch's loads and store over the
    # same batch without the classification; torch's 1 GiB device copy beside it
    probe = stream_ceiling_gbps(e, w, b, out, bpt, a.steps)
    cp = torch_copy_gbps()
    line["roofline"]["measured_stream_gbps"] = {"probe": probe, "copy": cp}
    line["roofline"]["frac_of_measured_stream"] = round(achieved / probe, 4)

    # Self-check of every rank's shard (after the timed region), whatever the world size: the
    # timed run's verdicts of the shard's first --check-tuples tuples against the oracle, and a
    # counted pass over them whose hit counters must equal the oracle's histogram
    check_threads = max(1, host_cores() // world)
    par = shard_check(w, b, out, base, a.check_tuples, check_threads) if not a.no_check else None
    # statscollector path (torchrun launches): the per-rule hit counters of one counted pass over
    # every rank's whole shard, summed by RCCL through the library's own communicator
    # (pg_allreduce_counters) and checked against torch.distributed's sum of the same local
    # histograms
    if launched:
        line.update(counter_allreduce(e, w, b, out, rank, world))
    if par is not None:
        pars = VD.gather_objects(par)
        line["parity_sample"] = {"ranks": world, "tuples": sum(p["tuples"] for p in pars),
                                 "bit_exact_action_and_rule_index": all(p["bit_exact_action_and_rule_index"]
                                                                        for p in pars),
                                 "counters_equal_oracle_histogram": all(p["counters_equal_oracle_histogram"]
                                                                        for p in pars)}
        line["parity_per_rank"] = pars
    if rank == 0 and world == 1 and not a.no_cpu:
        line["cpu_baseline"] = cpu_baseline(w, b, out, a.cpu_sample, a.faithful_seconds, a.cpu_seconds)
    side = a.side if a.side != "auto" else ("3,4,5" if a.config == 2 and not a.rules and not a.counters and
                                             not a.tuples and not a.per_table else "none")
    if side != "none":
        del b, out, counters
        torch.cuda.empty_cache()
        for c in side.split(","):
            line["side_config%s" % c] = side_line(a, int(c), rank, world, local, launched, check_threads)
            torch.cuda.empty_cache()
    if rank == 0:
        print(json.dumps(line), file=json_out, flush=True)
    if launched:
        dist.destroy_process_group()


def side_line(a, config, rank, world, local, launched, check_threads):
    """A labelled side block of the bench line: config `config` (its default shape, per-GPU
    tuples, scaling as the main line) timed exactly like `value` -- a.warmup untimed launches, then
    a.steps launches between barriers + synchronize, max over ranks -- with its roofline fraction
    and every rank's self-check. Reported beside `value`, never as it."""
    w = W.CONFIGS[config](local)
    e = w.engine
    base, n = shard_of(argparse.Namespace(**dict(vars(a), tuples=0)), w, rank, world)
    b = D.TupleBatch(n, with_sport=(w.mode == 2))
    D.gen_tuples(e, b, index_base=base, **w.gen)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    cptr = torch.zeros(e.num_counter_slots(), dtype=torch.int64, device="cuda") if w.counters else None
    torch.cuda.synchronize()
    for _ in range(a.warmup):
        D.classify(e, w.mode, w.table_id, b, out, counters=cptr)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    if launched:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(a.steps):
        D.classify(e, w.mode, w.table_id, b, out, counters=cptr)
    ev1.record()
    torch.cuda.synchronize()
    if launched:
        dist.barrier()
    torch.cuda.synchronize()
    wall = VD.max_over_ranks(time.perf_counter() - t0, "cuda")
    kern_ms = ev0.elapsed_time(ev1) / a.steps
    bpt, fields = bytes_per_tuple(w)
    achieved = n * bpt / (kern_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic("%d" % config, n, False)
    res = {"note": "side block: timed like `value` (%d warm-ups, %d steps), not the bench value" % (a.warmup, a.steps),
           "workload": "config%d: %s" % (config, w.desc), "mode": MODE_NAME[w.mode], "counters": bool(w.counters),
           "tuples_per_gpu": n, "rules": w.stats()["rules"], "tables": w.stats()["tables"],
           "value": round(VD.sum_over_ranks(n, "cuda") * a.steps / wall / 1e6, 1), "unit": "Mpps",
           "ms_per_step": round(wall * 1e3 / a.steps, 4),
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                        "bytes_per_tuple": bpt, "fields": fields, "kernel_ms": round(kern_ms, 4)}}
    if not a.no_check:
        pars = VD.gather_objects(shard_check(w, b, out, base, a.check_tuples, check_threads))
        res["parity_sample"] = {"ranks": world, "tuples": sum(p["tuples"] for p in pars),
                                "bit_exact_action_and_rule_index": all(p["bit_exact_action_and_rule_index"]
                                                                       for p in pars),
                                "counters_equal_oracle_histogram": all(p["counters_equal_oracle_histogram"]
                                                                       for p in pars)}
    return res


def steady_state(e, w, b, out, cptr, n, world, settle=60, timed=20):
    """settle + timed back-to-back launches after the timed region; the timed ones' mean (HIP
    events on the launch stream) and the whole-job rate it implies. A reported side figure, not
    `value`: it shows what the driver's short window loses to the clock ramp of a burst."""
    sink = torch.empty_like(out)  # `out` keeps the timed run's verdicts (checked later)
    for _ in range(settle):
        D.classify(e, w.mode, w.table_id, b, sink, counters=cptr)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(timed):
        D.classify(e, w.mode, w.table_id, b, sink, counters=cptr)
    e1.record()
    torch.cuda.synchronize()
    del sink
    ms = VD.max_over_ranks(e0.elapsed_time(e1) / timed / 1e3, "cuda") * 1e3
    return {"launches_before": settle, "launches_timed": timed, "kernel_ms": round(ms, 4),
            "value": round(VD.sum_over_ranks(n, "cuda") / (ms * 1e-3) / 1e6, 1), "unit": "Mpps",
            "note": "after the timed region and %d more launches; not the bench value" % settle}


def counter_allreduce(e, w, b, out, rank, world):
    """One counted classify pass per rank over its whole shard into the context's own
    counters, then pg_allreduce_counters over an RCCL communicator the library holds (unique id
    from rank 0 over torch.distributed). Checked (every rank): SINGLE / PERPOD local counters
    == the histogram of the pass's verdict slots (one evaluation per tuple); the RCCL sum ==
    torch.distributed's all_reduce of the same local histograms; the local counters unchanged
    by the reduction; SINGLE / PERPOD sum == every tuple of every rank."""
    res = {}
    try:
        uid = [D.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        D.comm_init_rank(e, world, uid[0], rank)
        D.reset_counters(e)
        D.classify(e, w.mode, w.table_id, b, out, counters=D.counters_device_ptr(e))
        torch.cuda.synchronize()
        local = D.read_counters(e).astype(np.int64)
        checks = {}
        if w.mode != 2:
            h = torch.bincount((out & 0x3FFFFFFF).long(), minlength=len(local)).cpu().numpy()
            checks["local_equals_verdict_histogram"] = bool(np.array_equal(h, local))
        dist.barrier()
        t1 = time.perf_counter()
        summed = D.allreduce_counters(e).astype(np.int64)
        res["counter_allreduce_ms"] = round((time.perf_counter() - t1) * 1e3, 3)
        ref = torch.from_numpy(local).cuda()
        dist.all_reduce(ref)
        checks["rccl_sum_equals_torch_sum"] = bool(np.array_equal(summed, ref.cpu().numpy()))
        checks["local_unchanged_by_reduction"] = bool(np.array_equal(D.read_counters(e).astype(np.int64), local))
        total = VD.sum_over_ranks(b.n, "cuda")
        checks["sum_accounts_for_every_tuple"] = bool(int(summed.sum()) == total if w.mode != 2
                                                      else int(summed.sum()) >= total)
        per_rank = VD.gather_objects(checks)
        res["counter_allreduce_check"] = all(all(c.values()) for c in per_rank)
        res["counter_allreduce_checks_per_rank"] = per_rank
        res["counter_slots"] = int(len(summed))
        res["counter_evaluations_total"] = int(summed.sum())
    except Exception as ex:  # reported, not fatal: the throughput line still prints
        res["counter_allreduce_error"] = str(ex)[:300]
        res["counter_allreduce_check"] = False
    return res


def shard_check(w, b, out, base, k, threads):
    """Self-check of this rank's shard (after the timed region; the oracle is the checker, never
    the thing measured): the timed run's verdicts of the shard's first k tuples (global indices
    base .. base + k) against the oracle, bit for bit (action and deciding rule slot), and a
    counted classify pass over those k tuples whose per-rule hit counters must equal the
    oracle's histogram -- one count per evalACL, so CONN's up-to-four evaluations per
    connection are checked too (aclengine_mock.go:448-491)."""
    from oracle import world as OW  # checker leg
    e = w.engine
    k = min(k, b.n)
    tup = b.numpy(k)
    got = out[:k].cpu().numpy().view(np.uint32)
    t0 = time.perf_counter()
    act, slot, hist = OW.expected(e, w.mode, w.table_id, w.local_ifs, w.node_if, *tup, threads=threads)
    dt = time.perf_counter() - t0
    ok = bool(np.array_equal(got >> 30, act.astype(np.uint32)) and np.array_equal(got & 0x3FFFFFFF, slot))
    sink = torch.empty(k, dtype=torch.int32, device="cuda")
    D.reset_counters(e)
    D.classify(e, w.mode, w.table_id, b, sink, counters=D.counters_device_ptr(e), n=k)
    cnt = D.read_counters(e).astype(np.int64)
    same = bool(np.array_equal(sink.cpu().numpy().view(np.uint32), got))
    return {"index_base": int(base), "tuples": int(k), "bit_exact_action_and_rule_index": ok,
            "counters_equal_oracle_histogram": bool(np.array_equal(cnt, hist)) and same,
            "evaluations": int(hist.sum()), "oracle_s": round(dt, 2), "oracle_threads": threads}


def dry_run(a, rank, world):
    """CPU rehearsal of the multi-rank path (gloo): same launcher, sharding, barriers,
    max-over-ranks timing, per-rank self-check and counter all-reduce as on GPUs; the per-tuple
    code is the product's, run on the host (pg_debug_classify_host); inputs are the oracle's
    restatement of the device generator (oracle/gen.py) at the rank's global index range.
    Prints the same JSON line with "dry_run": true."""
    from oracle import gen
    from oracle import world as OW
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if world > 1:
        dist.init_process_group("gloo")
    kw = {"n_tuples": a.tuples or 1 << 14}
    if a.rules:
        kw["n_rules"] = a.rules
    w = W.CONFIGS[a.config](0, **kw)
    e = w.engine
    base, n = shard_of(a, w, rank, world)
    rules = e.GetACLByName(e.ACLNames()[w.table_id])["rules"] if w.table_id >= 0 else None
    src, dst, sport, dport, proto = gen.gen_tuples(n, index_base=base, rules=rules, **w.gen)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.warmup + a.steps):
        out, cnt = e.debug_classify_host(w.mode, w.table_id, src, dst, sport, dport, proto, counters=True)
    if world > 1:
        dist.barrier()
    wall = VD.max_over_ranks(time.perf_counter() - t0, "cpu")
    local = cnt.astype(np.int64)
    # per-rank self-check: verdicts and hit counters of the whole (small) shard vs the oracle
    act, slot, hist = OW.expected(e, w.mode, w.table_id, w.local_ifs, w.node_if, src, dst, sport, dport, proto,
                                  threads=2)
    par = {"index_base": int(base), "tuples": int(n),
           "bit_exact_action_and_rule_index": bool(np.array_equal(out >> 30, act.astype(np.uint32)) and
                                                   np.array_equal(out & 0x3FFFFFFF, slot)),
           "counters_equal_oracle_histogram": bool(np.array_equal(local, hist)), "evaluations": int(hist.sum())}
    pars = VD.gather_objects(par)
    counters = torch.from_numpy(local.copy())
    t1 = time.perf_counter()
    VD.allreduce_counters(counters)
    ms = (time.perf_counter() - t1) * 1e3
    # the all-reduced counters == the oracle's histogram over the whole job's index range
    total = VD.sum_over_ranks(n, "cpu")
    ora = torch.from_numpy(hist.copy())
    VD.allreduce_counters(ora)
    check = bool(torch.equal(counters, ora)) and (int(counters.sum()) == total if w.mode != 2
                                                  else int(counters.sum()) >= total)
    line = {"metric": METRIC, "value": round(total * a.steps / wall / 1e6, 3), "unit": "Mpps", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "scaling": a.scaling, "dry_run": True,
            "config": {"workload": "config%d: %s" % (a.config, w.desc), "tuples_per_gpu": n, "tuples_total": total,
                       "parallelism": "dp%d" % world},
            "counter_allreduce_ms": round(ms, 3), "counter_allreduce_check": check,
            "parity_sample": {"ranks": world, "tuples": sum(p["tuples"] for p in pars),
                              "bit_exact_action_and_rule_index": all(p["bit_exact_action_and_rule_index"]
                                                                     for p in pars),
                              "counters_equal_oracle_histogram": all(p["counters_equal_oracle_histogram"]
                                                                     for p in pars)},
            "parity_per_rank": pars,
            "counters_sha": __import__("hashlib").sha1(counters.numpy().tobytes()).hexdigest()[:16]}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _median_ms(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


def stream_ceiling_gbps(e, w, b, out, bpt, reps):
    """pg_stream_probe over the timed batch: the loads of exactly the fields the classify launch
    reads (dst unless the table is dst-free, sport in CONN mode) and its verdict store, with
    the same vector widths and grid; algorithmic bytes / median launch time"""
    fields = (0 if bpt == 11 and w.mode == 0 else 1) | (2 if w.mode == 2 else 0)
    sink = torch.empty_like(out)  # the verdicts in `out` are checked against the CPU oracle later
    # the best of 2 / 3 / 4 resident 512-thread workgroups per CU (the classify launches run 1-4)
    best = 1e30
    for bpc in (2, 3, 4):
        e.set_tuning("blocks_per_cu", bpc)
        best = min(best, _median_ms(lambda: D.stream_probe(e, fields, b, sink), max(reps, 5)))
    e.set_tuning("blocks_per_cu", 0)
    del sink
    return round(b.n * bpt / (best * 1e-3) / 1e9, 1)


def torch_copy_gbps(nbytes=1 << 30, reps=10):
    """torch's own device-to-device copy of a 1 GiB buffer (bytes read + written / time)"""
    x = torch.ones(nbytes // 4, dtype=torch.float32, device="cuda")
    y = torch.empty_like(x)
    ms = _median_ms(lambda: y.copy_(x), reps)
    del x, y
    return round(2 * nbytes / (ms * 1e-3) / 1e9, 1)


def bytes_per_tuple(w):
    """Algorithmic bytes per tuple: the tuple fields the classification reads
    plus the 4-B verdict. SINGLE / PERPOD read src 4 + dst 4 + dport 2 + proto 1 = 11 B (15 B
    with the verdict), CONN also sport (17 B) -- except SINGLE over a table no rule of which
    tests dst (kFlagDstFree; FD tables among them): its verdict cannot depend on dst and the
    kernel does not read that stream, so 7 B in + 4 B out = 11 B."""
    if w.mode == 0 and w.engine.table_stats(w.table_id)["dst_free"]:
        return 11, "src 4 + dport 2 + proto 1 in, verdict 4 out (no rule tests dst: dst not read)"
    if w.mode == 2:
        return 17, "src 4 + dst 4 + sport 2 + dport 2 + proto 1 in, verdict 4 out"
    return 15, "src 4 + dst 4 + dport 2 + proto 1 in, verdict 4 out"


def classifier(w, per_table):
    """the structure the timed kernel walks"""
    e = w.engine
    if w.mode == 0:
        return "table blob: %s" % json.dumps(e.table_stats(w.table_id))
    ns = None if per_table else e.node_stats()
    if ns is None:
        return "per-table blobs + IPv4 hash"
    return "node: %s" % json.dumps(ns)


def pmc_traffic(label, n, other_shape):
    """HBM bytes per classify launch from the committed rocprofv3 PMC summary of this config
    (profiles/rNN_*_config<label>_pmc.json, label = C or CrM for config C at M rules,
    FETCH_SIZE/WRITE_SIZE passes, gfx950-corrected by tools/prof_summary.py), scaled to this
    launch's tuple count; None when there is none."""
    import glob
    import re
    # newest round / version first by number (r01_v12 after r01_v9)
    nat = lambda p: [int(x) if x.isdigit() else x for x in re.split(r"(\d+)", os.path.basename(p))]
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_config%s_pmc.json" % label)), key=nat)
    if not files or other_shape:  # the committed summary is of the default shape only
        return None, None
    with open(files[-1]) as f:
        p = json.load(f)
    return int(p["hbm_traffic_bytes_per_launch"] * n / p["tuples_per_launch"]), os.path.basename(files[-1])


def host_cores():
    """CPUs this process may use: its affinity set, capped by a cgroup-v2 CPU quota when one is
    set (a GPU box's share of a larger host)"""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(q) // int(p)))
    except (OSError, ValueError):
        pass
    return max(1, n)


def _timed_rate(fn, k_max, budget_s, cal):
    """fn(k) run on a calibration sample of `cal` tuples, then on a sample sized to about
    budget_s seconds (at most k_max) -> (tuples/s, sample size, result of the timed call)"""
    t0 = time.perf_counter()
    fn(min(cal, k_max))
    rate = min(cal, k_max) / max(time.perf_counter() - t0, 1e-9)
    k = int(min(k_max, max(min(cal, k_max), rate * budget_s)))
    t0 = time.perf_counter()
    r = fn(k)
    return k / (time.perf_counter() - t0), k, r


def cpu_baseline(w, b, out, k_max, faithful_s=8.0, budget_s=10.0):
    """The oracle's evalACL / testConnection (oracle/oracle.c, rules pre-parsed: BASELINE.md's
    B2) timed on this host's cores -- at one thread and at every core the process may use --
    over the first tuples of the same workload, each sample sized by a calibration run to
    about budget_s (one thread: half of it); and the reference-faithful variant of the same call
    (CIDR strings parsed on every rule visit, as evalACL does -- in every mode, so per-pod
    evalACL and testConnection too; one thread). The verdicts of each sample are compared with
    the GPU's."""
    from oracle import fast, world  # cpu_baseline leg: the checker, never the thing measured on GPU

    e = w.engine
    cores = host_cores()
    k_max = min(k_max, b.n)
    src, dst, sport, dport, proto = b.numpy(k_max)
    extra = {}
    if w.mode == 0:
        wd = world.World(e, {}, None)
        t = wd.tids.index(w.table_id)
        ora = wd.acls[t]
        run = lambda k, th: fast.eval_acl(ora, src[:k], dst[:k], dport[:k], proto[:k], threads=th)
        to_slot = lambda r: wd.slots(np.full(len(r[1]), t, np.int64), r[1])
        kind = "evalACL over the same ACL (rules pre-parsed)"
    else:
        wd = world.World(e, w.local_ifs, w.node_if)
        # interface lookup kept outside the timed call; CONN: the reference's Connection* end-point
        # rules (no evaluation for remote pod <-> non-pod and non-pod <-> non-pod, World.conn_ifs)
        sif, dif = wd.conn_ifs(src, dst) if w.mode == 2 else (None, wd.resolve(dst))
        if w.mode == 1:
            run = lambda k, th: fast.perpod(wd.acls, wd.if_out, dif[:k], src[:k], dst[:k], dport[:k], proto[:k], th)
            kind = "evalACL(outbound ACL of the dst interface), rules pre-parsed, interfaces resolved beforehand"
        else:
            run = lambda k, th: fast.test_connection(wd.acls, wd.if_in, wd.if_out, sif[:k], dif[:k], src[:k], dst[:k],
                                                     sport[:k], dport[:k], proto[:k], th)
            kind = "testConnection (up to 4 evalACL), rules pre-parsed, interfaces resolved beforehand"
        to_slot = lambda r: wd.slots(r[1], r[2])
    rate_n, k_n, res = _timed_rate(lambda k: run(k, cores), k_max, budget_s, 4096 * cores)
    rate_1, k_1, _ = _timed_rate(lambda k: run(k, 1), k_max, budget_s / 2, 4096)
    got = out[:k_n].cpu().numpy().view(np.uint32)
    ok = bool(((got >> 30) == res[0].astype(np.uint32)).all() and ((got & 0x3FFFFFFF) == to_slot(res)).all())
    # the reference-faithful variant of the same call: every evalACL parses its rules' CIDR strings
    # on each rule visit (aclengine_mock.go:535, 549), at one thread and at every core (one engine
    # per thread over a slice of the tuples: BASELINE.md B1, GOMAXPROCS=1 and GOMAXPROCS=$(nproc))
    if w.mode == 0:
        rules = e.GetACLByName(e.ACLNames()[w.table_id])["rules"]
        frun = lambda k, th: fast.eval_acl_faithful(rules, src[:k], dst[:k], dport[:k], proto[:k], threads=th)
        fslot = lambda r: wd.slots(np.full(len(r[1]), t, np.int64), r[1])
        fcal = 64 if len(rules) > 20000 else 4096
    else:
        if w.mode == 1:
            frun = lambda k, th: fast.perpod(wd.acls, wd.if_out, dif[:k], src[:k], dst[:k], dport[:k], proto[:k],
                                             threads=th, faithful=True)
        else:
            frun = lambda k, th: fast.test_connection(wd.acls, wd.if_in, wd.if_out, sif[:k], dif[:k], src[:k],
                                                      dst[:k], sport[:k], dport[:k], proto[:k], threads=th,
                                                      faithful=True)
        fslot = to_slot
        fcal = 4096
    fkind = kind.replace("rules pre-parsed", "CIDR strings parsed per rule visit")

    def fcheck(k, r):  # (against the GPU's verdicts of the same k tuples)
        g = out[:k].cpu().numpy().view(np.uint32)
        return bool(((g >> 30) == r[0].astype(np.uint32)).all() and ((g & 0x3FFFFFFF) == fslot(r)).all())
    fr, kf, fres = _timed_rate(lambda k: frun(k, 1), k_max, faithful_s, fcal)
    extra["faithful_1thread_mpps"] = round(fr / 1e6, 4)
    extra["faithful_sample"] = kf
    extra["faithful_kind"] = fkind + ", 1 thread"
    extra["faithful_variant_bit_exact"] = fcheck(kf, fres)
    frn, kfn, fresn = _timed_rate(lambda k: frun(k, cores), k_max, faithful_s, fcal * cores)
    extra["faithful_nthreads_mpps"] = round(frn / 1e6, 4)
    extra["faithful_nthreads_cores"] = cores
    extra["faithful_nthreads_sample"] = kfn
    extra["faithful_nthreads_kind"] = fkind + ", %d threads (one engine per thread)" % cores
    extra["faithful_nthreads_bit_exact"] = fcheck(kfn, fresn)
    if w.mode == 0:
        idx = res[1]
        # rules the reference's first-match loop (aclengine_mock.go:510-649) visits per tuple
        nr = len(rules)
        visited = np.where(idx >= 0, idx.astype(np.int64) + 1, nr)
        extra["reference_rules_visited"] = {"mean": round(float(visited.mean()), 1),
                                            "p99": int(np.percentile(visited, 99)), "rules": nr}
        # ... and the loads the GPU walk makes of the compiled structure per tuple (the kernels'
        # walk code on the host with counting loaders), LDS-staged vs gathered from HBM / L2
        ks = min(k_n, 1 << 20)
        nl, nm, stage = e.debug_walk_stats(w.table_id, src[:ks], dst[:ks], dport[:ks], proto[:ks])
        extra["gpu_loads_per_tuple"] = {"lds_mean": round(float(nl.mean()), 3),
                                        "gather_mean": round(float(nm.mean()), 3),
                                        "gather_p99": int(np.percentile(nm, 99)), "gather_max": int(nm.max()),
                                        "stage": stage, "sample": ks}
    base = {"value": round(rate_n / 1e6, 3), "unit": "Mpps", "cores": cores, "host_cpus": os.cpu_count(),
            "kind": "port", "sample": "first %d tuples of the same workload; %s, %d threads" % (k_n, kind, cores),
            "single_thread": {"value": round(rate_1 / 1e6, 3), "unit": "Mpps", "cores": 1, "sample": k_1},
            "sample_bit_exact_vs_gpu": ok}
    base.update(extra)
    return base


if __name__ == "__main__":
    main()
