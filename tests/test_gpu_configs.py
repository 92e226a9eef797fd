"""BASELINE configs 2 and 4 at their real rule counts on the GPU, bit-exact against the C
oracle (evalACL, mock/aclengine/aclengine_mock.go:503-652), through every launch shape the
engine picks for them; the reference's renderer test scenarios (acl_renderer_test.go,
testdata.go Ts1..Ts7) classified by k_classify in SINGLE / PERPOD / CONN modes; and the C
ABI's multi-context / multi-thread / RCCL boundary.

Verdict = (ACLAction or ConnAction, deciding counter slot): slots map back to (ACL, rule
index), so the matched-rule index is compared too."""
import random
import threading

import numpy as np
import pytest
import torch

import kat_driver as kd
from oracle import fast, gen

pytestmark = pytest.mark.gpu

from vpp_amd import _capi  # noqa: E402
from vpp_amd import device as D  # noqa: E402
from vpp_amd import renderer as R  # noqa: E402
from vpp_amd import workloads as W  # noqa: E402
from vpp_amd._capi import MODE_CONN, MODE_PERPOD, MODE_SINGLE  # noqa: E402

N_BIG = 4 << 20


def _expected_single(w, src, dst, dport, proto):
    e = w.engine
    rules = e.GetACLByName(e.ACLNames()[w.table_id])["rules"]
    act, idx = fast.eval_acl(fast.OraACL(rules), src, dst, dport, proto, threads=16)
    slot = np.where(idx >= 0, e.slot_of_rule(w.table_id, 0) + idx.astype(np.int64),
                    e.slot_of_rule(w.table_id, -1)).astype(np.uint32)
    return act.astype(np.uint32), slot, rules


def _classify(w, b, counters=False, **tune):
    e = w.engine
    out = torch.empty(b.n, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(e.num_counter_slots(), dtype=torch.int64, device="cuda") if counters else None
    with e.tuning(**tune):
        D.classify(e, w.mode, w.table_id, b, out, counters=cnt)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32), (cnt.cpu().numpy() if counters else None)


@pytest.fixture(scope="module", params=[2, 4], ids=["config2_1k_rules", "config4_100k_rules"])
def big(request):
    w = W.CONFIGS[request.param](0, n_tuples=N_BIG)
    b = D.TupleBatch(w.n_tuples, with_sport=False)
    D.gen_tuples(w.engine, b, **w.gen)
    torch.cuda.synchronize()
    src, dst, sport, dport, proto = b.numpy(b.n)
    act, slot, rules = _expected_single(w, src, dst, dport, proto)
    return request.param, w, b, (src, dst, sport, dport, proto), act, slot, rules


def test_config_generator_equals_restatement(big):
    """k_gen's "inside a rule" sampling (uniform / Zipf rule choice) == oracle/gen.py, on a
    slice of the batch and on a shard far into the index range"""
    cfg, w, b, tup, _, _, rules = big
    k = 200003
    exp = gen.gen_tuples(k, rules=rules, **w.gen)
    for g, x in zip(tup, exp):
        if g is tup[2]:
            continue  # no sport stream in SINGLE mode
        assert np.array_equal(np.asarray(g[:k]), np.asarray(x))
    b2 = D.TupleBatch(65537, with_sport=True)
    D.gen_tuples(w.engine, b2, index_base=7 * (1 << 30) + 11, **w.gen)
    torch.cuda.synchronize()
    exp2 = gen.gen_tuples(b2.n, index_base=7 * (1 << 30) + 11, rules=rules, **w.gen)
    for g, x in zip(b2.numpy(b2.n), exp2):
        assert np.array_equal(np.asarray(g), np.asarray(x))


def test_config_default_launch_bit_exact(big):
    cfg, w, b, tup, act, slot, _ = big
    got, _ = _classify(w, b)
    assert np.array_equal(got >> 30, act), np.nonzero((got >> 30) != act)[0][:10]
    assert np.array_equal(got & 0x3FFFFFFF, slot), np.nonzero((got & 0x3FFFFFFF) != slot)[0][:10]
    # the workload exercises both verdicts and many rules
    assert len(np.unique(got >> 30)) >= 2 and len(np.unique(slot)) >= (500 if cfg == 2 else 5000)


def test_config_with_counters_bit_exact(big):
    cfg, w, b, tup, act, slot, _ = big
    got, cnt = _classify(w, b, counters=True)
    assert np.array_equal(got >> 30, act) and np.array_equal(got & 0x3FFFFFFF, slot)
    assert np.array_equal(cnt, np.bincount(slot, minlength=len(cnt)))


@pytest.mark.parametrize("shape", ["root_staged", "hbm_only"])
def test_config_hbm_launches_bit_exact(big, shape):
    """config 2's blob normally sits in LDS (STAGE 1): here it is read from HBM with only its
    src-trie root staged, or with nothing staged; config 4's (4.6 MB) normally has its root
    staged (STAGE 2): here nothing is. With and without counters."""
    cfg, w, b, tup, act, slot, _ = big
    tune = {"stage_max_words": 0} if shape == "root_staged" else {"stage_max_words": 0, "stage_root_max_words": 0}
    for counters in (False, True):
        got, cnt = _classify(w, b, counters=counters, **tune)
        assert np.array_equal(got >> 30, act) and np.array_equal(got & 0x3FFFFFFF, slot), (shape, counters)
        if counters:
            assert np.array_equal(cnt, np.bincount(slot, minlength=len(cnt)))


def test_config_ragged_and_offset(big):
    """a ragged sub-batch at an odd element offset (scalar loads, one-tuple tail loop)"""
    cfg, w, b, tup, act, slot, _ = big
    out = torch.zeros(b.n, dtype=torch.int32, device="cuda")
    n = 1000003
    D.classify(w.engine, w.mode, w.table_id, b, out, offset=3, n=n)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)[3:3 + n]
    assert np.array_equal(got >> 30, act[3:3 + n]) and np.array_equal(got & 0x3FFFFFFF, slot[3:3 + n])


# ---- the reference's renderer scenarios through k_classify ----------------------------------
SCENARIOS = kd.load("acl_renderer_kats.json")


def _scenario_world(be, setup):
    from oracle.world import World
    e = be.engine
    local, no_if = {}, []
    for pod, ip, another in setup["pods"]:
        if another:
            continue
        v = W.ip_u32(ip)
        if pod in setup["pod_ifs"]:
            local[v] = setup["pod_ifs"][pod]
        else:
            no_if.append(v)
    node_if = setup["vxlan_bvi"] or setup["main_if"] or None
    return World(e, local, node_if, no_if), local


@pytest.mark.parametrize("sc", SCENARIOS, ids=[s["name"] for s in SCENARIOS])
def test_renderer_scenarios_through_k_classify(sc):
    """After every phase of each acl_renderer_test.go scenario (Ts1..Ts7 rule sets, resyncs,
    pod removal, renderer restart), 64k tuples drawn around the scenario's pods, the Internet
    hosts and ports of testdata.go are classified by k_classify: SINGLE mode on every installed
    ACL, PERPOD and CONN modes over the node's interfaces, with and without counters, each
    bit-exact against the oracle."""
    be = kd.ProductBackend(gpu=True)
    setup = sc["setup"]
    be.setup(setup)
    rng = np.random.default_rng(__import__("zlib").crc32(sc["name"].encode()))
    anchors = [W.ip_u32(ip) for _, ip, _ in setup["pods"]] + [W.ip_u32(x) for x in
                                                                ("8.8.8.8", "192.168.1.1", "10.0.0.5", "10.10.50.1")]
    ports = np.array([0, 22, 53, 67, 80, 161, 443, 500, 514, 600, 8080], np.uint16)
    checked = 0
    for phase in sc["phases"]:
        for st in phase["steps"]:
            if st["op"] == "restart":
                be.restart()
            else:
                assert be.txn(st["resync"], st["renders"]) is None
        e = be.engine
        n = 1 << 16
        pick = lambda: np.where(rng.random(n) < 0.7, np.asarray(anchors, np.uint32)[rng.integers(0, len(anchors), n)],
                                rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32))  # noqa: E731
        src, dst = pick(), pick()
        sport = np.where(rng.random(n) < 0.5, ports[rng.integers(0, len(ports), n)],
                         rng.integers(0, 1 << 16, n)).astype(np.uint16)
        dport = np.where(rng.random(n) < 0.6, ports[rng.integers(0, len(ports), n)],
                         rng.integers(0, 1 << 16, n)).astype(np.uint16)
        proto = rng.choice(np.array([0, 1, 2, 3], np.uint8), n, p=[0.45, 0.4, 0.1, 0.05])
        b = D.TupleBatch.from_numpy(src, dst, sport, dport, proto)
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        for name in e.ACLNames():
            tid = e.table_id(name)
            D.classify(e, MODE_SINGLE, tid, b, out)
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(np.uint32)
            a, i = fast.eval_acl(fast.OraACL(e.GetACLByName(name)["rules"]), src, dst, dport, proto)
            s = np.where(i >= 0, e.slot_of_rule(tid, 0) + i.astype(np.int64), e.slot_of_rule(tid, -1))
            assert np.array_equal(got >> 30, a.astype(np.uint32)), (phase.get("name"), name)
            assert np.array_equal(got & 0x3FFFFFFF, s.astype(np.uint32)), (phase.get("name"), name)
            checked += 1
        wd, local = _scenario_world(be, setup)
        for mode in (MODE_PERPOD, MODE_CONN):
            if mode == MODE_PERPOD:
                ea, es = wd.perpod(src, dst, dport, proto)
            else:
                ea, es = wd.conn(src, dst, sport, dport, proto)
            for counters in (False, True):
                cnt = torch.zeros(e.num_counter_slots(), dtype=torch.int64, device="cuda") if counters else None
                D.classify(e, mode, -1, b, out, counters=cnt)
                torch.cuda.synchronize()
                got = out.cpu().numpy().view(np.uint32)
                assert np.array_equal(got >> 30, ea.astype(np.uint32)), (sc["name"], mode)
                assert np.array_equal(got & 0x3FFFFFFF, es), (sc["name"], mode)
                if counters and mode == MODE_PERPOD:
                    assert np.array_equal(cnt.cpu().numpy(), np.bincount(es, minlength=cnt.numel()))
    assert checked > 0


# ---- the C ABI boundary: contexts, threads, RCCL ------------------------------------------
def _small_engine(seed):
    import acl_fuzz as fz
    rnd = random.Random(seed)
    rules = fz.rand_acl(rnd, 80, fz.ANCHORS, weird=True, tail="deny")
    e = R.Engine(0)
    e.SetMainInterfaceName("GbE")
    e.ApplyTxn(True, [("config/vpp/acls/v2/acl/x", {"name": "x", "rules": rules, "ingress": [], "egress": ["t"]})])
    return e, rules


def test_two_contexts_used_alternately_from_two_threads():
    """Two contexts on device 0, each driven by its own OS thread, calls interleaved: every
    call makes the context's device current and restores the caller's, uploads and
    launches stay with their context, and the verdicts equal the single-threaded oracle."""
    import acl_fuzz as fz
    engines = [_small_engine(s) for s in (1, 2)]
    tup = fz.rand_tuples(np.random.default_rng(3), 200001, fz.ANCHORS, any_pct=0.02)
    expect = []
    for e, rules in engines:
        a, i = fast.eval_acl(fast.OraACL(rules), tup[0], tup[1], tup[3], tup[4])
        tid = e.table_id("x")
        expect.append((a.astype(np.uint32), np.where(i >= 0, e.slot_of_rule(tid, 0) + i, e.slot_of_rule(tid, -1))))
    turn = threading.Condition()
    state = {"turn": 0, "errors": []}

    def run(k):
        try:
            e, _ = engines[k]
            torch.cuda.set_device(0)
            b = D.TupleBatch.from_numpy(*tup)
            stream = torch.cuda.Stream()
            for it in range(6):
                with turn:
                    turn.wait_for(lambda: state["turn"] % 2 == k)
                    out = torch.empty(b.n, dtype=torch.int32, device="cuda")
                    if it == 3:  # a table change mid-way: recompiled and re-uploaded by this thread
                        e.set_tuning("root_bits_max", 8)
                    D.classify(e, MODE_SINGLE, e.table_id("x"), b, out, stream=stream)
                    stream.synchronize()
                    got = out.cpu().numpy().view(np.uint32)
                    a, s = expect[k]
                    if not (np.array_equal(got >> 30, a) and np.array_equal(got & 0x3FFFFFFF, s.astype(np.uint32))):
                        state["errors"].append((k, it))
                    assert e.device == 0 and torch.cuda.current_device() == 0
                    state["turn"] += 1
                    turn.notify_all()
        except Exception as ex:  # pragma: no cover - reported below
            state["errors"].append((k, repr(ex)))
            with turn:
                state["turn"] += 1
                turn.notify_all()

    th = [threading.Thread(target=run, args=(k,)) for k in (0, 1)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not state["errors"], state["errors"]
    assert engines[0][0].get_tuning("root_bits_max") == 8 and R.Engine(0).get_tuning("root_bits_max") == 16


def test_rccl_counter_allreduce_single_rank():
    """pg_comm_init_rank (a one-rank communicator: the box has one GPU) and pg_comm_init_all
    over one context: the layout check passes, the all-reduced counters equal the local
    histogram, and the host snapshot (pg_counters_snapshot, no GPU access) holds them."""
    import acl_fuzz as fz
    e, rules = _small_engine(9)
    assert len(D.counters_snapshot(e)) == 0  # nothing read yet
    tup = fz.rand_tuples(np.random.default_rng(9), 300000, fz.ANCHORS)
    b = D.TupleBatch.from_numpy(*tup)
    out = torch.empty(b.n, dtype=torch.int32, device="cuda")
    tid = e.table_id("x")
    D.reset_counters(e)
    D.classify(e, MODE_SINGLE, tid, b, out, counters=D.counters_device_ptr(e))
    torch.cuda.synchronize()
    hist = np.bincount(out.cpu().numpy().view(np.uint32) & 0x3FFFFFFF, minlength=e.num_counter_slots())
    D.comm_init_rank(e, 1, D.comm_unique_id(), 0)
    summed = D.allreduce_counters(e)
    assert np.array_equal(summed, hist) and np.array_equal(D.read_counters(e), hist)
    assert np.array_equal(D.counters_snapshot(e), hist)
    # a second reduction (a periodic gauge) sums the same local counts again: no compounding,
    # and the local counters are still this rank's own
    assert np.array_equal(D.allreduce_counters(e), hist) and np.array_equal(D.read_counters(e), hist)
    # with a communicator the gauge snapshot is the cluster sum: a later pg_read_counters (this
    # rank's own, now ahead of the last reduction) refreshes only the LOCAL snapshot, so the
    # gauge never jumps between local and summed counts (a monotonic source)
    D.classify(e, MODE_SINGLE, tid, b, out, counters=D.counters_device_ptr(e))
    assert np.array_equal(D.read_counters(e), 2 * hist)
    assert np.array_equal(D.counters_snapshot(e), hist)
    assert np.array_equal(D.counters_snapshot_range(e, _capi.SNAP_LOCAL, 0, len(hist))[0], 2 * hist)
    assert np.array_equal(D.counters_snapshot_range(e, _capi.SNAP_CLUSTER, 0, len(hist))[0], hist)
    base, nr, dflt = e.table_info(tid)
    for i in range(nr):
        assert D.counter_of_rule(e, _capi.SNAP_GAUGE, "x", i)[0] == hist[base + i]
    assert D.counter_of_rule(e, _capi.SNAP_GAUGE, "x", -1)[0] == hist[dflt]
    assert np.array_equal(D.allreduce_counters(e), 2 * hist) and np.array_equal(D.counters_snapshot(e), 2 * hist)
    assert torch.cuda.current_device() == 0
    e2, _ = _small_engine(10)
    D.comm_init_all([e2])
    D.reset_counters(e2)
    D.classify(e2, MODE_SINGLE, e2.table_id("x"), b, out, counters=D.counters_device_ptr(e2))
    s2 = D.allreduce_counters_all([e2])[0]
    assert int(s2.sum()) == b.n


def test_counters_survive_a_commit():
    """Device hit counters across Commits (statscollector gauge, plugin_impl_statscollector.go:
    248-261): count, commit a change to another ACL, count again -- the unchanged ACL's counts
    (rules and default deny, read back and through its gauge) are the sum of both passes, the
    changed ACL's only the second pass's. Three shapes of recompile: more slots (a new ACL), the
    same slot count (one rule's action flipped: remapped in place), nothing changed (a compiler
    knob: the counters stay where they are)."""
    import acl_fuzz as fz
    rnd = random.Random(21)
    acls = {"b": fz.rand_acl(rnd, 60, fz.ANCHORS, weird=False, tail="deny"),
            "d": fz.rand_acl(rnd, 40, fz.ANCHORS, weird=False, tail="permit")}
    e = R.Engine(0)
    e.SetMainInterfaceName("GbE")

    def apply(a):
        e.ApplyTxn(True, [("config/vpp/acls/v2/acl/" + n, {"name": n, "rules": r, "ingress": [], "egress": ["if-" + n]})
                          for n, r in a.items()])

    apply(acls)
    tup = fz.rand_tuples(np.random.default_rng(21), 200000, fz.ANCHORS, any_pct=0.01)
    b = D.TupleBatch.from_numpy(*tup)
    out = torch.empty(b.n, dtype=torch.int32, device="cuda")

    def count(names):  # one counted pass per table into the context's counters -> this pass's histogram
        h = np.zeros(e.num_counter_slots(), np.int64)
        for n in names:
            D.classify(e, MODE_SINGLE, e.table_id(n), b, out, counters=D.counters_device_ptr(e))
            torch.cuda.synchronize()
            h += np.bincount(out.cpu().numpy().view(np.uint32) & 0x3FFFFFFF, minlength=len(h))
        return h

    def acl_slots(n):
        base, nr, dflt = e.table_info(e.table_id(n))
        return list(range(base, base + nr)) + [dflt]

    D.reset_counters(e)
    h1 = count(["b", "d"])
    assert np.array_equal(D.read_counters(e), h1)
    b1 = h1[acl_slots("b")]
    # 1: a new ACL sorted first (every slot moves, more slots) and d changed (a rule dropped)
    acls2 = {"a": fz.rand_acl(rnd, 30, fz.ANCHORS, weird=False, tail="deny"), "b": acls["b"], "d": acls["d"][1:]}
    apply(acls2)
    h2 = count(["a", "b", "d"])
    got = D.read_counters(e)
    assert np.array_equal(got[acl_slots("b")], b1 + h2[acl_slots("b")])
    assert np.array_equal(got[acl_slots("d")], h2[acl_slots("d")])
    assert np.array_equal(got[acl_slots("a")], h2[acl_slots("a")])
    ns = e.num_counter_slots()
    assert got[ns - 2] == h1[len(h1) - 2] + h2[ns - 2] and got[ns - 1] == h1[len(h1) - 1] + h2[ns - 1]
    for i, s in enumerate(acl_slots("b")[:-1]):
        assert D.counter_of_rule(e, _capi.SNAP_GAUGE, "b", i)[0] == got[s]
    assert D.counter_of_rule(e, _capi.SNAP_GAUGE, "b", -1)[0] == got[acl_slots("b")[-1]]
    # 2: the same slot count (d's first rule's action flipped): b and a carried, d restarts
    d3 = [dict(r) for r in acls2["d"]]
    d3[0]["action"] = 0 if d3[0]["action"] == 1 else 1
    apply(dict(acls2, d=d3))
    assert e.num_counter_slots() == ns
    h3 = count(["b", "d"])
    got3 = D.read_counters(e)
    assert np.array_equal(got3[acl_slots("b")], got[acl_slots("b")] + h3[acl_slots("b")])
    assert np.array_equal(got3[acl_slots("a")], got[acl_slots("a")])
    assert np.array_equal(got3[acl_slots("d")], h3[acl_slots("d")])
    # 3: a compiler knob (recompiled, nothing changed): every count stays
    e.set_tuning("fd", 0)
    h4 = count(["b"])
    assert np.array_equal(D.read_counters(e), got3 + h4)


# ---- rule-count sweep: gen-policy-shaped tables of 10k / 100k rules and the whole policy ----
@pytest.mark.parametrize("n_rules", [10000, 100000])
def test_rule_count_sweep_tables_bit_exact(n_rules):
    """config 2's shape at 10k and 100k rules: FD blobs too large for LDS (prefix staged,
    STAGE 5; and the generic walk with nothing staged), with and without counters."""
    w = W.config2(0, n_tuples=2 << 20, n_rules=n_rules)
    assert w.engine.table_stats(w.table_id)["structure"] == "fd"
    b = D.TupleBatch(w.n_tuples, with_sport=False)
    D.gen_tuples(w.engine, b, **w.gen)
    torch.cuda.synchronize()
    src, dst, sport, dport, proto = b.numpy(b.n)
    act, slot, rules = _expected_single(w, src, dst, dport, proto)
    for tune in ({}, {"stage_root_max_words": 0}):
        for counters in (False, True):
            got, cnt = _classify(w, b, counters=counters, **tune)
            assert np.array_equal(got >> 30, act) and np.array_equal(got & 0x3FFFFFFF, slot), (tune, counters)
            if counters:
                assert np.array_equal(cnt, np.bincount(slot, minlength=len(cnt)))
    assert len(np.unique(slot)) > n_rules // 4


def test_full_gen_policy_through_configurator():
    """config 7: the whole gen-policy.py policy (1000 CIDRs x 5 excepts x 20 ports, both
    directions) through the configurator; the pod's ~466k-rule table classified on the GPU
    and checked against the oracle on a sample."""
    w = W.config7(0, n_tuples=1 << 20)
    e = w.engine
    assert e.table_info(w.table_id)[1] > 400000
    b = D.TupleBatch(w.n_tuples, with_sport=False)
    D.gen_tuples(e, b, **w.gen)
    got, _ = _classify(w, b)
    k = 131072
    src, dst, sport, dport, proto = b.numpy(k)
    act, slot, _ = _expected_single(w, src, dst, dport, proto)
    assert np.array_equal(got[:k] >> 30, act) and np.array_equal(got[:k] & 0x3FFFFFFF, slot)
    assert len(np.unique(act)) == 2


@pytest.mark.parametrize("fields", [0, 1, 2, 3])
def test_stream_probe_reads_the_fields_it_is_told_to(fields):
    """pg_stream_probe (bench.py's stream ceiling): out = src ^ dport ^ proto (^ dst when
    fields & 1, ^ sport when fields & 2) over a ragged batch (vector groups + remainder)."""
    e, _ = _small_engine(3)
    n = (1 << 20) + 13
    rng = np.random.default_rng(fields)
    src = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    sport = rng.integers(0, 1 << 16, n).astype(np.uint16)
    dport = rng.integers(0, 1 << 16, n).astype(np.uint16)
    proto = rng.integers(0, 4, n).astype(np.uint8)
    b = D.TupleBatch.from_numpy(src, dst, sport, dport, proto)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    D.stream_probe(e, fields, b, out)
    torch.cuda.synchronize()
    exp = src ^ dport.astype(np.uint32) ^ proto.astype(np.uint32)
    if fields & 1:
        exp ^= dst
    if fields & 2:
        exp ^= sport.astype(np.uint32)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), exp)
