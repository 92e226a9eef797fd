"""Bit-exact parity of the HIP kernels against the CPU oracle (oracle/oracle.c, pinned to
the reference's KATs through oracle/aclengine.py).

Verdict = (ACLAction or ConnAction, deciding counter slot); slots map back to
(ACL, rule index) through pg_slot_info, so "matched rule index" parity is checked too.
"""
import random

import numpy as np
import pytest
import torch

import acl_fuzz as fz
from oracle import fast

pytestmark = pytest.mark.gpu

from vpp_amd import device as D  # noqa: E402
from vpp_amd import renderer as R  # noqa: E402
from vpp_amd._capi import MODE_CONN, MODE_PERPOD, MODE_SINGLE  # noqa: E402


def make_engine(acls_by_if, pods=(), node_if="VXLAN-BVI"):
    """acls_by_if: {ifname: (inbound rules|None, outbound rules|None)} -> Engine."""
    e = R.Engine(0)
    e.SetMainInterfaceName("GbE")
    e.SetVxlanBVIIfName(node_if)
    e.SetHostInterconnectIfName("VPP-Host")
    for pod, ip, ifn, another in pods:
        if ifn:
            e.SetPodIfName(pod, ifn)
        e.RegisterPod(pod, ip, another)
    ops = []
    for ifn, (inb, outb) in sorted(acls_by_if.items()):
        if inb is not None:
            ops.append(("config/vpp/acls/v2/acl/in-" + ifn, {"name": "in-" + ifn, "rules": inb, "ingress": [ifn],
                                                             "egress": []}))
        if outb is not None:
            ops.append(("config/vpp/acls/v2/acl/out-" + ifn, {"name": "out-" + ifn, "rules": outb, "ingress": [],
                                                              "egress": [ifn]}))
    e.ApplyTxn(True, ops)
    e.sync()
    return e


def slot_map(e):
    """(table id, rule index) -> slot; (table, -1) -> default slot; (-1,-1) no ACL."""
    m = {}
    for s in range(e.num_counter_slots()):
        m[e.slot_info(s)] = s
    return m


def run_single(e, tid, tup, counters=False):
    n = len(tup[0])
    b = D.TupleBatch.from_numpy(*tup)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    cnt = None
    if counters:
        D.reset_counters(e)
        cnt = D.counters_device_ptr(e)
    D.classify(e, MODE_SINGLE, tid, b, out, counters=cnt)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32), b


def expected_single(e, tid, rules, tup):
    src, dst, sport, dport, proto = tup
    a, i = fast.eval_acl(fast.OraACL(rules), src, dst, dport, proto)
    sm = slot_map(e)
    slots = np.array([sm[(tid, int(x))] if x >= 0 else sm[(tid, -1)] for x in i], np.uint32)
    return a.astype(np.uint32), slots


@pytest.mark.parametrize("seed", range(8))
def test_single_mode_random_acls_bit_exact(seed):
    rnd = random.Random(seed)
    acls = {"if%d" % k: (None, fz.rand_acl(rnd, rnd.choice([1, 5, 30, 120]), fz.ANCHORS, weird=True,
                                           tail=rnd.choice([None, "deny", "permit"]))) for k in range(3)}
    e = make_engine(acls)
    tup = fz.rand_tuples(np.random.default_rng(seed), 40000 + seed, fz.ANCHORS, any_pct=0.03)
    for ifn, (_, rules) in acls.items():
        tid = e.table_id("out-" + ifn)
        got, _ = run_single(e, tid, tup)
        ea, es = expected_single(e, tid, rules, tup)
        assert ((got >> 30) == ea).all(), np.nonzero((got >> 30) != ea)[0][:10]
        assert ((got & 0x3FFFFFFF) == es).all(), np.nonzero((got & 0x3FFFFFFF) != es)[0][:10]


@pytest.mark.parametrize("seed", range(3))
def test_linear_kernel_equals_indexed_kernel(seed):
    rnd = random.Random(100 + seed)
    rules = fz.rand_acl(rnd, 200, fz.ANCHORS, weird=True, tail="deny")
    e = make_engine({"x": (None, rules)})
    tid = e.table_id("out-x")
    tup = fz.rand_tuples(np.random.default_rng(seed), 100003, fz.ANCHORS, any_pct=0.02)
    got, b = run_single(e, tid, tup)
    lin = torch.empty(b.n, dtype=torch.int32, device="cuda")
    D.classify_linear(e, tid, b, lin)
    torch.cuda.synchronize()
    assert (lin.cpu().numpy().view(np.uint32) == got).all()


def test_counters_equal_verdict_histogram_and_oracle():
    rnd = random.Random(7)
    rules = fz.rand_acl(rnd, 60, fz.ANCHORS, weird=False, tail="deny")
    e = make_engine({"x": (None, rules)})
    tid = e.table_id("out-x")
    tup = fz.rand_tuples(np.random.default_rng(7), 300000, fz.ANCHORS)
    got, _ = run_single(e, tid, tup, counters=True)
    cnt = D.read_counters(e)
    hist = np.bincount(got & 0x3FFFFFFF, minlength=len(cnt))
    assert (cnt == hist).all()
    _, es = expected_single(e, tid, rules, tup)
    assert (np.bincount(es, minlength=len(cnt)) == cnt).all()


@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 5, 7, 9, 255, 257, 1023, 4099])
def test_ragged_sizes_and_tails(n):
    rnd = random.Random(n)
    rules = fz.rand_acl(rnd, 25, fz.ANCHORS, weird=True, tail="deny")
    e = make_engine({"x": (None, rules)})
    tid = e.table_id("out-x")
    tup = fz.rand_tuples(np.random.default_rng(n), max(n, 1), fz.ANCHORS)
    tup = tuple(a[:n] for a in tup)
    if n == 0:
        b = D.TupleBatch(0)
        out = torch.empty(0, dtype=torch.int32, device="cuda")
        D.classify(e, MODE_SINGLE, tid, b, out)
        return
    got, _ = run_single(e, tid, tup)
    ea, es = expected_single(e, tid, rules, tup)
    assert ((got >> 30) == ea).all() and ((got & 0x3FFFFFFF) == es).all()


def test_misaligned_pointers_take_scalar_path():
    rnd = random.Random(11)
    rules = fz.rand_acl(rnd, 40, fz.ANCHORS, weird=True, tail="deny")
    e = make_engine({"x": (None, rules)})
    tid = e.table_id("out-x")
    tup = fz.rand_tuples(np.random.default_rng(11), 10001, fz.ANCHORS)
    b = D.TupleBatch.from_numpy(*tup)
    out = torch.zeros(b.n, dtype=torch.int32, device="cuda")
    D.classify(e, MODE_SINGLE, tid, b, out, offset=1)  # every pointer off by one element
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)[1:]
    ea, es = expected_single(e, tid, rules, tuple(a[1:] for a in tup))
    assert ((got >> 30) == ea).all() and ((got & 0x3FFFFFFF) == es).all()


def _topology(rnd, n_pods=12, weird=False):
    pods = []
    acls = {}
    for k in range(n_pods):
        ip = 0x0A0A0000 | (k + 1)
        another = k >= n_pods - 2
        ifn = "tap%d" % k if not another else None
        pods.append(("ns/p%d" % k, "%d.%d.%d.%d" % (ip >> 24, ip >> 16 & 255, ip >> 8 & 255, ip & 255), ifn, another))
        if ifn:
            inb = fz.rand_acl(rnd, rnd.randint(0, 8), fz.ANCHORS + [ip], weird) if rnd.random() < 0.6 else None
            outb = fz.rand_acl(rnd, rnd.randint(0, 12), fz.ANCHORS + [ip], weird, tail="deny") if rnd.random() < 0.7 \
                else None
            if inb is not None and rnd.random() < 0.5:
                inb = [{"action": 2, "src": "", "dst": ""}]          # reflective ACL
            acls[ifn] = (inb, outb)
    acls["VXLAN-BVI"] = (fz.rand_acl(rnd, 3, fz.ANCHORS, weird) if rnd.random() < 0.5 else None,
                         fz.rand_acl(rnd, 20, fz.ANCHORS, weird, tail="permit"))
    return pods, acls


def _resolve(e, pods, ips):
    """IPv4 -> interface index as the device does it (local pod TAP else node interface)."""
    names = {}
    for pod, ip, ifn, another in pods:
        if not another:
            names[fz_ip(ip)] = ifn
    return names


def fz_ip(s):
    a, b, c, d = (int(x) for x in s.split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


def _oracle_world(e, acls):
    names = sorted(n for n in e.ACLNames())
    ora = [fast.OraACL(e.GetACLByName(n)["rules"]) for n in names]
    tid = {n: i for i, n in enumerate(names)}
    return names, ora, tid


@pytest.mark.parametrize("seed", range(5))
def test_conn_and_perpod_modes_random_topology(seed):
    rnd = random.Random(1000 + seed)
    pods, acls = _topology(rnd, weird=seed % 2 == 1)
    e = make_engine(acls, pods)
    names, ora, tid = _oracle_world(e, acls)
    assert [e.table_id(n) for n in names] == list(range(len(names)))
    pod_ips = [fz_ip(p[1]) for p in pods]
    n = 60001 + seed  # ragged: the one-tuple tail loop too
    rng = np.random.default_rng(seed)
    tup = list(fz.rand_tuples(rng, n, fz.ANCHORS + pod_ips))
    for k in (0, 1):  # 60 % of endpoints are pods
        m = rng.random(n) < 0.6
        tup[k][m] = np.array(pod_ips, np.uint32)[rng.integers(0, len(pod_ips), int(m.sum()))]
    tup = tuple(tup)
    local = {fz_ip(ip): ifn for pod, ip, ifn, another in pods if not another}
    ifnames = sorted(set(list(acls) + [p[2] for p in pods if p[2]] + ["GbE", "VPP-Host"]))
    ifx = {x: i for i, x in enumerate(ifnames)}
    node = ifx["VXLAN-BVI"]
    if_in = [tid.get("in-" + x, -1) for x in ifnames]
    if_out = [tid.get("out-" + x, -1) for x in ifnames]
    sif = np.array([ifx[local[int(s)]] if int(s) in local else node for s in tup[0]], np.int32)
    dif = np.array([ifx[local[int(d)]] if int(d) in local else node for d in tup[1]], np.int32)
    # a remote pod paired with a non-pod address, or two non-pod addresses: no Connection* call
    # evaluates them (aclengine_mock.go:343-347, 388-392) -> FAILURE before any evaluation
    remote = {fz_ip(ip) for pod, ip, ifn, another in pods if another}
    kind = lambda a: np.array([0 if int(x) in local else (1 if int(x) in remote else 2) for x in a])  # noqa: E731
    invalid = kind(tup[0]) + kind(tup[1]) >= 3
    assert 0 < invalid.sum() < n
    sif[invalid] = -1
    src, dst, sport, dport, proto = tup
    b = D.TupleBatch.from_numpy(*tup)
    sm = slot_map(e)

    # CONN, with hit counters: one count per evalACL each connection makes
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(e.num_counter_slots(), dtype=torch.int64, device="cuda")
    D.classify(e, MODE_CONN, -1, b, out, counters=cnt)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    conn, lt, li, evt, evi = fast.test_connection(ora, if_in, if_out, sif, dif, src, dst, sport, dport, proto,
                                                  trace=True)
    to_slot = lambda t, i: (sm[(int(t), int(i))] if t >= 0 and i >= 0 else  # noqa: E731
                            sm[(int(t), -1)] if t >= 0 else sm[(-1, -2)] if t == -2 else sm[(-1, -1)])
    exp_slot = np.array([to_slot(t, i) for t, i in zip(lt, li)], np.uint32)
    assert ((got >> 30) == conn.astype(np.uint32)).all(), np.nonzero((got >> 30) != conn)[0][:10]
    assert ((got & 0x3FFFFFFF) == exp_slot).all()
    made = evt != -3
    assert np.array_equal((evt == -2).any(axis=1), invalid)  # the only unresolved connections
    hist = np.bincount([to_slot(t, i) for t, i in zip(evt[made], evi[made])], minlength=cnt.numel())
    assert np.array_equal(cnt.cpu().numpy(), hist)

    # PERPOD: evalACL(outbound ACL of dst's interface)
    D.classify(e, MODE_PERPOD, -1, b, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    ea = np.empty(n, np.int64)
    es = np.empty(n, np.int64)
    for t_if in np.unique(dif):
        m = dif == t_if
        t = if_out[t_if]
        a, i = fast.eval_acl(ora[t] if t >= 0 else None, src[m], dst[m], dport[m], proto[m])
        ea[m] = a
        es[m] = [sm[(t, int(x))] if t >= 0 and x >= 0 else (sm[(t, -1)] if t >= 0 else sm[(-1, -1)]) for x in i]
    assert ((got >> 30) == ea).all() and ((got & 0x3FFFFFFF) == es).all()


def test_generator_matches_numpy_restatement():
    """k_gen (pool/uniform modes) == oracle/gen.py for two shards of a global index range."""
    from oracle import gen
    from vpp_amd import workloads as W
    w = W.config1(0, n_tuples=1 << 16)
    for base in (0, 12345678901):
        b = D.TupleBatch(50001, with_sport=True)
        D.gen_tuples(w.engine, b, index_base=base, **w.gen)
        torch.cuda.synchronize()
        got = b.numpy(b.n)
        exp = gen.gen_tuples(b.n, index_base=base, **w.gen)
        for g, x in zip(got, exp):
            assert np.array_equal(np.asarray(g), np.asarray(x))


@pytest.mark.parametrize("config,mode", [(3, None), (5, None), (8, None), (8, MODE_CONN), (9, None), (9, MODE_CONN)],
                         ids=["3", "5", "8", "8conn", "9", "9conn"])
def test_cluster_configs_gpu_vs_oracle(config, mode):
    """Configs 3 (PERPOD) and 5 (CONN) at full topology (1k pods, ~10k rules), config 8 -- the
    same cluster with 20 apps per namespace: 202 per-pod tables, past the 64 one common-row mask
    bit each covers (grouped marks) -- and config 9 -- 50 apps per namespace: 502 tables, past
    the 254 whose ids fit a byte of a class record (wide records) -- in both modes; 2M
    device-generated tuples, with hit counters (and the uncounted launch), bit-exact against the
    C oracle through oracle.world."""
    from oracle.world import World
    from vpp_amd import workloads as W
    w = W.CONFIGS[config](0, n_tuples=2 << 20)
    e = w.engine
    mode = w.mode if mode is None else mode
    if config in (8, 9):
        ns = e.node_stats()
        assert e.num_tables() > 64 and ns["uniform"] and ns["common_row_pairs"] > 0.5 * ns["table_ipclass_pairs"], ns
        assert ns["wide_records"] == (config == 9), ns
    b = D.TupleBatch(w.n_tuples, with_sport=(mode == MODE_CONN))
    D.gen_tuples(e, b, **w.gen)
    out = torch.empty(b.n, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(e.num_counter_slots(), dtype=torch.int64, device="cuda")
    D.classify(e, mode, -1, b, out, counters=cnt)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    src, dst, sport, dport, proto = b.numpy(b.n)
    wd = World(e, w.local_ifs, w.node_if)
    if mode == MODE_PERPOD:
        act, slot = wd.perpod(src, dst, dport, proto, threads=16)
        # one evaluation per tuple: the counters are the histogram of the verdict slots
        assert np.array_equal(cnt.cpu().numpy(), np.bincount(got & 0x3FFFFFFF, minlength=cnt.numel()))
    else:
        # the per-rule hit counters (the statscollector stream) equal the oracle's histogram of
        # every evalACL the connections made (aclengine_mock.go:448-491, up to four each)
        act, slot, hist = wd.conn(src, dst, sport, dport, proto, threads=16, hist=True)
        c = cnt.cpu().numpy()
        assert np.array_equal(c, hist), np.nonzero(c != hist)[0][:10]
        assert int(c.sum()) > b.n  # some connections evaluate more than one ACL
    assert ((got >> 30) == act.astype(np.uint32)).all()
    assert ((got & 0x3FFFFFFF) == slot).all()
    assert len(np.unique(got >> 30)) >= 2
    D.classify(e, mode, -1, b, out)  # the launch without counters: the same verdicts
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), got)


@pytest.mark.parametrize("any_pct", [0.05, 1.0])
def test_conn_any_protocol_packets_deferred(any_pct):
    """CONN over the uniform node (config 5's topology) classifies ANY-protocol packets (proto
    codes > 2: evalACL skips the L4 test) after its main loop through the per-table path
    (device.hip PG_CONN_DEFER_ANY): verdicts and the per-evaluation counters equal the oracle,
    for a few such packets and for a batch of nothing else, ragged tail included."""
    from oracle.world import World
    from vpp_amd import workloads as W
    w = W.config5(0, n_tuples=(1 << 18) + 7)
    e = w.engine
    assert e.node_stats()["uniform"]
    b0 = D.TupleBatch(w.n_tuples, with_sport=True)
    D.gen_tuples(e, b0, **w.gen)
    src, dst, sport, dport, proto = b0.numpy(b0.n)
    rng = np.random.default_rng(11)
    m = rng.random(b0.n) < any_pct
    proto = proto.copy()
    proto[m] = rng.choice(np.array([3, 7, 255], np.uint8), int(m.sum()))
    b = D.TupleBatch.from_numpy(src, dst, sport, dport, proto)
    out = torch.empty(b.n, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(e.num_counter_slots(), dtype=torch.int64, device="cuda")
    D.classify(e, MODE_CONN, -1, b, out, counters=cnt)
    out0 = torch.empty(b.n, dtype=torch.int32, device="cuda")
    D.classify(e, MODE_CONN, -1, b, out0)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    assert np.array_equal(out0.cpu().numpy().view(np.uint32), got)
    act, slot, hist = World(e, w.local_ifs, w.node_if).conn(src, dst, sport, dport, proto, threads=16, hist=True)
    assert ((got >> 30) == act.astype(np.uint32)).all(), np.nonzero((got >> 30) != act)[0][:10]
    assert ((got & 0x3FFFFFFF) == slot).all()
    c = cnt.cpu().numpy()
    assert np.array_equal(c, hist), np.nonzero(c != hist)[0][:10]


def test_conn_any_protocol_concurrent_streams():
    """k_conn_any finds its own launch's mark: CONN launches on two streams in flight together,
    one batch with ANY-protocol packets and one without, then the other way round; every
    verdict equals the oracle's."""
    from oracle.world import World
    from vpp_amd import workloads as W
    w = W.config5(0, n_tuples=(1 << 17) + 3)
    e = w.engine
    wd = World(e, w.local_ifs, w.node_if)
    b0 = D.TupleBatch(w.n_tuples, with_sport=True)
    D.gen_tuples(e, b0, **w.gen)
    src, dst, sport, dport, proto = b0.numpy(b0.n)
    rng = np.random.default_rng(12)
    proto_any = proto.copy()
    m = rng.random(b0.n) < 0.03
    proto_any[m] = 7
    batches = [D.TupleBatch.from_numpy(src, dst, sport, dport, proto_any), D.TupleBatch.from_numpy(src, dst, sport, dport, proto)]
    expect = [wd.conn(src, dst, sport, dport, p, threads=16)[0] for p in (proto_any, proto)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for order in ((0, 1), (1, 0)):
        outs = [torch.empty(b0.n, dtype=torch.int32, device="cuda") for _ in range(2)]
        torch.cuda.synchronize()
        for k in order:
            with torch.cuda.stream(streams[k]):
                for _ in range(3):  # several launches per stream: several ring slots in flight
                    D.classify(e, MODE_CONN, -1, batches[k], outs[k])
        torch.cuda.synchronize()
        for k in range(2):
            got = outs[k].cpu().numpy().view(np.uint32)
            assert ((got >> 30) == expect[k].astype(np.uint32)).all(), (order, k)


@pytest.mark.parametrize("config", [2, 3, 4, 5])
def test_launch_split_equals_one_launch(config):
    """A batch classified in several launches gives the verdicts and hit counters of one launch:
    Tuning launch_max_tuples = 64 x 1001 over a ragged batch (dev_classify splits a batch above
    2^30 - 64 tuples, the most a launch's 32-bit stream offsets allow, the same way), CONN with
    ANY-protocol packets among the tuples (their deferred pass runs per launch)."""
    from vpp_amd import workloads as W
    w = W.CONFIGS[config](0, n_tuples=(1 << 20) + 37)
    e = w.engine
    b = D.TupleBatch(w.n_tuples, with_sport=True)
    D.gen_tuples(e, b, **w.gen)
    if w.mode == MODE_CONN:
        b.proto[::97] = 7
    res = []
    for cap in (0, 64 * 1001):
        with e.tuning(launch_max_tuples=cap):
            out = torch.empty(b.n, dtype=torch.int32, device="cuda")
            cnt = torch.zeros(e.num_counter_slots(), dtype=torch.int64, device="cuda")
            D.classify(e, w.mode, w.table_id, b, out, counters=cnt)
            torch.cuda.synchronize()
            res.append((out.cpu().numpy(), cnt.cpu().numpy()))
    assert np.array_equal(res[0][0], res[1][0])
    assert np.array_equal(res[0][1], res[1][1])
    assert int(res[0][1].sum()) >= b.n


def test_batch_past_32bit_stream_offsets():
    """A batch of 2^30 + 4103 tuples (config 2's table, device-generated; ~19 GB of HBM): the
    library splits it at 2^30 - 64 tuples, so the first launch reads its src stream up to byte
    2^32 - 260 through 32-bit offsets (PG_IDX32). Its verdicts equal those of launches of 2^29
    tuples (launch_max_tuples), and the tuples around the split and at the end equal the
    oracle's."""
    from oracle.world import expected
    from vpp_amd import workloads as W
    if torch.cuda.get_device_properties(0).total_memory < (64 << 30):
        pytest.skip("needs a large-HBM GPU")
    w = W.config2(0, n_tuples=1024)
    e = w.engine
    n = (1 << 30) + 4103
    b = D.TupleBatch(n, with_sport=False)
    D.gen_tuples(e, b, **w.gen)
    outs = []
    for cap in (0, 1 << 29):
        with e.tuning(launch_max_tuples=cap):
            out = torch.empty(n, dtype=torch.int32, device="cuda")
            D.classify(e, w.mode, w.table_id, b, out)
            torch.cuda.synchronize()
            outs.append(out)
    assert torch.equal(outs[0], outs[1])
    split = (1 << 30) - 64
    for lo, hi in ((split - 4096, split + 4096), (n - 8192, n)):
        tup = tuple(x[lo:hi].cpu().numpy().view(dt) for x, dt in
                    ((b.src, np.uint32), (b.dst, np.uint32), (b.dport, np.uint16), (b.proto, np.uint8)))
        src, dst, dport, proto = tup
        act, slot, _ = expected(e, w.mode, w.table_id, w.local_ifs, w.node_if, src, dst,
                                np.zeros(hi - lo, np.uint16), dport, proto)
        got = outs[0][lo:hi].cpu().numpy().view(np.uint32)
        assert ((got >> 30) == act.astype(np.uint32)).all() and ((got & 0x3FFFFFFF) == slot).all()
    del outs, b
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n_tables", [252, 253])
def test_node_kernels_at_the_narrow_wide_record_boundary(n_tables):
    """The kernels on both sides of the class records' byte-wide table ids (252 tables: narrow
    records; 253: the "no ACL" pseudo-table's id rounds up to 256, wide records -- see
    test_node_host.py): PERPOD and CONN with counters equal the host run of the same per-tuple
    code, which test_node_host.py pins to the oracle; ragged batch, ANY-protocol packets in."""
    from test_node_host import _many_tables, tuples
    e, local, pod_ips = _many_tables(n_tables, 900 + n_tables)
    assert e.node_stats()["wide_records"] == (n_tables > 252)
    tup = tuples(n_tables, (1 << 16) + 5, pod_ips)
    b = D.TupleBatch.from_numpy(*tup)
    for mode in (MODE_PERPOD, MODE_CONN):
        out = torch.empty(b.n, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(e.num_counter_slots(), dtype=torch.int64, device="cuda")
        D.classify(e, mode, -1, b, out, counters=cnt)
        torch.cuda.synchronize()
        host, hc = e.debug_classify_host(mode, -1, *tup, counters=True, node=True)
        assert np.array_equal(out.cpu().numpy().view(np.uint32), host), mode
        assert np.array_equal(cnt.cpu().numpy(), hc.astype(np.int64)), mode


@pytest.mark.parametrize("mode", [MODE_PERPOD, MODE_CONN])
def test_half_cell_histogram_past_0x8000(mode):
    """Config 8's 202-table set counts into 16-bit LDS cells (k_classify STAGE + 256: its 32-bit
    histogram would leave LDS for one workgroup per CU). 48M copies of one connection: every
    workgroup takes each of its slots past 0x8000 several times, each crossing moving 0x8000 to
    the global counter; the counters equal the host run of that one connection times 48M."""
    from vpp_amd import workloads as W
    w = W.config8(0, n_tuples=1 << 10)
    e = w.engine
    ips = sorted(w.local_ifs)
    tup = (np.array([ips[3]], np.uint32), np.array([ips[7]], np.uint32), np.array([40000], np.uint16),
           np.array([80], np.uint16), np.array([0], np.uint8))
    host, hc = e.debug_classify_host(mode, -1, *tup, counters=True, node=True)
    n = 48 << 20
    b = D.TupleBatch(n, with_sport=True)
    i32 = lambda x: int(x) - (1 << 32) if int(x) >= (1 << 31) else int(x)  # noqa: E731
    b.src.fill_(i32(tup[0][0]))
    b.dst.fill_(i32(tup[1][0]))
    b.sport.fill_(40000 - 65536)
    b.dport.fill_(80)
    b.proto.fill_(0)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(e.num_counter_slots(), dtype=torch.int64, device="cuda")
    D.classify(e, mode, -1, b, out, counters=cnt)
    torch.cuda.synchronize()
    assert int((out != i32(host[0])).sum()) == 0
    assert np.array_equal(cnt.cpu().numpy(), hc.astype(np.int64) * n), np.nonzero(cnt.cpu().numpy() != hc * n)
    assert int(hc.sum()) >= 1


@pytest.mark.parametrize("mode", [MODE_PERPOD, MODE_CONN])
def test_k8s_object_cluster_gpu_vs_oracle(mode):
    """The cluster given as K8s objects (policy cache -> processor -> configurator -> renderer,
    SURVEY.md §8 f3; 4 namespaces x 30 pods, namespace-wide selectors): 1M device-generated
    tuples classified on the GPU, bit-exact against the C oracle through oracle.world."""
    from oracle.world import World
    from vpp_amd import workloads as W
    e, r, local, pool, keep = W.cluster_engine_k8s(0, 4, 30, 5)
    gen = dict(seed=0xC0DE0006, ip_pool=pool, pool_pct=85, dst_pool_pct=88,
               port_pool=np.array(W.CLUSTER_PORTS + [8000, 8001, 8002, 8003, 8004], np.uint16), port_pool_pct=80,
               tcp_pct=60, udp_pct=30)
    b = D.TupleBatch(1 << 20, with_sport=(mode == MODE_CONN))
    D.gen_tuples(e, b, **gen)
    out = torch.empty(b.n, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(e.num_counter_slots(), dtype=torch.int64, device="cuda")
    D.classify(e, mode, -1, b, out, counters=cnt)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    src, dst, sport, dport, proto = b.numpy(b.n)
    wd = World(e, local, "VXLAN-BVI")
    if mode == MODE_PERPOD:
        act, slot = wd.perpod(src, dst, dport, proto, threads=16)
        assert np.array_equal(cnt.cpu().numpy(), np.bincount(got & 0x3FFFFFFF, minlength=cnt.numel()))
    else:
        act, slot, hist = wd.conn(src, dst, sport, dport, proto, threads=16, hist=True)
        assert np.array_equal(cnt.cpu().numpy(), hist)
    assert ((got >> 30) == act.astype(np.uint32)).all()
    assert ((got & 0x3FFFFFFF) == slot).all()
    assert len(np.unique(got >> 30)) >= 2


def _classify_with(e, mode, b, node_path, stage_words=16384, counters=False, common_lds=80 << 10):
    with e.tuning(node_path=node_path, node_stage_max_words=stage_words, node_common_lds_max=common_lds):
        out = torch.empty(b.n, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(e.num_counter_slots(), dtype=torch.int64, device="cuda") if counters else None
        D.classify(e, mode, -1, b, out, counters=cnt)
        torch.cuda.synchronize()
        return out.cpu().numpy().view(np.uint32), (cnt.cpu().numpy() if counters else None)


@pytest.mark.parametrize("config", [3, 5])
def test_node_kernel_equals_per_table_kernel(config):
    """The node classifier (LDS-staged and read from HBM) and the per-table blobs + IPv4 hash
    give identical verdicts and hit counters on the cluster configs, and both equal the
    host run of the same per-tuple code (pg_debug_classify_host) on a ragged batch."""
    from vpp_amd import workloads as W
    w = W.CONFIGS[config](0, n_tuples=(1 << 20) + 3)
    e = w.engine
    assert e.node_stats() is not None
    b = D.TupleBatch(w.n_tuples, with_sport=True)
    D.gen_tuples(e, b, **w.gen)
    staged, c1 = _classify_with(e, w.mode, b, 1, counters=True)
    hbm, c2 = _classify_with(e, w.mode, b, 1, stage_words=0, counters=True)
    table, c3 = _classify_with(e, w.mode, b, 0, counters=True)
    assert np.array_equal(staged, hbm) and np.array_equal(staged, table)
    assert np.array_equal(c1, c2) and np.array_equal(c1, c3)
    # the image's common-row section staged next to the histogram (STAGE 3), and left out
    common, c4 = _classify_with(e, w.mode, b, 1, counters=True, common_lds=160 << 10)
    base, c5 = _classify_with(e, w.mode, b, 1, counters=True, common_lds=0)
    nocnt, _ = _classify_with(e, w.mode, b, 1)  # STAGE 3 at the default budget
    assert np.array_equal(common, staged) and np.array_equal(base, staged) and np.array_equal(nocnt, staged)
    assert np.array_equal(c4, c1) and np.array_equal(c5, c1)
    host = e.debug_classify_host(w.mode, -1, *b.numpy(b.n), node=True)
    assert np.array_equal(host, staged)


@pytest.mark.parametrize("config", [3, 5])
def test_node_launch_variants(config):
    """Every node launch shape, with and without counters, equals the default launch and the
    host run. List-verdict table form (default): with and without the common-row section. Record
    form (node_list_table=0): the image with its common rows but without the dst records
    (records from the cross array), and a build without common rows (records staged right after
    the base image, or left in the cross array)."""
    from vpp_amd import workloads as W
    w = W.CONFIGS[config](0, n_tuples=(1 << 19) + 5)
    e = w.engine
    b = D.TupleBatch(w.n_tuples, with_sport=True)
    D.gen_tuples(e, b, **w.gen)
    ref, cref = _classify_with(e, w.mode, b, 1, counters=True)
    ref0, _ = _classify_with(e, w.mode, b, 1)
    assert np.array_equal(ref, ref0)
    assert np.array_equal(e.debug_classify_host(w.mode, -1, *b.numpy(b.n), node=True), ref)
    ns = e.node_stats()
    assert ns["list_table_bytes"] and not ns["list_record_bytes"] and ns["common_row_pairs"]
    hist = (e.num_counter_slots() + 2) * 4
    with e.tuning(node_common=0):  # the table form without common rows (STAGE 1)
        assert e.node_stats()["common_row_pairs"] == 0
        for counters in (True, False):
            got, c = _classify_with(e, w.mode, b, 1, counters=counters)
            assert np.array_equal(got, ref) and (not counters or np.array_equal(c, cref))
    with e.tuning(node_list_table=0):
        ns = e.node_stats()
        assert ns["list_records_in_image"] and ns["list_record_bytes"] and ns["common_row_pairs"]
        norec = ns["image_bytes"] - ns["list_record_bytes"]
        for counters in (True, False):
            h = hist if counters else 0
            got, c = _classify_with(e, w.mode, b, 1, counters=counters)  # everything staged
            assert np.array_equal(got, ref) and (not counters or np.array_equal(c, cref))
            # the common rows staged, the records not (lrec cleared: read from the cross array)
            got, c = _classify_with(e, w.mode, b, 1, counters=counters, common_lds=h + norec + 16)
            assert np.array_equal(got, ref) and (not counters or np.array_equal(c, cref))
        with e.tuning(node_common=0):
            ns2 = e.node_stats()
            assert ns2["common_row_pairs"] == 0 and ns2["list_records_in_image"]
            base = ns2["base_image_bytes"] // 4
            for counters in (True, False):
                got, c = _classify_with(e, w.mode, b, 1, counters=counters)  # STAGE 1, records staged
                assert np.array_equal(got, ref) and (not counters or np.array_equal(c, cref))
                # STAGE 1 with the base image only: records from the cross array
                got, c = _classify_with(e, w.mode, b, 1, stage_words=base, counters=counters)
                assert np.array_equal(got, ref) and (not counters or np.array_equal(c, cref))


def test_large_table_root_staged_and_hbm_walks_equal_oracle():
    """A table whose blob exceeds LDS (candidate mode, level-compressed tries): the launch
    that stages only the src-trie root (STAGE 2) and the one that reads everything from HBM
    both equal evalACL."""
    rnd = random.Random(42)
    rules = []
    for k in range(20000):
        rules.append({"action": k % 2, "src": "10.%d.%d.%d/%d" % (k // 4096, (k // 16) % 256, (k % 16) * 16,
                                                                    rnd.choice([28, 29, 30, 31, 32])), "dst": "",
                      "udp": {"src": [0, 65535], "dst": [k % 1000, k % 1000 + 5]}})
    rules += fz.rand_acl(rnd, 50, fz.ANCHORS, weird=True, tail="deny")
    e = make_engine({"big": (None, rules)})
    tid = e.table_id("out-big")
    assert e.table_stats(tid)["structure"] == "cand" and e.table_stats(tid)["blob_bytes"] > (64 << 10)
    anchors = [(10 << 24) | (k << 4) for k in range(0, 20000, 13)] + fz.ANCHORS
    tup = fz.rand_tuples(np.random.default_rng(42), 200003, anchors, any_pct=0.02)
    ea, es = expected_single(e, tid, rules, tup)
    outs = []
    for root_words in (16400, 0):
        with e.tuning(stage_root_max_words=root_words):
            got, _ = run_single(e, tid, tup)
        assert ((got >> 30) == ea).all() and ((got & 0x3FFFFFFF) == es).all()
        outs.append(got)
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.parametrize("n_tuples", [122880, 122917, 200003])
def test_candi_window_edges_vs_oracle(n_tuples):
    """CANDI window (Tuning candi_window_bits): config 4's table shape at 20k rules with nested
    lower-priority prefixes in the window, every address of the window and a window's width either
    side, walked by the launch that stages root + window (STAGE 6), with and without counters, and
    with the window off: verdicts and hit counters equal evalACL's. Batch sizes: a multiple of
    64 lanes x 4 tuples, and two that are not (the last wave of the grid-stride loop then runs
    with only its first lanes active: the compacted walks must go to those lanes only)."""
    rnd = random.Random(91)
    rules, addr = [], 10 << 24
    for k in range(20000):
        pl = rnd.randint(26, 32)
        addr = (addr + (1 << (32 - pl)) - 1) & ~((1 << (32 - pl)) - 1)
        r = {"action": rnd.randrange(2), "src": "%d.%d.%d.%d/%d" % (addr >> 24, addr >> 16 & 255, addr >> 8 & 255,
                                                                     addr & 255, pl), "dst": ""}
        addr += 1 << (32 - pl)
        lo = rnd.randrange(1, 60000)
        if k % 5 < 2:
            r["tcp"] = {"src": [0, 65535], "dst": [lo, lo + rnd.choice([0, 10, 500])]}
        elif k % 5 < 4:
            r["udp"] = {"src": [0, 65535], "dst": [lo, lo + rnd.choice([0, 10, 500])]}
        if k % 97 == 50:
            addr += 256
        rules.append(r)
    rules.insert(5000, {"action": 1, "src": "10.0.0.0/22", "dst": "", "tcp": {"src": [0, 65535], "dst": [0, 30000]}})
    rules.insert(5001, {"action": 0, "src": "10.0.2.0/23", "dst": "", "udp": {"src": [0, 65535], "dst": [53, 53]}})
    e = make_engine({"big": (None, rules)})
    tid = e.table_id("out-big")
    span, base = 1 << 11, 10 << 24
    src = np.tile((base - span + np.arange(3 * span)).astype(np.uint32), -(-n_tuples // (3 * span)))[:n_tuples]
    n = len(src)
    g = np.random.default_rng(92)
    proto = g.choice(np.array([0, 1, 2, 7], np.uint8), n, p=[0.45, 0.44, 0.10, 0.01])
    dport = np.where(g.random(n) < 0.3, 53, g.integers(0, 65536, n)).astype(np.uint16)
    tup = (src, g.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32), np.zeros(n, np.uint16), dport, proto)
    ea, es = expected_single(e, tid, rules, tup)
    hist = np.bincount(es, minlength=e.num_counter_slots())
    for wb in (11, 0):
        e.set_tuning("candi_window_bits", wb)
        assert e.table_stats(tid)["structure"] == "candi"
        for counters in (False, True):
            got, _ = run_single(e, tid, tup, counters=counters)
            assert ((got >> 30) == ea).all() and ((got & 0x3FFFFFFF) == es).all(), (wb, counters)
            if counters:
                assert np.array_equal(D.read_counters(e), hist), wb


@pytest.mark.parametrize("mode", [MODE_PERPOD, MODE_CONN])
def test_large_node_set_counter_cache_vs_oracle(mode):
    """Config 6 (K8s objects -> 52 tables, 64.6k rules: more counter slots than the full LDS
    histogram) with hit counters through the node classifier: the LDS slot cache (8192 / the
    default 256 / 64 cells -- a tiny cache spills most slots to global atomics --; 0 = global
    atomics only) gives counters equal to the oracle's histogram (PERPOD: of the verdict slots;
    CONN: of every evaluation), and the verdicts stay bit-exact."""
    from oracle import world as OW
    from vpp_amd import workloads as W
    w = W.config6(0, n_tuples=1 << 20)
    e = w.engine
    assert e.num_counter_slots() > 16382 and e.node_stats() is not None
    b = D.TupleBatch(w.n_tuples, with_sport=True)
    D.gen_tuples(e, b, **w.gen)
    torch.cuda.synchronize()
    tup = b.numpy(b.n)
    act, slot, hist = OW.expected(e, mode, -1, w.local_ifs, w.node_if, *tup, threads=16)
    for cells in (8192, 256, 64, 0):
        e.set_tuning("node_hist_cells", cells)
        out = torch.empty(b.n, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(e.num_counter_slots(), dtype=torch.int64, device="cuda")
        D.classify(e, mode, -1, b, out, counters=cnt)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        assert ((got >> 30) == act.astype(np.uint32)).all() and ((got & 0x3FFFFFFF) == slot).all(), cells
        c = cnt.cpu().numpy()
        assert np.array_equal(c, hist), (cells, np.nonzero(c != hist)[0][:10])
