"""The IP-keyed connection mode (pg_classify CONN: both end points resolved from the packet's
addresses) against the reference's Connection* calls, over every end-point pair.

A CONN tuple (src IP, dst IP, ...) stands for the reference call its two end points select
(mock/aclengine/aclengine_mock.go:273-420):

  pod  -> pod       ConnectionPodToPod      (a pod on another node enters/leaves by the
                                             node-output interface, :291-299 / :309-317)
  pod  -> non-pod   ConnectionPodToInternet (FAILURE for a pod on another node, :343-347)
  non-pod -> pod    ConnectionInternetToPod (FAILURE for a pod on another node, :388-392)
  non-pod -> non-pod  no reference call: FAILURE by the engine's convention

The expected answers come from oracle/aclengine.py's Connection* (the restatement the 284
acl_renderer_test.go KATs pin, tests/test_oracle_kats.py), run on the state of every phase of
every KAT scenario, for every ordered pair of the scenario's pods (plus a pod of this node
without an interface and a second remote pod) and some non-pod addresses, every protocol and a
set of ports. Checked: the ConnAction, the deciding counter slot (the slot of the last
evaluation the call made, "unresolved" for a preamble FAILURE) and the per-rule hit counters
(one count per evaluation, aclengine_mock.go:448-491). CPU: the product's per-tuple code on the
host (pg_debug_classify_host). GPU: k_classify, and also pg_connections (the device
Connection* path the KATs run through) on the same pairs.
"""
import itertools

import numpy as np
import pytest

import kat_driver as kd
from oracle import aclengine as OA
from oracle import gonet

EXTRA_PODS = [("default/podx", "10.10.3.3", False),      # this node, no interface: FAILURE
              ("namespace3/pod9", "10.10.20.2", True)]   # a second pod on another node
INTERNET = ["8.8.8.8", "10.10.50.1", "192.168.1.1", "10.200.0.1"]
PORTS = [0, 22, 53, 67, 80, 161, 443, 514, 8080]
PROTOS = [0, 1, 2, 3]  # TCP, UDP, OTHER, ANY


def _ip(s):
    return gonet.ipv4_u32(gonet.to4(gonet.parse_ip(s)))


def _phases(sc, gpu):
    """(oracle backend, product backend) after each phase of scenario sc."""
    ob, pb = kd.OracleBackend(), kd.ProductBackend(gpu=gpu)
    setup = dict(sc["setup"])
    setup["pods"] = list(setup["pods"]) + [list(p) for p in EXTRA_PODS]
    for b in (ob, pb):
        b.setup(setup)
    for phase in sc["phases"]:
        for st in phase["steps"]:
            for b in (ob, pb):
                if st["op"] == "restart":
                    b.restart()
                else:
                    assert b.txn(st["resync"], st["renders"]) is None
        yield setup, ob, pb


def _reference(ob, setup, rng):
    """Tuples over every end-point pair and the oracle's answers:
    (src, dst, sport, dport, proto, kinds, conn, per-connection trace)."""
    pods = [(p, ip) for p, ip, _ in setup["pods"]]
    ends = [("pod", p, ip) for p, ip in pods] + [("inet", ip, ip) for ip in INTERNET]
    e = ob.engine
    rows = []
    for (ka, a, ipa), (kb, b, ipb) in itertools.product(ends, ends):
        for proto in PROTOS:
            for sport, dport in zip(rng.choice(PORTS, 4), rng.choice(PORTS, 4)):
                sport, dport = int(sport), int(dport)
                tr = []
                if ka == "pod" and kb == "pod":
                    kind = "PodToPod"
                    c = _pod_to_pod(e, a, b, proto, sport, dport, tr)
                elif ka == "pod":
                    kind = "PodToInternet"
                    c = _pod_to_inet(e, a, ipb, proto, sport, dport, tr)
                elif kb == "pod":
                    kind = "InternetToPod"
                    c = _inet_to_pod(e, ipa, b, proto, sport, dport, tr)
                else:
                    kind, c = None, OA.CONN_FAILURE
                rows.append((_ip(ipa), _ip(ipb), sport, dport, proto, (kind, a, b), c, tr))
    return rows


# The oracle's Connection* calls, with the evaluations their testConnection makes recorded
# (the preamble is the oracle's own, aclengine.py, pinned by the KATs).
def _with_trace(e, tr, call):
    orig = e.test_connection
    e.test_connection = lambda *a, **k: orig(*a, trace=tr)
    try:
        return call()
    finally:
        e.test_connection = orig


def _pod_to_pod(e, a, b, proto, sport, dport, tr):
    return _with_trace(e, tr, lambda: e.connection_pod_to_pod(a, b, proto, sport, dport))


def _pod_to_inet(e, a, ip, proto, sport, dport, tr):
    return _with_trace(e, tr, lambda: e.connection_pod_to_internet(a, ip, proto, sport, dport))


def _inet_to_pod(e, ip, b, proto, sport, dport, tr):
    return _with_trace(e, tr, lambda: e.connection_internet_to_pod(ip, b, proto, sport, dport))


def _expected(pe, rows):
    """(ConnAction, deciding slot) per row and the hit-counter histogram, in the product
    engine's slot numbering (pg_table_info / pg_num_counter_slots)."""
    ns = pe.num_counter_slots()
    noacl, unresolved = ns - 2, ns - 1

    def slot(acl, idx):
        if acl is None:
            return noacl
        base, _, dflt = pe.table_info(pe.table_id(acl.name))
        return dflt if idx == OA.NO_RULE else base + idx

    conn = np.array([r[6] for r in rows], np.uint32)
    last = np.array([slot(r[7][-1][0], r[7][-1][2]) if r[7] else unresolved for r in rows], np.uint32)
    hist = np.zeros(ns, np.int64)
    for r in rows:
        if not r[7]:
            hist[unresolved] += 1
        for acl, _, idx in r[7]:
            hist[slot(acl, idx)] += 1
    return conn, last, hist


def _arrays(rows):
    return (np.array([r[0] for r in rows], np.uint32), np.array([r[1] for r in rows], np.uint32),
            np.array([r[2] for r in rows], np.uint16), np.array([r[3] for r in rows], np.uint16),
            np.array([r[4] for r in rows], np.uint8))


def _cases():
    return [(sc["name"], sc) for sc in kd.load("acl_renderer_kats.json")]


@pytest.mark.parametrize("name,sc", _cases(), ids=[n for n, _ in _cases()])
def test_conn_mode_every_endpoint_pair_host(name, sc):
    from vpp_amd._capi import MODE_CONN
    rng = np.random.default_rng(len(name))
    kinds_seen = set()
    for setup, ob, pb in _phases(sc, gpu=False):
        rows = _reference(ob, setup, rng)
        pe = pb.engine
        conn, last, hist = _expected(pe, rows)
        for node in (True, False):  # node classifier and per-table (iphash) path
            got, cnt = pe.debug_classify_host(MODE_CONN, -1, *_arrays(rows), counters=True, node=node)
            bad = np.nonzero((got >> 30) != conn)[0]
            assert not len(bad), [(rows[i][5], int(got[i] >> 30), int(conn[i])) for i in bad[:5]]
            assert np.array_equal(got & 0x3FFFFFFF, last)
            assert np.array_equal(cnt.astype(np.int64), hist)
        kinds_seen |= {(r[5][0], r[6]) for r in rows}
    # the scenario exercised the reference's preamble FAILUREs as well as evaluated outcomes
    assert ("PodToInternet", OA.CONN_FAILURE) in kinds_seen and ("InternetToPod", OA.CONN_FAILURE) in kinds_seen
    assert any(k[0] == "PodToPod" and k[1] != OA.CONN_FAILURE for k in kinds_seen)


@pytest.mark.gpu
@pytest.mark.parametrize("name,sc", _cases(), ids=[n for n, _ in _cases()])
def test_conn_mode_every_endpoint_pair_gpu(name, sc):
    """k_classify CONN (verdict, slot, counters) == the oracle's Connection* answers ==
    pg_connections (the device Connection* path) on every end-point pair with a reference call."""
    import torch
    from vpp_amd import device as D
    from vpp_amd._capi import MODE_CONN
    rng = np.random.default_rng(len(name))
    for setup, ob, pb in _phases(sc, gpu=True):
        rows = _reference(ob, setup, rng)
        pe = pb.engine
        conn, last, hist = _expected(pe, rows)
        b = D.TupleBatch.from_numpy(*_arrays(rows))
        out = torch.empty(b.n, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(pe.num_counter_slots(), dtype=torch.int64, device="cuda")
        D.classify(pe, MODE_CONN, -1, b, out, counters=cnt)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        assert np.array_equal(got >> 30, conn)
        assert np.array_equal(got & 0x3FFFFFFF, last)
        assert np.array_equal(cnt.cpu().numpy(), hist)
        qi = [i for i, r in enumerate(rows) if r[5][0] is not None]
        qs = []
        for i in qi:
            kind, a, bb = rows[i][5]
            qs.append((kind, a, bb, int(rows[i][4]), int(rows[i][2]), int(rows[i][3])))
        pc, ps = pe.connections(qs)
        assert np.array_equal(np.array(pc, np.uint32), conn[qi])
        assert np.array_equal(np.array(ps, np.uint32), last[qi])
