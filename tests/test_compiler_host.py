"""The table compiler (C++ fastpath.cpp) checked against the oracle without a GPU.

pg_debug_walk_blob walks a compiled classification blob on the host with the same walk
code the kernels instantiate (vpp_amd/csrc/blobwalk.hpp); its verdicts -- ACLAction and
matched rule (counter slot) -- must equal evalACL's for every structure the compiler can
choose: cross product, cross product with dst lists, candidate mode, and empty tables.
"""
import random

import numpy as np
import pytest

import acl_fuzz as fz
from oracle import fast
from vpp_amd import renderer as R


def engine_with(rules_by_name):
    e = R.Engine(0)
    ops = [("config/vpp/acls/v2/acl/" + n, {"name": n, "rules": r, "ingress": [], "egress": ["if-" + n]})
           for n, r in sorted(rules_by_name.items())]
    e.ApplyTxn(True, ops)
    return e


def check(e, name, rules, tup):
    src, dst, sport, dport, proto = tup
    got = e.debug_walk(name, src, dst, dport, proto)
    for pred in (True, False):  # pg_classify's SINGLE-mode code, LDS (predicated) and HBM walks
        host = e.debug_classify_host(0, e.table_id(name), src, dst, sport, dport, proto, pred=pred)
        assert np.array_equal(host, got)
    a, i = fast.eval_acl(fast.OraACL(rules), src, dst, dport, proto)
    names = e.ACLNames()
    base = sum(len(e.GetACLByName(n)["rules"]) for n in names[:names.index(name)])
    nr = sum(len(e.GetACLByName(n)["rules"]) for n in names)
    slot = np.where(i >= 0, base + i, nr + names.index(name)).astype(np.uint32)
    bad = np.nonzero(((got >> 30) != a) | ((got & 0x3FFFFFFF) != slot))[0]
    assert len(bad) == 0, (name, bad[:8], got[bad[:4]] >> 30, a[bad[:4]])


@pytest.mark.parametrize("seed", range(16))
def test_random_weird_acls(seed):
    rnd = random.Random(seed)
    acls = {"t%d" % k: fz.rand_acl(rnd, rnd.choice([0, 1, 3, 12, 60, 250]), fz.ANCHORS, weird=True,
                                   tail=rnd.choice([None, "deny", "permit"])) for k in range(3)}
    e = engine_with(acls)
    tup = fz.rand_tuples(np.random.default_rng(seed), 20000, fz.ANCHORS, any_pct=0.03)
    for n, r in acls.items():
        check(e, n, r, tup)


def test_dst_specific_rules_use_lists():
    rnd = random.Random(5)
    rules = []
    for k in range(40):          # global-table shape: src = pod /32, dst = peer nets, ports
        src = "10.1.0.%d/32" % (k % 8 + 1)
        dst = rnd.choice(["10.2.0.0/16", "10.2.%d.0/24" % k, "8.8.8.8/32", ""])
        rules.append({"action": rnd.choice([0, 1]), "src": src, "dst": dst,
                      "tcp": {"src": [0, 65535], "dst": [80, 80 + k % 3]}})
    rules.append({"action": 1, "src": "", "dst": ""})
    e = engine_with({"g": rules})
    assert e.table_stats(0)["structure"] == "cross+lists"
    anchors = [0x0A010001 + k for k in range(8)] + [0x0A020000, 0x0A020500, 0x08080808]
    tup = fz.rand_tuples(np.random.default_rng(5), 50000, anchors)
    check(e, "g", rules, tup)


def test_large_table_uses_candidate_mode():
    rules = []
    for k in range(20000):       # > 16384 rules: no cross product
        rules.append({"action": k % 2, "src": "10.%d.%d.0/24" % (k // 256, k % 256), "dst": "",
                      "udp": {"src": [0, 65535], "dst": [k % 1000, k % 1000 + 5]}})
    e = engine_with({"big": rules})
    assert e.table_stats(0)["structure"] == "cand"
    anchors = [(10 << 24) | (k << 8) for k in range(0, 20000, 37)]
    tup = fz.rand_tuples(np.random.default_rng(9), 30000, anchors)
    check(e, "big", rules, tup)


def test_empty_and_catch_all_tables():
    e = engine_with({"empty": [], "all": [{"action": 2, "src": "", "dst": ""}]})
    tup = fz.rand_tuples(np.random.default_rng(1), 5000, fz.ANCHORS, any_pct=0.1)
    check(e, "empty", [], tup)
    check(e, "all", [{"action": 2, "src": "", "dst": ""}], tup)
