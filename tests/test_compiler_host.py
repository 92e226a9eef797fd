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


class tuning:
    """pg_set_tuning for the tables compiled inside the block"""

    def __init__(self, key, value, default):
        self.k, self.v, self.d = key.encode(), value, default

    def __enter__(self):
        assert R.lib.pg_set_tuning(self.k, self.v) == 0

    def __exit__(self, *a):
        R.lib.pg_set_tuning(self.k, self.d)


def test_large_table_uses_candidate_mode():
    rules = []
    for k in range(20000):       # > 16384 rules, 20k src x 1k key classes: no product fits
        rules.append({"action": k % 2, "src": "10.%d.%d.0/24" % (k // 256, k % 256), "dst": "",
                      "udp": {"src": [0, 65535], "dst": [k % 1000, k % 1000 + 5]}})
    anchors = [(10 << 24) | (k << 8) for k in range(0, 20000, 37)]
    tup = fz.rand_tuples(np.random.default_rng(9), 30000, anchors)
    # no rule tests dst: the inline-candidate form (CANDI); with it off, the record form
    for candi, want in ((1, "candi"), (0, "cand")):
        with tuning("candi", candi, 1):
            e = engine_with({"big": rules})
            assert e.table_stats(0)["structure"] == want
        check(e, "big", rules, tup)


@pytest.mark.parametrize("seed", range(3))
def test_candi_nested_prefixes_and_defaults(seed):
    """CANDI (dst-free candidate tables read from HBM): src classes with no candidate (the
    table's default inline), one candidate (inline: key range, action, rule), and several
    (nested /16 /24 /30 prefixes: the leaf points at the record list, whose last record carries
    the last-record flag); unconditional rules ending lists; ANY-protocol packets (linear);
    classes reached through root leaves (records)."""
    rnd = random.Random(300 + seed)
    rules = []
    for k in range(18000):
        a, b = rnd.randrange(6), rnd.randrange(64)
        src = rnd.choice(["10.%d.0.0/16" % a, "10.%d.%d.0/24" % (a, b), "10.%d.%d.%d/30" % (a, b, 4 * rnd.randrange(64)),
                          "10.%d.%d.%d/32" % (a, b, rnd.randrange(256)), "172.%d.0.0/12" % (16 + 16 * (k % 2))])
        r = {"action": rnd.randrange(2), "src": src, "dst": ""}
        kind = rnd.random()
        if kind < 0.4:
            lo = rnd.randrange(1, 60000)
            r["tcp"] = {"src": [0, 65535], "dst": [lo, lo + rnd.choice([0, 3, 100])]}
        elif kind < 0.8:
            lo = rnd.randrange(1, 60000)
            r["udp"] = {"src": [0, 65535], "dst": [lo, lo + rnd.choice([0, 3, 100])]}
        rules.append(r)
    if seed == 1:
        rules.append({"action": 1, "src": "", "dst": ""})
    with tuning("cross_max_rules", 0, 1 << 20), tuning("pair", 0, 1):  # (its cross product would fit)
        e = engine_with({"big": rules})
        assert e.table_stats(0)["structure"] == "candi"
    anchors = [(10 << 24) | (a << 16) | (b << 8) for a in range(7) for b in range(0, 66, 3)] + \
              [(172 << 24) | (k << 20) for k in range(4)]
    tup = fz.rand_tuples(np.random.default_rng(400 + seed), 40000, anchors, any_pct=0.02)
    check(e, "big", rules, tup)


@pytest.mark.parametrize("wbits", [11, 8])
def test_candi_window(wbits):
    """CANDI window (fastpath.cpp, Tuning candi_window_bits): the terminal entries of the aligned
    2^bits-address window where the earliest rules sit, staged with the root. Every address of
    the window and past both of its edges, with classes of no candidate, one (inline) and several
    (record list: nested lower-priority prefixes): the same verdicts as evalACL with and without
    the window, and in the window no trie gather (an inline candidate reads LDS only)."""
    rnd = random.Random(77)
    rules, addr = [], 10 << 24
    for k in range(6000):  # config 4's shape: disjoint /26../32 packed from 10.0.0.0 up
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
        if k % 97 == 50:  # a hole: addresses no rule covers (the default, inline)
            addr += 256
        rules.append(r)
    rules.insert(3000, {"action": 1, "src": "10.0.0.0/22", "dst": "", "tcp": {"src": [0, 65535], "dst": [0, 30000]}})
    rules.insert(3001, {"action": 0, "src": "10.0.2.0/23", "dst": "", "udp": {"src": [0, 65535], "dst": [53, 53]}})
    base, span = 10 << 24, 1 << wbits
    n = 3 * span
    src = (base - span + np.arange(n)).astype(np.uint32)  # the window and a window's width either side
    g = np.random.default_rng(78)
    proto = g.choice(np.array([0, 1, 2], np.uint8), n, p=[0.45, 0.45, 0.10])
    dport = np.where(g.random(n) < 0.3, 53, g.integers(0, 65536, n)).astype(np.uint16)
    tup = (src, g.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32), np.zeros(n, np.uint16), dport, proto)
    gathers = {}
    for wb in (wbits, 0):
        with tuning("cross_max_rules", 0, 1 << 20), tuning("pair", 0, 1), tuning("candi_window_bits", wb, 11), \
                tuning("lc_root_bits", 12, 13):  # (the root a window caps at 12 bits, both ways)
            e = engine_with({"big": rules})
            assert e.table_stats(0)["structure"] == "candi"
        check(e, "big", rules, tup)
        nl, nm, stage = e.debug_walk_stats(0, *tup[:2], tup[3], tup[4])
        assert stage == 2
        gathers[wb] = nm
    inw = (src >= base) & (src < base + span)
    assert (gathers[0] >= 1).all()  # no window: every lookup gathers
    assert (gathers[wbits][~inw] == gathers[0][~inw]).all()
    assert (gathers[wbits][inw] == 0).mean() > 0.3  # inline candidates and the default: LDS only
    assert (gathers[wbits][inw] <= gathers[0][inw] - 1).all()


def test_long_dst_lists_use_pair_mode():
    """global-table shape with long dst lists (egress to many pod /32s per port): PAIR mode,
    and the same verdicts with it disabled (cross product + dst lists)"""
    rnd = random.Random(11)
    pods = [0x0A010000 | k for k in range(1, 400)]
    rules = []
    for s in range(12):
        src = "10.1.0.%d/32" % (s + 1)
        rules.append({"action": 1, "src": src, "dst": "", "tcp": {"src": [0, 65535], "dst": [443, 443]}})
        for p in rnd.sample(pods, 300):
            port = rnd.choice([8000, 8001, 8002])
            rules.append({"action": 1, "src": src, "dst": "%d.%d.%d.%d/32" % (p >> 24, p >> 16 & 255, p >> 8 & 255,
                                                                            p & 255),
                          "tcp": {"src": [0, 65535], "dst": [port, port]}})
        rules.append({"action": 1, "src": src, "dst": "10.96.0.10/32", "udp": {"src": [0, 65535], "dst": [53, 53]}})
        rules.append({"action": 0, "src": src, "dst": ""})
    rules.append({"action": 1, "src": "", "dst": ""})
    anchors = pods[:40] + [0x0A010001 + k for k in range(12)] + [0x0A60000A]
    tup = fz.rand_tuples(np.random.default_rng(11), 40000, anchors)
    for pair, want in ((1, "pair"), (0, "cross+lists")):
        with tuning("pair", pair, 1):
            e = engine_with({"g": rules})
            assert e.table_stats(0)["structure"] == want
        check(e, "g", rules, tup)


@pytest.mark.parametrize("seed", range(12))
def test_random_weird_acls_pair_mode(seed):
    """every random weird ACL compiled into PAIR mode (pair = 2) walks to evalACL's verdicts"""
    rnd = random.Random(100 + seed)
    acls = {"t%d" % k: fz.rand_acl(rnd, rnd.choice([1, 3, 12, 60, 250]), fz.ANCHORS, weird=True,
                                   tail=rnd.choice([None, "deny", "permit"])) for k in range(3)}
    with tuning("pair", 2, 1):
        e = engine_with(acls)
        e.table_stats(0)  # compiles the tables under the tuning
    tup = fz.rand_tuples(np.random.default_rng(100 + seed), 20000, fz.ANCHORS, any_pct=0.03)
    for n, r in acls.items():
        assert e.table_stats(e.table_id(n))["structure"] in ("pair", "linear")
        check(e, n, r, tup)


def test_empty_and_catch_all_tables():
    e = engine_with({"empty": [], "all": [{"action": 2, "src": "", "dst": ""}]})
    tup = fz.rand_tuples(np.random.default_rng(1), 5000, fz.ANCHORS, any_pct=0.1)
    check(e, "empty", [], tup)
    check(e, "all", [{"action": 2, "src": "", "dst": ""}], tup)


def test_candidate_mode_multi_record_lists():
    """CAND lists of several candidates (nested src prefixes, dst-specific rules) whose last
    record carries the last-record flag instead of a match-all terminator, empty lists
    (sources no rule covers), and unconditional rules that end a list early."""
    rnd = random.Random(23)
    rules = []
    for k in range(17000):
        a, b = rnd.randrange(8), rnd.randrange(64)
        src = rnd.choice(["10.%d.0.0/16" % a, "10.%d.%d.0/24" % (a, b), "10.%d.%d.%d/30" % (a, b, 4 * rnd.randrange(64))])
        r = {"action": rnd.randrange(2), "src": src,
             "dst": rnd.choice(["", "", "192.168.%d.0/24" % rnd.randrange(4), "192.168.0.%d/32" % rnd.randrange(8)])}
        kind = rnd.random()
        if kind < 0.45:
            lo = rnd.randrange(1, 60000)
            r["tcp"] = {"src": [0, 65535], "dst": [lo, lo + rnd.choice([0, 3, 100])]}
        elif kind < 0.9:
            lo = rnd.randrange(1, 60000)
            r["udp"] = {"src": [0, 65535], "dst": [lo, lo + rnd.choice([0, 3, 100])]}
        rules.append(r)
    e = engine_with({"big": rules})
    assert e.table_stats(0)["structure"] == "cand"
    anchors = [(10 << 24) | (a << 16) | (b << 8) for a in range(9) for b in range(0, 66, 3)] + \
              [(192 << 24) | (168 << 16) | (k << 8) for k in range(5)]
    tup = fz.rand_tuples(np.random.default_rng(24), 30000, anchors)
    check(e, "big", rules, tup)


@pytest.mark.parametrize("seed", range(10))
def test_fd_tables_dst_free(seed):
    """Tables where no rule tests dst (the renderer's pod tables, config 2) compile to the FD
    form (fixed-depth walks, no dst stream; fastpath.cpp build_fd_blob) and classify like
    evalACL -- ANY-protocol packets included -- and like the same tables compiled without it."""
    rnd = random.Random(700 + seed)
    rules = fz.rand_acl(rnd, rnd.choice([1, 5, 40, 300, 1000]), fz.ANCHORS, weird=(seed % 2 == 1),
                        tail=rnd.choice([None, "deny", "permit"]))
    for r in rules:
        r["dst"] = ""
    plain = [r for r in rules if not any(r.get(k) for k in ("macip", "icmp")) and r.get("ip_rule", True)
             and r.get("ip", True) and not (r.get("tcp") and r.get("udp"))]
    rules = plain or [{"action": 1, "src": "", "dst": ""}]
    e = engine_with({"fd": rules})
    st = e.table_stats(0)
    tup = fz.rand_tuples(np.random.default_rng(seed), 30000, fz.ANCHORS, any_pct=0.05)
    check(e, "fd", rules, tup)
    got = e.debug_walk("fd", *[tup[k] for k in (0, 1, 3, 4)])
    # the verdict does not depend on dst
    tup2 = (tup[0], np.random.default_rng(seed + 1).integers(0, 1 << 32, len(tup[0]), dtype=np.uint64).astype(
        np.uint32)) + tup[2:]
    assert np.array_equal(e.debug_walk("fd", *[tup2[k] for k in (0, 1, 3, 4)]), got)
    e0 = R.Engine(0)
    e0.set_tuning("fd", 0)
    e0.ApplyTxn(True, [("config/vpp/acls/v2/acl/fd", {"name": "fd", "rules": rules, "ingress": [],
                                                       "egress": ["if-fd"]})])
    assert e0.table_stats(0)["structure"] != "fd"
    assert np.array_equal(e0.debug_walk("fd", *[tup[k] for k in (0, 1, 3, 4)]), got)
    # not FD only when the FD form would not fit LDS (or the table is no cross product)
    assert st["structure"] == "fd" or st["structure"] in ("cand", "pair", "linear") or st["blob_bytes"] > 48 << 10, st


def test_config2_table_is_fd():
    from vpp_amd import workloads as W
    w = W.config2(0, n_tuples=1 << 10)
    st = w.engine.table_stats(w.table_id)
    assert st["structure"] == "fd" and st["blob_bytes"] <= 64 << 10 and st["key_classes"] == 21, st


def test_launch_max_tuples_knob():
    """Tuning launch_max_tuples (device.hip dev_classify: the most tuples one k_classify launch
    takes; 0 = the 32-bit stream offsets' limit, 2^30 - 64): multiples of 64 up to that limit,
    anything else PG_EINVAL; a context's value reads back."""
    e = R.Engine(0)
    assert e.get_tuning("launch_max_tuples") == 0
    for v in (64, 64 * 1001, (1 << 30) - 64, 0):
        e.set_tuning("launch_max_tuples", v)
        assert e.get_tuning("launch_max_tuples") == v
    for v in (1, 63, 65, 1 << 30, -64):
        with pytest.raises(Exception):
            e.set_tuning("launch_max_tuples", v)
    assert e.get_tuning("launch_max_tuples") == 0
