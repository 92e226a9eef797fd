"""Host-side parity of the product renderer (C++ via the C ABI) against the CPU oracle.

No GPU needed: the renderer cache, the ACL renderer and ACL installation run on the host;
only evalACL/testConnection run on the device (tests/test_gpu_*.py). Checked here:
  * the C ABI library loads and exports every symbol include/policygpu.h declares;
  * for every acl_renderer_test.go scenario, every non-Connection* assertion, and the full
    set of installed ACLs (names = FNV-64a table IDs, rules, port ranges, interfaces) after
    every transaction, equal the oracle's;
  * the same on randomised multi-pod transactions (adds, updates, removals, resyncs,
    renderer restarts) built from the reference's own rule vocabulary.
"""
import random
import re

import pytest

import kat_driver as kd
from oracle import gonet, policy

ROOT_HDR = __import__("os").path.join(__import__("os").path.dirname(__file__), "..", "include", "policygpu.h")


def test_library_exports_every_declared_symbol():
    import ctypes
    from vpp_amd import _capi
    hdr = open(ROOT_HDR).read()
    declared = sorted(set(re.findall(r"\b(pg_[a-z0-9_]+)\s*\(", hdr)))
    lib = ctypes.CDLL(_capi.LIB_PATH)
    missing = [n for n in declared if not hasattr(lib, n)]
    assert not missing, missing
    assert set(declared) == set(_capi.EXPORTED)


def oracle_acls(engine):
    out = {}
    for name, acl in engine.cfg.by_name.items():
        rules = []
        for r in acl.rules:
            def sec(s):
                if s is None:
                    return None
                return {"src": [s.src_range.lower, s.src_range.upper], "dst": [s.dst_range.lower, s.dst_range.upper]}
            rules.append({"action": r.action, "src": r.src_network, "dst": r.dst_network, "tcp": sec(r.tcp),
                          "udp": sec(r.udp)})
        out[name] = {"ingress": sorted(acl.ingress), "egress": sorted(acl.egress), "rules": rules}
    return out


def product_acls(engine):
    out = {}
    for name in engine.ACLNames():
        a = engine.GetACLByName(name)
        out[name] = {"ingress": sorted(a["ingress"]), "egress": sorted(a["egress"]),
                     "rules": [{"action": r["action"], "src": r["src"], "dst": r["dst"], "tcp": r["tcp"],
                                "udp": r["udp"]} for r in a["rules"]]}
    return out


def bindings(engine, pods, ifs):
    return {i: engine._if_acls(i) for i in ifs}


SCENARIOS = kd.load("acl_renderer_kats.json")


@pytest.mark.parametrize("sc", SCENARIOS, ids=[s["name"] for s in SCENARIOS])
def test_product_renderer_matches_reference_kats_host(sc):
    prod = kd.ProductBackend(gpu=False)
    bad = [(c, g) for c, g in kd.run_scenario(prod, sc) if not c["kind"].startswith("Connection")]
    assert not bad, bad[:3]


@pytest.mark.parametrize("sc", SCENARIOS, ids=[s["name"] for s in SCENARIOS])
def test_product_acls_equal_oracle_acls(sc):
    ora, prod = kd.OracleBackend(), kd.ProductBackend(gpu=False)
    ora.setup(sc["setup"])
    prod.setup(sc["setup"])
    for phase in sc["phases"]:
        for st in phase["steps"]:
            if st["op"] == "restart":
                ora.restart()
                prod.restart()
            else:
                assert ora.txn(st["resync"], st["renders"]) is None
                assert prod.txn(st["resync"], st["renders"]) is None
        assert product_acls(prod.engine) == oracle_acls(ora.engine)
        assert prod.num_acl_changes() == ora.num_acl_changes()


# ---- randomised renderer transactions -------------------------------------------------
def _vocab():
    td = kd.load("testdata.json")
    rules = list(td["ts"].values())
    for v in td["ts7"].values():
        rules += v
    ips = td["pod_ips"]
    extra = []
    for ip in ips[:4]:
        extra += [kd.R("PERMIT", ip + "/32", "", "TCP", 0, 80), kd.R("PERMIT", ip + "/32", "", "UDP", 0, 53),
                  kd.R("PERMIT", "", ip + "/32", "TCP", 0, 8080), kd.R("PERMIT", ip + "/32", "", "ANY", 0, 0)]
    extra += [kd.R("PERMIT", "10.10.2.0/24", "", "UDP", 0, 0), kd.R("PERMIT", "", "10.10.1.0/24", "TCP", 0, 443),
              kd.R("PERMIT", "", "", "TCP", 0, 22), kd.R("DENY", "", "", "ANY", 0, 0)]
    return rules + extra


kd.R = lambda a, s, d, p, sp, dp: {"action": a, "src": s, "dst": d, "proto": p, "sport": sp, "dport": dp}


@pytest.mark.parametrize("seed", range(12))
def test_random_renderer_transactions_match_oracle(seed):
    rnd = random.Random(seed)
    td = kd.load("testdata.json")
    vocab = _vocab()
    setup = {"main_if": "GbE", "vxlan_bvi": rnd.choice(["VXLAN-BVI", ""]), "host_interconnect": "VPP-Host",
             "other_ifs": rnd.choice([[], ["other0"]]),
             "pod_ifs": dict(zip(td["pods"][:5], td["pod_ifs"][:5])),
             "pods": [[p, ip, i == 5] for i, (p, ip) in enumerate(zip(td["pods"], td["pod_ips"]))]}
    ora, prod = kd.OracleBackend(), kd.ProductBackend(gpu=False)
    ora.setup(setup)
    prod.setup(setup)
    live = set()
    for step in range(8):
        if rnd.random() < 0.15:
            ora.restart()
            prod.restart()
        resync = step == 0 or rnd.random() < 0.2
        renders = []
        pods = rnd.sample(range(5), rnd.randint(1, 4))
        for i in pods:
            pod, ip = td["pods"][i], td["pod_ips"][i]
            removed = (not resync) and pod in live and rnd.random() < 0.25
            if removed:
                renders.append({"pod": pod, "ip": ip, "ingress": [], "egress": [], "removed": True})
                live.discard(pod)
                continue
            ing = [r for r in rnd.sample(vocab, rnd.randint(0, 4)) if r["src"] == ""]
            eg = [r for r in rnd.sample(vocab, rnd.randint(0, 4)) if r["dst"] == ""]
            if rnd.random() < 0.5:
                ing.append(kd.R("DENY", "", "", "ANY", 0, 0))
            if rnd.random() < 0.5:
                eg.append(kd.R("DENY", "", "", "ANY", 0, 0))
            renders.append({"pod": pod, "ip": ip, "ingress": ing, "egress": eg, "removed": False})
            live.add(pod)
        if resync:
            live = {r["pod"] for r in renders if not r["removed"]}
        e1 = ora.txn(resync, renders)
        e2 = prod.txn(resync, renders)
        assert (e1 is None) == (e2 is None), (e1, e2)
        assert product_acls(prod.engine) == oracle_acls(ora.engine), step
        assert prod.num_acl_changes() == ora.num_acl_changes()
        assert prod.committed_txns() == ora.committed_txns()


@pytest.mark.parametrize("seed", range(4))
def test_acl_ingestion_roundtrip(seed):
    """ApplyTxn (vpp_acl key space) keeps every field evalACL reads, incl. missing ranges."""
    import acl_fuzz as fz
    from vpp_amd import renderer as R
    rnd = random.Random(seed)
    e = R.Engine(0)
    acls = []
    for k in range(3):
        rules = fz.rand_acl(rnd, 30, fz.ANCHORS, weird=True)
        acls.append({"name": "a%d" % k, "rules": rules, "ingress": ["if%d" % k], "egress": []})
    e.ApplyTxn(True, [("config/vpp/acls/v2/acl/" + a["name"], a) for a in acls])
    for a in acls:
        got = e.GetACLByName(a["name"])
        for r0, r1 in zip(a["rules"], got["rules"]):
            assert r1["action"] == r0["action"] and r1["src"] == r0["src"] and r1["dst"] == r0["dst"]
            for f in ("tcp", "udp"):
                if r0.get(f) is None:
                    assert r1[f] is None
                else:
                    assert r1[f] == {"src": r0[f].get("src"), "dst": r0[f].get("dst")}
            for f, d in (("macip", False), ("ip_rule", True), ("ip", True), ("icmp", False)):
                assert r1[f] == r0.get(f, d)
    with pytest.raises(R.PolicyError):
        e.ApplyTxn(False, [("config/vpp/interfaces/x", None)])
    with pytest.raises(R.PolicyError):
        e.ApplyTxn(False, [("config/vpp/acls/v2/acl/missing", None)])
    with pytest.raises(R.PolicyError):
        e.ApplyTxn(False, [("config/vpp/acls/v2/acl/noifs", {"name": "noifs", "rules": [], "ingress": [],
                                                             "egress": []})])
