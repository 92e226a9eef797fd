"""Pin the CPU oracle to the reference's own known-answer tests (runs on CPU).

* acl_renderer_test.go: 284 Connection* verdicts + ACL counts/changes/placement checks.
* cache_test.go: ordered local/global tables of all 14 scenarios (both orientations).
"""
import pytest

import kat_driver as kd
from oracle import gonet, policy

ACL_SCENARIOS = kd.load("acl_renderer_kats.json")
CACHE_SCENARIOS = kd.load("cache_tables.json")


@pytest.mark.parametrize("sc", ACL_SCENARIOS, ids=[s["name"] for s in ACL_SCENARIOS])
def test_oracle_acl_renderer_kats(sc):
    bad = kd.run_scenario(kd.OracleBackend(), sc)
    assert not bad, bad[:5]


def test_oracle_kat_count():
    n = sum(1 for s in ACL_SCENARIOS for p in s["phases"] for c in p["checks"] if c["kind"].startswith("Connection"))
    assert n == 284


def _rule(d):
    return policy.ContivRule(kd.ACTION[d["action"]], gonet.ip_network(d["src"]), gonet.ip_network(d["dst"]),
                             kd.PROTO[d["proto"]], d["sport"], d["dport"])


def _same(table_rules, expected):
    exp = [_rule(d) for d in expected]
    return policy.compare_rule_lists(table_rules, exp) == 0


@pytest.mark.parametrize("sc", CACHE_SCENARIOS, ids=[s["name"] for s in CACHE_SCENARIOS])
def test_oracle_cache_tables(sc):
    orient = policy.EGRESS_ORIENTATION if sc["orientation"] == "egress" else policy.INGRESS_ORIENTATION
    cache = policy.RendererCache(orient)
    if "resync" in sc:
        tables = []
        for t in sc["resync"]:
            tab = policy.ContivRuleTable(policy.GLOBAL if t["type"] == "global" else policy.LOCAL)
            tab.pods = set(t["pods"])
            for r in t["rules"]:
                tab.insert_rule(_rule(r))
            tables.append(tab)
        assert cache.resync(tables) is None
    for txn_spec in sc["txns"]:
        txn = cache.new_txn()
        for pod, c in txn_spec["updates"].items():
            txn.update(pod, policy.PodConfig(gonet.one_host_subnet(c["ip"]), [_rule(r) for r in c["ingress"]],
                                             [_rule(r) for r in c["egress"]], c["removed"]))
        assert len(txn.get_changes()) == txn_spec["changes"]
        txn.commit()
        assert len(txn.get_changes()) == 0
        exp = txn_spec["expect"]
        for pod, rules in exp["local"].items():
            t = cache.get_local_table_by_pod(pod)
            if rules is None:
                assert t is None, pod
            else:
                assert t is not None and _same(t.rules, rules), (pod, [r.string() for r in t.rules] if t else None)
                assert pod in t.pods and t.type == policy.LOCAL
        assert _same(cache.get_global_table().rules, exp["global"]), [r.string() for r in cache.get_global_table().rules]
        assert cache.get_isolated_pods() == set(exp["isolated"])
    if sc.get("flush_after"):
        cache.flush()
        assert cache.get_global_table().num_rules == 0
        assert not cache.get_isolated_pods()
