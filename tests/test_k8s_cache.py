"""K8s policy cache and policy processor.

* The reference's cache tests (cache_test.go, match_label_test.go, match_expression_test.go,
  podidx / namespaceidx / policyidx tests: 189 assertions, transcribed as data by
  tests/golden/make_k8s_cache_golden.py) replayed against the product (C++ cache behind the C
  ABI, objects passed in protobuf wire form) and against the oracle restatement.
* Random K8s states: every selector query of the product equals the oracle's.
* Random states + event sequences through the processor: the ContivRule lists the product
  configures (mock renderer) equal those of the oracle chain (oracle processor -> oracle
  configurator -> oracle mock renderer) after every event. The processor itself has no
  reference tests: parity unpinned beyond the cache and configurator KATs it builds on.
"""
import json
import os
import random

import pytest

from oracle import configurator as OC
from oracle import k8s_policy as OK
from vpp_amd import configurator as CF
from vpp_amd import k8s as K

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "k8s_cache_kats.json")))["scenarios"]
KIND = {"pod": 0, "namespace": 1, "policy": 2}
STORE_KIND = {"podmodel": 0, "namespace": 1, "policymodel": 2}


class Product:
    def __init__(self):
        self.c = K.PolicyCache()

    def register(self, kind, id_, obj):
        self.c.Register(kind, id_, obj)

    def unregister(self, kind, id_):
        self.c.Unregister(kind, id_)

    def update(self, kind, prev, new):
        assert self.c.Update(kind, prev, new) is None

    def resync(self, store):
        by = {0: [], 1: [], 2: []}
        for key, obj in store.items():
            by[STORE_KIND[key.split(":")[0]]].append(obj)
        assert self.c.Resync(by[0], by[1], by[2]) is None

    def lookup(self, kind, id_):
        found, raw = {0: self.c.LookupPod, 1: self.c.LookupNamespace, 2: self.c.LookupPolicy}[kind](id_)
        return found, raw

    def same_object(self, got, expected, kind):
        return got == K.ENCODE[kind](expected)

    def call(self, method, args, index_kind):
        c = self.c
        idx = {"LookupPodsByNSKey": K.Q_IDX_POD_NS_KEY, "LookupPodsByNSLabelSelector": K.Q_IDX_POD_NS_LABEL,
               "LookupPodsByLabelSelector": K.Q_IDX_POD_LABEL, "LookupPodsByLabelKey": K.Q_IDX_POD_KEY,
               "LookupNamespacesByLabelSelector": K.Q_IDX_NS_LABEL, "LookupNamespacesByKey": K.Q_IDX_NS_KEY,
               "LookupPolicyByNSLabelSelector": K.Q_IDX_POLICY_NS_LABEL,
               "LookupPolicyByLabelSelector": K.Q_IDX_POLICY_LABEL}
        if index_kind is not None:  # a single ConfigIndex
            if method == "ListAll":
                return c.query({0: K.Q_ALL_PODS, 1: K.Q_ALL_NAMESPACES, 2: K.Q_ALL_POLICIES}[index_kind])
            if method == "LookupPodsByNamespace":
                return c.LookupPodsByNamespace(args[0])
            if method in idx:
                return c.query(idx[method], args[0])
        return getattr(c, method)(*args)


class Oracle:
    def __init__(self):
        self.c = OK.PolicyCache()

    def _t(self, kind):
        return (self.c.pods, self.c.namespaces, self.c.policies)[kind]

    def register(self, kind, id_, obj):
        self._t(kind)[id_] = obj

    def unregister(self, kind, id_):
        self._t(kind).pop(id_, None)

    def update(self, kind, prev, new):
        self.c.update(kind, prev, new)

    def resync(self, store):
        by = {0: [], 1: [], 2: []}
        for key, obj in store.items():
            by[STORE_KIND[key.split(":")[0]]].append(obj)
        self.c.resync(by[0], by[1], by[2])

    def lookup(self, kind, id_):
        return self.c.lookup(kind, id_)

    def same_object(self, got, expected, kind):
        return got == expected

    def call(self, method, args, index_kind):
        c = self.c
        if index_kind is not None:
            field = {"LookupPodsByNSKey": ("pod", "nskey"), "LookupPodsByNSLabelSelector": ("pod", "nslabel"),
                     "LookupPodsByLabelSelector": ("pod", "label"), "LookupPodsByLabelKey": ("pod", "key"),
                     "LookupPodsByNamespace": ("pod", "ns"), "LookupNamespacesByLabelSelector": ("ns", "label"),
                     "LookupNamespacesByKey": ("ns", "key"), "LookupPolicyByNSLabelSelector": ("policy", "nslabel"),
                     "LookupPolicyByLabelSelector": ("policy", "label")}
            if method == "ListAll":
                return sorted(self._t(index_kind))
            if method in field:
                t, f = field[method]
                return {"pod": c.pods_by, "ns": c.ns_by, "policy": c.policies_by}[t](f, args[0])
        m = {"LookupPodsByLabelSelectorInsideNs": c.pods_by_label_selector_inside_ns,
             "LookupPodsByNsLabelSelector": c.pods_by_ns_label_selector,
             "LookupPodsByNamespace": c.pods_in_ns, "ListAllPods": c.all_pods,
             "LookupPoliciesByPod": c.policies_by_pod, "ListAllNamespaces": lambda: sorted(c.namespaces),
             "ListAllPolicies": lambda: sorted(c.policies),
             "getMatchLabelPodsInsideNs": c.match_label_pods_inside_ns, "getPodsByNsLabelSelector": c.pods_by_ns_labels,
             "getMatchExpressionPodsInsideNs": c.match_expression_pods_inside_ns,
             "getPodsByNsMatchExpression": c.pods_by_ns_expressions}
        return m[method](*args)


LOOKUPS = {"LookupPod": 0, "LookupNamespace": 1, "LookupPolicy": 2}


def replay(backend, sc):
    ops = list(sc["ops"])
    n_checked = 0

    def run_ops(upto):
        while ops and ops[0][4] <= upto:
            op, kind, a, b, _ = ops.pop(0)
            if op == "register":
                backend.register(KIND[kind], a, b)
            elif op == "unregister":
                backend.unregister(KIND[kind], a)
            elif op == "update":
                backend.update(KIND[kind], a, b)
            else:
                backend.resync(b)

    for ci, chk in enumerate(sc["checks"]):
        run_ops(ci)
        method, args = chk["method"], chk["args"]
        ik = KIND.get(sc["index_kind"])
        if method in LOOKUPS:
            kind = LOOKUPS[method] if ik is None else ik
            found, data = backend.lookup(kind, args[0])
            vals = dict(zip(chk["vars"], (found, data)))
        else:
            kind = None
            vals = {chk["vars"][0]: backend.call(method, args, ik)}
        for a in chk["asserts"]:
            v, what, exp = vals[a["var"]], a["kind"], a["value"]
            where = "%s line %d" % (sc["source"], chk["line"])
            if what == "contains":
                assert exp in v, where
            elif what == "empty":
                assert len(v) == 0, where
            elif what == "nil":
                assert v is None or (isinstance(v, list) and not v), where
            elif what in ("true", "false"):
                assert v is (what == "true"), where
            elif isinstance(exp, list):
                assert sorted(v) == sorted(exp), where
            else:
                assert backend.same_object(v, exp, kind), where
            n_checked += 1
    run_ops(len(sc["checks"]) + 1)
    return n_checked


@pytest.mark.parametrize("sc", FIX, ids=[s["name"] for s in FIX])
def test_cache_kats_product(sc):
    replay(Product(), sc)


@pytest.mark.parametrize("sc", FIX, ids=[s["name"] for s in FIX])
def test_cache_kats_oracle(sc):
    replay(Oracle(), sc)


def test_kat_count():
    assert sum(len(c["asserts"]) for s in FIX for c in s["checks"]) == 189
    assert sum(replay(Oracle(), s) for s in FIX) == 189


def test_protobuf_roundtrip_and_nil():
    c = K.PolicyCache()
    pod = {"Name": "p", "Namespace": "n", "Label": [{"Key": "a", "Value": ""}], "IpAddress": "10.0.0.1",
           "Container": [{"Name": "c", "Port": [{"Name": "http", "ContainerPort": 8080, "Protocol": 1}]}]}
    c.Register(K.POD, "n/p", pod)
    assert c.LookupPod("n/p") == (True, K.encode_pod(pod))
    assert c.query(K.Q_IDX_POD_NS_LABEL, "n/a/") == ["n/p"]
    c.Register(K.POLICY, "n/x", None)  # a nil object indexes nothing but is found
    assert c.LookupPolicy("n/x") == (True, None)
    assert c.ListAllPolicies() == ["n/x"]
    assert c.Unregister(K.POLICY, "n/x") and not c.Unregister(K.POLICY, "n/x")
    # truncated field: rejected, and nothing is registered under the ID
    assert K.lib.pg_policy_cache_register(c.h, K.POD, b"bad", b"\x0a\x05ab", 4) == K._capi.PG_EINVAL
    assert not c.LookupPod("bad")[0]


# ---- random K8s states ------------------------------------------------------------------------
KEYS = ["app", "role", "tier", "env"]
VALS = ["a", "b", "c", "db", "web"]


def rand_labels(rnd, n=3):
    return [{"Key": rnd.choice(KEYS), "Value": rnd.choice(VALS)} for _ in range(rnd.randint(0, n))]


def rand_selector(rnd):
    sel = {}
    if rnd.random() < 0.6:
        sel["MatchLabel"] = rand_labels(rnd, 2)
    if rnd.random() < 0.5:
        sel["MatchExpression"] = [{"Key": rnd.choice(KEYS + ["zz"]), "Operator": rnd.randint(0, 3),
                                   "Value": rnd.sample(VALS + [""], rnd.randint(0, 3))}
                                  for _ in range(rnd.randint(1, 3))]
    return sel


def rand_state(rnd, n_ns=4, n_pods=14, n_pol=6):
    nss = ["ns%d" % i for i in range(n_ns)] + ["kube-system"]
    namespaces = [{"Name": n, "Label": rand_labels(rnd)} for n in nss if rnd.random() < 0.85]
    pods = []
    for i in range(n_pods):
        ns = rnd.choice(nss)
        ip = "10.1.%d.%d" % (rnd.choice([1, 1, 1, 2]), i + 2) if rnd.random() < 0.85 else ""
        cont = [{"Name": "c", "Port": [{"Name": rnd.choice(["http", "dns", "db"]), "ContainerPort": rnd.choice(
            [80, 53, 5432, 8080]), "Protocol": rnd.choice([0, 1])} for _ in range(rnd.randint(0, 2))]}]
        pods.append({"Name": "pod%d" % i, "Namespace": ns, "Label": rand_labels(rnd), "IpAddress": ip,
                     "Container": cont})
    policies = [rand_policy(rnd, nss, k) for k in range(n_pol)]
    return pods, namespaces, policies


def rand_peer(rnd):
    peer = {}
    x = rnd.random()
    if x < 0.4:
        peer["Pods"] = rand_selector(rnd)
    elif x < 0.7:
        peer["Namespaces"] = rand_selector(rnd)
    elif x < 0.8:
        peer["Pods"], peer["Namespaces"] = rand_selector(rnd), rand_selector(rnd)
    if rnd.random() < 0.3:
        peer["IpBlock"] = {"Cidr": rnd.choice(["10.0.0.0/8", "10.1.0.0/16", "192.168.0.0/16"]),
                           "Except": rnd.sample(["10.1.1.0/24", "10.1.2.128/25", "192.168.5.5/32"], rnd.randint(0, 2))}
    return peer


def rand_rule(rnd, key):
    ports = []
    for _ in range(rnd.choice([0, 0, 1, 2])):
        if rnd.random() < 0.3:
            pn = {"Type": 1, "Name": rnd.choice(["http", "dns", "nope"])}
        else:
            pn = {"Type": 0, "Number": rnd.choice([53, 80, 443, 8080])}
        ports.append({"Protocol": rnd.choice([0, 1]), "Port": pn})
    return {"Port": ports, key: [rand_peer(rnd) for _ in range(rnd.choice([0, 1, 1, 2]))]}


def rand_policy(rnd, nss, k, name=None):
    return {"Name": name or "pol%d" % k, "Namespace": rnd.choice(nss), "Pods": rand_selector(rnd),
            "PolicyType": rnd.randint(0, 3),
            "IngressRule": [rand_rule(rnd, "From") for _ in range(rnd.choice([0, 1, 1, 2]))],
            "EgressRule": [rand_rule(rnd, "To") for _ in range(rnd.choice([0, 0, 1, 2]))]}


@pytest.mark.parametrize("seed", range(20))
def test_random_queries_product_equals_oracle(seed):
    rnd = random.Random(seed)
    pods, nss, pols = rand_state(rnd)
    p, o = K.PolicyCache(), OK.PolicyCache()
    assert p.Resync(pods, nss, pols) is None
    o.resync(pods, nss, pols)
    for ns in ["ns0", "ns1", "ns2", "kube-system", "nope"]:
        for _ in range(8):
            sel = rand_selector(rnd)
            assert p.LookupPodsByLabelSelectorInsideNs(ns, sel) == o.pods_by_label_selector_inside_ns(ns, sel)
    for _ in range(30):
        sel = rand_selector(rnd)
        assert p.LookupPodsByNsLabelSelector(sel) == sorted(o.pods_by_ns_label_selector(sel))
    for pod in o.all_pods():
        assert p.LookupPoliciesByPod(pod) == o.policies_by_pod(pod)
    assert p.ListAllPods() == o.all_pods()


def rules_of(mock, pod, d):
    from test_configurator import rule_str
    return [rule_str(r) for r in mock.Rules(pod, d)]


def compare_chain(pm, om, pods):
    for pod in pods:
        if pod in om.config:
            for d in (0, 1):
                assert rules_of(pm, pod, d) == [
                    __import__("test_configurator").rule_str(r) for r in om.config[pod][1 + d]], (pod, d)
        else:
            assert pm.Rules(pod, 0) is None, pod


def make_chain(subnet="10.1.1.0/24"):
    cache, cfg, mock = K.PolicyCache(), CF.PolicyConfigurator(), CF.MockRenderer()
    cfg.SetNatLoopbackIP("10.1.1.254")
    assert cfg.RegisterRenderer(mock) is None
    proc = K.PolicyProcessor(cache, cfg, subnet)
    ocache = OK.PolicyCache()
    ocfg = OC.PolicyConfigurator({}, "10.1.1.254")
    omock = OC.MockRenderer()
    ocfg.renderers.append(omock)
    oproc = OK.PolicyProcessor(ocache, ocfg, subnet)
    return (cache, cfg, mock, proc), (ocache, ocfg, omock, oproc)


@pytest.mark.parametrize("seed", range(25))
def test_processor_resync_and_events(seed):
    rnd = random.Random(1000 + seed)
    pods, nss, pols = rand_state(rnd)
    (cache, cfg, mock, proc), (ocache, ocfg, omock, oproc) = make_chain()
    assert cache.Resync(pods, nss, pols) is None
    ocache.resync(pods, nss, pols)
    names = lambda: sorted(set(ocache.all_pods()) | {"%s/%s" % (p["Namespace"], p["Name"]) for p in pods})  # noqa
    compare_chain(mock, omock, names())
    live_pods = {("%s/%s" % (p["Namespace"], p["Name"])): p for p in pods}
    live_pols = {("%s/%s" % (p["Namespace"], p["Name"])): p for p in pols}
    live_ns = {n["Name"]: n for n in nss}
    for step in range(25):
        x = rnd.random()
        if x < 0.3:  # pod add / update / delete
            key = rnd.choice(sorted(live_pods)) if live_pods and rnd.random() < 0.7 else None
            if key is None:
                i = 100 + step
                new = {"Name": "pod%d" % i, "Namespace": rnd.choice(["ns0", "ns1"]), "Label": rand_labels(rnd),
                       "IpAddress": "10.1.1.%d" % (100 + step), "Container": []}
                ev = (K.POD, None, new)
            elif rnd.random() < 0.4:
                ev = (K.POD, live_pods[key], None)
            else:
                old = live_pods[key]
                new = dict(old, Label=rand_labels(rnd), IpAddress=rnd.choice([old["IpAddress"], "", "10.1.1.77",
                                                                              "10.1.2.9"]))
                ev = (K.POD, old, new)
        elif x < 0.7:  # policy
            key = rnd.choice(sorted(live_pols)) if live_pols and rnd.random() < 0.7 else None
            if key is None:
                ev = (K.POLICY, None, rand_policy(rnd, ["ns0", "ns1", "ns2"], 0, name="new%d" % step))
            elif rnd.random() < 0.3:
                ev = (K.POLICY, live_pols[key], None)
            else:
                old = live_pols[key]
                new = rand_policy(rnd, [old["Namespace"]], 0, name=old["Name"])
                ev = (K.POLICY, old, new)
        else:  # namespace update (labels)
            if not live_ns:
                continue
            old = live_ns[rnd.choice(sorted(live_ns))]
            ev = (K.NAMESPACE, old, dict(old, Label=rand_labels(rnd)))
        kind, old, new = ev
        assert cache.Update(kind, old, new) is None
        ocache.update(kind, old, new)
        live = {K.POD: live_pods, K.POLICY: live_pols, K.NAMESPACE: live_ns}[kind]
        idf = (lambda o: o["Name"]) if kind == K.NAMESPACE else (lambda o: "%s/%s" % (o["Namespace"], o["Name"]))
        if old is not None:
            live.pop(idf(old), None)
        if new is not None:
            live[idf(new)] = new
        compare_chain(mock, omock, sorted(set(names()) | set(live_pods)))


def test_processor_host_filter_and_named_ports():
    pods = [{"Name": "web", "Namespace": "default", "Label": [{"Key": "app", "Value": "web"}], "IpAddress": "10.1.1.2",
             "Container": [{"Name": "c", "Port": [{"Name": "http", "ContainerPort": 8080}]}]},
            {"Name": "db", "Namespace": "default", "Label": [{"Key": "app", "Value": "db"}], "IpAddress": "10.1.1.3",
             "Container": [{"Name": "c", "Port": [{"Name": "pg", "ContainerPort": 5432}]}]},
            {"Name": "remote", "Namespace": "default", "Label": [{"Key": "app", "Value": "web"}],
             "IpAddress": "10.1.2.4"}]
    pol = {"Name": "db-allow", "Namespace": "default", "Pods": {"MatchLabel": [{"Key": "app", "Value": "db"}]},
           "PolicyType": 3,
           "IngressRule": [{"Port": [{"Protocol": 0, "Port": {"Type": 1, "Name": "pg"}}],
                            "From": [{"Pods": {"MatchLabel": [{"Key": "app", "Value": "web"}]}}]}],
           "EgressRule": [{"Port": [{"Protocol": 0, "Port": {"Type": 1, "Name": "http"}}], "To": []}]}
    (cache, cfg, mock, proc), (ocache, ocfg, omock, oproc) = make_chain()
    assert cache.Resync(pods, [{"Name": "default"}], [pol]) is None
    ocache.resync(pods, [{"Name": "default"}], [pol])
    assert mock.Rules("default/remote", 0) is None  # not on this node
    ing = mock.Rules("default/db", 0)  # traffic from the pod: egress match
    egr = mock.Rules("default/db", 1)
    assert egr[0].DestPort == 5432 and egr[0].Protocol == 0  # named ingress port of the target pod
    assert any(r.DestPort == 8080 for r in ing)              # named egress port of the peer pod
    compare_chain(mock, omock, ["default/web", "default/db", "default/remote"])
    assert mock.TestTraffic("default/db", CF.EgressTraffic, "10.1.1.2", "10.1.1.3", 0, 999, 5432) == CF.AllowedTraffic
    assert mock.TestTraffic("default/db", CF.EgressTraffic, "10.1.1.2", "10.1.1.3", 0, 999, 80) == CF.DeniedTraffic
