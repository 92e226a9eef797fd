"""Replays the reference's renderer/engine known-answer tests against a backend.

The scenarios and expected answers live in tests/golden/acl_renderer_kats.json (made by
tests/golden/make_golden.py from /root/reference/plugins/policy/renderer/acl/
acl_renderer_test.go). A backend is either the CPU oracle (``OracleBackend`` here) or the
product's C-ABI renderer+device engine (tests/test_gpu_kats.py); both are driven by the
same ``run_scenario`` so the parity tests read like the reference's own tests.
"""
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CONN = {"ConnActionDenySyn": 0, "ConnActionDenySynAck": 1, "ConnActionAllow": 2, "ConnActionFailure": 3}
PROTO = {"TCP": 0, "UDP": 1, "OTHER": 2, "ANY": 3}
ACTION = {"DENY": 0, "PERMIT": 1}


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def node_output_ifs_test_order(setup):
    """acl_renderer_test.go:120-131 nodeOutputInterfaces (test helper order)."""
    ifs = []
    if setup["main_if"]:
        ifs.append(setup["main_if"])
    ifs += setup["other_ifs"]
    ifs.append(setup["vxlan_bvi"])
    ifs.append(setup["host_interconnect"])
    return ifs


def run_scenario(backend, sc, on_check=None):
    """Run one acl_renderer_test scenario; returns list of (check, got) mismatches."""
    setup = sc["setup"]
    backend.setup(setup)
    bad = []
    for phase in sc["phases"]:
        for st in phase["steps"]:
            if st["op"] == "restart":
                backend.restart()
            else:
                err = backend.txn(st["resync"], st["renders"])
                assert err is None, "commit error: %s" % err
        conn_checks = [c for c in phase["checks"] if c["kind"].startswith("Connection")]
        got_conn = backend.connections(conn_checks) if conn_checks else []
        gi = 0
        for c in phase["checks"]:
            k = c["kind"]
            if k.startswith("Connection"):
                got = got_conn[gi]
                gi += 1
                ok = got == CONN[c["expect"]]
            elif k == "NumACLs":
                got = backend.num_acls()
                ok = got == c["expect"]
            elif k == "NumACLChanges":
                got = backend.num_acl_changes()
                ok = got == c["expect"]
            elif k == "CommittedTxns":
                got = backend.committed_txns()
                ok = got == c["expect"]
            elif k == "PendingTxns":
                got, ok = 0, c["expect"] == 0
            elif k == "ReflectiveACL":
                got = backend.inbound_acl(c["if"])
                ok = check_reflective(got, setup, c)
            elif k == "GlobalACL":
                got = backend.acl_by_name("contiv-policy-NODE-GLOBAL")
                ok = check_global(got, setup, c)
            else:
                raise AssertionError(k)
            if on_check:
                on_check(c, got, ok)
            if not ok:
                bad.append((c, got))
    return bad


def check_reflective(acl, setup, c):
    """acl_renderer_test.go:133-166 verifyReflectiveACL. ``acl`` is a dict or None."""
    if not c["expect"]:
        return acl is None
    if acl is None or acl["name"] != "contiv-policy-REFLECTION" or len(acl["rules"]) != 1:
        return False
    ifs = (node_output_ifs_test_order(setup) if c["on_output_ifs"] else []) + [c["if"]]
    if any(i not in acl["ingress"] for i in ifs) or len(acl["egress"]) != 0:
        return False
    r = acl["rules"][0]
    return (r["action"] == 2 and r["src"] == "" and r["dst"] == "" and not r["tcp"] and not r["udp"]
            and not r.get("icmp") and not r.get("macip") and r.get("ip_rule", True) and r.get("ip", True))


def check_global(acl, setup, c):
    """acl_renderer_test.go:168-184 verifyGlobalTable."""
    if not c["expect"]:
        return acl is None
    ifs = node_output_ifs_test_order(setup)
    return (acl is not None and len(acl["rules"]) > 0 and len(acl["ingress"]) == 0
            and all(i in acl["egress"] for i in ifs) and len(acl["egress"]) == len(ifs))


# --- CPU oracle backend -------------------------------------------------------
class OracleBackend:
    def __init__(self):
        from oracle import policy, aclengine, gonet
        self.policy, self.aclengine, self.gonet = policy, aclengine, gonet

    def rule(self, d):
        pol, g = self.policy, self.gonet
        return pol.ContivRule(ACTION[d["action"]], g.ip_network(d["src"]), g.ip_network(d["dst"]),
                              PROTO[d["proto"]], d["sport"], d["dport"])

    def setup(self, s):
        pol = self.policy
        self.ifaces = pol.NodeIfaces(pod_if=dict(s["pod_ifs"]), host_interconnect=s["host_interconnect"],
                                     main_if=s["main_if"], other_ifs=list(s["other_ifs"]),
                                     vxlan_bvi=s["vxlan_bvi"])
        self.engine = self.aclengine.MockACLEngine(self.ifaces)
        for pod, ip, another in s["pods"]:
            self.engine.register_pod(pod, ip, another)
        self.restart()

    def restart(self):
        self.base_txns = self.engine.committed_txns
        self.renderer = self.policy.AclRenderer(self.ifaces, self.engine.apply_txn)

    def txn(self, resync, renders):
        t = self.renderer.new_txn(resync)
        for r in renders:
            ip = self.gonet.one_host_subnet(r["ip"])
            t.render(r["pod"], ip, [self.rule(x) for x in r["ingress"]], [self.rule(x) for x in r["egress"]],
                     r["removed"])
        return t.commit()

    def connections(self, checks):
        e = self.engine
        out = []
        for c in checks:
            a = c["args"]
            proto = PROTO[a[2]]
            if c["kind"] == "ConnectionPodToPod":
                out.append(e.connection_pod_to_pod(a[0], a[1], proto, a[3], a[4]))
            elif c["kind"] == "ConnectionPodToInternet":
                out.append(e.connection_pod_to_internet(a[0], a[1], proto, a[3], a[4]))
            else:
                out.append(e.connection_internet_to_pod(a[0], a[1], proto, a[3], a[4]))
        return out

    def num_acls(self):
        return self.engine.num_acls()

    def num_acl_changes(self):
        return self.engine.num_acl_changes()

    def committed_txns(self):
        return self.engine.committed_txns - self.base_txns

    @staticmethod
    def acl_dict(acl):
        if acl is None:
            return None
        return {"name": acl.name, "ingress": list(acl.ingress), "egress": list(acl.egress),
                "rules": [{"action": r.action, "src": r.src_network, "dst": r.dst_network,
                           "tcp": r.tcp is not None, "udp": r.udp is not None} for r in acl.rules]}

    def inbound_acl(self, ifn):
        return self.acl_dict(self.engine.inbound_acl(ifn))

    def acl_by_name(self, name):
        return self.acl_dict(self.engine.acl_by_name(name))


# --- product backend (C ABI) ----------------------------------------------------
class ProductBackend:
    """Drives vpp_amd (C++ renderer + device engine). With ``gpu=False`` the Connection*
    verdicts are not evaluated (they need the device); everything else runs on the host."""

    def __init__(self, gpu=True):
        import vpp_amd.renderer as R
        self.R = R
        self.gpu = gpu

    def rule(self, d):
        R = self.R
        return R.ContivRule(ACTION[d["action"]], R.IPNet(d["src"]), R.IPNet(d["dst"]), PROTO[d["proto"]],
                            d["sport"], d["dport"])

    def setup(self, s):
        R = self.R
        self.engine = R.Engine(0)
        e = self.engine
        e.SetMainInterfaceName(s["main_if"])
        e.SetVxlanBVIIfName(s["vxlan_bvi"])
        e.SetHostInterconnectIfName(s["host_interconnect"])
        e.SetOtherVPPInterfaces(s["other_ifs"])
        for pod, ifn in s["pod_ifs"].items():
            e.SetPodIfName(pod, ifn)
        for pod, ip, another in s["pods"]:
            e.RegisterPod(pod, ip, another)
        self.restart()

    def restart(self):
        self.base_txns = self.engine.NumCommittedTxns()
        self.renderer = self.R.Renderer(self.engine)

    def txn(self, resync, renders):
        t = self.renderer.NewTxn(resync)
        for r in renders:
            t.Render(r["pod"], self.R.IPNet.host(r["ip"]), [self.rule(x) for x in r["ingress"]],
                     [self.rule(x) for x in r["egress"]], r["removed"])
        return t.Commit()

    def connections(self, checks):
        if not self.gpu:
            return [None] * len(checks)
        qs = []
        for c in checks:
            a = c["args"]
            kind = c["kind"].replace("Connection", "")
            qs.append((kind, a[0], a[1], PROTO[a[2]], a[3], a[4]))
        return self.engine.connections(qs)[0]

    def num_acls(self):
        return self.engine.GetNumOfACLs()

    def num_acl_changes(self):
        return self.engine.GetNumOfACLChanges()

    def committed_txns(self):
        return self.engine.NumCommittedTxns() - self.base_txns

    @staticmethod
    def acl_dict(acl):
        if acl is None:
            return None
        return {"name": acl["name"], "ingress": acl["ingress"], "egress": acl["egress"],
                "rules": [{"action": r["action"], "src": r["src"], "dst": r["dst"], "tcp": r["tcp"] is not None,
                           "udp": r["udp"] is not None, "icmp": r["icmp"], "macip": r["macip"],
                           "ip_rule": r["ip_rule"], "ip": r["ip"]} for r in acl["rules"]]}

    def inbound_acl(self, ifn):
        return self.acl_dict(self.engine.GetInboundACL(ifn))

    def acl_by_name(self, name):
        return self.acl_dict(self.engine.GetACLByName(name))
