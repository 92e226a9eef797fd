"""The installed ACLs and interface bindings of an engine, restated for the C oracle
(TEST INFRASTRUCTURE ONLY; see oracle/__init__.py).

Interface resolution follows MockACLEngine (aclengine_mock.go:273-420): an IP of a local pod
leaves/enters through that pod's TAP; any other IP (remote pod, Internet) through the
node-output interface (VXLAN BVI if set, else the main interface). In connection mode the
pair of end points also picks the reference's call: pod <-> pod is ConnectionPodToPod
(:273-327), local pod <-> non-pod ConnectionPodToInternet / ConnectionInternetToPod; a pod
registered on another node paired with a non-pod address is those calls' "invalid scenario"
and returns ConnActionFailure before any evaluation (:343-347, :388-392). Non-pod <-> non-pod
has no reference call; the engine's convention is the same FAILURE. Both count
once at the "unresolved" slot, like the other preamble failures. The engine is only read
through its public introspection calls (ACL names, ACL dumps, interface bindings, slot
layout) and the pod registrations the test made (RegisterPod), never through its classifier.
"""
import numpy as np

from . import fast
from . import gonet

LOCAL, REMOTE, INET = 0, 1, 2  # end-point kinds


class World:
    def __init__(self, engine, local_ifs, node_if, no_if_ips=(), remote_ips=None):
        """local_ifs: {IPv4 u32: TAP name} of the pods on this node; node_if: name or None;
        no_if_ips: IPv4s of pods on this node whose interface is unknown (unresolvable:
        "Missing interface for ... pod", aclengine_mock.go:302-306 -> FAILURE); remote_ips:
        IPv4s of pods on another node (default: the engine's RegisterPod calls with
        anotherNode set)."""
        self.names = engine.ACLNames()
        self.acls = [fast.OraACL(engine.GetACLByName(n)["rules"]) for n in self.names]
        tix = {n: i for i, n in enumerate(self.names)}
        ifnames = sorted(set(local_ifs.values()) | ({node_if} if node_if else set()))
        self.ifx = {x: i for i, x in enumerate(ifnames)}
        bind = [engine._if_acls(x) for x in ifnames]
        self.if_in = np.array([tix.get(b[0], -1) for b in bind], np.int32)
        self.if_out = np.array([tix.get(b[1], -1) for b in bind], np.int32)
        ips = sorted(set(local_ifs) | set(no_if_ips))
        self.local_ips = np.array(ips, np.uint32)
        self.local_if = np.array([self.ifx[local_ifs[ip]] if ip in local_ifs else -1 for ip in ips], np.int32)
        self.node = self.ifx[node_if] if node_if else -1
        if remote_ips is None:
            remote_ips = []
            for ip, another in getattr(engine, "registered_pods", {}).values():
                v4 = gonet.to4(gonet.parse_ip(ip) or b"")
                if another and v4 is not None:
                    remote_ips.append(gonet.ipv4_u32(v4))
        self.remote_ips = np.array(sorted(set(int(x) for x in remote_ips) - set(ips)), np.uint32)
        # slot layout of the engine (pg_table_info / pg_num_counter_slots)
        self.tids = [engine.table_id(n) for n in self.names]  # engine table id of each oracle table
        info = [engine.table_info(t) for t in self.tids]
        self.base = np.array([b for b, _, _ in info] + [0], np.int64)
        self.dflt = np.array([d for _, _, d in info] + [0], np.int64)
        ns = engine.num_counter_slots()
        self.slot_noacl, self.slot_unresolved = ns - 2, ns - 1

    def resolve(self, ips):
        ips = np.ascontiguousarray(ips, np.uint32)
        if len(self.local_ips) == 0:
            return np.full(len(ips), self.node, np.int32)
        k = np.minimum(np.searchsorted(self.local_ips, ips), len(self.local_ips) - 1)
        return np.where(self.local_ips[k] == ips, self.local_if[k], self.node).astype(np.int32)

    def kind(self, ips):
        """end-point kind of each address: LOCAL (a pod of this node), REMOTE, INET."""
        ips = np.ascontiguousarray(ips, np.uint32)
        out = np.full(len(ips), INET, np.int32)
        for arr, kd in ((self.remote_ips, REMOTE), (self.local_ips, LOCAL)):
            if len(arr):
                k = np.minimum(np.searchsorted(arr, ips), len(arr) - 1)
                out[arr[k] == ips] = kd
        return out

    def conn_ifs(self, src, dst):
        """(src interface, dst interface) of each connection for testConnection, -1 where the
        reference makes no evaluation: no Connection* call exists for remote pod <-> non-pod
        (aclengine_mock.go:343-347, 388-392) nor for non-pod <-> non-pod -- FAILURE before any
        evaluation, counted like an unresolved interface."""
        sif = self.resolve(src)
        sif[self.kind(src) + self.kind(dst) >= 3] = -1
        return sif, self.resolve(dst)

    def slots(self, table, idx):
        """(oracle table, matched index) -> engine counter slot."""
        table = np.asarray(table, np.int64)
        idx = np.asarray(idx, np.int64)
        t = np.where(table >= 0, table, len(self.names))
        s = np.where(idx >= 0, self.base[t] + idx, self.dflt[t])
        s = np.where(table == -1, self.slot_noacl, s)
        s = np.where(table == -2, self.slot_unresolved, s)
        return s.astype(np.uint32)

    def perpod(self, src, dst, dport, proto, threads=1):
        """-> (ACLAction, slot) of evalACL(outbound ACL of dst's interface)."""
        act, lt, li = fast.perpod(self.acls, self.if_out, self.resolve(dst), src, dst, dport, proto, threads)
        return act, self.slots(lt, li)

    def single(self, table_id, src, dst, dport, proto, threads=1):
        """-> (ACLAction, slot) of evalACL over the engine's table `table_id`."""
        t = self.tids.index(table_id)
        act, idx = fast.eval_acl(self.acls[t], src, dst, dport, proto, threads=threads)
        return act, self.slots(np.full(len(idx), t, np.int64), idx)

    def conn(self, src, dst, sport, dport, proto, threads=1, hist=False):
        """-> (ConnAction, slot of the deciding evaluation) of testConnection; hist=True also
        the per-rule hit-counter histogram of the batch: one count per evalACL every
        connection makes (up to four, aclengine_mock.go:448-491), at the slot of the rule that
        decided that evaluation (its table's default slot when none matched, "no ACL" for a
        nil ACL), and one "unresolved" count per connection with an unknown interface."""
        sif, dif = self.conn_ifs(src, dst)
        r = fast.test_connection(self.acls, self.if_in, self.if_out, sif, dif,
                                 src, dst, sport, dport, proto, threads, trace=hist)
        if not hist:
            c, lt, li = r
            return c, self.slots(lt, li)
        c, lt, li, evt, evi = r
        made = evt.ravel() != -3
        ev_slots = self.slots(evt.ravel()[made], evi.ravel()[made])
        h = np.bincount(ev_slots, minlength=self.slot_unresolved + 1).astype(np.int64)
        return c, self.slots(lt, li), h


def expected(engine, mode, table_id, local_ifs, node_if, src, dst, sport, dport, proto, threads=1):
    """The oracle's answer for a batch in any mode (0 SINGLE: evalACL over table_id; 1 PERPOD:
    evalACL over the outbound ACL of dst's interface; 2 CONN: testConnection) -> (action,
    deciding slot, per-rule hit-counter histogram). SINGLE and PERPOD make one evaluation per
    tuple, so their histogram is that of the slots; CONN counts every evaluation it makes."""
    wd = World(engine, local_ifs, node_if)
    if mode == 0:
        act, slot = wd.single(table_id, src, dst, dport, proto, threads)
    elif mode == 1:
        act, slot = wd.perpod(src, dst, dport, proto, threads)
    else:
        return wd.conn(src, dst, sport, dport, proto, threads, hist=True)
    return act, slot, np.bincount(slot, minlength=wd.slot_unresolved + 1).astype(np.int64)
