"""K8s policy cache and policy processor (TEST INFRASTRUCTURE ONLY; see oracle/__init__.py).

CPU restatement of:
  * plugins/policy/cache/cache_impl.go:33-234         PolicyCache lookups
  * plugins/policy/cache/match_label.go:23-74          label selectors
  * plugins/policy/cache/match_expression.go:23-271    expression selectors
  * plugins/policy/cache/data_change.go, data_resync.go  Update / Resync events
  * plugins/policy/cache/{podidx,namespaceidx,policyidx}/*.go  secondary indexes
  * plugins/policy/utils/utils.go:33-160               set helpers (Difference is the
                                                       count==1 rule, i.e. a symmetric difference)
  * plugins/policy/processor/processor.go:73-527       Process + event handlers, filterHostPods
  * plugins/policy/processor/matches_calculator.go     calculateMatches, portNameToNumber
  * plugins/policy/processor/match_label_selector.go   the event-time selector matching, with its
                                                       key-building quirks kept
Pinned by the 189 assertions of the reference's cache tests (tests/golden/k8s_cache_kats.json);
the processor has no reference tests ("parity unpinned" beyond the cache it builds on: it is
checked against the product on random K8s states and event sequences).

Objects are dicts with the Go field names (see vpp_amd/k8s.py). Go map iteration order is
replaced by sorted order; a policy's named ingress port is resolved against the first pod
(sorted) that selects it, as in the product.
"""
from __future__ import annotations

from . import gonet

POD, NAMESPACE, POLICY = 0, 1, 2
IN, NOT_IN, EXISTS, DOES_NOT_EXIST = 0, 1, 2, 3


def _labels(o):
    return (o or {}).get("Label") or []


def intersect(a, b):
    if not a or not b:
        return []
    sa = set(a)
    return sorted(x for x in b if x in sa)


def difference(a, b):
    m = {x: 1 for x in a}
    for x in b:
        m[x] = m.get(x, 0) + 1
    return sorted(k for k, v in m.items() if v == 1)


def unstring(pid):
    parts = pid.split("/")
    return (parts[0], parts[1]) if len(parts) >= 2 else None


class PolicyCache:
    def __init__(self):
        self.reset()
        self.watchers = []

    def reset(self):
        self.pods, self.namespaces, self.policies = {}, {}, {}

    # ---- index functions (podmap.go, namespacemap.go, policymap.go) ----
    @staticmethod
    def pod_index(p):
        if p is None:
            return {}
        ns = p.get("Namespace", "")
        ls = _labels(p)
        return {"label": {l.get("Key", "") + "/" + l.get("Value", "") for l in ls},
                "key": {l.get("Key", "") for l in ls},
                "ns": {ns},
                "nslabel": {ns + "/" + l.get("Key", "") + "/" + l.get("Value", "") for l in ls},
                "nskey": {ns + "/" + l.get("Key", "") for l in ls}}

    @staticmethod
    def ns_index(n):
        if n is None:
            return {}
        ls = _labels(n)
        return {"label": {l.get("Key", "") + "/" + l.get("Value", "") for l in ls},
                "key": {l.get("Key", "") for l in ls}}

    @staticmethod
    def policy_index(p):
        if p is None:
            return {}
        ml = (p.get("Pods") or {}).get("MatchLabel") or []
        return {"label": {l.get("Key", "") + "/" + l.get("Value", "") for l in ml},
                "nslabel": {p.get("Namespace", "") + "/" + l.get("Key", "") + "/" + l.get("Value", "") for l in ml}}

    def _list(self, table, index, field, value):
        return sorted(name for name, obj in table.items() if value in index(obj).get(field, ()))

    def pods_by(self, field, value):
        return self._list(self.pods, self.pod_index, field, value)

    def ns_by(self, field, value):
        return self._list(self.namespaces, self.ns_index, field, value)

    def policies_by(self, field, value):
        return self._list(self.policies, self.policy_index, field, value)

    # ---- PolicyCacheAPI ----
    def lookup(self, kind, id_):
        t = (self.pods, self.namespaces, self.policies)[kind]
        return (True, t[id_]) if id_ in t else (False, None)

    def pods_in_ns(self, ns):
        return self.pods_by("ns", ns)

    def all_pods(self):
        return sorted(self.pods)

    def match_label_pods_inside_ns(self, ns, labels):
        if not labels:
            return []
        cur = self.pods_by("nslabel", ns + "/" + labels[0]["Key"] + "/" + labels[0]["Value"])
        for l in labels[1:]:
            cur = intersect(cur, self.pods_by("nslabel", ns + "/" + l["Key"] + "/" + l["Value"]))
            if not cur:
                break
        return cur

    def pods_by_ns_labels(self, labels):
        if not labels:
            return []
        cur = self.ns_by("label", labels[0]["Key"] + "/" + labels[0]["Value"])
        for l in labels[1:]:
            cur = intersect(cur, self.ns_by("label", l["Key"] + "/" + l["Value"]))
            if not cur:
                break
        return [p for ns in cur for p in self.pods_in_ns(ns)]

    @staticmethod
    def _combine(exprs, pod_set_of):
        sets = {IN: [], NOT_IN: [], EXISTS: [], DOES_NOT_EXIST: []}
        for x in exprs:
            op = x.get("Operator", 0)
            if op not in sets:
                continue
            ps = pod_set_of(x, op)
            if ps is None:
                return []
            if not sets[op]:
                sets[op] = list(ps)
            sets[op] = intersect(sets[op], ps)
            if not sets[op]:
                return []
        final = [s for s in (sets[IN], sets[NOT_IN], sets[EXISTS], sets[DOES_NOT_EXIST]) if s]
        if not final:
            return []
        r = final[0]
        for s in final[1:]:
            r = intersect(r, s)
        return r

    def match_expression_pods_inside_ns(self, ns, exprs):
        if not exprs:
            return []

        def pod_set(x, op):
            k = x.get("Key", "")
            if op in (IN, NOT_IN):
                s = sorted({p for v in x.get("Value") or [] for p in self.pods_by("nslabel", ns + "/" + k + "/" + v)})
                return s if op == IN else difference(self.pods_in_ns(ns), s)
            s = self.pods_by("nskey", ns + "/" + k)
            if op == EXISTS:
                return s or None  # an empty EXISTS set ends the lookup
            return difference(self.pods_in_ns(ns), s)

        return self._combine(exprs, pod_set)

    def pods_by_ns_expressions(self, exprs):
        if not exprs:
            return []

        def pod_set(x, op):
            k = x.get("Key", "")
            if op in (IN, NOT_IN):
                nss = sorted({n for v in x.get("Value") or [] for n in self.ns_by("label", k + "/" + v)})
                if op == NOT_IN:
                    nss = difference(sorted(self.namespaces), nss)
            else:
                nss = sorted(set(self.ns_by("key", k)))
                if op == DOES_NOT_EXIST:
                    nss = difference(sorted(self.namespaces), nss)
            return [p for n in nss for p in self.pods_in_ns(n)]

        return self._combine(exprs, pod_set)

    def pods_by_label_selector_inside_ns(self, ns, sel):
        sel = sel or {}
        ml, me = sel.get("MatchLabel") or [], sel.get("MatchExpression") or []
        if not ml and not me:
            return self.pods_in_ns(ns)
        a, b = self.match_label_pods_inside_ns(ns, ml), self.match_expression_pods_inside_ns(ns, me)
        if ml and me:
            return intersect(a, b)
        return a if ml else b

    def pods_by_ns_label_selector(self, sel):
        sel = sel or {}
        ml, me = sel.get("MatchLabel") or [], sel.get("MatchExpression") or []
        if not ml and not me:
            return difference(self.all_pods(), self.pods_in_ns("kube-system"))
        a, b = self.pods_by_ns_labels(ml), self.pods_by_ns_expressions(me)
        if ml and me:
            return intersect(a, b)
        return a if ml else b

    def policies_by_pod(self, pod):
        want = unstring(pod)
        out = []
        for pid in sorted(self.policies):
            p = self.policies[pid]
            if p is None:
                continue
            for x in self.pods_by_label_selector_inside_ns(p.get("Namespace", ""), p.get("Pods")):
                if unstring(x) == want:
                    out.append(p.get("Namespace", "") + "/" + p.get("Name", ""))
        return sorted(out)

    # ---- events ----
    @staticmethod
    def obj_id(kind, o):
        return o.get("Name", "") if kind == NAMESPACE else o.get("Namespace", "") + "/" + o.get("Name", "")

    def update(self, kind, prev, new):
        t = (self.pods, self.namespaces, self.policies)[kind]
        if prev is None:
            t[self.obj_id(kind, new)] = new
            ev = ("add", new)
        elif new is None:
            t.pop(self.obj_id(kind, prev), None)
            ev = ("del", prev)
        else:
            t.pop(self.obj_id(kind, prev), None)
            t[self.obj_id(kind, new)] = new
            ev = ("update", prev, new)
        for w in self.watchers:
            w.on_event(kind, ev)

    def resync(self, pods=(), namespaces=(), policies=()):
        self.reset()
        for p in pods:
            self.pods[self.obj_id(POD, p)] = p
        for n in namespaces:
            self.namespaces[self.obj_id(NAMESPACE, n)] = n
        for p in policies:
            self.policies[self.obj_id(POLICY, p)] = p
        for w in self.watchers:
            w.on_resync(pods)


# ---- processor ----
def _is_match_label(labels, exists, prefix):
    return all(prefix + l.get("Key", "") + "/" + l.get("Value", "") in exists for l in labels)


def _is_match_expression(exprs, exists, prefix):
    match = False
    for x in exprs:
        op, k = x.get("Operator", 0), x.get("Key", "")
        if op == IN:
            for v in x.get("Value") or []:
                match = (prefix + k + v) in exists
                if match:
                    break
            if not match:
                return False
        elif op == NOT_IN:
            if any(prefix + k + v in exists for v in x.get("Value") or []):
                return False
            match = True
        elif op == EXISTS:
            if prefix + k not in exists:
                return False
            match = True
        elif op == DOES_NOT_EXIST:
            if prefix + k in exists:
                return False
            match = True
    return match


def _selector_match(sel, label_match, expr_match):
    hl, he = bool(sel.get("MatchLabel")), bool(sel.get("MatchExpression"))
    if hl and he:
        return label_match() and expr_match()
    if he:
        return expr_match()
    if hl:
        return label_match()
    return True


class PolicyProcessor:
    def __init__(self, cache: PolicyCache, configurator, pod_subnet):
        """configurator: oracle.configurator.PolicyConfigurator; its pod_ips are refreshed from
        the cache before every commit (the reference configurator reads the cache)."""
        self.cache, self.cfg = cache, configurator
        self.subnet = gonet.parse_cidr(pod_subnet)[1]
        self.pod_ip_map = {}
        cache.watchers.append(self)

    def filter_host_pods(self, pods):
        out = []
        for pid in pods:
            found, p = self.cache.lookup(POD, pid)
            if not found or p is None or not p.get("IpAddress"):
                if pid not in self.pod_ip_map:
                    continue
                ip = self.pod_ip_map[pid]
            else:
                ip = gonet.parse_ip(p["IpAddress"])
            if ip is None or not gonet.contains(self.subnet, ip):
                continue
            out.append(pid)
        return out

    def pods_assigned(self, policy):
        return self.cache.pods_by_label_selector_inside_ns(policy.get("Namespace", ""), policy.get("Pods"))

    def calculate_matches(self, policy, pod):
        c = self.cache
        ns = policy.get("Namespace", "")
        matches = []

        def named(p, name):
            found, pd = c.lookup(POD, p)
            if pd is None:
                return []
            return [q.get("ContainerPort", 0) for ct in pd.get("Container") or [] for q in ct.get("Port") or []
                    if q.get("Name", "") == name]

        for mtype, rules, key in ((0, policy.get("IngressRule") or [], "From"),
                                  (1, policy.get("EgressRule") or [], "To")):
            for r in rules:
                peers = r.get(key) or []
                pods, blocks, ports = ([], [], []) if peers else (None, None, [])
                for peer in peers:
                    if peer.get("Pods") is not None:
                        pods += c.pods_by_label_selector_inside_ns(ns, peer["Pods"])
                    if peer.get("Namespaces") is not None:
                        pods += c.pods_by_ns_label_selector(peer["Namespaces"])
                    ib = peer.get("IpBlock")
                    if ib is None:
                        continue
                    blocks.append({"network": ib.get("Cidr", ""), "except": list(ib.get("Except") or [])})
                for rp in r.get("Port") or []:
                    proto = 1 if rp.get("Protocol", 0) == 1 else 0
                    pn = rp.get("Port") or {}
                    if pn.get("Type", 0) == 0:
                        ports.append({"protocol": proto, "number": pn.get("Number", 0) & 0xFFFF})
                    elif mtype == 0:
                        ports += [{"protocol": proto, "number": n & 0xFFFF} for n in named(pod, pn.get("Name", ""))]
                    else:
                        for t in (pods if pods else c.all_pods()):
                            for n in named(t, pn.get("Name", "")):
                                matches.append({"type": 1, "pods": [t], "blocks": [],
                                                "ports": [{"protocol": proto, "number": n & 0xFFFF}]})
                matches.append({"type": mtype, "pods": pods, "blocks": blocks, "ports": ports})
        return matches

    def process(self, resync, pods):
        pods = ["%s/%s" % u for u in sorted({unstring(p) for p in pods} - {None})]  # RemoveDuplicatePodIDs
        pods = self.filter_host_pods(pods)
        if not pods:
            return
        self.cfg.pod_ips = {pid: (p or {}).get("IpAddress", "") for pid, p in self.cache.pods.items()}
        txn = self.cfg.new_txn(resync)
        processed = {}
        for pod in pods:
            lst = []
            for pol_id in self.cache.policies_by_pod(pod):
                if pol_id not in processed:
                    found, pd = self.cache.lookup(POLICY, pol_id)
                    if not found or pd is None:
                        continue
                    ptype = {2: 1, 3: 2}.get(pd.get("PolicyType", 0), 0)
                    processed[pol_id] = {"id": pol_id, "type": ptype, "matches": self.calculate_matches(pd, pod)}
                lst.append(processed[pol_id])
            txn.configure(pod, lst)
        txn.commit()

    def policies_referencing_pod(self, pod):
        ns = pod.get("Namespace", "")
        lab = {ns + l.get("Key", "") + "/" + l.get("Value", "") for l in _labels(pod)}
        expr = {ns + "/" + l.get("Key", "") + "/" + l.get("Value", "") for l in _labels(pod)} | \
               {ns + "/" + l.get("Key", "") for l in _labels(pod)}
        nsd = self.cache.namespaces.get(ns)
        nlab = {l.get("Key", "") + "/" + l.get("Value", "") for l in _labels(nsd)}
        nexpr = nlab | {l.get("Key", "") for l in _labels(nsd)}
        out = {}
        for pid in sorted(self.cache.policies):
            p = self.cache.policies[pid]
            if p is None:
                continue
            key = p.get("Namespace", "") + "/" + p.get("Name", "")
            prefix = p.get("Namespace", "") + "/"
            for rules, pk in ((p.get("IngressRule") or [], "From"), (p.get("EgressRule") or [], "To")):
                if not rules:
                    out[key] = p
                    continue
                for r in rules:
                    for peer in r.get(pk) or []:
                        s = peer.get("Pods")
                        if s is not None:
                            if _selector_match(s, lambda: _is_match_label(s.get("MatchLabel") or [], lab, prefix),
                                               lambda: _is_match_expression(s.get("MatchExpression") or [], expr,
                                                                            prefix)):
                                out[key] = p
                        elif peer.get("Namespaces") is not None:
                            s = peer["Namespaces"]
                            if _selector_match(s, lambda: _is_match_label(s.get("MatchLabel") or [], nlab, ""),
                                               lambda: _is_match_expression(s.get("MatchExpression") or [], nexpr,
                                                                            "")):
                                out[key] = p
        return [out[k] for k in sorted(out)]

    def policies_referencing_namespace(self, ns):
        nsd = self.cache.namespaces.get(ns.get("Name", ""))
        lab = {l.get("Key", "") + "/" + l.get("Value", "") for l in _labels(nsd)}
        expr = lab | {l.get("Key", "") for l in _labels(nsd)}
        out = {}
        for pid in sorted(self.cache.policies):
            p = self.cache.policies[pid]
            if p is None:
                continue
            key = p.get("Namespace", "") + "/" + p.get("Name", "")
            for rules, pk in ((p.get("IngressRule") or [], "From"), (p.get("EgressRule") or [], "To")):
                if not rules:
                    out[key] = p
                    continue
                for r in rules:
                    for peer in r.get(pk) or []:
                        s = peer.get("Namespaces")
                        if s is not None and _selector_match(
                                s, lambda: _is_match_label(s.get("MatchLabel") or [], lab, ""),
                                lambda: _is_match_expression(s.get("MatchExpression") or [], expr, "")):
                            out[key] = p
        return [out[k] for k in sorted(out)]

    # ---- watcher callbacks ----
    def on_resync(self, pods):
        self.pod_ip_map = {}
        for p in pods:
            if p.get("IpAddress"):
                self.pod_ip_map[p.get("Namespace", "") + "/" + p.get("Name", "")] = gonet.parse_ip(p["IpAddress"])
        self.process(True, self.cache.all_pods())

    def _assigned_of(self, policies):
        return [x for p in policies for x in self.pods_assigned(p)]

    def on_event(self, kind, ev):
        if kind == POD:
            if ev[0] == "add":
                p = ev[1]
                pid = PolicyCache.obj_id(POD, p)
                if not p.get("IpAddress"):
                    return
                self.pod_ip_map[pid] = gonet.parse_ip(p["IpAddress"])
                self.process(False, self._assigned_of(self.policies_referencing_pod(p)) + [pid])
            elif ev[0] == "del":
                p = ev[1]
                pid = PolicyCache.obj_id(POD, p)
                self.process(False, self._assigned_of(self.policies_referencing_pod(p)) + [pid])
                self.pod_ip_map.pop(pid, None)
            else:
                old, new = ev[1], ev[2]
                pid = PolicyCache.obj_id(POD, new)
                if new.get("IpAddress"):
                    self.pod_ip_map[pid] = gonet.parse_ip(new["IpAddress"])
                elif not old.get("IpAddress"):
                    return
                pods = []
                for p in (old, new):
                    if p.get("IpAddress"):
                        pods += self._assigned_of(self.policies_referencing_pod(p))
                if new.get("IpAddress", "") != old.get("IpAddress", ""):
                    pods.append(pid)
                self.process(False, pods)
        elif kind == POLICY:
            pods = [x for p in ev[1:] for x in self.pods_assigned(p)]
            self.process(False, pods)
        elif kind == NAMESPACE and ev[0] == "update":
            pods = [x for n in ev[1:] for x in self._assigned_of(self.policies_referencing_namespace(n))]
            self.process(False, pods)
