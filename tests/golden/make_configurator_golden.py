#!/usr/bin/env python3
"""Generate tests/golden/configurator_kats.json from the reference's configurator tests.

Run here (the reference is at /root/reference; it does not exist on the GPU box):

    python tests/golden/make_configurator_golden.py

plugins/policy/configurator/configurator_test.go holds 10 scenarios. Each builds pods (in the
mock policy cache), ContivPolicy literals, one or more mock renderers, runs one configurator
transaction and asserts GetPodIP and MockRenderer.TestTraffic results (174 of them). This
script reads the test source as text and extracts, per scenario, only data:

  * pods:      {"ns/name": IP or null (pod not in the cache)}
  * nat:       the IPAM NAT-loopback address
  * policies:  {var: {id, type, matches: [{type, pods|null, blocks|null, ports}]}}
  * renderers: mock renderer variables in registration order
  * txn:       {resync, configure: [[pod, [policy var, ...]], ...]}
  * pod_ip:    GetPodIP expectations [renderer, pod, ip, masklen]
  * traffic:   TestTraffic expectations [renderer, pod, direction, src, dst, proto, sport,
               dport, expected action]  (test source line cited per entry)

The Go composite literals are read by a small tokenizer/parser of the subset they use.
"""
import json
import os
import re

REF = "/root/reference/plugins/policy/configurator/configurator_test.go"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "configurator_kats.json")

TOK = re.compile(r'\s*(?:(?P<str>"[^"]*")|(?P<num>\d+)|(?P<id>[A-Za-z_][\w.]*)|(?P<p>\[\]|[{}()\[\]:,&*]))')


def tokenize(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)  # Go comments (no string here holds them)
    s = re.sub(r"//[^\n]*", " ", s)
    out, i = [], 0
    while i < len(s):
        m = TOK.match(s, i)
        if not m or m.end() == i:
            if s[i:].strip() == "":
                break
            raise ValueError("cannot tokenize at %r" % s[i:i + 30])
        i = m.end()
        kind = m.lastgroup
        out.append((kind, m.group(kind)))
    return out


class Parser:
    """value := ['&'] [type] '{' elems '}' | ident '(' args ')' | string | number | ident
    type := ident | '[]' ['*'] type"""

    def __init__(self, toks):
        self.t, self.i = toks, 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else (None, None)

    def take(self, v=None):
        tok = self.t[self.i]
        if v is not None and tok[1] != v:
            raise ValueError("expected %r got %r" % (v, tok))
        self.i += 1
        return tok

    def typ(self):
        if self.peek()[1] == "[]":
            self.take("[]")
            if self.peek()[1] == "*":
                self.take("*")
            return "[]" + self.typ()
        return self.take()[1]

    def value(self):
        kind, v = self.peek()
        if v == "&":
            self.take("&")
            return self.value()
        if kind == "str":
            self.take()
            return v[1:-1]
        if kind == "num":
            self.take()
            return int(v)
        if v == "{":  # elided type (element of a typed slice)
            return self.composite(None)
        if v == "[]":
            return self.composite(self.typ())
        if kind == "id":
            nxt = self.peek(1)[1]
            if nxt == "{":
                self.take()
                return self.composite(v)
            if nxt == "(":
                self.take()
                self.take("(")
                args = []
                while self.peek()[1] != ")":
                    args.append(self.value())
                    if self.peek()[1] == ",":
                        self.take(",")
                self.take(")")
                return {"call": v, "args": args}
            self.take()
            return {"ident": v}
        raise ValueError("unexpected %r" % (self.peek(),))

    def composite(self, typ):
        self.take("{")
        fields, items = {}, []
        while self.peek()[1] != "}":
            if self.peek()[0] == "id" and self.peek(1)[1] == ":":
                key = self.take()[1]
                self.take(":")
                fields[key] = self.value()
            else:
                items.append(self.value())
            if self.peek()[1] == ",":
                self.take(",")
        self.take("}")
        return {"type": typ, "fields": fields, "items": items}


def literal_at(body, start):
    """text of the brace-balanced literal starting at body[start] (which is '&' or a type)"""
    i = body.index("{", start)
    depth = 0
    for j in range(i, len(body)):
        if body[j] == "{":
            depth += 1
        elif body[j] == "}":
            depth -= 1
            if depth == 0:
                return body[start:j + 1]
    raise ValueError("unbalanced literal")


def main():
    src = open(REF).read()
    starts = [m.start() for m in re.finditer(r"^func (Test\w+)\(", src, re.M)] + [len(src)]
    scenarios = []
    total = 0
    for a, b in zip(starts, starts[1:]):
        body = src[a:b]
        line0 = src[:a].count("\n") + 1
        name = re.match(r"func (Test\w+)", body).group(1)
        consts = dict(re.findall(r'^\s*(\w+)\s*=\s*"([^"]*)"', body, re.M))
        consts["natLoopbackIP"] = re.search(r'natLoopbackIP = "([^"]*)"', src).group(1)

        def cv(x):
            if x.startswith('"'):
                return x[1:-1]
            return consts[x] if x in consts else x

        pods = {}
        for var, nm, ns in re.findall(r"(\w+) := podmodel\.ID\{Name: (\w+), Namespace: (\w+)\}", body):
            pods[var] = "%s/%s" % (cv(ns), cv(nm))

        def pod_of(v):
            return pods[v["ident"]]

        policies = {}
        for m in re.finditer(r"(\w+) := &ContivPolicy\{", body):
            lit = Parser(tokenize(literal_at(body, m.start() + len(m.group(1)) + 4))).value()
            f = lit["fields"]
            pid = f["ID"]["fields"]
            matches = []
            for mt in f.get("Matches", {"items": []})["items"]:
                mf = mt["fields"]
                pods_v = [pod_of(x) for x in mf["Pods"]["items"]] if "Pods" in mf else None
                blocks = None
                if "IPBlocks" in mf:
                    blocks = []
                    for bl in mf["IPBlocks"]["items"]:
                        bf = bl["fields"]
                        blocks.append({"network": bf["Network"]["args"][0],
                                       "except": [e["args"][0] for e in bf.get("Except", {"items": []})["items"]]})
                ports = [{"protocol": p["fields"]["Protocol"]["ident"], "number": p["fields"]["Number"]}
                         for p in mf.get("Ports", {"items": []})["items"]]
                matches.append({"type": mf["Type"]["ident"], "pods": pods_v, "blocks": blocks, "ports": ports})
            policies[m.group(1)] = {"id": "%s/%s" % (cv(pid["Namespace"]["ident"]) if isinstance(pid["Namespace"], dict)
                                                     else pid["Namespace"], pid["Name"]),
                                    "type": f["Type"]["ident"], "matches": matches}
        plists = {v: [x.strip() for x in items.split(",") if x.strip()]
                  for v, items in re.findall(r"(\w+) := \[\]\*ContivPolicy\{([^}]*)\}", body)}
        in_cache = {pods[p]: cv(ip) for p, ip in re.findall(r"cache\.AddPodConfig\((\w+), (\w+)\)", body)}
        all_pods = {pods[v]: in_cache.get(pods[v]) for v in pods}
        nat = cv(re.search(r"ipam\.SetNatLoopbackIP\((\w+)\)", body).group(1))
        rvars = {v: n for v, n in re.findall(r'(\w+) := NewMockRenderer\("(\w+)"', body)}
        registered = re.findall(r"configurator\.RegisterRenderer\((\w+)\)", body)
        resync = re.search(r"configurator\.NewTxn\((true|false)\)", body).group(1) == "true"
        configure = [[pods[p], plists[l]] for p, l in re.findall(r"txn\.Configure\((\w+), (\w+)\)", body)]
        pod_ip = [[r, pods[p], cv(ip), 32] for r, p, ip in re.findall(
            r"ip, masklen\s*:?= (\w+)\.GetPodIP\((\w+)\)\s*\n\s*gomega\.Expect\(masklen\)\.To\(gomega\.BeEquivalentTo\("
            r"net\.IPv4len \* 8\)\)\s*\n\s*gomega\.Expect\(ip\)\.To\(gomega\.BeEquivalentTo\((\w+)\)\)", body)]
        traffic = []
        for m in re.finditer(r"action :?= (\w+)\.TestTraffic\((\w+), (\w+),\s*parseIP\((\w+|\"[^\"]*\")\), parseIP\((\w+|\"[^\"]*\")\), "
                             r"rendererAPI\.(\w+), (\d+), (\d+)\)\s*\n\s*gomega\.Expect\(action\)\.To\("
                             r"gomega\.BeEquivalentTo\((\w+)\)\)", body):
            r, p, d, s_, t_, proto, sp, dp, exp = m.groups()
            traffic.append({"renderer": r, "pod": pods[p], "direction": d, "src": cv(s_), "dst": cv(t_),
                            "proto": proto, "sport": int(sp), "dport": int(dp), "expect": exp,
                            "line": line0 + body[:m.start()].count("\n")})
        assert len(traffic) == body.count(".TestTraffic("), name
        total += len(traffic)
        scenarios.append({"name": name, "line": line0, "pods": all_pods, "nat": nat, "policies": policies,
                          "renderers": registered, "renderer_names": rvars, "txn": {"resync": resync,
                                                                                    "configure": configure},
                          "pod_ip": pod_ip, "traffic": traffic})
    with open(OUT, "w") as f:
        json.dump({"source": "plugins/policy/configurator/configurator_test.go", "scenarios": scenarios}, f, indent=1)
    print("wrote %s: %d scenarios, %d TestTraffic KATs" % (OUT, len(scenarios), total))


if __name__ == "__main__":
    main()
