#!/usr/bin/env python3
"""Generate tests/golden/vpptcp_kats.json from the reference's VPPTCP renderer tests.

Run here (the reference is at /root/reference; it does not exist on the GPU box):

    python tests/golden/make_vpptcp_golden.py

plugins/policy/renderer/vpptcp/vpptcp_renderer_test.go holds 6 scenarios. Each registers pods
with VPP application-namespace indexes, builds ContivRule literals, runs renderer transactions
(some after a simulated restart, i.e. a new renderer over the same session-rule tables, with
resync) and asserts the session-rule tables: request / error counts, rule counts and HasRule.
This script reads the test source as text and emits, per scenario, only data -- an ordered
list of steps:

  {"op": "appns", "pod": [ns, name], "index": N}
  {"op": "clear"}                                          mockSessionRules.Clear()
  {"op": "renderer", "buf": N}                             new Renderer + Init (0 = default)
  {"op": "txn", "resync": b, "render": [[pod, ip, [ingress rules], [egress rules], removed]]}
  {"op": "expect", "what": "err_count"|"req_count", "value": N, "line": L}
  {"op": "expect", "what": "num_rules", "scope": "local"|"global", "ns": N, "value": N, "line": L}
  {"op": "expect", "what": "has_rule", "scope": ..., "ns": N,
   "args": [lclIP, lclPort, rmtIP, rmtPort, proto, action], "value": true, "line": L}

Rules are [action, src CIDR or "", dst CIDR or "", protocol, src port, dst port] with the
reference's enum values (ActionDeny 0 / Permit 1; TCP 0, UDP 1, OTHER 2, ANY 3).
"""
import json
import os
import re

REF = "/root/reference/plugins/policy/renderer/vpptcp/vpptcp_renderer_test.go"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "vpptcp_kats.json")

ACTIONS = {"renderer.ActionDeny": 0, "renderer.ActionPermit": 1}
PROTOS = {"renderer.TCP": 0, "renderer.UDP": 1, "renderer.OTHER": 2, "renderer.ANY": 3}


def parse_scenario(name, body, line0):
    consts, pods, rules, lists, steps = {}, {}, {}, {}, []
    txn = None

    def val(tok):
        tok = tok.strip()
        if tok.startswith('"'):
            return tok.strip('"')
        if re.fullmatch(r"\d+", tok):
            return int(tok)
        return consts[tok]

    lines = body.split("\n")
    i = 0
    in_const = False
    while i < len(lines):
        ln = lines[i].strip()
        lno = line0 + i
        i += 1
        if ln.startswith("const ("):
            in_const = True
            continue
        if in_const:
            if ln == ")":
                in_const = False
                continue
            m = re.fullmatch(r"(\w+)\s*=\s*(.+)", ln)
            if m:
                consts[m.group(1)] = val(m.group(2))
            continue
        m = re.fullmatch(r"(\w+) := podmodel\.ID\{Name: (\w+), Namespace: (\w+)\}", ln)
        if m:
            pods[m.group(1)] = [val(m.group(3)), val(m.group(2))]
            continue
        m = re.fullmatch(r"(\w+) := &renderer\.ContivRule\{", ln)
        if m:
            fields = {}
            while lines[i].strip() != "}":
                f = re.fullmatch(r"(\w+):\s*(.+),", lines[i].strip())
                fields[f.group(1)] = f.group(2)
                i += 1
            i += 1

            def net(s):
                return re.fullmatch(r'ipNetwork\("([^"]*)"\)', s).group(1)

            rules[m.group(1)] = [ACTIONS[fields["Action"]], net(fields["SrcNetwork"]), net(fields["DestNetwork"]),
                                 PROTOS[fields["Protocol"]], int(fields["SrcPort"]), int(fields["DestPort"])]
            continue
        m = re.fullmatch(r"(\w+) :?= \[\]\*renderer\.ContivRule\{(.*)\}", ln)
        if m:
            names = [x.strip() for x in m.group(2).split(",") if x.strip()]
            lists[m.group(1)] = [rules[x] for x in names]
            continue
        m = re.fullmatch(r"ipv4Net\.SetPodAppNsIndex\((\w+), (\w+)\)", ln)
        if m:
            steps.append({"op": "appns", "pod": pods[m.group(1)], "index": val(m.group(2))})
            continue
        if ln == "mockSessionRules.Clear()":
            steps.append({"op": "clear"})
            continue
        if re.fullmatch(r"vppTCPRenderer :?= &Renderer\{", ln):
            buf = 0
            while not lines[i].strip().startswith("vppTCPRenderer.Init()"):
                f = re.search(r"GoVPPChanBufSize:\s*(\d+)", lines[i])
                if f:
                    buf = int(f.group(1))
                i += 1
            i += 1
            steps.append({"op": "renderer", "buf": buf})
            continue

        def render_args(s):
            a = [x.strip() for x in s.split(",")]
            ip = re.fullmatch(r"GetOneHostSubnet\((\w+)\)", a[1]).group(1)
            return [pods[a[0]], val(ip), lists[a[2]], lists[a[3]], a[4] == "true"]

        m = re.fullmatch(r"vppTCPRenderer\.NewTxn\((true|false)\)\.Render\((.*)\)\.Commit\(\)", ln)
        if m:
            steps.append({"op": "txn", "resync": m.group(1) == "true", "render": [render_args(m.group(2))]})
            continue
        m = re.fullmatch(r"txn :?= vppTCPRenderer\.NewTxn\((true|false)\)", ln)
        if m:
            txn = {"op": "txn", "resync": m.group(1) == "true", "render": []}
            continue
        m = re.fullmatch(r"txn\.Render\((.*)\)", ln)
        if m:
            txn["render"].append(render_args(m.group(1)))
            continue
        if ln == "txn.Commit()":
            steps.append(txn)
            txn = None
            continue
        m = re.fullmatch(r"gomega\.Expect\(mockSessionRules\.(.*)\)\.To\(gomega\.(BeEquivalentTo\((\d+)\)|BeTrue\(\))\)"
                         r"(\s*//.*)?", ln)
        if m:
            expr = m.group(1)
            value = int(m.group(3)) if m.group(3) is not None else True
            if expr == "GetErrCount()":
                steps.append({"op": "expect", "what": "err_count", "value": value, "line": lno})
                continue
            if expr == "GetReqCount()":
                steps.append({"op": "expect", "what": "req_count", "value": value, "line": lno})
                continue
            t = re.fullmatch(r"(LocalTable\((\w+)\)|GlobalTable\(\))\.(NumOfRules\(\)|HasRule\((.*)\))", expr)
            scope = "local" if t.group(1).startswith("Local") else "global"
            ns = val(t.group(2)) if t.group(2) else 0
            if t.group(3) == "NumOfRules()":
                steps.append({"op": "expect", "what": "num_rules", "scope": scope, "ns": ns, "value": value,
                              "line": lno})
            else:
                a = [x.strip() for x in t.group(4).split(",")]
                args = [val(a[0]), int(a[1]), val(a[2]), int(a[3]), val(a[4]), val(a[5])]
                steps.append({"op": "expect", "what": "has_rule", "scope": scope, "ns": ns, "args": args,
                              "value": value, "line": lno})
            continue
        if ("gomega.Expect(vppChan)" in ln or ln.startswith("vppChan :=") or ln.startswith("ipv4Net :=")
                or ln == "gomega.RegisterTestingT(t)"):
            continue
        if ln.startswith("gomega.") or ln.startswith("mockSessionRules") or "Render(" in ln:
            raise ValueError("%s:%d unhandled statement: %s" % (name, lno, ln))
    return {"name": name, "steps": steps}


def main():
    src = open(REF).read()
    out = []
    for m in re.finditer(r"^func (Test\w+)\(t \*testing\.T\) \{\n(.*?)^\}", src, flags=re.S | re.M):
        if m.group(1) == "TestMain":
            continue
        line0 = src[:m.start(2)].count("\n") + 1
        out.append(parse_scenario(m.group(1), m.group(2), line0))
    n = sum(1 for s in out for st in s["steps"] if st["op"] == "expect")
    with open(OUT, "w") as f:
        json.dump({"source": "plugins/policy/renderer/vpptcp/vpptcp_renderer_test.go", "n_checks": n,
                   "scenarios": out}, f, indent=1)
    print("%d scenarios, %d checks -> %s" % (len(out), n, OUT))


if __name__ == "__main__":
    main()
