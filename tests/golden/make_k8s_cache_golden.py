#!/usr/bin/env python3
"""Generate tests/golden/k8s_cache_kats.json from the reference's policy-cache tests.

Run here (the reference is at /root/reference; it does not exist on the GPU box):

    python tests/golden/make_k8s_cache_golden.py

Sources (plugins/policy/cache/): cache_test.go, match_label_test.go, match_expression_test.go,
podidx/podmap_test.go, namespaceidx/namespace_test.go, policyidx/policymap_test.go, with the
shared objects of testdata/testdata.go. Each test function becomes one scenario holding only
data, in execution order:

  * ops:    ["register", kind, id, object|null] / ["unregister", kind, id] /
            ["update", kind, prev|null, next|null]  (datasync Put/Delete events replayed against a
            key -> value store, so `prev` is what the store held)
  * checks: {"target": "pc"|"idx", "method", "args", "vars", "asserts": [{"var", "kind", "value"}]}
            with kind one of contains / empty / nil / true / false / equals

Objects keep the Go field names (Name, Namespace, Label [{Key, Value}], Pods {MatchLabel,
MatchExpression [{Key, Operator, Value}]}, PolicyType, IngressRule, EgressRule, ...); IDs are
"ns/name" strings (namespace IDs: the name). The Go composite literals are read by the small
parser of make_configurator_golden.py.
"""
import importlib.util
import json
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/plugins/policy/cache"
OUT = os.path.join(HERE, "k8s_cache_kats.json")
FILES = [("cache_test.go", None), ("match_label_test.go", None), ("match_expression_test.go", None),
         ("podidx/podmap_test.go", "pod"), ("namespaceidx/namespace_test.go", "namespace"),
         ("policyidx/policymap_test.go", "policy")]

_spec = importlib.util.spec_from_file_location("mcg", os.path.join(HERE, "make_configurator_golden.py"))
mcg = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mcg)

ENUMS = {"IN": 0, "NOT_IN": 1, "EXISTS": 2, "DOES_NOT_EXIST": 3}
KIND = {"Pod": "pod", "Namespace": "namespace", "Policy": "policy"}


def strip_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def fold_strings(s, consts):
    for k, v in consts.items():
        s = re.sub(r"(?<![\w.\"])%s(?![\w\"])" % re.escape(k), '"%s"' % v, s)
    prev = None
    while prev != s:
        prev = s
        s = re.sub(r'"([^"]*)"\s*\+\s*"([^"]*)"', r'"\1\2"', s)
    return s


class Env:
    def __init__(self, parent=None):
        self.v, self.parent = {}, parent

    def get(self, name):
        if name in self.v:
            return self.v[name]
        if self.parent is not None:
            return self.parent.get(name)
        raise KeyError(name)


def conv(x, env):
    """parsed Go value -> JSON value"""
    if isinstance(x, (str, int)):
        return x
    if "ident" in x:
        name = x["ident"]
        if name == "nil":
            return None
        m = re.search(r"_(IN|NOT_IN|EXISTS|DOES_NOT_EXIST)$", name)
        if m:
            return ENUMS[m.group(1)]
        if name in ("true", "false"):
            return name == "true"
        return resolve(name, env)
    if "call" in x:
        fn, args = x["call"], [conv(a, env) for a in x["args"]]
        if fn.endswith(".GetID"):
            o = args[0]
            return o["Name"] if fn.startswith("namespace") else "%s/%s" % (o.get("Namespace", ""), o.get("Name", ""))
        if fn.endswith(".ID"):
            return args[0]
        if fn.endswith(".Key"):
            return "%s:%s" % (fn.split(".")[0], "/".join(str(a) for a in args))
        return fn  # e.g. KeyPrefix(): irrelevant here
    typ = x["type"] or ""
    if x["items"] and not x["fields"]:
        return [conv(i, env) for i in x["items"]]
    if typ.endswith(".ID"):
        f = {k: conv(v, env) for k, v in x["fields"].items()}
        return "%s/%s" % (f.get("Namespace", ""), f.get("Name", ""))
    if typ.startswith("[]") and not x["fields"]:
        return []
    return {k: conv(v, env) for k, v in x["fields"].items()}


def resolve(name, env):
    if name.startswith("testdata."):
        name = name[len("testdata."):]
    parts = name.split(".")
    v = env.get(parts[0])
    for p in parts[1:]:
        if isinstance(v, str):  # an ID held as "ns/name"
            v = v.split("/", 1)[0 if p == "Namespace" else 1]
        else:
            v = v[p]
    return v


def parse_value(text, env):
    return conv(mcg.Parser(mcg.tokenize(text)).value(), env)


def split_args(text):
    p = mcg.Parser(mcg.tokenize("f(%s)" % text))
    return p.value()["args"]


def load_testdata():
    src = strip_comments(open(os.path.join(REF, "testdata/testdata.go")).read())
    consts = dict(re.findall(r'^\s*(\w+)\s*=\s*"([^"]*)"', src, re.M))
    src = fold_strings(src, consts)
    env = Env()
    env.v.update(consts)
    # NAME = <literal> (top level or inside var ( ... ) groups), NAME = LIST[i]
    for m in re.finditer(r"^\s*(?:var\s+)?(\w+)\s*=\s*(?=&|\[\]|[\w.]+\{)", src, re.M):
        lit = mcg.literal_at(src, m.end())
        env.v[m.group(1)] = parse_value(lit, env)
    for name, lst, i in re.findall(r"^\s*(\w+)\s*=\s*(\w+)\[(\d+)\]", src, re.M):
        env.v[name] = env.v[lst][int(i)]
    return env


def scenario(body, name, line0, td, index_kind):
    env = Env(td)
    ops, checks, by_var = [], [], {}
    store = {}  # datasync mock: key -> value
    text = body
    i = 0
    while i < len(text):
        nl = text.find("\n", i)
        nl = len(text) if nl < 0 else nl
        line = text[i:nl]
        s = line.strip()
        nxt = nl + 1
        m_const = re.match(r"const\s*\(", s)
        if m_const:
            end = text.index(")", i)
            for k, v in re.findall(r'(\w+)\s*=\s*"([^"]*)"', text[i:end]):
                env.v[k] = v
            i = end + 1
            continue
        m = re.match(r"^([\w, ]+?)\s*(?::=|=)\s*(.*)$", s)
        if m and not s.startswith("gomega"):
            lhs = [v.strip() for v in m.group(1).split(",")]
            rhs = m.group(2)
            start = i + line.index(rhs) if rhs else i
            mcall = re.match(r"(pc|idx|datasnc)\.(\w+)\((.*)\)$", rhs)
            if re.match(r"(&|\[\]|[\w.]+\{)", rhs) and "{" in rhs and not mcall:
                lit = mcg.literal_at(text, start)
                if not rhs.startswith("&PolicyCache"):
                    env.v[lhs[0]] = parse_value(lit, env)
                i = start + len(lit)
                continue
            if mcall:
                tgt, meth, args = mcall.groups()
                if tgt == "datasnc" or meth == "ResyncEvent":
                    a = [conv(x, env) for x in split_args(args)] if meth in ("PutEvent", "DeleteEvent") else []
                    if meth == "PutEvent":
                        key, obj = a
                        env.v[lhs[0]] = ("put", key, store.get(key), obj)
                        store[key] = obj
                    elif meth == "DeleteEvent":
                        key = a[0]
                        env.v[lhs[0]] = ("del", key, store.get(key), None)
                        store.pop(key, None)
                    elif meth == "ResyncEvent":
                        env.v[lhs[0]] = ("resync", dict(store))
                    i = nxt
                    continue
                if meth == "NewMockDataSync" or meth.startswith("New"):
                    i = nxt
                    continue
                a = [conv(x, env) for x in split_args(args)] if args.strip() else []
                chk = {"target": tgt, "method": meth, "args": a, "vars": lhs, "asserts": [],
                       "line": line0 + text[:i].count("\n")}
                checks.append(chk)
                for v in lhs:
                    by_var[v] = chk
                i = nxt
                continue
            if rhs.startswith("NewConfigIndex") or rhs.startswith("datasync.") or rhs.startswith("logrus"):
                i = nxt
                continue
            if rhs.startswith("[]string{"):
                lit = mcg.literal_at(text, start)
                env.v[lhs[0]] = parse_value(lit, env)
                i = start + len(lit)
                continue
            env.v[lhs[0]] = parse_value(rhs, env)
            i = nxt
            continue
        mreg = re.match(r"(?:pc\.configured(?:Pods|Namespaces|Policies)|idx)\.(Register|Unregister|UnRegister)"
                        r"(Pod|Namespace|Policy)\((.*)\)$", s)
        if mreg:
            verb, kind, args = mreg.groups()
            a = [conv(x, env) for x in split_args(args)]
            if verb == "Register":
                ops.append(["register", KIND[kind], a[0], a[1], len(checks)])
            else:
                ops.append(["unregister", KIND[kind], a[0], None, len(checks)])
            i = nxt
            continue
        mupd = re.match(r"gomega\.Expect\(pc\.(Update|Resync)\((\w+)(?:\.KubeState)?\)\)\.To\(gomega\.BeNil\(\)\)$", s)
        if mupd:
            ev = env.get(mupd.group(2))
            if ev[0] == "resync":
                ops.append(["resync", None, None, ev[1], len(checks)])
            else:
                kind = ev[1].split(":")[0]
                kind = {"podmodel": "pod", "namespace": "namespace", "policymodel": "policy"}[kind]
                ops.append(["update", kind, ev[2], ev[3], len(checks)])
            i = nxt
            continue
        mexp = re.match(r"gomega\.Expect\((\w+)\)\.(To|NotTo)\(gomega\.(\w+)\((.*)\)\)$", s)
        if mexp:
            var, how, matcher, arg = mexp.groups()
            if var in by_var and how == "To":
                kind = {"ContainElement": "contains", "BeEmpty": "empty", "BeNil": "nil", "BeTrue": "true",
                        "BeFalse": "false", "BeEquivalentTo": "equals", "BeIdenticalTo": "equals"}[matcher]
                val = parse_value(arg, env) if arg.strip() else None
                by_var[var]["asserts"].append({"var": var, "kind": kind, "value": val})
            i = nxt
            continue
        i = nxt
    return {"name": name, "line": line0, "index_kind": index_kind, "ops": ops, "checks": checks}


def main():
    td = load_testdata()
    out, n_asserts = [], 0
    for rel, index_kind in FILES:
        src = open(os.path.join(REF, rel)).read()
        starts = [m.start() for m in re.finditer(r"^func (Test\w+)\(", src, re.M)] + [len(src)]
        for a, b in zip(starts, starts[1:]):
            body = strip_comments(src[a:b])
            name = re.match(r"func (Test\w+)", body).group(1)
            sc = scenario(body, "%s:%s" % (rel, name), src[:a].count("\n") + 1, td, index_kind)
            sc["source"] = rel
            n_asserts += sum(len(c["asserts"]) for c in sc["checks"])
            out.append(sc)
    with open(OUT, "w") as f:
        json.dump({"source": "plugins/policy/cache/*_test.go", "scenarios": out}, f, indent=1)
    print("wrote %s: %d scenarios, %d assertions" % (OUT, len(out), n_asserts))


if __name__ == "__main__":
    main()
