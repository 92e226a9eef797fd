// KSR model decoding and the policy cache (see k8s.hpp for the reference map).
#include "k8s.hpp"

#include <algorithm>

namespace pg {

const char* const kPodLabel = "podLabelSelectorKey";
const char* const kPodKey = "podKeySelectorKey";
const char* const kPodNSKey = "podNSKeySelectorKey";
const char* const kPodNSLabel = "podNamespaceLabelKey";
const char* const kPodNamespace = "podNamespaceKey";
const char* const kNsLabel = "namespaceLabelSelectorKey";
const char* const kNsKey = "namespaceKeySelectorKey";
const char* const kPolicyLabel = "policyPodLabelKey";
const char* const kPolicyNSLabel = "policyPodNSLabelKey";

// ---- protobuf wire format -------------------------------------------------------------------
namespace {

struct Pb {
    const uint8_t* p;
    const uint8_t* e;
    bool ok = true;
    Pb(const uint8_t* b, size_t n) : p(b), e(b + n) {}
    bool more() const { return ok && p < e; }
    uint64_t varint() {
        uint64_t v = 0;
        for (int s = 0; s < 64; s += 7) {
            if (p >= e) break;
            const uint8_t b = *p++;
            v |= (uint64_t)(b & 0x7F) << s;
            if (!(b & 0x80)) return v;
        }
        ok = false;
        return 0;
    }
    // next field header; false at the end or on error
    bool field(uint32_t* num, uint32_t* wt) {
        if (!more()) return false;
        const uint64_t k = varint();
        *num = (uint32_t)(k >> 3);
        *wt = (uint32_t)(k & 7);
        return ok && *num != 0;
    }
    Pb sub() {
        const uint64_t n = varint();
        if (!ok || n > (uint64_t)(e - p)) {
            ok = false;
            return Pb(p, 0);
        }
        Pb s(p, (size_t)n);
        p += n;
        return s;
    }
    std::string str() {
        Pb s = sub();
        return ok ? std::string((const char*)s.p, (size_t)(s.e - s.p)) : std::string();
    }
    void skip(uint32_t wt) {
        switch (wt) {
            case 0: varint(); break;
            case 1: if (e - p < 8) ok = false; else p += 8; break;
            case 2: sub(); break;
            case 5: if (e - p < 4) ok = false; else p += 4; break;
            default: ok = false;
        }
    }
};

// Each decoder: for every field, take it when (number, wire type) is known, skip otherwise.
bool dec_label(Pb m, K8sLabel* l) {
    uint32_t f, wt;
    while (m.field(&f, &wt)) {
        if (f == 1 && wt == 2) l->key = m.str();
        else if (f == 2 && wt == 2) l->value = m.str();
        else m.skip(wt);
    }
    return m.ok;
}

bool dec_expr(Pb m, K8sLabelExpr* x) {
    uint32_t f, wt;
    while (m.field(&f, &wt)) {
        if (f == 1 && wt == 2) x->key = m.str();
        else if (f == 2 && wt == 0) x->op = (int)(int32_t)m.varint();
        else if (f == 3 && wt == 2) x->values.push_back(m.str());
        else m.skip(wt);
    }
    return m.ok;
}

bool dec_selector(Pb m, K8sLabelSelector* s) {
    uint32_t f, wt;
    while (m.field(&f, &wt)) {
        if (f == 1 && wt == 2) {
            s->match_label.emplace_back();
            if (!dec_label(m.sub(), &s->match_label.back())) return false;
        } else if (f == 2 && wt == 2) {
            s->match_expression.emplace_back();
            if (!dec_expr(m.sub(), &s->match_expression.back())) return false;
        } else {
            m.skip(wt);
        }
    }
    return m.ok;
}

bool dec_cport(Pb m, K8sContainerPort* c) {
    uint32_t f, wt;
    while (m.field(&f, &wt)) {
        if (f == 1 && wt == 2) c->name = m.str();
        else if (f == 2 && wt == 0) c->host_port = (int32_t)m.varint();
        else if (f == 3 && wt == 0) c->container_port = (int32_t)m.varint();
        else if (f == 4 && wt == 0) c->protocol = (int)(int32_t)m.varint();
        else if (f == 5 && wt == 2) c->host_ip = m.str();
        else m.skip(wt);
    }
    return m.ok;
}

bool dec_container(Pb m, K8sContainer* c) {
    uint32_t f, wt;
    while (m.field(&f, &wt)) {
        if (f == 1 && wt == 2) {
            c->name = m.str();
        } else if (f == 2 && wt == 2) {
            c->ports.emplace_back();
            if (!dec_cport(m.sub(), &c->ports.back())) return false;
        } else {
            m.skip(wt);
        }
    }
    return m.ok;
}

bool dec_pport(Pb m, K8sPolicyPort* p) {
    uint32_t f, wt;
    while (m.field(&f, &wt)) {
        if (f == 1 && wt == 2) {  // PortNameOrNumber
            Pb s = m.sub();
            uint32_t g, wt2;
            while (s.field(&g, &wt2)) {
                if (g == 1 && wt2 == 0) p->type = (int)(int32_t)s.varint();
                else if (g == 2 && wt2 == 0) p->number = (int32_t)s.varint();
                else if (g == 3 && wt2 == 2) p->name = s.str();
                else s.skip(wt2);
            }
            if (!s.ok) return false;
        } else if (f == 3 && wt == 0) {
            p->protocol = (int)(int32_t)m.varint();
        } else {
            m.skip(wt);
        }
    }
    return m.ok;
}

bool dec_peer(Pb m, K8sPeer* p) {
    uint32_t f, wt;
    while (m.field(&f, &wt)) {
        if ((f == 1 || f == 2) && wt == 2) {
            auto& sel = f == 1 ? p->pods : p->namespaces;
            if (!sel) sel.emplace();
            if (!dec_selector(m.sub(), &*sel)) return false;  // repeated message fields merge
        } else if (f == 3 && wt == 2) {
            if (!p->ip_block) p->ip_block.emplace();
            Pb s = m.sub();
            uint32_t g, wt2;
            while (s.field(&g, &wt2)) {
                if (g == 1 && wt2 == 2) p->ip_block->cidr = s.str();
                else if (g == 2 && wt2 == 2) p->ip_block->except.push_back(s.str());
                else s.skip(wt2);
            }
            if (!s.ok) return false;
        } else {
            m.skip(wt);
        }
    }
    return m.ok;
}

bool dec_rule(Pb m, K8sPolicyRule* r) {
    uint32_t f, wt;
    while (m.field(&f, &wt)) {
        if (f == 1 && wt == 2) {
            r->ports.emplace_back();
            if (!dec_pport(m.sub(), &r->ports.back())) return false;
        } else if (f == 2 && wt == 2) {
            r->peers.emplace_back();
            if (!dec_peer(m.sub(), &r->peers.back())) return false;
        } else {
            m.skip(wt);
        }
    }
    return m.ok;
}

}  // namespace

bool decode_label_selector(const uint8_t* p, size_t n, K8sLabelSelector* out) {
    return dec_selector(Pb(p, n), out);
}

bool decode_pod(const uint8_t* p, size_t n, K8sPod* out) {
    Pb m(p, n);
    uint32_t f, wt;
    while (m.field(&f, &wt)) {
        if (f == 1 && wt == 2) out->name = m.str();
        else if (f == 2 && wt == 2) out->ns = m.str();
        else if (f == 3 && wt == 2) {
            out->labels.emplace_back();
            if (!dec_label(m.sub(), &out->labels.back())) return false;
        } else if (f == 4 && wt == 2) out->ip = m.str();
        else if (f == 5 && wt == 2) out->host_ip = m.str();
        else if (f == 6 && wt == 2) {
            out->containers.emplace_back();
            if (!dec_container(m.sub(), &out->containers.back())) return false;
        } else m.skip(wt);
    }
    return m.ok;
}

bool decode_namespace(const uint8_t* p, size_t n, K8sNamespace* out) {
    Pb m(p, n);
    uint32_t f, wt;
    while (m.field(&f, &wt)) {
        if (f == 1 && wt == 2) out->name = m.str();
        else if (f == 3 && wt == 2) {
            out->labels.emplace_back();
            if (!dec_label(m.sub(), &out->labels.back())) return false;
        } else m.skip(wt);
    }
    return m.ok;
}

bool decode_policy(const uint8_t* p, size_t n, K8sPolicy* out) {
    Pb m(p, n);
    uint32_t f, wt;
    while (m.field(&f, &wt)) {
        if (f == 1 && wt == 2) out->name = m.str();
        else if (f == 2 && wt == 2) out->ns = m.str();
        else if (f == 3 && wt == 2) {
            out->labels.emplace_back();
            if (!dec_label(m.sub(), &out->labels.back())) return false;
        } else if (f == 4 && wt == 2) {
            if (!out->pods) out->pods.emplace();
            if (!dec_selector(m.sub(), &*out->pods)) return false;
        } else if (f == 5 && wt == 0) out->policy_type = (int)(int32_t)m.varint();
        else if ((f == 6 || f == 7) && wt == 2) {
            auto& v = f == 6 ? out->ingress : out->egress;
            v.emplace_back();
            if (!dec_rule(m.sub(), &v.back())) return false;
        } else m.skip(wt);
    }
    return m.ok;
}

// ---- utils.go set helpers -------------------------------------------------------------------
Names names_unique(Names v) {
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    return v;
}

Names names_intersect(const Names& a, const Names& b) {  // utils.go:63-83
    if (a.empty() || b.empty()) return {};
    std::set<std::string> ha(a.begin(), a.end());
    Names out;
    for (auto& x : b)
        if (ha.count(x)) out.push_back(x);
    std::sort(out.begin(), out.end());
    return out;
}

Names names_difference(const Names& a, const Names& b) {  // utils.go:86-105
    std::map<std::string, int> m;
    for (auto& x : a) m[x] = 1;
    for (auto& x : b) m[x] += 1;
    Names out;
    for (auto& kv : m)
        if (kv.second == 1) out.push_back(kv.first);
    return out;
}

bool unstring_id(const std::string& s, std::string* ns, std::string* name) {
    const size_t a = s.find('/');
    if (a == std::string::npos) return false;  // Go would index out of range
    const size_t b = s.find('/', a + 1);
    *ns = s.substr(0, a);
    *name = s.substr(a + 1, b == std::string::npos ? std::string::npos : b - a - 1);
    return true;
}

// ---- index functions ------------------------------------------------------------------------
void PolicyCache::register_pod(const std::string& id, std::shared_ptr<const K8sPod> pod, std::string raw) {
    NamedIndex<K8sPod>::Entry e;  // podmap.go:95-125
    if (pod) {
        Names labels, keys, ns_labels, ns_keys;
        for (auto& l : pod->labels) {
            labels.push_back(l.key + "/" + l.value);
            keys.push_back(l.key);
            ns_labels.push_back(pod->ns + "/" + l.key + "/" + l.value);
            ns_keys.push_back(pod->ns + "/" + l.key);
        }
        e.fields[kPodLabel] = labels;
        e.fields[kPodKey] = names_unique(keys);
        e.fields[kPodNamespace] = {pod->ns};
        e.fields[kPodNSLabel] = ns_labels;
        e.fields[kPodNSKey] = names_unique(ns_keys);
    }
    e.obj = std::move(pod);
    e.raw = std::move(raw);
    pods.put(id, std::move(e));
}

void PolicyCache::register_namespace(const std::string& id, std::shared_ptr<const K8sNamespace> ns,
                                     std::string raw) {
    NamedIndex<K8sNamespace>::Entry e;  // namespacemap.go:78-99
    if (ns) {
        Names labels, keys;
        for (auto& l : ns->labels) {
            labels.push_back(l.key + "/" + l.value);
            keys.push_back(l.key);
        }
        e.fields[kNsLabel] = labels;
        e.fields[kNsKey] = names_unique(keys);
    }
    e.obj = std::move(ns);
    e.raw = std::move(raw);
    namespaces.put(id, std::move(e));
}

void PolicyCache::register_policy(const std::string& id, std::shared_ptr<const K8sPolicy> pol, std::string raw) {
    NamedIndex<K8sPolicy>::Entry e;  // policymap.go:82-102 (a nil pod selector indexes nothing)
    if (pol) {
        Names labels, ns_labels;
        if (pol->pods)
            for (auto& l : pol->pods->match_label) {
                labels.push_back(l.key + "/" + l.value);
                ns_labels.push_back(pol->ns + "/" + l.key + "/" + l.value);
            }
        e.fields[kPolicyLabel] = labels;
        e.fields[kPolicyNSLabel] = ns_labels;
    }
    e.obj = std::move(pol);
    e.raw = std::move(raw);
    policies.put(id, std::move(e));
}

void PolicyCache::reset() {
    pods = NamedIndex<K8sPod>();
    namespaces = NamedIndex<K8sNamespace>();
    policies = NamedIndex<K8sPolicy>();
}

// ---- lookups (cache_impl.go) ----------------------------------------------------------------
const K8sPod* PolicyCache::lookup_pod(const std::string& id, bool* found) const {
    const auto* e = pods.get(id);
    *found = e != nullptr;
    return e ? e->obj.get() : nullptr;
}
const K8sPolicy* PolicyCache::lookup_policy(const std::string& id, bool* found) const {
    const auto* e = policies.get(id);
    *found = e != nullptr;
    return e ? e->obj.get() : nullptr;
}
const K8sNamespace* PolicyCache::lookup_namespace(const std::string& id, bool* found) const {
    const auto* e = namespaces.get(id);
    *found = e != nullptr;
    return e ? e->obj.get() : nullptr;
}

Names PolicyCache::match_label_pods_inside_ns(const std::string& ns, const std::vector<K8sLabel>& labels) const {
    if (labels.empty()) return {};  // match_label.go:23-46
    Names current = pods.list(kPodNSLabel, ns + "/" + labels[0].key + "/" + labels[0].value);
    for (size_t i = 1; i < labels.size(); i++) {
        current = names_intersect(current, pods.list(kPodNSLabel, ns + "/" + labels[i].key + "/" + labels[i].value));
        if (current.empty()) break;
    }
    return current;
}

Names PolicyCache::pods_by_ns_label_selector(const std::vector<K8sLabel>& labels) const {
    if (labels.empty()) return {};  // match_label.go:48-74
    Names current = namespaces.list(kNsLabel, labels[0].key + "/" + labels[0].value);
    for (size_t i = 1; i < labels.size(); i++) {
        current = names_intersect(current, namespaces.list(kNsLabel, labels[i].key + "/" + labels[i].value));
        if (current.empty()) break;
    }
    Names out;
    for (auto& ns : current) {
        Names p = pods.list(kPodNamespace, ns);
        out.insert(out.end(), p.begin(), p.end());
    }
    return out;
}

namespace {
// The four per-operator accumulators of match_expression.go: the first result seeds the set,
// later ones intersect it; an empty set ends the whole evaluation with no pods.
struct ExprSets {
    Names sets[4];
    bool add(int op, const Names& pod_set) {
        Names& s = sets[op];
        if (s.empty()) s = pod_set;
        s = names_intersect(s, pod_set);
        return !s.empty();
    }
    Names result() const {
        std::vector<const Names*> f;
        for (auto& s : sets)
            if (!s.empty()) f.push_back(&s);
        if (f.empty()) return {};
        Names r = *f[0];
        for (size_t i = 1; i < f.size(); i++) r = names_intersect(r, *f[i]);
        return r;
    }
};
}  // namespace

Names PolicyCache::match_expression_pods_inside_ns(const std::string& ns,
                                                   const std::vector<K8sLabelExpr>& exprs) const {
    if (exprs.empty()) return {};  // match_expression.go:30-134
    ExprSets acc;
    for (const auto& x : exprs) {
        Names pod_set;
        switch (x.op) {
            case kOpIn:
            case kOpNotIn:
                for (auto& v : x.values) {
                    Names p = pods.list(kPodNSLabel, ns + "/" + x.key + "/" + v);
                    pod_set.insert(pod_set.end(), p.begin(), p.end());
                }
                pod_set = names_unique(pod_set);
                if (x.op == kOpNotIn) pod_set = names_difference(pods.list(kPodNamespace, ns), pod_set);
                break;
            case kOpExists:
                pod_set = pods.list(kPodNSKey, ns + "/" + x.key);
                if (pod_set.empty()) return {};
                break;
            case kOpDoesNotExist:
                pod_set = names_difference(pods.list(kPodNamespace, ns), pods.list(kPodNSKey, ns + "/" + x.key));
                break;
            default:
                continue;
        }
        if (!acc.add(x.op, pod_set)) return {};
    }
    return acc.result();
}

Names PolicyCache::pods_by_ns_match_expression(const std::vector<K8sLabelExpr>& exprs) const {
    if (exprs.empty()) return {};  // match_expression.go:136-271
    ExprSets acc;
    for (const auto& x : exprs) {
        Names ns_set;
        switch (x.op) {
            case kOpIn:
            case kOpNotIn:
                for (auto& v : x.values) {
                    Names n = namespaces.list(kNsLabel, x.key + "/" + v);
                    ns_set.insert(ns_set.end(), n.begin(), n.end());
                }
                ns_set = names_unique(ns_set);
                if (x.op == kOpNotIn) ns_set = names_difference(namespaces.all(), ns_set);
                break;
            case kOpExists:
                ns_set = names_unique(namespaces.list(kNsKey, x.key));
                break;
            case kOpDoesNotExist:
                ns_set = names_difference(namespaces.all(), names_unique(namespaces.list(kNsKey, x.key)));
                break;
            default:
                continue;
        }
        Names pod_set;
        for (auto& ns : ns_set) {
            Names p = pods.list(kPodNamespace, ns);
            pod_set.insert(pod_set.end(), p.begin(), p.end());
        }
        if (!acc.add(x.op, pod_set)) return {};
    }
    return acc.result();
}

Names PolicyCache::lookup_pods_by_label_selector_inside_ns(const std::string& ns,
                                                           const K8sLabelSelector& sel) const {
    // cache_impl.go:81-105
    if (sel.match_expression.empty() && sel.match_label.empty()) return pods.list(kPodNamespace, ns);
    Names ml = match_label_pods_inside_ns(ns, sel.match_label);
    Names me = match_expression_pods_inside_ns(ns, sel.match_expression);
    if (!sel.match_label.empty() && !sel.match_expression.empty()) return names_intersect(ml, me);
    return sel.match_label.empty() ? me : ml;
}

Names PolicyCache::lookup_pods_by_ns_label_selector(const K8sLabelSelector& sel) const {
    // cache_impl.go:107-136: an empty selector = every pod outside kube-system
    if (sel.match_expression.empty() && sel.match_label.empty())
        return names_difference(pods.all(), pods.list(kPodNamespace, "kube-system"));
    Names ml = pods_by_ns_label_selector(sel.match_label);
    Names me = pods_by_ns_match_expression(sel.match_expression);
    if (!sel.match_label.empty() && !sel.match_expression.empty()) return names_intersect(ml, me);
    return sel.match_label.empty() ? me : ml;
}

Names PolicyCache::lookup_policies_by_pod(const std::string& pod_id) const {
    // cache_impl.go:169-196
    std::string ns, name, pns, pname;
    if (!unstring_id(pod_id, &ns, &name)) return {};
    static const K8sLabelSelector kEmpty;
    Names out;
    for (auto& kv : policies.items) {
        const K8sPolicy* p = kv.second.obj.get();
        if (!p) continue;
        for (auto& id : lookup_pods_by_label_selector_inside_ns(p->ns, p->pods ? *p->pods : kEmpty))
            if (unstring_id(id, &pns, &pname) && pns == ns && pname == name) out.push_back(policy_key(*p));
    }
    return out;
}

// ---- events (data_change.go, data_resync.go) ------------------------------------------------
std::string PolicyCache::update_pod(std::shared_ptr<const K8sPod> prev, std::shared_ptr<const K8sPod> next,
                                    std::string raw) {
    if (!prev && !next) return "no pod given";
    if (!prev) {
        const std::string id = pod_key(*next);
        register_pod(id, next, std::move(raw));
        for (auto* w : watchers)
            if (auto err = w->add_pod(id, *next); !err.empty()) return err;
    } else if (!next) {
        const std::string id = pod_key(*prev);
        pods.del(id);
        for (auto* w : watchers)
            if (auto err = w->del_pod(id, *prev); !err.empty()) return err;
    } else {
        pods.del(pod_key(*prev));
        const std::string id = pod_key(*next);
        register_pod(id, next, std::move(raw));
        for (auto* w : watchers)
            if (auto err = w->update_pod(id, *prev, *next); !err.empty()) return err;
    }
    return "";
}

std::string PolicyCache::update_namespace(std::shared_ptr<const K8sNamespace> prev,
                                          std::shared_ptr<const K8sNamespace> next, std::string raw) {
    if (!prev && !next) return "no namespace given";
    if (!prev) {
        register_namespace(next->name, next, std::move(raw));
        for (auto* w : watchers)
            if (auto err = w->add_namespace(*next); !err.empty()) return err;
    } else if (!next) {
        namespaces.del(prev->name);
        for (auto* w : watchers)
            if (auto err = w->del_namespace(*prev); !err.empty()) return err;
    } else {
        namespaces.del(prev->name);
        register_namespace(next->name, next, std::move(raw));
        for (auto* w : watchers)
            if (auto err = w->update_namespace(*prev, *next); !err.empty()) return err;
    }
    return "";
}

std::string PolicyCache::update_policy(std::shared_ptr<const K8sPolicy> prev, std::shared_ptr<const K8sPolicy> next,
                                       std::string raw) {
    if (!prev && !next) return "no policy given";
    if (!prev) {
        register_policy(policy_key(*next), next, std::move(raw));
        for (auto* w : watchers)
            if (auto err = w->add_policy(*next); !err.empty()) return err;
    } else if (!next) {
        policies.del(policy_key(*prev));
        for (auto* w : watchers)
            if (auto err = w->del_policy(*prev); !err.empty()) return err;
    } else {
        policies.del(policy_key(*prev));
        register_policy(policy_key(*next), next, std::move(raw));
        for (auto* w : watchers)
            if (auto err = w->update_policy(*prev, *next); !err.empty()) return err;
    }
    return "";
}

std::string PolicyCache::resync(const ResyncData& d) {
    reset();
    auto raw = [](const std::vector<std::string>& v, size_t i) { return i < v.size() ? v[i] : std::string(); };
    for (size_t i = 0; i < d.pods.size(); i++) register_pod(pod_key(*d.pods[i]), d.pods[i], raw(d.pod_raw, i));
    for (size_t i = 0; i < d.namespaces.size(); i++)
        register_namespace(d.namespaces[i]->name, d.namespaces[i], raw(d.ns_raw, i));
    for (size_t i = 0; i < d.policies.size(); i++)
        register_policy(policy_key(*d.policies[i]), d.policies[i], raw(d.policy_raw, i));
    for (auto* w : watchers) w->resync(d);  // cache_impl.go:69-77 ignores watcher errors
    return "";
}

}  // namespace pg
