// C ABI of the K8s policy cache and processor (include/policygpu.h).
#include <algorithm>
#include <cstring>
#include <new>

#include "capi_internal.hpp"
#include "k8s.hpp"
#include "processor.hpp"

using namespace pg;

struct pg_policy_cache {
    PolicyCache c;
    std::string last_error;
};
struct pg_policy_processor {
    std::unique_ptr<PolicyProcessor> p;
    std::string last_error;
};

namespace {

template <class T>
std::shared_ptr<const T> decode(int kind, const uint8_t* pb, size_t len, bool* ok) {
    auto obj = std::make_shared<T>();
    if constexpr (std::is_same_v<T, K8sPod>) *ok = decode_pod(pb, len, obj.get());
    else if constexpr (std::is_same_v<T, K8sNamespace>) *ok = decode_namespace(pb, len, obj.get());
    else *ok = decode_policy(pb, len, obj.get());
    (void)kind;
    return obj;
}

std::string raw_of(const uint8_t* pb, size_t len) { return pb ? std::string((const char*)pb, len) : std::string(); }

int put_names(const Names& names, char* out, size_t cap, size_t* out_len) {
    size_t n = 0;
    for (size_t i = 0; i < names.size(); i++) n += names[i].size() + (i ? 1 : 0);
    if (out_len) *out_len = n;
    if (out && n <= cap) {
        size_t o = 0;
        for (size_t i = 0; i < names.size(); i++) {
            if (i) out[o++] = '\n';
            std::memcpy(out + o, names[i].data(), names[i].size());
            o += names[i].size();
        }
    }
    return (int)names.size();
}

template <class E>
int lookup_entry(const E* e, uint8_t* out, size_t cap, size_t* out_len) {
    if (!e) return 0;
    if (!e->obj) {
        if (out_len) *out_len = (size_t)-1;
        return 1;
    }
    if (out_len) *out_len = e->raw.size();
    if (out && e->raw.size() <= cap) std::memcpy(out, e->raw.data(), e->raw.size());
    return 1;
}

}  // namespace

extern "C" {

pg_policy_cache* pg_policy_cache_new(void) { return new (std::nothrow) pg_policy_cache(); }
void pg_policy_cache_free(pg_policy_cache* c) { delete c; }
const char* pg_policy_cache_last_error(const pg_policy_cache* c) { return c ? c->last_error.c_str() : "null"; }

int pg_policy_cache_register(pg_policy_cache* c, int kind, const char* id, const uint8_t* pb, size_t len) {
    if (!c || !id) return PG_EINVAL;
    bool ok = true;
    switch (kind) {
        case PG_K8S_POD:
            c->c.register_pod(id, pb ? decode<K8sPod>(kind, pb, len, &ok) : nullptr, raw_of(pb, len));
            break;
        case PG_K8S_NAMESPACE:
            c->c.register_namespace(id, pb ? decode<K8sNamespace>(kind, pb, len, &ok) : nullptr, raw_of(pb, len));
            break;
        case PG_K8S_POLICY:
            c->c.register_policy(id, pb ? decode<K8sPolicy>(kind, pb, len, &ok) : nullptr, raw_of(pb, len));
            break;
        default:
            return PG_EINVAL;
    }
    if (!ok) {  // keep the index consistent: a malformed object is not registered
        pg_policy_cache_unregister(c, kind, id);
        return PG_EINVAL;
    }
    return PG_OK;
}

int pg_policy_cache_unregister(pg_policy_cache* c, int kind, const char* id) {
    if (!c || !id) return PG_EINVAL;
    switch (kind) {
        case PG_K8S_POD: return c->c.pods.del(id) ? 1 : 0;
        case PG_K8S_NAMESPACE: return c->c.namespaces.del(id) ? 1 : 0;
        case PG_K8S_POLICY: return c->c.policies.del(id) ? 1 : 0;
        default: return PG_EINVAL;
    }
}

int pg_policy_cache_update(pg_policy_cache* c, int kind, const uint8_t* prev, size_t prev_len, const uint8_t* next,
                           size_t next_len) {
    if (!c || (!prev && !next)) return PG_EINVAL;
    bool ok1 = true, ok2 = true;
    std::string err;
    switch (kind) {
        case PG_K8S_POD: {
            auto a = prev ? decode<K8sPod>(kind, prev, prev_len, &ok1) : nullptr;
            auto b = next ? decode<K8sPod>(kind, next, next_len, &ok2) : nullptr;
            if (!ok1 || !ok2) return PG_EINVAL;
            err = c->c.update_pod(a, b, raw_of(next, next_len));
            break;
        }
        case PG_K8S_NAMESPACE: {
            auto a = prev ? decode<K8sNamespace>(kind, prev, prev_len, &ok1) : nullptr;
            auto b = next ? decode<K8sNamespace>(kind, next, next_len, &ok2) : nullptr;
            if (!ok1 || !ok2) return PG_EINVAL;
            err = c->c.update_namespace(a, b, raw_of(next, next_len));
            break;
        }
        case PG_K8S_POLICY: {
            auto a = prev ? decode<K8sPolicy>(kind, prev, prev_len, &ok1) : nullptr;
            auto b = next ? decode<K8sPolicy>(kind, next, next_len, &ok2) : nullptr;
            if (!ok1 || !ok2) return PG_EINVAL;
            err = c->c.update_policy(a, b, raw_of(next, next_len));
            break;
        }
        default:
            return PG_EINVAL;
    }
    c->last_error = err;
    return err.empty() ? PG_OK : PG_EFAULT;
}

int pg_policy_cache_resync(pg_policy_cache* c, const int* kinds, const uint8_t* const* objs, const size_t* lens,
                           size_t n) {
    if (!c || (n && (!kinds || !objs || !lens))) return PG_EINVAL;
    ResyncData d;
    for (size_t i = 0; i < n; i++) {
        if (!objs[i]) return PG_EINVAL;
        bool ok = true;
        switch (kinds[i]) {
            case PG_K8S_POD:
                d.pods.push_back(decode<K8sPod>(kinds[i], objs[i], lens[i], &ok));
                d.pod_raw.push_back(raw_of(objs[i], lens[i]));
                break;
            case PG_K8S_NAMESPACE:
                d.namespaces.push_back(decode<K8sNamespace>(kinds[i], objs[i], lens[i], &ok));
                d.ns_raw.push_back(raw_of(objs[i], lens[i]));
                break;
            case PG_K8S_POLICY:
                d.policies.push_back(decode<K8sPolicy>(kinds[i], objs[i], lens[i], &ok));
                d.policy_raw.push_back(raw_of(objs[i], lens[i]));
                break;
            default:
                return PG_EINVAL;
        }
        if (!ok) return PG_EINVAL;
    }
    c->last_error = c->c.resync(d);
    return c->last_error.empty() ? PG_OK : PG_EFAULT;
}

int pg_policy_cache_lookup(const pg_policy_cache* c, int kind, const char* id, uint8_t* out, size_t cap,
                           size_t* out_len) {
    if (!c || !id) return PG_EINVAL;
    switch (kind) {
        case PG_K8S_POD: return lookup_entry(c->c.pods.get(id), out, cap, out_len);
        case PG_K8S_NAMESPACE: return lookup_entry(c->c.namespaces.get(id), out, cap, out_len);
        case PG_K8S_POLICY: return lookup_entry(c->c.policies.get(id), out, cap, out_len);
        default: return PG_EINVAL;
    }
}

int pg_policy_cache_query(const pg_policy_cache* c, int query, const char* arg, const uint8_t* selector,
                          size_t selector_len, char* out, size_t cap, size_t* out_len) {
    if (!c) return PG_EINVAL;
    const std::string a = arg ? arg : "";
    K8sLabelSelector sel;
    if (selector && !decode_label_selector(selector, selector_len, &sel)) return PG_EINVAL;
    const PolicyCache& pc = c->c;
    Names r;
    switch (query) {
        case PG_Q_PODS_BY_LABEL_SELECTOR_INSIDE_NS: r = pc.lookup_pods_by_label_selector_inside_ns(a, sel); break;
        case PG_Q_PODS_BY_NS_LABEL_SELECTOR: r = pc.lookup_pods_by_ns_label_selector(sel); break;
        case PG_Q_PODS_BY_NAMESPACE: r = pc.lookup_pods_by_namespace(a); break;
        case PG_Q_ALL_PODS: r = pc.list_all_pods(); break;
        case PG_Q_POLICIES_BY_POD: r = pc.lookup_policies_by_pod(a); break;
        case PG_Q_ALL_POLICIES: r = pc.list_all_policies(); break;
        case PG_Q_ALL_NAMESPACES: r = pc.list_all_namespaces(); break;
        case PG_Q_MATCH_LABEL_PODS_INSIDE_NS: r = pc.match_label_pods_inside_ns(a, sel.match_label); break;
        case PG_Q_PODS_BY_NS_LABELS: r = pc.pods_by_ns_label_selector(sel.match_label); break;
        case PG_Q_MATCH_EXPRESSION_PODS_INSIDE_NS: r = pc.match_expression_pods_inside_ns(a, sel.match_expression); break;
        case PG_Q_PODS_BY_NS_EXPRESSIONS: r = pc.pods_by_ns_match_expression(sel.match_expression); break;
        case PG_Q_IDX_POD_LABEL: r = pc.pods.list(kPodLabel, a); break;
        case PG_Q_IDX_POD_KEY: r = pc.pods.list(kPodKey, a); break;
        case PG_Q_IDX_POD_NS_LABEL: r = pc.pods.list(kPodNSLabel, a); break;
        case PG_Q_IDX_POD_NS_KEY: r = pc.pods.list(kPodNSKey, a); break;
        case PG_Q_IDX_NS_LABEL: r = pc.namespaces.list(kNsLabel, a); break;
        case PG_Q_IDX_NS_KEY: r = pc.namespaces.list(kNsKey, a); break;
        case PG_Q_IDX_POLICY_LABEL: r = pc.policies.list(kPolicyLabel, a); break;
        case PG_Q_IDX_POLICY_NS_LABEL: r = pc.policies.list(kPolicyNSLabel, a); break;
        default: return PG_EINVAL;
    }
    std::sort(r.begin(), r.end());
    return put_names(r, out, cap, out_len);
}

pg_policy_processor* pg_policy_processor_new(pg_policy_cache* c, pg_configurator* cfg, const pg_ipnet* pod_subnet) {
    if (!c || !cfg || !pod_subnet || !pod_subnet->family) return nullptr;
    auto* p = new (std::nothrow) pg_policy_processor();
    if (!p) return nullptr;
    p->p = std::make_unique<PolicyProcessor>(&c->c, &cfg->c, to_ipnet(*pod_subnet));
    return p;
}

void pg_policy_processor_free(pg_policy_processor* p) { delete p; }

int pg_policy_processor_process(pg_policy_processor* p, int resync, const char* const* pods, size_t n) {
    if (!p || (n && !pods)) return PG_EINVAL;
    std::vector<std::string> v;
    for (size_t i = 0; i < n; i++) {
        if (!pods[i]) return PG_EINVAL;
        v.push_back(pods[i]);
    }
    p->last_error = p->p->process(resync != 0, v);
    return p->last_error.empty() ? PG_OK : PG_EFAULT;
}

const char* pg_policy_processor_last_error(const pg_policy_processor* p) {
    return p ? p->last_error.c_str() : "null";
}

}  // extern "C"
