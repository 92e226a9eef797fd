// extern "C" boundary of the VPPTCP renderer and the VPP session-rule tables
// (include/policygpu.h "VPPTCP renderer"; vpptcp.hpp for the reference map).
#include <cstring>
#include <stdexcept>

#include "capi_internal.hpp"
#include "vpptcp.hpp"

using namespace pg;

struct pg_session_rules {
    SessionRuleTables t;
    explicit pg_session_rules(const char* prefix) : t(prefix ? prefix : kSessionRuleTagPrefix) {}
};
struct pg_appns {
    AppNsIndex m;
};
struct pg_vpptcp_renderer {
    std::unique_ptr<VppTcpRenderer> r;
    std::string last_error;
};
struct pg_vpptcp_txn {
    pg_vpptcp_renderer* r;
    std::unique_ptr<VppTcpRendererTxn> t;
};

namespace {

std::string sv(const char* s) { return s ? std::string(s) : std::string(); }

ContivRule to_rule(const pg_contiv_rule& c) {
    ContivRule r;
    r.action = c.action;
    r.protocol = c.protocol;
    r.src_port = c.src_port;
    r.dst_port = c.dst_port;
    r.src = to_ipnet(c.src);
    r.dst = to_ipnet(c.dst);
    return r;
}

pg_session_rule to_pg(const SessionRule& s) {
    pg_session_rule o{};
    o.transport_proto = s.transport_proto;
    o.is_ip4 = s.is_ip4;
    std::memcpy(o.lcl_ip, s.lcl_ip, 16);
    o.lcl_plen = s.lcl_plen;
    std::memcpy(o.rmt_ip, s.rmt_ip, 16);
    o.rmt_plen = s.rmt_plen;
    o.lcl_port = s.lcl_port;
    o.rmt_port = s.rmt_port;
    o.action_index = s.action_index;
    o.appns_index = s.appns_index;
    o.scope = s.scope;
    std::memcpy(o.tag, s.tag, 64);
    return o;
}

SessionRule from_pg(const pg_session_rule& o) {
    SessionRule s;
    s.transport_proto = o.transport_proto;
    s.is_ip4 = o.is_ip4;
    std::memcpy(s.lcl_ip, o.lcl_ip, 16);
    s.lcl_plen = o.lcl_plen;
    std::memcpy(s.rmt_ip, o.rmt_ip, 16);
    s.rmt_plen = o.rmt_plen;
    s.lcl_port = o.lcl_port;
    s.rmt_port = o.rmt_port;
    s.action_index = o.action_index;
    s.appns_index = o.appns_index;
    s.scope = o.scope;
    std::memcpy(s.tag, o.tag, 64);
    return s;
}

int copy_out(const std::vector<SessionRule>& v, pg_session_rule* out, size_t cap) {
    if (out)
        for (size_t i = 0; i < v.size() && i < cap; i++) out[i] = to_pg(v[i]);
    return (int)v.size();
}

}  // namespace

extern "C" {

pg_session_rules* pg_session_rules_new(const char* tag_prefix) {
    try {
        return new pg_session_rules(tag_prefix);
    } catch (...) {
        return nullptr;
    }
}
void pg_session_rules_free(pg_session_rules* s) { delete s; }
int pg_session_rules_clear(pg_session_rules* s) {
    if (!s) return PG_EINVAL;
    s->t.clear();
    return PG_OK;
}
int pg_session_rules_counts(const pg_session_rules* s, int* req_count, int* err_count) {
    if (!s) return PG_EINVAL;
    if (req_count) *req_count = s->t.req_count;
    if (err_count) *err_count = s->t.err_count;
    return PG_OK;
}
int pg_session_rule_add_del(pg_session_rules* s, const pg_session_rule* rule, int is_add) {
    if (!s || !rule) return PG_EINVAL;
    try {
        return s->t.add_del(from_pg(*rule), is_add != 0);
    } catch (...) {
        return PG_ENOMEM;
    }
}
int pg_session_rules_table(const pg_session_rules* s, int scope, uint32_t ns_index, pg_session_rule* out, size_t cap) {
    if (!s) return PG_EINVAL;
    const std::vector<SessionRule>* t = s->t.table(scope, ns_index);
    if (!t) return 0;
    return copy_out(*t, out, cap);
}
int pg_session_rules_has_rule(const pg_session_rules* s, int scope, uint32_t ns_index, const char* lcl_ip,
                              uint16_t lcl_port, const char* rmt_ip, uint16_t rmt_port, const char* proto,
                              const char* action) {
    if (!s) return PG_EINVAL;
    try {
        return s->t.has_rule(scope, ns_index, sv(lcl_ip), lcl_port, sv(rmt_ip), rmt_port, sv(proto), sv(action)) ? 1
                                                                                                                : 0;
    } catch (...) {
        return PG_ENOMEM;
    }
}

pg_appns* pg_appns_new(void) {
    try {
        return new pg_appns();
    } catch (...) {
        return nullptr;
    }
}
void pg_appns_free(pg_appns* a) { delete a; }
int pg_appns_set(pg_appns* a, const char* ns, const char* name, uint32_t ns_index) {
    if (!a || !ns || !name) return PG_EINVAL;
    a->m.by_pod[PodID{ns, name}] = ns_index;
    return PG_OK;
}

int pg_export_session_rules(const pg_appns* a, const pg_contiv_rule* rules, size_t n, const char* pod_namespace,
                            const char* pod_name, const pg_ipnet* pod_ip, pg_session_rule* out, size_t cap) {
    if (!a || (n && !rules)) return PG_EINVAL;
    try {
        std::vector<ContivRule> v;
        for (size_t i = 0; i < n; i++) v.push_back(to_rule(rules[i]));
        PodID pod{sv(pod_namespace), sv(pod_name)};
        Bytes ip;
        if (pod_ip) ip = to_ipnet(*pod_ip).ip;
        return copy_out(export_session_rules(v, pod_name ? &pod : nullptr, ip, a->m), out, cap);
    } catch (...) {
        return PG_ENOMEM;
    }
}

pg_vpptcp_renderer* pg_vpptcp_renderer_new(pg_session_rules* vpp, const pg_appns* ipv4net, int chan_buf_size) {
    if (!vpp || !ipv4net) return nullptr;
    try {
        auto* r = new pg_vpptcp_renderer();
        r->r = std::make_unique<VppTcpRenderer>(&ipv4net->m, &vpp->t, chan_buf_size);
        return r;
    } catch (...) {
        return nullptr;
    }
}
void pg_vpptcp_renderer_free(pg_vpptcp_renderer* r) { delete r; }
const char* pg_vpptcp_last_error(const pg_vpptcp_renderer* r) { return r ? r->last_error.c_str() : "null renderer"; }

pg_vpptcp_txn* pg_vpptcp_new_txn(pg_vpptcp_renderer* r, int resync) {
    if (!r) return nullptr;
    try {
        auto* t = new pg_vpptcp_txn();
        t->r = r;
        t->t = std::make_unique<VppTcpRendererTxn>(r->r.get(), resync != 0);
        return t;
    } catch (...) {
        return nullptr;
    }
}
int pg_vpptcp_txn_render(pg_vpptcp_txn* t, const char* pod_namespace, const char* pod_name, const pg_ipnet* pod_ip,
                         const pg_contiv_rule* ingress, size_t n_ingress, const pg_contiv_rule* egress,
                         size_t n_egress, int removed) {
    if (!t || !pod_namespace || !pod_name || (n_ingress && !ingress) || (n_egress && !egress)) return PG_EINVAL;
    try {
        std::vector<ContivRule> in, eg;
        for (size_t i = 0; i < n_ingress; i++) in.push_back(to_rule(ingress[i]));
        for (size_t i = 0; i < n_egress; i++) eg.push_back(to_rule(egress[i]));
        IPNet ip;
        if (pod_ip) ip = to_ipnet(*pod_ip);
        t->t->render(PodID{pod_namespace, pod_name}, pod_ip ? &ip : nullptr, in, eg, removed != 0);
        return PG_OK;
    } catch (...) {
        return PG_ENOMEM;
    }
}
int pg_vpptcp_txn_commit(pg_vpptcp_txn* t) {
    if (!t) return PG_EINVAL;
    pg_vpptcp_renderer* r = t->r;
    int rc = PG_OK;
    try {
        std::string err = t->t->commit();
        r->last_error = err;
        if (!err.empty()) rc = PG_EFAULT;
    } catch (const std::exception& e) {
        r->last_error = e.what();
        rc = PG_ENOMEM;
    }
    delete t;
    return rc;
}
void pg_vpptcp_txn_free(pg_vpptcp_txn* t) { delete t; }

int pg_session_table_install(pg_ctx* ctx, const pg_session_rules* s, int scope, uint32_t ns_index,
                             const char* acl_name) {
    if (!ctx || !s || !acl_name || !*acl_name) return PG_EINVAL;
    if (scope != kScopeLocal && scope != kScopeGlobal) return PG_EINVAL;
    try {
        const std::vector<SessionRule>* t = s->t.table(scope, ns_index);
        const std::vector<SessionRule> none;
        std::string err;
        ACLPtr acl = session_table_acl(t ? *t : none, scope, acl_name, &err);
        if (!acl) {
            ctx->eng.last_error = err;
            return PG_EINVAL;
        }
        AclOps ops;
        ops[acl_name] = acl;
        err = ctx->eng.apply_txn(false, ops);
        if (!err.empty()) {
            ctx->eng.last_error = err;
            return PG_EFAULT;
        }
        return PG_OK;
    } catch (const std::exception& e) {
        ctx->eng.last_error = e.what();
        return PG_ENOMEM;
    }
}

int pg_configurator_register_vpptcp(pg_configurator* c, pg_vpptcp_renderer* r) {
    if (!c || !r) return PG_EINVAL;
    c->c.renderers.push_back(r->r.get());
    return PG_OK;
}

}  // extern "C"
