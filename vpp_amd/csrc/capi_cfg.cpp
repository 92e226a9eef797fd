// extern "C" boundary of the policy configurator and the mock renderer
// (include/policygpu.h "policy configurator"; configurator.hpp for the reference map).
#include <cstring>
#include <stdexcept>

#include "capi_internal.hpp"

using namespace pg;

namespace {

// the GPU ACL renderer behind the configurator's renderer interface
struct AclRendererTxnAdapter : CfgRendererTxn {
    RendererTxn t;
    AclRendererTxnAdapter(Renderer* r, bool resync) : t(r, resync) {}
    void render(const PodID& pod, const IPNet* pod_ip, const std::vector<ContivRule>& ingress,
                const std::vector<ContivRule>& egress, bool removed) override {
        t.render(pod, pod_ip, ingress, egress, removed);
    }
    std::string commit() override { return t.commit(); }
};
struct AclRendererAdapter : CfgRenderer {
    Renderer* r;
    explicit AclRendererAdapter(Renderer* rr) : r(rr) {}
    std::unique_ptr<CfgRendererTxn> new_txn(bool resync) override {
        return std::make_unique<AclRendererTxnAdapter>(r, resync);
    }
};

std::string sv(const char* s) { return s ? std::string(s) : std::string(); }

int cfg_fail(pg_configurator* c, int code, const std::string& msg) {
    if (c) c->last_error = msg;
    return code;
}

CfgPolicy to_policy(const pg_policy& p) {
    CfgPolicy r;
    r.id = PodID{sv(p.id.ns), sv(p.id.name)};
    r.type = p.type;
    for (size_t m = 0; m < p.n_matches; m++) {
        const pg_match& x = p.matches[m];
        CfgMatch cm;
        cm.type = x.type;
        cm.pods_nil = x.pods_nil != 0;
        for (size_t i = 0; i < x.n_pods; i++) cm.pods.push_back(PodID{sv(x.pods[i].ns), sv(x.pods[i].name)});
        cm.blocks_nil = x.blocks_nil != 0;
        for (size_t i = 0; i < x.n_blocks; i++) {
            CfgIPBlock b;
            b.network = to_ipnet(x.blocks[i].network);
            for (size_t k = 0; k < x.blocks[i].n_except; k++) b.except.push_back(to_ipnet(x.blocks[i].except[k]));
            cm.blocks.push_back(std::move(b));
        }
        for (size_t i = 0; i < x.n_ports; i++) cm.ports.push_back(CfgPort{x.ports[i].protocol, x.ports[i].number});
        r.matches.push_back(std::move(cm));
    }
    return r;
}

}  // namespace

extern "C" {

pg_configurator* pg_configurator_new(void) { return new (std::nothrow) pg_configurator(); }
void pg_configurator_free(pg_configurator* c) { delete c; }
const char* pg_configurator_last_error(const pg_configurator* c) { return c ? c->last_error.c_str() : "null"; }

int pg_configurator_register_renderer(pg_configurator* c, pg_renderer* r) {
    if (!c || !r) return PG_EINVAL;
    c->adapters.push_back(std::make_unique<AclRendererAdapter>(r->r.get()));
    c->c.renderers.push_back(c->adapters.back().get());
    return PG_OK;
}
int pg_configurator_register_mock(pg_configurator* c, pg_mock_renderer* r) {
    if (!c || !r) return PG_EINVAL;
    c->c.renderers.push_back(&r->r);
    return PG_OK;
}
int pg_configurator_set_pod(pg_configurator* c, const char* ns, const char* name, const char* ip) {
    if (!c || !ns || !name) return PG_EINVAL;
    const PodID id{ns, name};
    if (ip) c->c.pod_data[id] = ip;
    else c->c.pod_data.erase(id);
    return PG_OK;
}
int pg_configurator_set_nat_loopback(pg_configurator* c, const char* ip) {
    if (!c) return PG_EINVAL;
    Bytes b;
    c->c.nat_loopback = (ip && parse_ip(ip, &b)) ? b : Bytes();
    return PG_OK;
}
pg_cfg_txn* pg_configurator_new_txn(pg_configurator* c, int resync) {
    if (!c) return nullptr;
    auto* t = new (std::nothrow) pg_cfg_txn();
    if (!t) return nullptr;
    t->c = c;
    t->t.reset(new PolicyConfiguratorTxn(&c->c, resync != 0));
    return t;
}
int pg_cfg_txn_configure(pg_cfg_txn* t, const char* ns, const char* name, const pg_policy* policies, size_t n) {
    if (!t || !ns || !name || (n && !policies)) return PG_EINVAL;
    try {
        CfgPolicies ps;
        for (size_t i = 0; i < n; i++) ps.push_back(std::make_shared<const CfgPolicy>(to_policy(policies[i])));
        t->t->configure(PodID{ns, name}, std::move(ps));
    } catch (const std::exception& e) {
        return cfg_fail(t->c, PG_EFAULT, e.what());
    }
    return PG_OK;
}
int pg_cfg_txn_commit(pg_cfg_txn* t) {
    if (!t) return PG_EINVAL;
    int rc = PG_OK;
    try {
        std::string e = t->t->commit();
        if (!e.empty()) rc = cfg_fail(t->c, PG_EFAULT, e);
    } catch (const std::exception& ex) {
        rc = cfg_fail(t->c, PG_EFAULT, ex.what());
    }
    delete t;
    return rc;
}
void pg_cfg_txn_free(pg_cfg_txn* t) { delete t; }

pg_mock_renderer* pg_mock_renderer_new(void) { return new (std::nothrow) pg_mock_renderer(); }
void pg_mock_renderer_free(pg_mock_renderer* r) { delete r; }

int pg_mock_renderer_pod_ip(pg_mock_renderer* r, const char* ns, const char* name, char* ip, size_t cap,
                            int* masklen) {  // renderer_mock.go:85-101
    if (!r || !ns || !name) return PG_EINVAL;
    std::string s;
    int ones = 0, bits = 0;
    auto it = r->r.config.find(PodID{ns, name});
    if (it != r->r.config.end() && it->second.has_ip && it->second.ip.ip.len) {
        s = ip_string(it->second.ip.ip);
        mask_size(it->second.ip.mask, &ones, &bits);
    }
    if (masklen) *masklen = ones;
    if (ip && cap) {
        std::strncpy(ip, s.c_str(), cap - 1);
        ip[cap - 1] = 0;
    }
    return (int)s.size() + 1;
}
int pg_mock_renderer_rules(pg_mock_renderer* r, const char* ns, const char* name, int direction,
                           pg_contiv_rule* out, size_t cap) {
    if (!r || !ns || !name) return PG_EINVAL;
    auto it = r->r.config.find(PodID{ns, name});
    if (it == r->r.config.end()) return PG_ENOENT;
    const auto& rules = direction == kIngressTraffic ? it->second.ingress : it->second.egress;
    for (size_t i = 0; i < rules.size() && i < cap && out; i++) {
        pg_contiv_rule& o = out[i];
        o.action = rules[i].action;
        o.protocol = rules[i].protocol;
        o.src_port = rules[i].src_port;
        o.dst_port = rules[i].dst_port;
        o.src = to_pg_ipnet(rules[i].src);
        o.dst = to_pg_ipnet(rules[i].dst);
    }
    return (int)rules.size();
}
int pg_mock_renderer_test_traffic(pg_mock_renderer* r, const char* ns, const char* name, int direction,
                                  const char* src_ip, const char* dst_ip, int protocol, uint16_t src_port,
                                  uint16_t dst_port) {  // renderer_mock.go:105-147
    if (!r || !ns || !name || !src_ip || !dst_ip) return PG_EINVAL;
    Bytes s, d;  // net.ParseIP; an unparsable address is a nil IP (contained by nothing)
    if (!parse_ip(src_ip, &s)) s = Bytes();
    if (!parse_ip(dst_ip, &d)) d = Bytes();
    return r->r.test_traffic(PodID{ns, name}, direction, s, d, protocol, src_port, dst_port);
}

int pg_mock_renderer_install(pg_ctx* ctx, const pg_mock_renderer* r, const char* ns, const char* name, int direction,
                             const char* acl_name) {
    if (!ctx || !r || !ns || !name || !acl_name || !*acl_name) return PG_EINVAL;
    try {
        std::string err;
        bool missing = false;
        ACLPtr acl = r->r.traffic_acl(PodID{ns, name}, direction, acl_name, &err, &missing);
        if (!acl) {
            ctx->eng.last_error = err;
            return missing ? PG_ENOENT : PG_EINVAL;
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

}  // extern "C"
