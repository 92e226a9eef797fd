// Policy configurator + mock renderer (see configurator.hpp for the reference map).
#include "configurator.hpp"

#include <algorithm>

namespace pg {

bool ContivRules::insert(const ContivRule& r) {  // configurator_impl.go:520-540
    if (!ordered.insert(r).second) return false;  // Compare == 0 with a rule already in
    rules.push_back(r);
    return true;
}

IPNet one_host_subnet(const Bytes& ip) {  // utils.go:283-291
    IPNet n;
    n.ip = ip;
    Bytes v4;
    n.mask = to4(ip, &v4) ? cidr_mask(32, 32) : cidr_mask(128, 128);
    return n;
}

std::vector<IPNet> subtract_subnet(const IPNet& net1, const IPNet& net2) {  // configurator_impl.go:562-594
    std::vector<IPNet> out;
    int ones1 = 0, ones2 = 0, bits = 0;
    mask_size(net1.mask, &ones1, &bits);
    mask_size(net2.mask, &ones2, &bits);
    if (ones1 > ones2) {  // net2 higher than net1 in the tree
        if (!contains(net2, net1.ip)) out.push_back(net1);
    } else if (ones1 == ones2) {  // same level
        if (!ip_equal(net1.ip, net2.ip)) out.push_back(net1);
    } else if (!contains(net1, net2.ip)) {
        out.push_back(net1);
    } else {  // net2 under net1: the siblings of every node on the path down to net2
        for (int bit = ones1; bit < ones2; bit++) {
            IPNet s;
            s.mask = cidr_mask(bit + 1, net2.mask.len * 8);
            if (!ip_mask(net2.ip, s.mask, &s.ip)) continue;  // (Go would index a nil IP)
            s.ip.b[bit / 8] ^= (uint8_t)(1u << (7 - bit % 8));
            out.push_back(s);
        }
    }
    return out;
}

// ---- mock renderer (renderer_mock.go) -------------------------------------------------
namespace {
struct MockTxn : CfgRendererTxn {
    MockRenderer* r;
    bool resync;
    std::map<PodID, MockRenderer::Cfg> config;
    MockTxn(MockRenderer* rr, bool rs) : r(rr), resync(rs) {}
    void render(const PodID& pod, const IPNet* pod_ip, const std::vector<ContivRule>& ingress,
                const std::vector<ContivRule>& egress, bool removed) override {  // :150-166
        if (removed) {
            config.erase(pod);
            return;
        }
        MockRenderer::Cfg c;
        c.has_ip = pod_ip != nullptr;
        if (pod_ip) c.ip = *pod_ip;
        c.ingress = ingress;
        c.egress = egress;
        config[pod] = std::move(c);
    }
    std::string commit() override {  // :169-185
        if (resync) {
            r->config = config;
        } else {
            for (auto& kv : config) r->config[kv.first] = kv.second;
        }
        return "";
    }
};
}  // namespace

std::unique_ptr<CfgRendererTxn> MockRenderer::new_txn(bool resync) { return std::make_unique<MockTxn>(this, resync); }

int MockRenderer::test_traffic(const PodID& pod, int direction, const Bytes& src, const Bytes& dst, int protocol,
                               uint16_t src_port, uint16_t dst_port) const {  // :105-147
    auto it = config.find(pod);
    if (it == config.end()) return kUnmatchedTraffic;
    const auto& rules = direction == kIngressTraffic ? it->second.ingress : it->second.egress;
    for (const ContivRule& r : rules) {
        if (r.src.ip.len > 0 && !contains(r.src, src)) continue;
        if (r.dst.ip.len > 0 && !contains(r.dst, dst)) continue;
        if (r.protocol != kANY) {
            if (r.protocol != protocol) continue;
            if (r.src_port != 0 && r.src_port != src_port) continue;
            if (r.dst_port != 0 && r.dst_port != dst_port) continue;
        }
        return r.action == kPermit ? kAllowedTraffic : kDeniedTraffic;
    }
    return kUnmatchedTraffic;
}

ACLPtr MockRenderer::traffic_acl(const PodID& pod, int direction, const std::string& name, std::string* err,
                                 bool* missing) const {
    *missing = false;
    auto it = config.find(pod);
    if (it == config.end()) {
        *missing = true;
        *err = "pod not rendered";
        return nullptr;
    }
    auto acl = std::make_shared<ACL>();
    acl->name = name;
    acl->ingress = {name};
    for (const ContivRule& r : direction == kIngressTraffic ? it->second.ingress : it->second.egress) {
        if (r.protocol == kOTHER || (r.protocol != kANY && r.src_port != 0)) {
            *err = "rule with protocol OTHER or a source port";
            return nullptr;
        }
        AclRule a;
        a.action = r.action == kPermit ? kAclPermit : kAclDeny;
        if (r.src.ip.len > 0) a.src_network = ipnet_string(r.src);
        if (r.dst.ip.len > 0) a.dst_network = ipnet_string(r.dst);
        if (r.protocol == kTCP || r.protocol == kUDP) {
            L4Section& l4 = r.protocol == kTCP ? a.tcp : a.udp;
            l4.present = l4.has_src = l4.has_dst = true;
            l4.src = PortRange{0, 0xFFFF};
            l4.dst = r.dst_port ? PortRange{r.dst_port, r.dst_port} : PortRange{0, 0xFFFF};
        }
        acl->rules.push_back(a);
    }
    return acl;
}

// ---- configurator ---------------------------------------------------------------------
PolicyConfiguratorTxn::PolicyConfiguratorTxn(PolicyConfigurator* c, bool rs) : cfg(c), resync(rs) {
    if (!resync) pod_ip_addresses = cfg->pod_ip_addresses;  // configurator_impl.go:119-124
}

namespace {
ContivRule permit_any() {
    ContivRule r;
    r.action = kPermit;
    r.protocol = kANY;
    return r;
}
int l4_proto(int port_proto) { return port_proto == kPortTCP ? kTCP : kUDP; }
}  // namespace

// configurator_impl.go:263-472
ContivRules PolicyConfiguratorTxn::generate_rules(int direction, const CfgPolicies& policies) const {
    ContivRules rules;
    bool has_policy = false, all_allowed = false;
    for (const auto& policy : policies) {
        if ((policy->type == kPolicyIngress && direction == kMatchEgress) ||
            (policy->type == kPolicyEgress && direction == kMatchIngress))
            continue;  // the policy does not apply to this direction
        has_policy = true;
        for (const CfgMatch& match : policy->matches) {
            if (match.type != direction) continue;
            // IPs of the pod peers known to the cache
            std::vector<IPNet> peers;
            for (const PodID& peer : match.pods) {
                std::string pd;
                if (!cfg->pod_ip(peer, &pd) || pd.empty()) continue;
                Bytes ip;
                if (!parse_ip(pd, &ip)) continue;
                peers.push_back(one_host_subnet(ip));
            }
            // IPBlocks minus their excepts
            std::vector<IPNet> all_subnets;
            for (const CfgIPBlock& block : match.blocks) {
                std::vector<IPNet> subnets{block.network};
                for (const IPNet& except : block.except) {
                    std::vector<IPNet> sub;
                    for (const IPNet& s : subnets) {
                        auto part = subtract_subnet(s, except);
                        sub.insert(sub.end(), part.begin(), part.end());
                    }
                    subnets.swap(sub);
                }
                all_subnets.insert(all_subnets.end(), subnets.begin(), subnets.end());
            }
            auto with_peer = [&](ContivRule r, const IPNet& n) {
                if (direction == kMatchIngress) r.src = n;
                else r.dst = n;
                return r;
            };
            // no pods and no blocks: anything on L3
            if (match.pods_nil && match.blocks_nil) {
                if (match.ports.empty()) {
                    rules.insert(permit_any());
                    all_allowed = true;
                } else {
                    for (const CfgPort& p : match.ports) {
                        ContivRule r = permit_any();
                        r.protocol = l4_proto(p.protocol);
                        r.dst_port = p.number;
                        rules.insert(r);
                    }
                }
            }
            for (const std::vector<IPNet>* nets : {&peers, &all_subnets}) {
                for (const IPNet& n : *nets) {
                    if (match.ports.empty()) {
                        rules.insert(with_peer(permit_any(), n));
                        continue;
                    }
                    for (const CfgPort& p : match.ports) {
                        ContivRule r = permit_any();
                        r.protocol = l4_proto(p.protocol);
                        r.dst_port = p.number;
                        rules.insert(with_peer(r, n));
                    }
                }
            }
        }
    }
    if (has_policy && !all_allowed) {
        if (direction == kMatchIngress) {  // access to a service from the pod itself (NAT loopback)
            ContivRule r = permit_any();
            r.src = one_host_subnet(cfg->nat_loopback);
            rules.insert(r);
        }
        ContivRule deny = permit_any();  // deny the rest
        deny.action = kDeny;
        rules.insert(deny);
    }
    return rules;
}

// configurator_impl.go:138-254
std::string PolicyConfiguratorTxn::commit() {
    struct Processed {
        CfgPolicies policies;
        ContivRules ingress, egress;
    };
    std::vector<Processed> processed;
    std::vector<std::unique_ptr<CfgRendererTxn>> txns;
    for (auto& kv : config) {
        const PodID& pod = kv.first;
        ContivRules ingress, egress;
        bool del = false;
        auto had = pod_ip_addresses.find(pod);
        const bool had_ip = had != pod_ip_addresses.end();
        IPNet pod_ip = had_ip ? had->second : IPNet();
        std::string pd;
        if (!cfg->pod_ip(pod, &pd) || pd.empty()) {  // removed pod
            if (!had_ip) continue;                              // already un-configured
            del = true;
            pod_ip_addresses.erase(pod);
        }
        if (!del) {
            Bytes ip;
            if (!parse_ip(pd, &ip)) continue;  // invalid IP address: skipped
            pod_ip = one_host_subnet(ip);
            pod_ip_addresses[pod] = pod_ip;
            CfgPolicies policies = kv.second;  // sorted by ID: the same set gives the same outcome
            std::sort(policies.begin(), policies.end(), [](const auto& a, const auto& b) { return a->id < b->id; });
            auto same = [&](const CfgPolicies& o) {
                if (o.size() != policies.size()) return false;
                for (size_t i = 0; i < o.size(); i++)
                    if (!(o[i]->id == policies[i]->id)) return false;
                return true;
            };
            bool done = false;
            for (const Processed& p : processed) {
                if (same(p.policies)) {
                    ingress = p.ingress, egress = p.egress;
                    done = true;
                }
            }
            if (!done) {
                // policy directions are from the pod's point of view, rules from the vswitch's
                egress = generate_rules(kMatchIngress, policies);
                ingress = generate_rules(kMatchEgress, policies);
                processed.push_back({policies, ingress, egress});
            }
        }
        if (txns.empty())
            for (CfgRenderer* r : cfg->renderers) txns.push_back(r->new_txn(resync));
        for (auto& t : txns) t->render(pod, &pod_ip, ingress.rules, egress.rules, del);
    }
    std::string err;
    for (auto& t : txns) {
        std::string e = t->commit();
        if (!e.empty()) err = e;
    }
    cfg->pod_ip_addresses = pod_ip_addresses;
    return err;
}

}  // namespace pg
