// The policy processor (see processor.hpp for the reference map).
#include "processor.hpp"

#include <algorithm>
#include <set>

#include "gonet.hpp"

namespace pg {

namespace {

const K8sLabelSelector kNoSelector;

// match_label_selector.go:276-296
bool is_match_label(const std::vector<K8sLabel>& labels, const std::set<std::string>& exists,
                    const std::string& prefix) {
    for (auto& l : labels)
        if (!exists.count(prefix + l.key + "/" + l.value)) return false;
    return true;
}

// match_label_selector.go:298-323 (the IN / NOT_IN keys lack the '/' between key and value)
bool is_match_expression(const std::vector<K8sLabelExpr>& exprs, const std::set<std::string>& exists,
                         const std::string& prefix) {
    bool match = false;
    for (auto& x : exprs) {
        switch (x.op) {
            case kOpIn:
                for (auto& v : x.values) {
                    match = exists.count(prefix + x.key + v) != 0;
                    if (match) break;
                }
                if (!match) return false;
                break;
            case kOpNotIn:
                for (auto& v : x.values)
                    if (exists.count(prefix + x.key + v)) return false;
                match = true;
                break;
            case kOpExists:
                if (!exists.count(prefix + x.key)) return false;
                match = true;
                break;
            case kOpDoesNotExist:
                if (exists.count(prefix + x.key)) return false;
                match = true;
                break;
            default:
                break;
        }
    }
    return match;
}

// the common shape of is{Pod,Ns,NsUpdate}LabelSelectorMatch
template <class L, class E>
bool selector_match(const K8sLabelSelector& sel, L label_match, E expr_match) {
    const bool hl = !sel.match_label.empty(), he = !sel.match_expression.empty();
    if (hl && he) return label_match() && expr_match();
    if (he) return expr_match();
    if (hl) return label_match();
    return true;
}

std::vector<const K8sPolicy*> all_policies(const PolicyCache& c) {
    std::vector<const K8sPolicy*> out;
    for (auto& kv : c.policies.items)
        if (kv.second.obj) out.push_back(kv.second.obj.get());
    return out;
}

std::vector<const K8sPolicy*> sorted_unique(std::map<std::string, const K8sPolicy*>& m) {
    std::vector<const K8sPolicy*> out;
    for (auto& kv : m) out.push_back(kv.second);
    return out;
}

}  // namespace

PolicyProcessor::PolicyProcessor(PolicyCache* c, PolicyConfigurator* cfg, const IPNet& subnet)
    : cache(c), configurator(cfg), pod_subnet_this_node(subnet) {
    cache->watchers.push_back(this);  // processor.go:61-66 (Init: Cache.Watch)
    PolicyCache* pc = cache;
    configurator->lookup_pod = [pc](const PodID& pod, std::string* ip) {  // the configurator's Cache.LookupPod
        bool found;
        const K8sPod* p = pc->lookup_pod(pod.str(), &found);
        if (!found) return false;
        *ip = p ? p->ip : std::string();
        return true;
    };
}

PolicyProcessor::~PolicyProcessor() {
    auto& w = cache->watchers;
    w.erase(std::remove(w.begin(), w.end(), static_cast<PolicyCacheWatcher*>(this)), w.end());
    configurator->lookup_pod = nullptr;
}

std::vector<std::string> PolicyProcessor::filter_host_pods(const std::vector<std::string>& pods) const {
    std::vector<std::string> out;  // processor.go:343-367
    for (auto& id : pods) {
        bool found;
        const K8sPod* p = cache->lookup_pod(id, &found);
        Bytes ip;
        if (!found || !p || p->ip.empty()) {
            auto it = pod_ip_address_map.find(id);
            if (it == pod_ip_address_map.end()) continue;
            ip = it->second;
        } else if (!parse_ip(p->ip, &ip)) {
            ip = Bytes();
        }
        if (!contains(pod_subnet_this_node, ip)) continue;
        out.push_back(id);
    }
    return out;
}

std::vector<std::string> PolicyProcessor::pods_assigned_to_policy(const K8sPolicy& policy) const {
    return cache->lookup_pods_by_label_selector_inside_ns(policy.ns, policy.pods ? *policy.pods : kNoSelector);
}

std::vector<CfgMatch> PolicyProcessor::calculate_matches(const K8sPolicy& policy, const std::string& pod_id,
                                                         std::string* err) const {
    std::vector<CfgMatch> matches;  // matches_calculator.go:14-191
    auto to_pods = [](const Names& ids, std::vector<PodID>* out) {
        for (auto& id : ids) {
            std::string ns, name;
            if (unstring_id(id, &ns, &name)) out->push_back(PodID{ns, name});
        }
    };
    auto port_of = [](const K8sPolicyPort& rp, int32_t number) {
        CfgPort p;
        p.protocol = rp.protocol == 1 ? kPortUDP : kPortTCP;
        p.number = (uint16_t)number;
        return p;
    };
    auto parse_block = [&](const K8sIPBlock& b, CfgIPBlock* out) {
        if (!parse_cidr(b.cidr, &out->network)) {
            *err = "invalid IPBlock CIDR " + b.cidr;
            return false;
        }
        for (auto& e : b.except) {
            IPNet n;
            if (!parse_cidr(e, &n)) {
                *err = "invalid IPBlock except " + e;
                return false;
            }
            out->except.push_back(n);
        }
        return true;
    };
    for (int dir = 0; dir < 2; dir++) {
        const auto& rules = dir == 0 ? policy.ingress : policy.egress;
        for (const K8sPolicyRule& rule : rules) {
            CfgMatch m;
            m.type = dir == 0 ? kMatchIngress : kMatchEgress;
            m.pods_nil = m.blocks_nil = rule.peers.empty();  // no peers: match anything on L3
            for (const K8sPeer& peer : rule.peers) {
                if (peer.pods) to_pods(cache->lookup_pods_by_label_selector_inside_ns(policy.ns, *peer.pods), &m.pods);
                if (peer.namespaces) to_pods(cache->lookup_pods_by_ns_label_selector(*peer.namespaces), &m.pods);
                if (!peer.ip_block) continue;
                CfgIPBlock b;
                if (!parse_block(*peer.ip_block, &b)) return {};
                m.blocks.push_back(b);
            }
            for (const K8sPolicyPort& rp : rule.ports) {
                if (rp.type == kPortNumber) {
                    m.ports.push_back(port_of(rp, rp.number));
                    continue;
                }
                if (dir == 0) {  // named ingress port: the target pod's container port of that name
                    bool found;
                    const K8sPod* pd = cache->lookup_pod(pod_id, &found);
                    if (!pd) continue;
                    for (auto& c : pd->containers)
                        for (auto& cp : c.ports)
                            if (cp.name == rp.name) m.ports.push_back(port_of(rp, cp.container_port));
                    continue;
                }
                // named egress port (portNameToNumber, matches_calculator.go:193-221): one match
                // per peer pod exposing it, ahead of the rule's own match
                std::vector<PodID> targets = m.pods;
                if (targets.empty()) to_pods(cache->list_all_pods(), &targets);
                for (const PodID& t : targets) {
                    bool found;
                    const K8sPod* pd = cache->lookup_pod(t.str(), &found);
                    if (!pd) continue;
                    for (auto& c : pd->containers)
                        for (auto& cp : c.ports)
                            if (cp.name == rp.name) {
                                CfgMatch pm;
                                pm.type = kMatchEgress;
                                pm.pods_nil = false;
                                pm.pods = {t};
                                pm.blocks_nil = false;
                                pm.ports = {port_of(rp, cp.container_port)};
                                matches.push_back(pm);
                            }
                }
            }
            matches.push_back(std::move(m));
        }
    }
    return matches;
}

std::string PolicyProcessor::process(bool resync, std::vector<std::string> pods) {
    // processor.go:73-149; RemoveDuplicatePodIDs
    {
        std::set<PodID> uniq;
        for (auto& id : pods) {
            std::string ns, name;
            if (unstring_id(id, &ns, &name)) uniq.insert(PodID{ns, name});
        }
        pods.clear();
        for (auto& p : uniq) pods.push_back(p.str());
    }
    pods = filter_host_pods(pods);
    if (pods.empty()) return "";
    PolicyConfiguratorTxn txn(configurator, resync);
    std::map<std::string, std::shared_ptr<const CfgPolicy>> processed;
    for (const std::string& pod : pods) {
        std::string ns, name;
        unstring_id(pod, &ns, &name);
        const PodID pid{ns, name};
        CfgPolicies list;
        for (const std::string& pol_id : cache->lookup_policies_by_pod(pod)) {
            auto it = processed.find(pol_id);
            if (it == processed.end()) {
                bool found;
                const K8sPolicy* pd = cache->lookup_policy(pol_id, &found);
                if (!found || !pd) continue;
                auto cp = std::make_shared<CfgPolicy>();
                cp->id = PodID{pd->ns, pd->name};
                switch (pd->policy_type) {
                    case kK8sEgress: cp->type = kPolicyEgress; break;
                    case kK8sIngressAndEgress: cp->type = kPolicyAll; break;
                    default: cp->type = kPolicyIngress; break;  // INGRESS and DEFAULT
                }
                std::string err;
                cp->matches = calculate_matches(*pd, pod, &err);
                if (!err.empty()) return err;
                it = processed.emplace(pol_id, cp).first;
            }
            list.push_back(it->second);
        }
        txn.configure(pid, std::move(list));
    }
    return txn.commit();
}

std::vector<const K8sPolicy*> PolicyProcessor::policies_referencing_pod(const K8sPod& pod) const {
    // processor.go:375-451 with match_label_selector.go:33-130
    std::set<std::string> pod_label_exists;  // isPodLabelMatch (namespace and key not separated)
    std::set<std::string> pod_expr_exists;   // isPodExpressionMatch
    for (auto& l : pod.labels) {
        pod_label_exists.insert(pod.ns + l.key + "/" + l.value);
        pod_expr_exists.insert(pod.ns + "/" + l.key + "/" + l.value);
        pod_expr_exists.insert(pod.ns + "/" + l.key);
    }
    std::set<std::string> ns_label_exists, ns_expr_exists;
    bool found;
    if (const K8sNamespace* nd = cache->lookup_namespace(pod.ns, &found))
        for (auto& l : nd->labels) {
            ns_label_exists.insert(l.key + "/" + l.value);
            ns_expr_exists.insert(l.key + "/" + l.value);
            ns_expr_exists.insert(l.key);
        }
    std::map<std::string, const K8sPolicy*> out;
    for (const K8sPolicy* p : all_policies(*cache)) {
        const std::string id = policy_key(*p);
        const std::string prefix = p->ns + "/";
        for (int dir = 0; dir < 2; dir++) {
            const auto& rules = dir == 0 ? p->ingress : p->egress;
            if (rules.empty()) {
                out[id] = p;
                continue;
            }
            for (auto& r : rules)
                for (auto& peer : r.peers) {
                    if (peer.pods) {
                        if (selector_match(
                                *peer.pods,
                                [&] { return is_match_label(peer.pods->match_label, pod_label_exists, prefix); },
                                [&] { return is_match_expression(peer.pods->match_expression, pod_expr_exists, prefix); }))
                            out[id] = p;
                    } else if (peer.namespaces) {
                        if (selector_match(
                                *peer.namespaces,
                                [&] { return is_match_label(peer.namespaces->match_label, ns_label_exists, ""); },
                                [&] { return is_match_expression(peer.namespaces->match_expression, ns_expr_exists, ""); }))
                            out[id] = p;
                    }
                }
        }
    }
    return sorted_unique(out);
}

std::vector<const K8sPolicy*> PolicyProcessor::policies_referencing_namespace(const K8sNamespace& ns) const {
    // processor.go:453-527 with match_label_selector.go:216-274 (the namespace as now cached)
    std::set<std::string> label_exists, expr_exists;
    bool found;
    if (const K8sNamespace* nd = cache->lookup_namespace(ns.name, &found))
        for (auto& l : nd->labels) {
            label_exists.insert(l.key + "/" + l.value);
            expr_exists.insert(l.key + "/" + l.value);
            expr_exists.insert(l.key);
        }
    std::map<std::string, const K8sPolicy*> out;
    for (const K8sPolicy* p : all_policies(*cache)) {
        const std::string id = policy_key(*p);
        for (int dir = 0; dir < 2; dir++) {
            const auto& rules = dir == 0 ? p->ingress : p->egress;
            if (rules.empty()) {
                out[id] = p;
                continue;
            }
            for (auto& r : rules)
                for (auto& peer : r.peers)
                    if (peer.namespaces &&
                        selector_match(
                            *peer.namespaces,
                            [&] { return is_match_label(peer.namespaces->match_label, label_exists, ""); },
                            [&] { return is_match_expression(peer.namespaces->match_expression, expr_exists, ""); }))
                        out[id] = p;
        }
    }
    return sorted_unique(out);
}

// ---- cache events (processor.go:151-316) ----------------------------------------------------
std::string PolicyProcessor::resync(const ResyncData& data) {
    pod_ip_address_map.clear();
    for (auto& p : data.pods) {
        if (p->ip.empty()) continue;
        Bytes ip;
        if (!parse_ip(p->ip, &ip)) ip = Bytes();
        pod_ip_address_map[pod_key(*p)] = ip;
    }
    return process(true, cache->list_all_pods());
}

std::string PolicyProcessor::add_pod(const std::string& id, const K8sPod& pod) {
    if (pod.ip.empty()) return "";  // no IP address assigned yet
    Bytes ip;
    if (!parse_ip(pod.ip, &ip)) ip = Bytes();
    pod_ip_address_map[id] = ip;
    std::vector<std::string> pods;
    for (const K8sPolicy* p : policies_referencing_pod(pod)) {
        auto v = pods_assigned_to_policy(*p);
        pods.insert(pods.end(), v.begin(), v.end());
    }
    pods.push_back(id);
    return process(false, pods);
}

std::string PolicyProcessor::del_pod(const std::string& id, const K8sPod& pod) {
    std::vector<std::string> pods;
    for (const K8sPolicy* p : policies_referencing_pod(pod)) {
        auto v = pods_assigned_to_policy(*p);
        pods.insert(pods.end(), v.begin(), v.end());
    }
    pods.push_back(id);
    std::string err = process(false, pods);
    pod_ip_address_map.erase(id);
    return err;
}

std::string PolicyProcessor::update_pod(const std::string& id, const K8sPod& old_pod, const K8sPod& new_pod) {
    if (!new_pod.ip.empty()) {
        Bytes ip;
        if (!parse_ip(new_pod.ip, &ip)) ip = Bytes();
        pod_ip_address_map[id] = ip;
    } else if (old_pod.ip.empty()) {
        return "";  // still no IP address
    }
    std::vector<std::string> pods;
    for (const K8sPod* pod : {&old_pod, &new_pod}) {
        if (pod->ip.empty()) continue;
        for (const K8sPolicy* p : policies_referencing_pod(*pod)) {
            auto v = pods_assigned_to_policy(*p);
            pods.insert(pods.end(), v.begin(), v.end());
        }
    }
    if (new_pod.ip != old_pod.ip) pods.push_back(id);
    return process(false, pods);
}

std::string PolicyProcessor::add_policy(const K8sPolicy& p) { return process(false, pods_assigned_to_policy(p)); }
std::string PolicyProcessor::del_policy(const K8sPolicy& p) { return process(false, pods_assigned_to_policy(p)); }

std::string PolicyProcessor::update_policy(const K8sPolicy& old_p, const K8sPolicy& new_p) {
    std::vector<std::string> pods = pods_assigned_to_policy(old_p);
    auto v = pods_assigned_to_policy(new_p);
    pods.insert(pods.end(), v.begin(), v.end());
    return process(false, pods);
}

std::string PolicyProcessor::update_namespace(const K8sNamespace& old_ns, const K8sNamespace& new_ns) {
    std::vector<std::string> pods;
    for (const K8sNamespace* ns : {&old_ns, &new_ns})
        for (const K8sPolicy* p : policies_referencing_namespace(*ns)) {
            auto v = pods_assigned_to_policy(*p);
            pods.insert(pods.end(), v.begin(), v.end());
        }
    return process(false, pods);
}

}  // namespace pg
