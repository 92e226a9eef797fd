// K8s state as the policy plugin sees it: the KSR data model (pods,
// namespaces, network policies), decoded from their protobuf wire form, and the policy cache
// that indexes it and expands label / namespace selectors into pod sets.
//
// Reference (itaimlx/vpp):
//   ksr model            plugins/ksr/model/{pod/pod.proto, namespace/namespace.proto, policy/policy.proto}
//   PolicyCacheAPI       plugins/policy/cache/cache_api.go:30-116
//   PolicyCache          plugins/policy/cache/cache_impl.go:33-234
//   Update / Resync      plugins/policy/cache/data_change.go:24-148, data_resync.go:24-71
//   match labels         plugins/policy/cache/match_label.go:23-74
//   match expressions    plugins/policy/cache/match_expression.go:23-271
//   secondary indexes    plugins/policy/cache/{podidx/podmap.go, namespaceidx/namespacemap.go,
//                        policyidx/policymap.go} over cn-infra idxmap/mem (a named mapping whose
//                        ListNames(field, value) returns every name indexed under value)
//   set helpers          plugins/policy/utils/utils.go:33-160 (RemoveDuplicates, Intersect,
//                        Difference, Unstring*ID, ConstructLabels)
//
// Go map iteration order makes the reference's result lists unordered; here every lookup
// returns its names sorted, so the same state always gives the same answer.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <optional>
#include <set>
#include <string>
#include <vector>

namespace pg {

// ---- KSR model (field numbers = the .proto files) -------------------------------------------
struct K8sLabel {
    std::string key, value;
};
enum K8sOperator { kOpIn = 0, kOpNotIn = 1, kOpExists = 2, kOpDoesNotExist = 3 };
struct K8sLabelExpr {
    std::string key;
    int op = kOpIn;
    std::vector<std::string> values;
};
struct K8sLabelSelector {
    std::vector<K8sLabel> match_label;
    std::vector<K8sLabelExpr> match_expression;
};
struct K8sContainerPort {
    std::string name, host_ip;
    int32_t host_port = 0, container_port = 0;
    int protocol = 0;
};
struct K8sContainer {
    std::string name;
    std::vector<K8sContainerPort> ports;
};
struct K8sPod {
    std::string name, ns, ip, host_ip;
    std::vector<K8sLabel> labels;
    std::vector<K8sContainer> containers;
};
struct K8sNamespace {
    std::string name;
    std::vector<K8sLabel> labels;
};
enum K8sPolicyType { kK8sDefault = 0, kK8sIngress = 1, kK8sEgress = 2, kK8sIngressAndEgress = 3 };
enum K8sPortType { kPortNumber = 0, kPortName = 1 };
struct K8sPolicyPort {
    int protocol = 0;  // TCP 0, UDP 1
    int type = kPortNumber;
    int32_t number = 0;
    std::string name;
};
struct K8sIPBlock {
    std::string cidr;
    std::vector<std::string> except;
};
struct K8sPeer {
    std::optional<K8sLabelSelector> pods, namespaces;
    std::optional<K8sIPBlock> ip_block;
};
struct K8sPolicyRule {  // IngressRule (port, from) / EgressRule (port, to)
    std::vector<K8sPolicyPort> ports;
    std::vector<K8sPeer> peers;
};
struct K8sPolicy {
    std::string name, ns;
    std::vector<K8sLabel> labels;
    std::optional<K8sLabelSelector> pods;
    int policy_type = kK8sDefault;
    std::vector<K8sPolicyRule> ingress, egress;
};

// protobuf wire decoding (proto3; unknown fields skipped); false = malformed input
bool decode_pod(const uint8_t* p, size_t n, K8sPod* out);
bool decode_namespace(const uint8_t* p, size_t n, K8sNamespace* out);
bool decode_policy(const uint8_t* p, size_t n, K8sPolicy* out);
bool decode_label_selector(const uint8_t* p, size_t n, K8sLabelSelector* out);

using Names = std::vector<std::string>;

// utils.go set helpers with the reference's multiset semantics; results sorted
Names names_intersect(const Names& a, const Names& b);  // elements of b found in a
Names names_difference(const Names& a, const Names& b);  // count == 1 over {a as a set} + b
Names names_unique(Names v);

// cn-infra idxmap/mem named mapping: name -> (object, secondary index values per field)
template <class T>
struct NamedIndex {
    struct Entry {
        std::shared_ptr<const T> obj;  // null = registered as nil
        std::string raw;               // wire bytes as registered
        std::map<std::string, Names> fields;
    };
    std::map<std::string, Entry> items;
    std::map<std::string, std::map<std::string, std::set<std::string>>> index;  // field -> value -> names

    void put(const std::string& name, Entry e) {
        del(name);
        for (auto& f : e.fields)
            for (auto& v : f.second) index[f.first][v].insert(name);
        items[name] = std::move(e);
    }
    bool del(const std::string& name) {
        auto it = items.find(name);
        if (it == items.end()) return false;
        for (auto& f : it->second.fields)
            for (auto& v : f.second) {
                auto& m = index[f.first];
                auto s = m.find(v);
                if (s != m.end() && (s->second.erase(name), s->second.empty())) m.erase(s);
            }
        items.erase(it);
        return true;
    }
    const Entry* get(const std::string& name) const {
        auto it = items.find(name);
        return it == items.end() ? nullptr : &it->second;
    }
    Names list(const std::string& field, const std::string& value) const {
        auto f = index.find(field);
        if (f == index.end()) return {};
        auto v = f->second.find(value);
        return v == f->second.end() ? Names() : Names(v->second.begin(), v->second.end());
    }
    Names all() const {
        Names out;
        for (auto& kv : items) out.push_back(kv.first);
        return out;
    }
};

// Secondary index fields (podmap.go:29-35, namespacemap.go:27-30, policymap.go:27-32)
extern const char* const kPodLabel;     // "key/value"
extern const char* const kPodKey;       // "key"
extern const char* const kPodNSKey;     // "ns/key"
extern const char* const kPodNSLabel;   // "ns/key/value"
extern const char* const kPodNamespace; // "ns"
extern const char* const kNsLabel;      // "key/value"
extern const char* const kNsKey;        // "key"
extern const char* const kPolicyLabel;  // "key/value" of the policy's pod selector
extern const char* const kPolicyNSLabel;// "ns/key/value"

enum K8sKind { kK8sPod = 0, kK8sNamespace = 1, kK8sPolicy = 2 };

// data_resync.go DataResyncEvent
struct ResyncData {
    std::vector<std::shared_ptr<const K8sPod>> pods;
    std::vector<std::shared_ptr<const K8sNamespace>> namespaces;
    std::vector<std::shared_ptr<const K8sPolicy>> policies;
    std::vector<std::string> pod_raw, ns_raw, policy_raw;  // wire bytes (optional)
};

// cache_api.go:82-116 PolicyCacheWatcher; "" = ok
struct PolicyCacheWatcher {
    virtual ~PolicyCacheWatcher() = default;
    virtual std::string resync(const ResyncData& data) = 0;
    virtual std::string add_pod(const std::string& id, const K8sPod& pod) = 0;
    virtual std::string del_pod(const std::string& id, const K8sPod& pod) = 0;
    virtual std::string update_pod(const std::string& id, const K8sPod& old_pod, const K8sPod& new_pod) = 0;
    virtual std::string add_policy(const K8sPolicy& p) = 0;
    virtual std::string del_policy(const K8sPolicy& p) = 0;
    virtual std::string update_policy(const K8sPolicy& old_p, const K8sPolicy& new_p) = 0;
    virtual std::string add_namespace(const K8sNamespace& ns) = 0;
    virtual std::string del_namespace(const K8sNamespace& ns) = 0;
    virtual std::string update_namespace(const K8sNamespace& old_ns, const K8sNamespace& new_ns) = 0;
};

struct PolicyCache {
    NamedIndex<K8sPod> pods;
    NamedIndex<K8sNamespace> namespaces;
    NamedIndex<K8sPolicy> policies;
    std::vector<PolicyCacheWatcher*> watchers;

    // podidx / namespaceidx / policyidx Register* (index only, no watcher events)
    void register_pod(const std::string& id, std::shared_ptr<const K8sPod> pod, std::string raw = "");
    void register_namespace(const std::string& id, std::shared_ptr<const K8sNamespace> ns, std::string raw = "");
    void register_policy(const std::string& id, std::shared_ptr<const K8sPolicy> pol, std::string raw = "");
    void reset();

    // PolicyCacheAPI
    const K8sPod* lookup_pod(const std::string& pod_id, bool* found) const;
    const K8sPolicy* lookup_policy(const std::string& policy_id, bool* found) const;
    const K8sNamespace* lookup_namespace(const std::string& ns, bool* found) const;
    Names lookup_pods_by_label_selector_inside_ns(const std::string& ns, const K8sLabelSelector& sel) const;
    Names lookup_pods_by_ns_label_selector(const K8sLabelSelector& sel) const;
    Names lookup_pods_by_namespace(const std::string& ns) const { return pods.list(kPodNamespace, ns); }
    Names list_all_pods() const { return pods.all(); }
    Names lookup_policies_by_pod(const std::string& pod_id) const;
    Names list_all_policies() const { return policies.all(); }
    Names list_all_namespaces() const { return namespaces.all(); }

    // match_label.go / match_expression.go
    Names match_label_pods_inside_ns(const std::string& ns, const std::vector<K8sLabel>& labels) const;
    Names pods_by_ns_label_selector(const std::vector<K8sLabel>& labels) const;
    Names match_expression_pods_inside_ns(const std::string& ns, const std::vector<K8sLabelExpr>& exprs) const;
    Names pods_by_ns_match_expression(const std::vector<K8sLabelExpr>& exprs) const;

    // data_change.go: register the change (prev null = add, next null = delete), then notify
    // every watcher; "" = ok, else the first watcher error
    std::string update_pod(std::shared_ptr<const K8sPod> prev, std::shared_ptr<const K8sPod> next,
                           std::string raw = "");
    std::string update_namespace(std::shared_ptr<const K8sNamespace> prev, std::shared_ptr<const K8sNamespace> next,
                                 std::string raw = "");
    std::string update_policy(std::shared_ptr<const K8sPolicy> prev, std::shared_ptr<const K8sPolicy> next,
                              std::string raw = "");
    // data_resync.go: reset, register everything, then Resync every watcher
    std::string resync(const ResyncData& data);
};

inline std::string pod_key(const K8sPod& p) { return p.ns + "/" + p.name; }
inline std::string policy_key(const K8sPolicy& p) { return p.ns + "/" + p.name; }
// utils.UnstringPodID: "ns/name" split on '/' (parts[0], parts[1])
bool unstring_id(const std::string& s, std::string* ns, std::string* name);

}  // namespace pg
