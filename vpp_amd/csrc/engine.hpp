// The device ACL engine: the MI355X counterpart of mock/aclengine.MockACLEngine.
// Holds installed ACLs (ApplyTxn/PutACL/DelACL semantics, aclengine_mock.go:151-228,
// 655-712), compiles them into the device table set (device.hpp) and evaluates
// evalACL/testConnection on the GPU.
#pragma once
#include <map>
#include <string>
#include <vector>

#include "device.hpp"
#include "policy.hpp"

namespace pg {

struct PodReg {
    Bytes ip;
    bool another_node = false;
};

// Compiled form of one vpp_acl rule (evalACL semantics, aclengine_mock.go:510-649).
DevRule compile_acl_rule(const AclRule& r);

struct Engine {
    int device = 0;
    std::string last_error;
    NodeIfaces ifaces;
    std::map<PodID, PodReg> pods;

    // ACLConfig
    std::map<std::string, ACLPtr> by_name;
    std::map<std::string, std::pair<ACLPtr, ACLPtr>> by_if;  // {inbound, outbound}
    int changes = 0;
    int committed = 0;

    // compiled / device state
    bool dirty = true;     // device tables stale
    bool compiled = false; // `host` reflects the installed ACLs
    HostTableSet host;
    DeviceBuffers* cur = nullptr;
    std::map<std::string, int> table_of_acl;
    std::vector<std::string> table_names;
    std::map<std::string, int> iface_index;
    std::vector<int32_t> slot_table, slot_rule;
    unsigned long long* counters = nullptr;
    size_t counter_slots = 0;

    ~Engine();
    std::string apply_txn(bool resync, const AclOps& ops);
    std::string put_acl(const ACLPtr& acl);
    std::string del_acl(const std::string& name);
    int sync();      // compile + upload if dirty; returns PG_* code
    void compile();  // host image only (no GPU)
    void touch() { dirty = true, compiled = false; }
    const DevTableSet* view() const;
    int iface_of(const std::string& name) const;
    std::string node_if_name() const;
};

std::string engine_apply_cb(void* engine, bool resync, const AclOps& ops);

}  // namespace pg
