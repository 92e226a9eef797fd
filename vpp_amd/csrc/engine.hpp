// The device ACL engine: the MI355X counterpart of mock/aclengine.MockACLEngine.
// Holds installed ACLs (ApplyTxn/PutACL/DelACL semantics, aclengine_mock.go:151-228,
// 655-712), compiles them into the device table set (device.hpp) and evaluates
// evalACL/testConnection on the GPU.
#pragma once
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "device.hpp"
#include "policy.hpp"

namespace pg {

struct PodReg {
    Bytes ip;
    bool another_node = false;
};

// The counter-slot layout of one compiled table set, kept with every host snapshot of the
// counters, so a statscollector gauge keyed by a stable rule identity (ACL name, rule index)
// reads the slot that identity had in the snapshot it reads (slots are renumbered on every
// recompile).
struct SlotLayout {
    uint64_t gen = 0;  // Engine::layout_gen when compiled
    struct Tab {
        uint32_t base, n, dflt;
        uint64_t rules_hash;  // FNV-64a over the ACL's rules (acl_rules_hash)
    };
    std::map<std::string, Tab> tabs;  // ACL name -> its slots
    uint32_t noacl = 0, unresolved = 0, slots = 0;
};

// FNV-64a over every field of an ACL's rules, in order (the identity its counts carry over by)
uint64_t acl_rules_hash(const ACL& acl);

// Counts that survive a recompile (statscollector: a gauge is a monotonic source,
// plugin_impl_statscollector.go:248-261): map[new slot] = the slot of `from` whose count it
// continues, or kNoSlot (starts at zero). An ACL carries over when an ACL of the same name with
// the same rules (count and acl_rules_hash) exists in both layouts -- its rule slots and its
// default-deny slot; "no ACL" and "unresolved" always do. Identity: every slot maps to itself.
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
std::vector<uint32_t> slot_remap(const SlotLayout& from, const SlotLayout& to, bool* identity = nullptr);

// A host copy of the counters and the layout they were counted in.
struct CounterSnapshot {
    std::vector<uint64_t> v;
    std::shared_ptr<const SlotLayout> layout;  // null: never taken
};

// Compiled form of one vpp_acl rule (evalACL semantics, aclengine_mock.go:510-649).
DevRule compile_acl_rule(const AclRule& r);

struct Engine {
    int device = 0;
    Tuning tune = default_tuning();  // this context's knobs (pg_ctx_set_tuning)
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
    uint64_t layout_hash = 0;  // FNV-64a over (table name, rule count) in slot order

    // RCCL: one communicator per context (multi-process: pg_comm_init_rank; one process over
    // several GPUs: pg_comm_init_all). Before every counter all-reduce the ranks compare
    // (counter slots, layout hash) with a max all-reduce of this 4 x u64 device scratch.
    void* comm = nullptr;
    int comm_rank = -1, comm_nranks = 0;
    unsigned long long* comm_check = nullptr;
    // the all-reduce sums a copy of the counters (never the counters themselves), so the
    // local counts stay this rank's and repeated reductions do not compound
    unsigned long long* reduced = nullptr;
    size_t reduced_slots = 0;
    // slot layout of the compiled set; layout_gen counts the recompiles that renumbered slots
    // (published for pg_counter_layout_gen, which any thread may poll, through layout_gen_pub)
    std::shared_ptr<const SlotLayout> layout;
    uint64_t layout_gen = 0;
    std::atomic<uint64_t> layout_gen_pub{0};
    // the layout of the uploaded set, which the device counters are counted in: sync() carries
    // them over (slot_remap) to the next set's layout
    std::shared_ptr<const SlotLayout> counted_layout;
    // host copies of the counters, read by the statscollector gauges without touching the GPU
    // (pg_counters_snapshot*): this rank's own as of the last pg_read_counters, and the sum over
    // the communicator as of the last pg_allreduce_counters*. Gauges run on their own threads
    // (scrape time), so the snapshots sit behind snap_mu.
    mutable std::mutex snap_mu;
    CounterSnapshot snap_local, snap_cluster;

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
