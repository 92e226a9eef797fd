// Device-side data layout shared by the host compiler (engine.cpp, fastpath.cpp) and the
// HIP kernels (device.hip). Everything here is plain-old-data copied to HBM as flat arrays.
//
// Layout in HBM (one "table set"; a new set is uploaded and swapped in on every change):
//   rules   DevRule[NR]   all ACLs' rules concatenated, ACL order preserved (linear kernel,
//                         ANY-protocol packets, generator)
//   tabs    DevTable[T]   per-ACL header incl. everything the blob walk needs (one 32-B read)
//   blobs   u32[]         per-ACL classification blob (fastpath.cpp), 16-byte aligned
//   ifaces  int2[NI]      per interface {inbound table, outbound table} (-1 = no ACL)
//   iphash  uint4[cap]    IPv4 -> {ip, interface, inbound table, outbound table} of a local
//                         pod (open addressing; EMPTY: interface = 0xFFFFFFFF)
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace pg {

// Packet L4 key: TCP -> dport, UDP -> 0x10000|dport, OTHER -> 0x20000, else (ANY/invalid) 0x30000.
constexpr uint32_t kKeyUDP = 0x10000u, kKeyOTHER = 0x20000u, kKeyANY = 0x30000u, kKeyMax = 0x2FFFFu;
// ACLAction codes (aclengine_mock.go:56-71)
constexpr uint32_t kActDeny = 0, kActPermit = 1, kActReflect = 2, kActFailure = 3, kActNever = 0xF;

struct DevRule {           // 32 B, one compiled vpp_acl rule
    uint32_t snet, smask;  // src: (src & smask) == snet
    uint32_t dnet, dmask;  // dst
    uint32_t klo, khi;     // L4 key range (empty when klo > khi)
    uint32_t act;          // low nibble: action on key match; high nibble: action for ANY packets (F = never)
    uint32_t pad;
};

struct DevTable {          // 32 B: two 16-B loads
    uint32_t blob_off;     // in u32 words, multiple of 4
    uint32_t fsk;          // flags (blob[0]; 8 = linear) | s1 << 8 | k1 << 16
    uint32_t dflt;         // default verdict: DENY << 30 | default slot
    uint32_t kroot;        // blob[4]
    uint32_t xoff;         // blob[6]
    uint32_t nkc;          // blob[7]
    uint32_t rule_base;    // first rule (global index == counter slot)
    uint32_t n_rules;
};

// Node classifier (fastpath.cpp build_node; PERPOD / CONN modes): every table the node
// covers evaluated through one IPv4 trie and one L4-key trie shared by all tables, and one
// cross-table entry per evaluation.
//   img    u32[]  (tries: entries are byte addresses in the image, blobwalk.hpp node_child_byte)
//                 IPv4 trie (root at word 0, leaf -> the node IP class's record) | L4-key
//                 trie (leaf -> the node key class's record) | IPv4 class records: in the
//                 uniform layout 16 B {self, packed end point (classify.hpp node_end_packed),
//                 common-row mask lo, hi} from word ipinfo, else 4-B self words from word
//                 ipself | key class records (uniform: 32 B, else 4 B) from byte kself << shift
//                 (self = the leaf value pointing at the record: a lookup that reached a leaf
//                 above the trie's last level re-reads it, so every lookup has the trie's depth)
//                 | outside the uniform layout: ipinfo uint2[n_ipc] {interface, tin | tout << 16}
//                 | tabinfo
//                 uint4[T] {cross base, nkc | covered << 31, common row, 0} | kmap u16[T][2^gk_shift]
//                 (local key class) | the words up to img_words_base are the base image;
//                 then the common-row section (cmap != 0): per covered table its most
//                 frequent cross row (u32[nkc], at tabinfo.z) and a bitmap over [T][n_ipc]
//                 (rows of 2^cmap_shift words),
//                 bit set = that (table, ip class) row equals the table's common row, so the
//                 entry is read from the (LDS-staged) image instead of the cross table
//   cross  u32[]  per covered table, [ip class][local key class] -> verdict, or kNodeList |
//                 first dst record (16 B records, blobwalk.hpp, ending with a match-all one);
//                 per covered PAIR table its pair map [src class][dst class] -> pair class and
//                 its verdicts [pair class][local key class] (the image then holds, per node IP
//                 class, the table's src class | dst class << 16)
constexpr uint32_t kNodeList = 1u << 29, kNodeRecMask = kNodeList - 1u;
// tabinfo.y bit 30: a PAIR table (tabinfo = {pair map base, nkc | covered << 31 | 1 << 30,
// verdicts base, class map offset | ndc << 16}): (src class of the src-side IP class, dst class of
// the dst-side one) -> pair class by one cross-array entry, then x local key class -> verdict
constexpr uint32_t kNodePairFlag = 1u << 30;
struct DevNode {
    const uint32_t* img;   // null: no node classifier (the per-table path runs)
    const uint32_t* cross;
    uint32_t img_words;    // whole image (with the common-row section when cmap != 0, and the dst records)
    uint32_t img_words_base;  // image without the common-row section and the dst records
    uint32_t cmap;         // word offset of the common-row bitmap in img, 0 = none
    uint32_t ip_s1, key_root, key_k1;
    // fixed-depth tries (blobwalk.hpp node_child_byte): a leaf is its class record's byte
    // address r; class = (r >> record shift) - ipself / kself (blobwalk.hpp node_ip_rec_shift); every lookup
    // takes exactly ip_depth / key_depth reads
    uint32_t ip_depth, key_depth, ipself, kself;
    uint32_t ipinfo, tabinfo, kmap;  // word offsets in img (uniform: ipinfo = the IPv4 class records)
    uint32_t gk;           // node key classes
    // row strides as shifts (rows padded to powers of two, so a row address is one shifted add):
    // kmap: table t's u16 row at halfword (kmap * 2) + (t << gk_shift); common-row bitmap:
    // table t's row of n_ipc bits at word cmap + (t << cmap_shift)
    uint32_t gk_shift, cmap_shift;
    uint32_t n_ipc;        // node IP classes
    uint32_t n_pair;       // covered PAIR tables (0: the evaluations skip the PAIR steps)
    // dst records (kNodeList words): rec0 = word offset of the first record in the cross array
    // (the numbering list words use); lrec != 0: a copy of them ends the image, at word lrec
    // (record word p of the cross numbering is image word p - rec0 + lrec); launches that do not
    // stage that part of the image clear lrec and read the cross array
    uint32_t rec0, lrec;
    // uniform layout (every table covered, none in PAIR form, fewer than 65535 tables;
    // Tuning::node_uniform): table t's cross rows are over the node key classes, entry (t, ip
    // class g, key class k) at word (t * n_ipc + g) * gk + k, and its common row (when cmap != 0)
    // at image word crow0 + t * gk; tabinfo and kmap are not read, and the common-row marks are
    // one uint2 mask per IP class in its record (bit t >> gshift: that class's row of table t --
    // of every table of t's group -- is the common one; class g's at word cmap + (g << cmap_shift))
    uint32_t uniform, crow0;
    uint32_t tstride;      // uniform layout: cross words per table, n_ipc * gk (below 2^24)
    uint32_t gshift;       // uniform layout: common-row mark bit of table t is t >> gshift (> 64 tables)
    // uniform layout with 255 tables or more (wide records): a class record is {self, interface |
    // kind << 14, marks (32 bits: bit t >> gshift, T <= 32 << gshift), tin | tout << 16 (0xFFFF =
    // no ACL)} instead of {self, interface | kind << 14 | tin << 16 | tout << 24 (0xFF = no ACL),
    // marks lo, marks hi} (classify.hpp node_end_packed / node_end_wide)
    uint32_t wide;
    // uniform layout: the table id of "no ACL" in the class records -- narrow records: a pseudo-table
    // past the tables (T rounded up to 2^gshift) whose common row is PERMIT with the "no ACL" slot and
    // whose mark every class has (fastpath.cpp build_node / build_common_rows); wide: 0xFFFF
    uint32_t tnil;
    // list-verdict table (Tuning::node_list_table; 0 = the record form above): a kNodeList word's
    // low bits are a list id L, and its verdict for the rule's dst-side address is cross word
    // lv0 + L * n_ipc + (that address's node IP class) -- one gather, no record walk
    uint32_t lv0;
};

// table sets of up to this many counter slots are counted by a full LDS histogram (one cell per
// slot, 64 KiB with the two extra cells of a SINGLE window)
constexpr uint32_t kLdsHistCells = 16382;

// End-point kind of an IP-keyed lookup (iphash, node IP classes), in bits 29-28 of a resolved
// interface index >= 0: a local pod's TAP (0), a pod registered on another node (kEndRemote)
// or any other address (kEndInet), both of which leave by the node-output interface. The
// IP-keyed CONN mode picks the reference's Connection* call from the two kinds
// (aclengine_mock.go:273-420): a remote pod paired with a non-pod address is the "invalid
// scenario" of ConnectionPodToInternet / ConnectionInternetToPod (:343-347, :388-392) ->
// FAILURE without an evaluation; non-pod <-> non-pod has no reference call and is FAILURE too
// (DESIGN.md §1). Kinds add: the pair is valid iff kind(src) + kind(dst) < 3.
constexpr int32_t kEndRemote = 1 << 28, kEndInet = 2 << 28;
constexpr uint32_t kEndKindShift = 28;

// Streams that launched kernels reading one table set, one slot each (device.hip DeviceBuffers:
// the slot's completion events, and its launch-mark word). A PERPOD / CONN launch over a uniform
// node defers its ANY-protocol packets to k_node_any, launched after it on the same stream
// (device.hip PG_CONN_DEFER_ANY): the classify kernel writes its launch number into its
// stream's mark word when it deferred a packet, and k_node_any runs only when the word holds its
// own number. Both launches are on one stream, so stream order alone makes the mark the one of
// this launch; a stale number (an earlier launch, or a slot reassigned after clear()) can only
// equal a later launch's after 2^32 - 1 more draws, and then k_node_any makes a pass that finds
// nothing to do -- never a skipped packet. Host-only bookkeeping, tested without a GPU
// (pg_debug_stream_slots).
struct StreamSlots {
    static constexpr size_t kMax = 32;  // slots; past this many streams the caller drains and clears
    std::vector<const void*> streams;   // slot i serves streams[i]
    uint32_t seq[kMax] = {};            // last launch number drawn at each slot (kept across clear())
    // slot of stream s (added when unseen: *added); false when every slot serves another stream --
    // the caller waits for the launches recorded at the slots, then clear()s
    bool slot(const void* s, size_t* i, bool* added) {
        for (size_t k = 0; k < streams.size(); k++)
            if (streams[k] == s) return *i = k, *added = false, true;
        if (streams.size() >= kMax) return false;
        streams.push_back(s);
        return *i = streams.size() - 1, *added = true, true;
    }
    uint32_t draw(size_t i) {  // the next launch number of slot i (never 0: a fresh mark word holds 0)
        if (++seq[i] == 0) ++seq[i];
        return seq[i];
    }
    void clear() { streams.clear(); }
};

struct DevTableSet {       // device pointers (valid on the GPU)
    const DevRule* rules;
    const DevTable* tabs;
    const uint32_t* blobs;
    const int32_t* ifaces; // int2 pairs
    const uint32_t* iphash;// uint4 {ip, iface, in table, out table}
    uint32_t iphash_mask;
    int32_t node_if;       // end point of non-pod IPs: node-output interface | kEndInet, -1 = none (FAILURE)
    int32_t node_in, node_out;  // its ACL tables (-1 = none)
    uint32_t n_rules;      // NR
    uint32_t n_tables;     // T
    uint32_t n_ifaces;
    uint32_t slot_noacl;   // NR + T
    uint32_t slot_unresolved;
    uint32_t n_slots;
    // the last rule of the inbound ACL the most interfaces share (the renderer's reflective ACL
    // for the pods without an ingress policy), 0xFFFFFFFF = none: CONN kernels count it, like "no
    // ACL", in a register
    uint32_t slot_hot_in;
    DevNode node;
    // PERPOD / CONN launches: the launch stream's mark word and this launch's number (StreamSlots; set per
    // launch by pg_classify through dev_any_mark, null otherwise)
    uint32_t* any_mark;
    uint32_t any_seq;
    const DevTable* host_tabs;       // host copies (launch decisions; not dereferenced on the GPU)
    const uint32_t* host_blob_words;
    const uint32_t* host_blob_prefix;  // FD blobs: words of the prefix a STAGE 5 launch stages
};

// Host image of a table set, produced by the compiler and uploaded as one blob.
struct HostTableSet {
    std::vector<DevRule> rules;
    std::vector<DevTable> tabs;
    std::vector<uint32_t> blob_words;  // per table (0 = linear)
    std::vector<uint32_t> blob_prefix; // per table: FD blob prefix words (0 = not FD)
    std::vector<uint32_t> blobs;
    std::vector<int32_t> ifaces;
    std::vector<uint32_t> iphash;
    uint32_t iphash_mask = 0;
    int32_t node_if = -1, node_in = -1, node_out = -1;
    uint32_t slot_hot_in = 0xFFFFFFFFu;          // DevTableSet.slot_hot_in (engine.cpp compile)
    std::vector<uint32_t> node_img, node_cross;  // empty img: no node classifier
    std::vector<uint32_t> node_aux;              // uniform layout: tabinfo and kmap (host only)
    DevNode node{};                              // header fields (pointers unset)
    uint32_t node_rec_words = 0;                 // words of the node's dst records (build_node)
    uint32_t node_list_tab_words = 0;            // words of its list-verdict table (DevNode lv0)
};

// table blobs up to this many words are staged in LDS by default (64 KiB); larger ones are
// read from HBM and compiled with level-compressed tries
constexpr uint32_t kStageBlobWords = 16384;

// Knobs of one engine context (pg_ctx_set_tuning; pg_set_tuning sets the process defaults new
// contexts start from). Compiler knobs apply to the tables the context compiles next; launch
// knobs to its next launches. Keys and ranges: tuning_set (engine.cpp), include/policygpu.h.
struct Tuning {
    // table compiler
    uint32_t root_bits_max = 16;   // cap of the tries' root stride (4..16)
    uint32_t lc_lds = 4096;        // LC rebuild of LDS-sized blobs of at least this many words (0 = off)
    uint32_t lc_dense12 = 16;      // boundaries in a child's span that earn it a 12-bit stride
    uint32_t lc_max_stride = 16;   // widest level-compressed stride (12, 16, 18)
    uint32_t lc_root_bits = 13;    // src-trie root stride cap of HBM-resident (level-compressed) blobs
    uint32_t pair = 1;             // PAIR for tables CROSS cannot take (0 = CAND, 2 = wherever it fits)
    uint32_t node_build = 1;       // build the node classifier (PERPOD / CONN)
    uint32_t node_root_bits = 12;  // its IPv4 / key trie root stride cap (4..16)
    // uniform layout: cap of the key trie's root stride, rounded down to 2, 6 or 10 (the strides
    // build_node tries). 10 saves a level (config 3 +1 % in the driver's window) but its 4 KiB
    // push config 5's image + counter histogram past the 80 KiB that keep two 1024-thread
    // workgroups per CU (139 -> 94 Gpps)
    uint32_t node_key_root_bits = 6;
    uint32_t node_common = 1;      // common-row section of node images
    uint32_t fd = 1;               // FD form of dst-independent CROSS tables that fit LDS
    uint32_t candi = 1;            // CANDI form (inline candidates) of dst-independent HBM-resident CAND tables
    uint32_t candi_window_bits = 11;  // CANDI: LDS window of 2^bits addresses' terminal entries (0 = none)
    uint32_t candi_window_root_bits = 12;  // CANDI: root stride cap of a table with a window
    uint32_t cross_max_rules = 1u << 20;  // CROSS (cross product) considered up to this many rules (within budget)
    uint32_t node_hist_cells = 256;   // LDS slot-cache cells (rounded down to a power of two; < 16 = none)
                                      // of node launches whose set has more slots than the LDS histogram
    uint32_t node_list_words = 4096;  // node dst records up to this many words go into the image (0 = never)
    uint32_t node_uniform = 1;        // the node's uniform cross layout where it applies (DevNode uniform)
    uint32_t node_list_table = 1;     // node lists resolved by a list-verdict table (DevNode lv0), else records
    // launches
    uint32_t blocks_per_cu = 0;    // cap on resident workgroups per CU (0 = occupancy)
    uint32_t stage_max_words = kStageBlobWords;  // table blobs staged whole in LDS
    uint32_t node_stage_max_words = 16384;       // node images staged in LDS
    uint32_t stage_root_max_words = 16400;       // larger blobs: header + src root up to 2^14 entries
    uint32_t node_path = 1;        // PERPOD / CONN through the node classifier when built
    uint32_t node_common_lds_max = 80u << 10;    // LDS bytes up to which the common-row section is staged
    uint32_t block_stage = 0;      // workgroup size of LDS-staged launches (0 = per mode)
    uint32_t hist_window = 4096;   // LDS hit-counter cells when the slots exceed the LDS histogram
    uint32_t launch_max_tuples = 0;  // tuples per k_classify launch at most (0 = kMaxLaunchTuples)
};
// key -> field; 0 ok, -1 unknown key or value out of range. *compiler: the key changes how
// tables are compiled (the context recompiles on its next use).
int tuning_set(Tuning& t, const std::string& key, int value, bool* compiler = nullptr);
int tuning_get(const Tuning& t, const std::string& key, int* value);
// process defaults (contexts copy them when created), behind one lock: pg_set_tuning may race
// pg_create on another thread
Tuning default_tuning();
int default_tuning_set(const std::string& key, int value);

// fastpath.cpp: classification blob of one table (false = does not fit the budgets). When
// `an` is given it receives the table's class analysis for build_node.
struct TableAnalysis;
// lc: level-compressed tries (wider strides in dense subtrees) for blobs read from HBM
bool build_fast_table(const DevRule* rules, uint32_t n, uint32_t rule_base, uint32_t default_slot,
                      std::vector<uint32_t>& blob, uint64_t cross_budget, const Tuning& tu,
                      TableAnalysis** an = nullptr, bool lc = false);
void free_analysis(TableAnalysis* an);
// fastpath.cpp: the FD (fixed-depth, dst-independent) form of a CROSS table without dst lists,
// when it fits max_words (false otherwise; blobwalk.hpp fd_walk); a shape that fits lds_words
// (the kernel then stages it whole) is preferred over fewer levels
bool build_fd_blob(const TableAnalysis& an, uint32_t dflt, const Tuning& tu, std::vector<uint32_t>& blob,
                   uint32_t max_words, uint32_t lds_words);
// fastpath.cpp: the node classifier over the tables with an analysis (null = not covered).
// pods: {IPv4, interface (with its kEnd* kind), inbound table, outbound table} of registered
// pods; node_end: the same for every other address. false = over budget (h.node_img left empty).
struct NodePod {
    uint32_t ip;
    int32_t ifc, tin, tout;
};
bool build_node(HostTableSet& h, const std::vector<TableAnalysis*>& an, const std::vector<NodePod>& pods,
                const NodePod& node_end, const Tuning& tu);


struct GenParams {         // device view of pg_gen_spec
    uint64_t seed, index_base;
    int32_t table_id;
    uint32_t inside_pct, pool_pct, port_pool_pct, tcp_pct, udp_pct, nomatch_pct, dst_pool_pct;
    uint32_t n_ip_pool, n_port_pool;
    const uint32_t* ip_pool;
    const uint16_t* port_pool;
    const uint32_t* zipf_cdf;  // n_rules entries or null
};

struct ConnQueryDev {      // resolved Connection* query
    uint32_t src_ip, dst_ip;
    int32_t src_if, dst_if;
    uint32_t key_syn;      // L4 key with dport
    uint32_t key_synack;   // L4 key with sport
    uint32_t pad[2];
};

// ---- device API (device.hip) ----------------------------------------------------------
struct DeviceBuffers;  // opaque
DeviceBuffers* dev_upload(const HostTableSet& h, std::string* err);
void dev_free(DeviceBuffers* b);
const DevTableSet& dev_view(const DeviceBuffers* b);

int dev_classify(const DevTableSet& T, const Tuning& tu, int mode, int table_id, const uint32_t* src,
                 const uint32_t* dst, const uint16_t* sport, const uint16_t* dport, const uint8_t* proto, uint64_t n,
                 uint32_t* out, unsigned long long* counters, void* stream, std::string* err);
int dev_classify_linear(const DevTableSet& T, int table_id, const uint32_t* src, const uint32_t* dst,
                        const uint16_t* dport, const uint8_t* proto, uint64_t n, uint32_t* out, void* stream,
                        std::string* err);
// the stream ceiling of a classify launch: its loads (fields: 1 = dst, 2 = sport) and store only
int dev_stream_probe(const Tuning& tu, int fields, const uint32_t* src, const uint32_t* dst, const uint16_t* sport,
                     const uint16_t* dport, const uint8_t* proto, uint64_t n, uint32_t* out, void* stream,
                     std::string* err);
int dev_gen(const DevTableSet& T, const GenParams& g, uint64_t n, uint32_t* src, uint32_t* dst, uint16_t* sport,
            uint16_t* dport, uint8_t* proto, void* stream, std::string* err);
int dev_conn_queries(const DevTableSet& T, const ConnQueryDev* q_host, size_t n, uint32_t* out_host,
                     std::string* err);
int dev_set_device(int dev, std::string* err);
int dev_get_device(int* dev);
void* dev_alloc(size_t bytes, std::string* err);
void dev_release(void* p);
int dev_memset(void* p, int v, size_t bytes, void* stream, std::string* err);
int dev_copy_d2h(void* dst, const void* src, size_t bytes, std::string* err);
int dev_copy_h2d(void* dst, const void* src, size_t bytes, std::string* err);
int dev_copy_d2d_async(void* dst, const void* src, size_t bytes, void* stream, std::string* err);
int dev_sync(std::string* err);
int dev_stream_sync(void* stream, std::string* err);
// record that `stream` launched kernels reading table set b (dev_free / dev_wait_uses wait for them)
int dev_mark_use(DeviceBuffers* b, void* stream, bool fenced, std::string* err);
// dst[i] = map[i] == kNoSlot (engine.hpp) ? 0 : src[map[i]] for n slots (map: host), on the null
// stream (the caller synchronises)
int dev_counters_remap(unsigned long long* dst, const unsigned long long* src, const uint32_t* map, size_t n,
                       std::string* err);
// the launch-mark word of `stream` for table set b and the next launch number at it (StreamSlots)
uint32_t* dev_any_mark(DeviceBuffers* b, void* stream, uint32_t* seq, std::string* err);
int dev_wait_uses(DeviceBuffers* b, std::string* err);
// RCCL communicators (opaque ncclComm_t), librccl opened on first use
int dev_comm_unique_id(uint8_t* id /* 128 B */, std::string* err);
void* dev_comm_init_rank(int nranks, const uint8_t* id, int rank, std::string* err);
int dev_comm_init_all(void** comms, const int* devs, int n, std::string* err);
void dev_comm_destroy(void* comm);
int dev_comm_allreduce_u64(void* const* comms, unsigned long long* const* bufs, const int* devs,
                           void* const* streams, int k, size_t count, bool max, std::string* err);

}  // namespace pg
