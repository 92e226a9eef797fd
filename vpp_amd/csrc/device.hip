// gfx950 kernels of the policy classification path.
//
//  K1 k_linear       reference-shaped first-match scan: one lane per tuple, rules read
//                    wave-uniformly (scalar loads), wave exits when every lane matched.
//  K2 k_classify     the production path for SINGLE / PERPOD / CONN modes: per table a
//                    classification blob (fastpath.cpp: src/key multibit tries -> equivalence
//                    classes -> cross-product verdicts or candidate records), walked for 4
//                    tuples per lane in lockstep (blobwalk.hpp) after 16/8/4-byte coalesced,
//                    non-temporal SoA loads of the quad; SINGLE mode stages the blob in LDS;
//                    per-rule hit counters kept in an LDS histogram and flushed once per
//                    workgroup with u64 atomics.
//  K3 (inside K2)    PERPOD / CONN: IPv4 -> interface + its ACL tables by one 16-B hash probe;
//                    CONN fuses testConnection's up-to-4 evalACL steps
//                    (mock/aclengine/aclengine_mock.go:424-501), each in lockstep over the quad.
//  K5 k_gen          counter-based (splitmix64) synthetic 5-tuple generator.
//
// Semantics of one evaluation == evalACL (aclengine_mock.go:503-652) over the ACL the table
// was compiled from (engine.cpp compile_acl_rule); the output word packs the ACLAction (or
// ConnAction) in bits 31-30 and the deciding counter slot in bits 29-0.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <type_traits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <utility>

#include "classify.hpp"

namespace pg {

#define HIPCHK(expr)                                                         \
    do {                                                                     \
        hipError_t e_ = (expr);                                              \
        if (e_ != hipSuccess) {                                              \
            if (err) *err = std::string(#expr ": ") + hipGetErrorString(e_); \
            return -1;                                                       \
        }                                                                    \
    } while (0)

struct DeviceBuffers {
    void* blob = nullptr;
    DevTableSet view{};
    std::vector<DevTable> host_tabs;
    std::vector<uint32_t> host_blob_words, host_blob_prefix;
    // streams that launched kernels reading this set, with events recorded after the last
    // launch on each: the set is freed (and counters read) once those have completed, without
    // a device-wide synchronisation (dev_mark_use)
    struct Use {
        hipEvent_t plain, fenced;
        bool plain_rec, fenced_rec;
    };
    std::vector<Use> uses;  // uses[i]: the stream of slot i (StreamSlots)
    StreamSlots slots;
    uint32_t* marks = nullptr;  // device: StreamSlots::kMax launch-mark words (k_node_any)
};

const DevTableSet& dev_view(const DeviceBuffers* b) { return b->view; }

int dev_set_device(int dev, std::string* err) {
    HIPCHK(hipSetDevice(dev));
    return 0;
}
int dev_get_device(int* dev) { return hipGetDevice(dev) == hipSuccess ? 0 : -1; }
void* dev_alloc(size_t bytes, std::string* err) {
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
    if (e != hipSuccess) {
        if (err) *err = std::string("hipMalloc: ") + hipGetErrorString(e);
        return nullptr;
    }
    return p;
}
void dev_release(void* p) {
    if (p) (void)hipFree(p);
}
int dev_memset(void* p, int v, size_t bytes, void* stream, std::string* err) {
    HIPCHK(hipMemsetAsync(p, v, bytes, (hipStream_t)stream));
    return 0;
}
int dev_copy_d2h(void* dst, const void* src, size_t bytes, std::string* err) {
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return 0;
}
int dev_copy_h2d(void* dst, const void* src, size_t bytes, std::string* err) {
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return 0;
}
int dev_copy_d2d_async(void* dst, const void* src, size_t bytes, void* stream, std::string* err) {
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return 0;
}
int dev_sync(std::string* err) {
    HIPCHK(hipDeviceSynchronize());
    return 0;
}
int dev_stream_sync(void* stream, std::string* err) {
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
    return 0;
}

// Completion events per stream: `fenced` after launches that wrote hit counters (the
// system-scope release makes them visible to the counter read-back), a fence-free one after the
// others -- freeing a set needs only that its readers have finished, and a system-scope fence
// per record cost ~3 us per back-to-back launch on MI355X (tools/gap_probe.py: 130.2 -> 127.1 us
// per config-2 launch without it)
// The slot of `stream` (StreamSlots; its events created when new). Bounded: past kMax streams,
// wait for every recorded launch and start over.
static int use_slot(DeviceBuffers* b, hipStream_t s, size_t* i, std::string* err) {
    bool added = false;
    if (!b->slots.slot(s, i, &added)) {
        // wait for every recorded launch (keeping the first error), then destroy every event and
        // clear the list on both paths, so no destroyed event stays listed
        hipError_t first = hipSuccess;
        for (auto& u : b->uses) {
            hipError_t e1 = u.plain_rec ? hipEventSynchronize(u.plain) : hipSuccess;
            hipError_t e2 = u.fenced_rec ? hipEventSynchronize(u.fenced) : hipSuccess;
            if (first == hipSuccess) first = e1 != hipSuccess ? e1 : e2;
        }
        for (auto& u : b->uses) {
            (void)hipEventDestroy(u.plain);
            (void)hipEventDestroy(u.fenced);
        }
        b->uses.clear();
        b->slots.clear();
        if (first != hipSuccess) {
            if (err) *err = std::string("hipEventSynchronize: ") + hipGetErrorString(first);
            return -1;
        }
        b->slots.slot(s, i, &added);
    }
    if (added) {
        DeviceBuffers::Use u{nullptr, nullptr, false, false};
        hipError_t e = hipEventCreateWithFlags(&u.plain, hipEventDisableTiming | hipEventDisableSystemFence);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&u.fenced, hipEventDisableTiming);
        if (e != hipSuccess) {
            if (u.plain) (void)hipEventDestroy(u.plain);
            b->slots.streams.pop_back();  // (the slot just added: the lists stay aligned)
            if (err) *err = std::string("hipEventCreateWithFlags: ") + hipGetErrorString(e);
            return -1;
        }
        b->uses.push_back(u);
    }
    return 0;
}

int dev_mark_use(DeviceBuffers* b, void* stream, bool fenced, std::string* err) {
    const hipStream_t s = (hipStream_t)stream;
    size_t i = 0;
    if (use_slot(b, s, &i, err) != 0) return -1;
    DeviceBuffers::Use& u = b->uses[i];
    HIPCHK(hipEventRecord(fenced ? u.fenced : u.plain, s));
    (fenced ? u.fenced_rec : u.plain_rec) = true;
    return 0;
}

uint32_t* dev_any_mark(DeviceBuffers* b, void* stream, uint32_t* seq, std::string* err) {
    size_t i = 0;
    if (use_slot(b, (hipStream_t)stream, &i, err) != 0) return nullptr;
    *seq = b->slots.draw(i);
    return b->marks + i;
}

int dev_wait_uses(DeviceBuffers* b, std::string* err) {
    for (auto& u : b->uses) {
        if (u.plain_rec) HIPCHK(hipEventSynchronize(u.plain));
        if (u.fenced_rec) HIPCHK(hipEventSynchronize(u.fenced));
    }
    return 0;
}

DeviceBuffers* dev_upload(const HostTableSet& h, std::string* err) {
    // one blob, every array 256-byte aligned
    size_t off = 0;
    auto place = [&](size_t bytes) {
        size_t o = off;
        off += (bytes + 255) & ~(size_t)255;
        if (bytes == 0) off += 256;
        return o;
    };
    size_t o_rules = place(h.rules.size() * sizeof(DevRule));
    size_t o_tabs = place(h.tabs.size() * sizeof(DevTable));
    size_t o_blob = place(h.blobs.size() * 4);
    size_t o_if = place(h.ifaces.size() * 4);
    size_t o_ip = place(h.iphash.size() * 4);
    size_t o_nimg = place(h.node_img.size() * 4);
    size_t o_nx = place(h.node_cross.size() * 4);
    size_t o_mark = place(StreamSlots::kMax * 4);  // launch-mark words, zero
    std::vector<uint8_t> img(off, 0);
    auto put = [&](size_t o, const void* p, size_t n) {
        if (n) std::memcpy(img.data() + o, p, n);
    };
    put(o_rules, h.rules.data(), h.rules.size() * sizeof(DevRule));
    put(o_tabs, h.tabs.data(), h.tabs.size() * sizeof(DevTable));
    put(o_blob, h.blobs.data(), h.blobs.size() * 4);
    put(o_if, h.ifaces.data(), h.ifaces.size() * 4);
    put(o_ip, h.iphash.data(), h.iphash.size() * 4);
    put(o_nimg, h.node_img.data(), h.node_img.size() * 4);
    put(o_nx, h.node_cross.data(), h.node_cross.size() * 4);
    auto* b = new DeviceBuffers();
    b->blob = dev_alloc(off, err);
    if (!b->blob) {
        delete b;
        return nullptr;
    }
    if (dev_copy_h2d(b->blob, img.data(), off, err) != 0) {  // synchronous: the copy has landed
        dev_release(b->blob);
        delete b;
        return nullptr;
    }
    auto* base = (uint8_t*)b->blob;
    DevTableSet& v = b->view;
    v.rules = (const DevRule*)(base + o_rules);
    v.tabs = (const DevTable*)(base + o_tabs);
    v.blobs = (const uint32_t*)(base + o_blob);
    v.ifaces = (const int32_t*)(base + o_if);
    v.iphash = (const uint32_t*)(base + o_ip);
    v.iphash_mask = h.iphash_mask;
    v.node_if = h.node_if;
    v.node_in = h.node_in;
    v.node_out = h.node_out;
    v.n_rules = (uint32_t)h.rules.size();
    v.n_tables = (uint32_t)h.tabs.size();
    v.n_ifaces = (uint32_t)(h.ifaces.size() / 2);
    v.slot_noacl = v.n_rules + v.n_tables;
    v.slot_unresolved = v.slot_noacl + 1;
    v.n_slots = v.slot_unresolved + 1;
    v.slot_hot_in = h.slot_hot_in;
    v.node = h.node;
    v.node.img = h.node_img.empty() ? nullptr : (const uint32_t*)(base + o_nimg);
    v.node.cross = h.node_img.empty() ? nullptr : (const uint32_t*)(base + o_nx);
    v.any_mark = nullptr;
    v.any_seq = 0;
    b->marks = (uint32_t*)(base + o_mark);
    b->host_tabs = h.tabs;
    b->host_blob_words = h.blob_words;
    b->host_blob_prefix = h.blob_prefix;
    v.host_tabs = b->host_tabs.data();
    v.host_blob_words = b->host_blob_words.data();
    v.host_blob_prefix = b->host_blob_prefix.data();
    return b;
}

void dev_free(DeviceBuffers* b) {
    if (!b) return;
    for (auto& u : b->uses) {  // launches that read the set have completed
        if (u.plain_rec) (void)hipEventSynchronize(u.plain);
        if (u.fenced_rec) (void)hipEventSynchronize(u.fenced);
        (void)hipEventDestroy(u.plain);
        (void)hipEventDestroy(u.fenced);
    }
    dev_release(b->blob);
    delete b;
}

// ---- RCCL (counter all-reduce) ------------------------------------------------
// librccl is opened at first use (dlopen of the SONAME: a process that already holds one --
// e.g. torch's -- shares it), so contexts that never all-reduce need no RCCL.
namespace {
struct Rccl {
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGetErrorString) errstr = nullptr;
    std::string load_error;
};
const Rccl& rccl() {
    static const Rccl r = [] {
        Rccl x;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            const char* e = dlerror();
            x.load_error = std::string("dlopen librccl: ") + (e ? e : "?");
            return x;
        }
        auto sym = [&](auto& f, const char* name) { f = reinterpret_cast<std::decay_t<decltype(f)>>(dlsym(h, name)); };
        sym(x.get_id, "ncclGetUniqueId");
        sym(x.init_rank, "ncclCommInitRank");
        sym(x.init_all, "ncclCommInitAll");
        sym(x.all_reduce, "ncclAllReduce");
        sym(x.group_start, "ncclGroupStart");
        sym(x.group_end, "ncclGroupEnd");
        sym(x.destroy, "ncclCommDestroy");
        sym(x.errstr, "ncclGetErrorString");
        if (!x.get_id || !x.init_rank || !x.init_all || !x.all_reduce || !x.group_start || !x.group_end ||
            !x.destroy || !x.errstr)
            x.load_error = "librccl: missing symbols";
        return x;
    }();
    return r;
}
bool rccl_ok(std::string* err) {
    if (!rccl().load_error.empty()) {
        if (err) *err = rccl().load_error;
        return false;
    }
    return true;
}
}  // namespace

#define NCCLCHK(expr)                                                               \
    do {                                                                            \
        ncclResult_t r_ = (expr);                                                   \
        if (r_ != ncclSuccess) {                                                    \
            if (err) *err = std::string(#expr ": ") + rccl().errstr(r_);            \
            return -1;                                                              \
        }                                                                           \
    } while (0)

int dev_comm_unique_id(uint8_t* id, std::string* err) {
    if (!rccl_ok(err)) return -1;
    ncclUniqueId u;
    NCCLCHK(rccl().get_id(&u));
    std::memcpy(id, u.internal, sizeof(u.internal));
    return 0;
}

void* dev_comm_init_rank(int nranks, const uint8_t* id, int rank, std::string* err) {
    if (!rccl_ok(err)) return nullptr;
    ncclUniqueId u;
    std::memcpy(u.internal, id, sizeof(u.internal));
    ncclComm_t c = nullptr;
    const ncclResult_t r = rccl().init_rank(&c, nranks, u, rank);
    if (r != ncclSuccess) {
        if (err) *err = std::string("ncclCommInitRank: ") + rccl().errstr(r);
        return nullptr;
    }
    return c;
}

int dev_comm_init_all(void** comms, const int* devs, int n, std::string* err) {
    if (!rccl_ok(err)) return -1;
    std::vector<ncclComm_t> c(n, nullptr);
    NCCLCHK(rccl().init_all(c.data(), n, devs));
    for (int i = 0; i < n; i++) comms[i] = c[i];
    return 0;
}

void dev_comm_destroy(void* comm) {
    if (comm && rccl().destroy) (void)rccl().destroy((ncclComm_t)comm);
}

// In-place ncclAllReduce of k buffers (one per communicator of a group; k = 1 for one rank of
// a multi-process communicator), u64 max or sum, on the given streams; devs[i] is made current
// around each call (the caller restores its device).
int dev_comm_allreduce_u64(void* const* comms, unsigned long long* const* bufs, const int* devs,
                           void* const* streams, int k, size_t count, bool max, std::string* err) {
    if (!rccl_ok(err)) return -1;
    if (k > 1) NCCLCHK(rccl().group_start());
    for (int i = 0; i < k; i++) {
        HIPCHK(hipSetDevice(devs[i]));
        const ncclResult_t r = rccl().all_reduce(bufs[i], bufs[i], count, ncclUint64, max ? ncclMax : ncclSum,
                                                 (ncclComm_t)comms[i], (hipStream_t)streams[i]);
        if (r != ncclSuccess) {
            if (k > 1) (void)rccl().group_end();
            if (err) *err = std::string("ncclAllReduce: ") + rccl().errstr(r);
            return -1;
        }
    }
    if (k > 1) NCCLCHK(rccl().group_end());
    return 0;
}

constexpr int kBlock = 256;
constexpr uint32_t kLdsHistMax = kLdsHistCells + 2;  // hit-counter cells kept in LDS (64 KiB): a window + 2

// Tuple streams are read once and verdicts written once: issued with the non-temporal
// policy (A/B in one process with tools/sweep.py: +3-4 % on config 2; PG_NT_STREAM=0 builds
// the plain-policy variant).
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
#ifndef PG_NT_STREAM
#define PG_NT_STREAM 1
#endif
template <class V>
__device__ __forceinline__ V stream_load(const V* p) {
    if (PG_NT_STREAM) return __builtin_nontemporal_load(p);
    return *p;
}
template <class V>
__device__ __forceinline__ void stream_store(V v, V* p) {
    if (PG_NT_STREAM) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// STAGE (SINGLE mode): 1 = the table's blob (stage_words u32, multiple of 4) is copied into
// LDS once per workgroup and every lookup of the grid-stride loop reads it from there; 2 = a
// blob too large for LDS has its header and src-trie root (stage_words) copied, so the first
// dependent load of every lookup hits LDS and the rest read HBM / L2; 4 = an FD blob
// (fastpath.cpp build_fd_blob) staged like 1 and walked by classify_fd_q: fixed-depth reads,
// no per-lane branches, and no dst stream (no rule of an FD table tests dst); 5 = an FD blob
// too large for LDS: its prefix (header, src root, key trie) staged, the src levels below the
// root and the verdict rows read from HBM / L2.
// NODE (PERPOD / CONN): the node classifier; STAGE then copies the node image into LDS.
//
// Stream pipelining (PG_PREFETCH): 1 = the next group's loads are issued at the top of each
// iteration; 2 = (NODE) issued right after the cross-entry gathers of the group's first (or,
// PG_HOOK_LAST, last) chunk, so waiting for those gathers does not also wait for them (vmcnt
// retires in issue order); 3 = after the group's classification; 0 = none;
// -1 (default) = per mode: none for SINGLE over an LDS-staged blob (all lookups in LDS,
// occupancy hides the stream), top-of-iteration for SINGLE over a blob in HBM and for PERPOD /
// CONN (tools/sweep.py A/B on MI355X).
#ifndef PG_PREFETCH
#define PG_PREFETCH -1
#endif
#ifndef PG_PROBE_STREAM  // measurement build only: the streams with no classification
#define PG_PROBE_STREAM 0
#endif
#ifndef PG_PRED  // predicated (branch-free) trie walks on LDS-staged images (A/B: slower)
#define PG_PRED 0
#endif
// tuples of a group classified together (lockstep chunk), per mode, each dividing PG_TPL
// SINGLE: blob staged in LDS (STAGE 1) one tuple at a time (A/B on MI355X: config 2 331 / 343 /
// 348 Gpps at 4 / 2 / 1, with counters 307 / 316 / 325), blob in HBM four (config 4 with the
// inline-candidate form and a 12-bit staged root: 169.3 / 163.5 / 124 at 4 / 2 / 1)
#ifndef PG_QCANDI  // STAGE 6 without counters (A/B on MI355X, config 4: 188.5 vs 179.5 Gpps at 4; with
#define PG_QCANDI 2  // counters 4 stays: 113.5 vs 112)
#endif
#ifndef PG_FD_BS1024  // LDS-staged FD blobs that leave room for < 3 workgroups per CU: 1024 threads
#define PG_FD_BS1024 1
#endif
constexpr size_t kLdsPerCU = 160u << 10;
#ifndef PG_CANDI_LEAN  // SINGLE over a CANDI table with its root staged: the dedicated walk (STAGE 6)
#define PG_CANDI_LEAN 1
#endif
#ifndef PG_QSINGLE_LDS
#define PG_QSINGLE_LDS 1
#endif
#ifndef PG_QSINGLE
#define PG_QSINGLE 4
#endif
#ifndef PG_QPOD  // PERPOD: 2 (A/B on MI355X, config 3: 237 vs 198 Gpps at 4 -- fewer registers)
#define PG_QPOD 2
#endif
#ifndef PG_QPOD_FULLH  // PERPOD counting into an LDS histogram of every slot (64 registers, 1024
#define PG_QPOD_FULLH 4     // threads): 4 (A/B on MI355X, config 3 with counters 282 -> 295 Gpps)
#endif
#ifndef PG_QCONN
#define PG_QCONN 1
#endif
#ifndef PG_QCONN_COUNT  // CONN with hit counters (A/B on MI355X, config 5: 2 = +9 % over 1, 4 = -6 % in
#define PG_QCONN_COUNT 1  // round 1; after the fixed-depth node walks 1 = +3.5 % over 2, tune1)
#endif
#ifndef PG_QSINGLE_FD  // SINGLE over an LDS-staged FD table (STAGE 4)
#define PG_QSINGLE_FD 1
#endif
#ifndef PG_QSINGLE_FDG  // SINGLE over an FD table read from HBM, its prefix staged (STAGE 5): 4 (A/B on
                        // MI355X with the finished-lane skip: 30k / 100k / config 7 +2 / +1.2 / +1.2 % over 2)
#define PG_QSINGLE_FDG 4
#endif
#ifndef PG_PREFETCH_FD  // STAGE 4 / 5: stream prefetch of the next group (see PG_PREFETCH)
#define PG_PREFETCH_FD 0
#endif
#ifndef PG_PF_DEPTH  // launches with stream prefetch: groups loaded ahead (1 or 2)
#define PG_PF_DEPTH 1
#endif
#ifndef PG_HOOK_LAST  // PF 2: the loads issued after the gathers of the group's last chunk (else its first)
#define PG_HOOK_LAST 0
#endif
#ifndef PG_CONN_HOT_REGS  // CONN full-histogram build: two hot slots counted in registers
#define PG_CONN_HOT_REGS 1
#endif
#ifndef PG_NODE_NOPAIR  // node sets without PAIR tables: the build without PAIR code (STAGE + 32)
#define PG_NODE_NOPAIR 1
#endif
#ifndef PG_NODE_HALF  // uniform node sets whose 32-bit histogram would crowd LDS: 16-bit cells (STAGE + 256)
#define PG_NODE_HALF 1
#endif
#ifndef PG_NODE_FULLH  // node kernels whose LDS histogram holds every slot: the specialised build (STAGE + 16)
#define PG_NODE_FULLH 1
#endif
// CONN over a uniform node (STAGE + 96): ANY-protocol packets, the only ones the node cannot
// classify, are deferred to k_node_any, launched after the classify kernel on the same stream
// (iphash end points, the ANY-protocol first match, global counter increments), so the
// classify kernel carries no per-table fallback. The out-of-line fallback call in the loop
// cost the kernel its SGPR allocation: 54 SGPRs spilled to VGPR lanes, a v_readlane per use;
// a pass after the loop in the same kernel still cost 6 % (A/B on MI355X, config 5 with
// counters: in-loop call 123, pass after the loop 129, no pass 137 Gpps; PERPOD unchanged by
// any of it, so it keeps the call). A launch that deferred a packet writes its number into its
// stream's mark word (device.hpp StreamSlots, DevTableSet any_mark / any_seq); the k_node_any
// launched after it on that stream classifies the batch's ANY-protocol packets when the word
// holds its number, and returns at once otherwise -- stream order makes the word this launch's.
#ifndef PG_CONN_DEFER_ANY
#define PG_CONN_DEFER_ANY 1
#endif
// PERPOD over a uniform node likewise (k_node_any<1>): without the fallback call the kernel needs
// no call frame, its SGPR block and the VGPRs the call saved (67 -> 64, no scratch)
#ifndef PG_POD_DEFER_ANY
#define PG_POD_DEFER_ANY 0
#endif
#ifndef PG_PROBE_NOANYLAUNCH
#define PG_PROBE_NOANYLAUNCH 0
#endif
template <int MODE>
constexpr bool defer_any() { return MODE == 2 ? PG_CONN_DEFER_ANY : (MODE == 1 ? PG_POD_DEFER_ANY : false); }
// any of the four protocol bytes of w above 2 (bytes >= 0x80 by their top bit, the rest by a
// carry-free add into it)
__device__ __forceinline__ bool any_proto_gt2(uint32_t w) {
    return ((((w & 0x7F7F7F7Fu) + 0x7D7D7D7Du) | w) & 0x80808080u) != 0u;
}

template <int MODE, bool COUNT>
__global__ __launch_bounds__(kBlock) void k_node_any(DevTableSet T, const uint32_t* __restrict__ src,
                                                  const uint32_t* __restrict__ dst, const uint8_t* __restrict__ proto,
                                                  uint64_t n, uint32_t* __restrict__ out, unsigned long long* counters) {
    if (*T.any_mark != T.any_seq) return;
    const Hist h{nullptr, counters};  // global increments (rare packets)
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        if (proto[i] > 2u) out[i] = MODE == 2 ? conn_any_1<COUNT>(T, src[i], dst[i], h) : pod_any_1<COUNT>(T, src[i], dst[i], h);
}
#ifndef PG_IDX32  // k_classify's group indices and stream offsets in 32 bits (launches below kMaxLaunchTuples)
#define PG_IDX32 1
#endif
// the most tuples one k_classify launch takes: every stream's byte offset below 2^32 (dev_classify
// splits larger batches into launches of at most this many; a multiple of 64, so the pieces stay
// vector-aligned)
constexpr uint64_t kMaxLaunchTuples = PG_IDX32 ? (1ull << 30) - 64 : ~0ull;
#ifndef PG_TPL  // tuples per lane per loop iteration (4 or 8)
#define PG_TPL 4
#endif
// ... in CONN mode: 4 (round 4 measured 8 ahead, 133.7 -> 137.7 Gpps for config 5 with counters;
// with the node walks' compile-time shapes (classify.hpp node_walks) 8 tuples per lane no longer
// fit the 64-register cap of the CONN build: 144 B of scratch per lane, 109 Gpps, vs 142 at 4)
#ifndef PG_TPL_CONN
#define PG_TPL_CONN 4
#endif
template <int MODE>
constexpr int tuples_per_lane() { return MODE == 2 ? PG_TPL_CONN : PG_TPL; }

// NW consecutive u32 of a stream with the widest loads / stores (NW = 1, 2, 4, 8)
template <int NW>
struct Words {
    uint32_t w[NW];
};
template <int NW>
__device__ __forceinline__ Words<NW> ld_words(const uint32_t* p) {
    Words<NW> r;
    if constexpr (NW == 1) {
        r.w[0] = stream_load(p);
    } else if constexpr (NW == 2) {
        const v2u v = stream_load(reinterpret_cast<const v2u*>(p));
        r.w[0] = v.x, r.w[1] = v.y;
    } else {
#pragma unroll
        for (int k = 0; k < NW / 4; k++) {
            const v4u v = stream_load(reinterpret_cast<const v4u*>(p) + k);
            r.w[4 * k] = v.x, r.w[4 * k + 1] = v.y, r.w[4 * k + 2] = v.z, r.w[4 * k + 3] = v.w;
        }
    }
    return r;
}
template <int NW>
__device__ __forceinline__ void st_words(const Words<NW>& v, uint32_t* p) {
#pragma unroll
    for (int k = 0; k < NW / 4; k++)
        stream_store(v4u{v.w[4 * k], v.w[4 * k + 1], v.w[4 * k + 2], v.w[4 * k + 3]}, reinterpret_cast<v4u*>(p) + k);
}
#ifndef PG_NODE_WPE  // node kernels: minimum waves per SIMD the register allocation must allow (1 = any)
#define PG_NODE_WPE 1
#endif
// CONN with hit counters (config 5): image + counter histogram (79 KB) leave LDS for two
// workgroups per CU; 1024-thread workgroups, registers held to 64 (8 waves per SIMD) and no
// stream prefetch (its 13 registers) put 32 waves per CU instead of 16 (A/B on MI355X,
// gpurun_out/abocc: 89.1 -> 103.4 Gpps; the same 64-register cap on PERPOD spills and loses)
#ifndef PG_POD_FULLH_WPE8  // PERPOD full-histogram build at 64 registers / 1024 threads / no prefetch
#define PG_POD_FULLH_WPE8 1
#endif
#ifndef PG_CONN_WPE8_ALL  // CONN without counters too (A/B on MI355X, config 5 without counters: 136 -> 146 Gpps)
#define PG_CONN_WPE8_ALL 1
#endif
#ifndef PG_CONN_COUNT_WPE
#define PG_CONN_COUNT_WPE 8
#endif
// SINGLE over a blob in HBM (STAGE 0 / 2, the dst-free variants included): 66 registers at four
// tuples per chunk hold it to three 512-thread workgroups per CU; a 64-register cap spills
#ifndef PG_HOT_SLOT  // SINGLE with counters: the table's last rule counted in a register (HistT::hot)
#define PG_HOT_SLOT 1
#endif
#ifndef PG_HOT_SLOT_NODE  // node kernels with counters: the node-output table's last rule in a register
#define PG_HOT_SLOT_NODE 1
#endif
#ifndef PG_SINGLE_HBM_WPE  // (A/B on MI355X, config 4: 8 = 164.6 Gpps with 2 spills, 1 = 175.7)
#define PG_SINGLE_HBM_WPE 1
#endif
#ifndef PG_NODE_WIDE_BS  // workgroup size of the wide node builds (node_wide)
#define PG_NODE_WIDE_BS 1024
#endif
#ifndef PG_NODE_WIDE_REC_BS  // ... and of the other builds over wide class records (STAGE + 128)
#define PG_NODE_WIDE_REC_BS 768
#endif
// node builds at 64 registers (wpe 8): 1024-thread workgroups and no stream prefetch (its
// registers): CONN, and PERPOD counting into an LDS histogram of every slot (image + histogram
// leave LDS for two workgroups per CU: 16 waves at 512 threads, 32 at 1024; A/B on MI355X,
// config 3 with counters 227 -> 260 Gpps; without counters, or through the slot cache, the
// prefetching 512-thread build stays ahead: config 3 317 vs 301, config 6 with counters 147 vs 142)
template <int MODE, bool COUNT, bool NODE, int STAGE = 1>
constexpr bool node_wide() {
    return NODE && ((MODE == 2 && (COUNT || PG_CONN_WPE8_ALL)) || (MODE == 1 && COUNT && (STAGE & 16) && PG_POD_FULLH_WPE8));
}
template <int MODE, bool COUNT, bool NODE, int STAGE = 1>
constexpr int kernel_wpe() {
    return !NODE ? (MODE == 0 && ((STAGE & 7) == 0 || (STAGE & 7) == 2) ? PG_SINGLE_HBM_WPE : 1)
                 : (node_wide<MODE, COUNT, NODE, STAGE>() ? PG_CONN_COUNT_WPE : PG_NODE_WPE);
}
// the most waves per SIMD the register scheduler should aim for: the node builds that are not
// register-capped are LDS-bound at three 512-thread workgroups per CU (6 waves per SIMD), so more
// than 6 buys nothing and only costs the scheduler latency hiding (PG_NODE_WPE_MAX)
#ifndef PG_NODE_WPE_MAX
#define PG_NODE_WPE_MAX 8
#endif
template <int MODE, bool COUNT, bool NODE, int STAGE = 1>
constexpr int kernel_wpe_max() {
    return NODE && !node_wide<MODE, COUNT, NODE, STAGE>() ? PG_NODE_WPE_MAX : 8;
}
// STAGE_ + 8 (SINGLE, STAGE 0-2): the table is dst-free (kFlagDstFree: no rule tests dst), so
// the dst stream is not read
// SINGLE over a CANDI table with root + window staged (STAGE 6), a group of P tuples per lane
// at once, the walks compacted across the wave (PG_CANDI_COMPACT). A lookup the window resolves
// (an inline candidate or the default) is done in LDS; every other walkable one -- a trie walk
// from the root, or a window record list -- is numbered wave-wide (ballot + mbcnt per tuple
// slot), its lane and slot written as one byte to the wave's 256-B LDS scratch, and the walks run
// over the numbered lookups: lane i takes lookups r0 + i and r0 + 64 + i, pulling their address
// and key from the owning lanes (ds_bpermute), then the owners pull the verdicts back. The wave
// then issues its gathers for the lookups that need them only, in one lockstep pass of two per
// lane for up to 128 of them, instead of P / 2 passes over every lane's every slot (the lanes the
// window resolved only exec-masked). ANY-protocol packets take the linear scan on their lane.
#ifndef PG_CANDI_COMPACT
#define PG_CANDI_COMPACT 1
#endif
// Active lanes: the grid-stride loop runs lane l of a wave while its group index q0 + l is below
// nfull, so the lanes that reach this function always form a prefix 0 .. na-1 of the wave (the
// last wave of a launch whose group count is not a multiple of 64 holds fewer). The walks are
// spread over those na lanes only: lane i takes lookups r0 + i and r0 + na + i, r0 stepping by
// 2 na, and the owner of lookup g pulls its verdict from lane (g - r0) mod na -- an inactive lane
// would never walk the lookups given to it.
template <bool COUNT, int P>
__device__ __forceinline__ void classify_candi_group(const DevTableSet& T, const DevTable& tab0, uint8_t* scr,
                                                     const uint32_t (&s)[P], const uint32_t (&dp)[P],
                                                     const uint32_t (&pr)[P], const Hist& h, uint32_t (&out)[P]) {
    // the scratch holds one byte per pending lookup (64 lanes x 4 slots = 256 B per wave, the
    // launcher's BS * 4 bytes) and a byte encodes its owner as lane * 4 + slot
    static_assert(P == 4, "classify_candi_group: 4 tuples per lane (scratch size, owner encoding)");
#if defined(__HIP_DEVICE_COMPILE__)  // (device code only: wave intrinsics)
    const uint32_t lane = __lane_id();
    const uint32_t na = (uint32_t)__popcll(__ballot(true));  // active lanes: 0 .. na-1
    const LdsLoader l0{};
    const DevLoader blob{T.blobs + tab0.blob_off};
    const uint32_t wb = tab0.kroot, wsz = tab0.nkc, woff = candi_window_off((tab0.fsk >> 8) & 0xFFu);
    uint32_t key[P], g[P];
    bool pend[P];
#pragma unroll
    for (int j = 0; j < P; j++) {
        key[j] = pkt_key(pr[j], dp[j]);
        pend[j] = key[j] < kWalkKeyLimit;
        out[j] = 0;
        const uint32_t wd = s[j] - wb;
        if (pend[j] && wd < wsz) {  // the window's terminal entry: an inline candidate or the default ends here
            const W2 v = l0.u2(woff + 2u * wd);
            if (!(v.y & kCandiNode)) {
                const uint32_t klo = v.x & 0x3FFFFu, khi = (v.x >> 18) | ((v.y & 15u) << 14);
                const uint32_t rel = (v.y >> 6) & kCandiDefault;
                const bool hit = key[j] >= klo && key[j] <= khi && rel != kCandiDefault;
                out[j] = hit ? (((v.y >> 4) & 3u) << 30) | (tab0.rule_base + rel) : tab0.dflt;
                pend[j] = false;
            }
        }
    }
    uint32_t M = 0;  // walks left in the wave (uniform)
#pragma unroll
    for (int j = 0; j < P; j++) {
        const unsigned long long m = __ballot(pend[j]);
        g[j] = M + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (pend[j]) scr[g[j]] = (uint8_t)(lane * 4u + (uint32_t)j);
        M += (uint32_t)__popcll(m);
    }
    const BlobTab tb1{tab0.fsk, tab0.dflt, tab0.kroot, tab0.xoff, tab0.nkc, tab0.rule_base};
    for (uint32_t r0 = 0; r0 < M; r0 += 2u * na) {
        uint32_t vs[2], vk[2], res[2] = {0u, 0u}, pos[2] = {0u, 0u};
        const uint32_t zero[2] = {0u, 0u};
        bool on[2], pd[2] = {false, false};
        const DevLoader ld[2] = {blob, blob};
        const LdsLoader ld0[2] = {l0, l0};
        const BlobTab tb[2] = {tb1, tb1};
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const uint32_t gi = r0 + na * (uint32_t)q + lane;
            on[q] = gi < M;
            const uint32_t id = on[q] ? (uint32_t)scr[gi] : 0u;
            const int a = (int)((id >> 2) << 2);  // the owning lane, as a byte address
            uint32_t xs = 0, xk = 0;
#pragma unroll
            for (int j = 0; j < P; j++) {
                const uint32_t ps = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)s[j]);
                const uint32_t pk = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)key[j]);
                if ((id & 3u) == (uint32_t)j) xs = ps, xk = pk;
            }
            vs[q] = xs;
            vk[q] = xk;
        }
        candi_walk(ld, ld0, tb, on, vs, vk, res, pd, pos);
        rec_walk(ld, tb, zero, vk, pd, pos, res);
#pragma unroll
        for (int j = 0; j < P; j++) {  // the owners pull their verdicts back
            const uint32_t rel = g[j] - r0;
            const bool hi = rel >= na;
            const int a = (int)(((hi ? rel - na : rel) & 63u) << 2);
            const uint32_t v0 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)res[0]);
            const uint32_t v1 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)res[1]);
            if (pend[j] && rel < 2u * na) out[j] = hi ? v1 : v0;
        }
    }
#pragma unroll
    for (int j = 0; j < P; j++)
        if (key[j] >= kWalkKeyLimit)
            out[j] = eval_linear(T.rules, tab0.rule_base, tab0.n_rules, tab0.dflt, s[j], 0u, key[j]);
    if (COUNT) {
#pragma unroll
        for (int j = 0; j < P; j++) h.inc(out[j] & kSlotMask);
    }
#endif
}

template <int MODE, bool COUNT, bool VEC, int STAGE_, bool NODE, int BS>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(kernel_wpe<MODE, COUNT, NODE, STAGE_>(),
                                                                    kernel_wpe_max<MODE, COUNT, NODE, STAGE_>())))
void k_classify(DevTableSet T, int32_t t, const uint32_t* __restrict__ src,
                                                     const uint32_t* __restrict__ dst,
                                                     const uint16_t* __restrict__ sport,
                                                     const uint16_t* __restrict__ dport,
                                                     const uint8_t* __restrict__ proto, uint64_t n,
                                                     uint32_t* __restrict__ out, unsigned long long* counters,
                                                     uint32_t stage_words, uint32_t hist_cells) {
    constexpr int STAGE = STAGE_ & 7;
    constexpr bool NODST = MODE == 0 && (STAGE_ & 8);
    // STAGE_ + 16 (node kernels with counters): the LDS histogram holds every slot (launcher)
    constexpr bool FULLH = NODE && COUNT && (STAGE_ & 16);
    // STAGE_ + 32 (node kernels): the node set has no PAIR tables -- the evaluation carries no
    // PAIR code (A/B on MI355X: config 5 with counters 118.9 -> 124.7 Gpps, config 3 +1 %)
    constexpr bool NOPAIR = NODE && (STAGE_ & 32);
    // STAGE_ + 64 (node kernels): the node's uniform cross layout (DevNode uniform; with + 32)
    constexpr bool UNIF = NODE && NOPAIR && (STAGE_ & 64);
    // PERPOD / CONN over a uniform node: ANY-protocol packets deferred to k_node_any
    // (PG_CONN_DEFER_ANY, PG_POD_DEFER_ANY)
    constexpr bool DEFER = UNIF && defer_any<MODE>();
    // STAGE_ + 128 (uniform node): its wide class records (DevNode wide: 255 tables or more)
    constexpr bool WIDE = UNIF && (STAGE_ & 128);
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t* hist = smem + (STAGE ? stage_words : 0u);
    // node kernels: the LDS histogram, when used, holds every slot (HistT<true>: no window test)
    // STAGE_ + 256 (with + 16): the histogram's cells are 16 bits (HistT kHalf)
    constexpr bool HALF = FULLH && (STAGE_ & 256);
    HistT<NODE, NODE && MODE == 1 && !FULLH, NODE && !FULLH, FULLH, FULLH && MODE == 2 && PG_CONN_HOT_REGS, HALF> h{nullptr,
                                                                                                  counters};
    DevTable tab0{};
    const uint32_t* blobs = T.blobs;
    // the node image: its LDS copy (at LDS address 0: LdsLoader) when staged, else global memory
    using ImgLoader = std::conditional_t<NODE && STAGE != 0, LdsLoader, DevLoader>;
    ImgLoader img{};
    if constexpr (NODE && STAGE == 0) img = DevLoader{T.node.img};
    if (NODE && STAGE) {
        const uint4* g = reinterpret_cast<const uint4*>(T.node.img);
        for (uint32_t i = threadIdx.x; i < stage_words / 4u; i += BS) reinterpret_cast<uint4*>(smem)[i] = g[i];
    }
    if (MODE == 0) {
        tab0 = load_tab(T.tabs, t);
        if (STAGE) {
            const uint4* g = reinterpret_cast<const uint4*>(T.blobs + tab0.blob_off);
            for (uint32_t i = threadIdx.x; i < stage_words / 4u; i += BS) reinterpret_cast<uint4*>(smem)[i] = g[i];
            if (STAGE == 1 || STAGE == 4) {  // (STAGE 5: the prefix in LDS, the rest read from HBM)
                blobs = smem;
                tab0.blob_off = 0;
            }
        }
    }
    // STAGE 2 / 6: only the header and src-trie root of a large blob are in LDS
    const uint32_t* rootb = (MODE == 0 && (STAGE == 2 || STAGE == 6)) ? smem : nullptr;
    // hit counters: an LDS histogram of the window [wbase, wbase + wn) of slots plus cells for
    // slots xslot and xslot1, flushed with one u64 atomic per non-zero cell; slots outside go to
    // global atomics. Every slot fits the window unless the table set has more than
    // kLdsHistMax - 2; then the window is a SINGLE table's first rules (first-match traffic
    // favours them: config 4's Zipf depth) and the extra cells its default-deny slot and its
    // last rule (a deny-the-rest / allow-all catch-all takes every unmatched packet: a single
    // global address would serialise them); node modes: "no ACL", "unresolved"
    // node kernels over more slots than the full histogram holds count through an LDS slot
    // cache of hist_cells (a power of two) cells (HistT kCache), else with global atomics only
    const bool lds_hist = FULLH || (COUNT && (!NODE || hist_cells >= T.n_slots));
    const bool cache = NODE && COUNT && !lds_hist && hist_cells != 0;
    const bool has_hist = COUNT && (!NODE || lds_hist || cache);  // an LDS histogram was allocated
    // STAGE 6 (PG_CANDI_COMPACT): each wave's 256-B scratch after the staged words and histogram
    // (cells + 2 words; a node slot cache would take 2 (cells + 1))
    const uint32_t hist_words = !has_hist ? 0u
                                : (cache ? 2u * (hist_cells + 1u) : (HALF ? (hist_cells + 1u) / 2u + 1u : hist_cells + 2u));
    uint8_t* const cscr = reinterpret_cast<uint8_t*>(smem + stage_words + hist_words) + (threadIdx.x >> 6) * 256u;
    const uint32_t wn = COUNT ? hist_cells : 0u;
    const uint32_t wbase = (MODE == 0 && wn < T.n_slots) ? min(tab0.rule_base, T.n_slots - wn) : 0u;
    const uint32_t xslot = MODE == 0 ? (tab0.dflt & kSlotMask) : T.slot_noacl;
    const uint32_t xslot1 = MODE == 0 ? (tab0.n_rules ? tab0.rule_base + tab0.n_rules - 1u : xslot) : T.slot_unresolved;
    if (COUNT) {
        if (has_hist && !cache)
            for (uint32_t i = threadIdx.x; i < hist_words; i += BS) hist[i] = 0;
        h.lds = lds_hist ? hist : nullptr;
        h.wbase = wbase;
        h.wn = wn;
        h.xslot = xslot;
        h.xslot1 = xslot1;
        h.full = wn >= T.n_slots;
        if (MODE == 0 && PG_HOT_SLOT) h.hot = xslot1;
        if (FULLH && MODE == 2 && PG_CONN_HOT_REGS) {  // "no ACL" and the most shared inbound ACL's last rule
            h.hot = T.slot_noacl;
            h.hot2 = T.slot_hot_in;
        }
        // node kernels whose table set has more slots than the LDS histogram holds: the
        // catch-all of the node-output interface's outbound table (traffic to remote pods and
        // the Internet) in a register -- config 6 with counters 0.4 -> 5.6 Gpps when every
        // increment was a global atomic; with the histogram in LDS it costs 2 % (configs 3, 5)
        if (MODE != 0 && PG_HOT_SLOT_NODE && !lds_hist && T.node_out >= 0) {
            const DevTable no = load_tab(T.tabs, T.node_out);
            if (no.n_rules) h.hot = no.rule_base + no.n_rules - 1u;
        }
        if (cache) {  // keys [0, wn] then counts [0, wn]; cell wn holds the register-counted hot slot
            for (uint32_t i = threadIdx.x; i <= wn; i += BS) {
                hist[i] = i == wn ? h.hot : kCacheEmpty;
                hist[wn + 1u + i] = 0u;
            }
            h.ckey = hist;
            h.cmask = wn - 1u;
            h.cshift = 32u - (uint32_t)__builtin_ctz(wn);
        }
    }
    if (STAGE || COUNT) __syncthreads();
    // group indices and stream offsets in 32 bits (PG_IDX32: the launcher keeps a launch below
    // kMaxLaunchTuples, so every byte offset of a stream fits 32 bits): a load is then the SGPR base
    // plus a 32-bit VGPR offset, with no 64-bit address arithmetic per stream and group
    using Idx = std::conditional_t<PG_IDX32 != 0, uint32_t, uint64_t>;
    const Idx stride = (Idx)gridDim.x * BS;
    const Idx first = (Idx)blockIdx.x * BS + threadIdx.x;
    // full groups of P tuples per lane (P = tuples_per_lane): SoA fields read with 16/8/4-byte loads per
    // lane (coalesced, non-temporal); prefetch 1/2: the next group's loads are in flight
    // while this group is classified
    constexpr int P = tuples_per_lane<MODE>();
    static_assert(P % 4 == 0, "a group's protocol bytes are loaded as whole words (PG_TPL, PG_TPL_CONN)");
    const Idx nfull = VEC ? (Idx)(n / P) : 0;
    // element i of a stream, its byte offset computed in Idx
    auto el = [](auto* base, Idx i) {
        using E = std::remove_pointer_t<decltype(base)>;
        using C = std::conditional_t<std::is_const<E>::value, const char, char>;
        return reinterpret_cast<decltype(base)>(reinterpret_cast<C*>(base) + (Idx)(i * (Idx)sizeof(E)));
    };
    struct Group {
        Words<P> s, d;
        Words<P / 2> dp, sp;
        Words<P / 4> pr;
    };
    // STAGE 4 / 5 (SINGLE over an FD table): no rule tests dst, so the dst stream is not read
    constexpr bool FD = MODE == 0 && (STAGE == 4 || STAGE == 5);
    constexpr bool NEED_DST = !FD && !NODST;
    const uint32_t* fd_blob = FD ? (STAGE == 4 ? smem : T.blobs + tab0.blob_off) : nullptr;
    auto load = [&](Idx q) {
        Group x;
        const Idx i0 = q * P;
        x.s = ld_words<P>(el(src, i0));
        if (NEED_DST) x.d = ld_words<P>(el(dst, i0));
        else x.d = Words<P>{};
        x.dp = ld_words<P / 2>(reinterpret_cast<const uint32_t*>(el(dport, i0)));
        x.pr = ld_words<P / 4>(reinterpret_cast<const uint32_t*>(el(proto, i0)));
        if (MODE == 2) x.sp = ld_words<P / 2>(reinterpret_cast<const uint32_t*>(el(sport, i0)));
        else x.sp = Words<P / 2>{};
        return x;
    };
    Idx q = first;
    Group cur;
    // default: SINGLE over an LDS-staged blob none, SINGLE over a blob in HBM (STAGE 0 / 2) and
    // the node modes the next group at the top of the iteration (A/B on MI355X, config 4 with
    // four tuples per chunk: 172.9 vs 169.3 Gpps)
    constexpr int PF0 = FD ? PG_PREFETCH_FD
                          : (PG_PREFETCH >= 0 ? PG_PREFETCH
                                              : ((MODE == 0 && STAGE != 0 && STAGE != 2 && STAGE != 6) ||
                                                 node_wide<MODE, COUNT, NODE, STAGE_>()
                                                     ? 0 : 1));
    constexpr int PF = (!NODE && PF0 == 2) ? 1 : PF0;  // (only node kernels have the gather hook)
    // PD = 2 (PG_PF_DEPTH): the loads run two groups ahead (group q + 2 * stride is
    // loaded while group q is classified). PF 3: the loads are issued after the group's
    // classification (its gathers waited for) and verdict store. Vector-memory
    // operations retire in issue order (MI355X_MICROARCH.md, vmcnt), so a cross-table gather
    // issued after a stream load waits for that load too.
    constexpr int PD = PF ? PG_PF_DEPTH : 1;
    // classification of one group (P tuples per lane, loaded), its verdicts stored; hk: called
    // once after the first chunk's cross-entry loads are issued (node kernels, PF 2)
    auto run_group = [&](const Group& g, Idx qq, auto&& hk) {
        uint32_t sv[P], dv[P], spv[P], dpv[P], prv[P], o[P];
        // (DEFER) a protocol code > 2 among the group's: this launch's number into its stream's
        // mark word for k_node_any (one test of the packed protocol word per group, no state
        // across groups)
        if constexpr (DEFER) {
            bool any = false;
#pragma unroll
            for (int k = 0; k < P / 4; k++) any |= any_proto_gt2(g.pr.w[k]);
            if (any) *T.any_mark = T.any_seq;
        }
#pragma unroll
        for (int j = 0; j < P; j++) {
            sv[j] = g.s.w[j];
            dv[j] = g.d.w[j];
            dpv[j] = (g.dp.w[j / 2] >> (16 * (j & 1))) & 0xFFFFu;
            spv[j] = (g.sp.w[j / 2] >> (16 * (j & 1))) & 0xFFFFu;
            prv[j] = (g.pr.w[j / 4] >> (8 * (j & 3))) & 0xFFu;
        }
#if PG_PROBE_STREAM
        for (int j = 0; j < P; j++) o[j] = sv[j] ^ dv[j] ^ dpv[j] ^ prv[j] ^ spv[j];
#else
        // per-mode chunk: the group's P tuples are classified QC at a time (less state per
        // lane, more waves per SIMD)
        constexpr int QC = MODE == 2 ? (COUNT ? PG_QCONN_COUNT : PG_QCONN)
                                     : (MODE == 1 ? (FULLH ? PG_QPOD_FULLH : PG_QPOD)
                                                  : (FD ? (STAGE == 4 ? PG_QSINGLE_FD : PG_QSINGLE_FDG)
                                                        : (STAGE == 1   ? PG_QSINGLE_LDS
                                                           : STAGE == 6 ? (COUNT ? PG_QSINGLE : PG_QCANDI)
                                                                        : PG_QSINGLE)));
        if constexpr (MODE == 0 && STAGE == 6 && PG_CANDI_COMPACT) {
            classify_candi_group<COUNT, P>(T, tab0, cscr, sv, dpv, prv, h, o);
        } else
#pragma unroll
        for (int c = 0; c < P; c += QC) {
            uint32_t cs[QC], cd[QC], csp[QC], cdp[QC], cpr[QC], co[QC];
#pragma unroll
            for (int j = 0; j < QC; j++)
                cs[j] = sv[c + j], cd[j] = dv[c + j], csp[j] = spv[c + j], cdp[j] = dpv[c + j], cpr[j] = prv[c + j];
            if constexpr (FD) {
                if constexpr (STAGE == 4) classify_fd_q<COUNT, QC>(T, LdsLoader{}, LdsLoader{}, tab0, cs, cdp, cpr, h, co);
                else classify_fd_q<COUNT, QC>(T, LdsLoader{}, DevLoader{fd_blob}, tab0, cs, cdp, cpr, h, co);
            } else if constexpr (MODE == 0 && STAGE == 6) {
                classify_candi_q<COUNT, QC>(T, LdsLoader{}, DevLoader{T.blobs + tab0.blob_off}, tab0, cs, cdp, cpr, h, co);
            } else if constexpr (NODE) {
                if (c == (PG_HOOK_LAST ? P - QC : 0))
                    classify_node_q<MODE, COUNT, QC, STAGE && PG_PRED, STAGE == 3, NOPAIR, UNIF, DEFER, WIDE>(T, T.node, img, cs, cd, csp, cdp, cpr, h, co, hk);
                else
                    classify_node_q<MODE, COUNT, QC, STAGE && PG_PRED, STAGE == 3, NOPAIR, UNIF, DEFER, WIDE>(T, T.node, img, cs, cd, csp, cdp, cpr, h, co);
            } else {
                classify_q<MODE, COUNT, QC, STAGE == 1 && PG_PRED>(T, blobs, tab0, cs, cd, csp, cdp, cpr, h, co, rootb);
            }
#pragma unroll
            for (int j = 0; j < QC; j++) o[c + j] = co[j];
        }
#endif
        Words<P> ow;
#pragma unroll
        for (int j = 0; j < P; j++) ow.w[j] = o[j];
        st_words<P>(ow, el(out, qq * P));
    };
    Group ahead{};
    if (PF && q < nfull) cur = load(q);
    if (PD == 2 && q + stride < nfull) ahead = load(q + stride);
    while (q < nfull) {
        const Idx qn = q + stride, qa = PD == 2 ? qn + stride : qn;  // qa: the group loaded now
        Group nxt = PD == 2 ? ahead : cur;
        if (!PF) cur = load(q);
        auto issue = [&]() {
            if (qa < nfull) {
                if constexpr (PD == 2) ahead = load(qa);
                else nxt = load(qa);
            }
        };
        if (PF == 1) issue();
        auto hook = [&]() {
            if (PF == 2) issue();
        };
        run_group(cur, q, hook);
        if (PF == 3) issue();  // (the loads after the group's classification and verdict store)
        cur = nxt;
        q = qn;
    }
    // remainder (or everything when the pointers are not vector-aligned): one tuple per lane
    for (uint64_t i = (uint64_t)nfull * P + first; i < n; i += stride) {
        const uint32_t s1[1] = {src[i]}, d1[1] = {NEED_DST ? dst[i] : 0u},
                       sp1[1] = {MODE == 2 ? (uint32_t)sport[i] : 0u}, dp1[1] = {dport[i]}, pr1[1] = {proto[i]};
        uint32_t o[1];
        if constexpr (FD && STAGE == 4) classify_fd_q<COUNT, 1>(T, LdsLoader{}, LdsLoader{}, tab0, s1, dp1, pr1, h, o);
        else if constexpr (FD) classify_fd_q<COUNT, 1>(T, LdsLoader{}, DevLoader{fd_blob}, tab0, s1, dp1, pr1, h, o);
        else if constexpr (MODE == 0 && STAGE == 6)
            classify_candi_q<COUNT, 1>(T, LdsLoader{}, DevLoader{T.blobs + tab0.blob_off}, tab0, s1, dp1, pr1, h, o);
        else if constexpr (NODE) classify_node_q<MODE, COUNT, 1, STAGE && PG_PRED, STAGE == 3, NOPAIR, UNIF, DEFER, WIDE>(T, T.node, img, s1, d1, sp1, dp1, pr1, h, o);
        else classify_q<MODE, COUNT, 1, STAGE == 1 && PG_PRED>(T, blobs, tab0, s1, d1, sp1, dp1, pr1, h, o, rootb);
        out[i] = o[0];
        if (DEFER && pr1[0] > 2u) *T.any_mark = T.any_seq;
    }
    // (the packets deferred above -- ANY protocol, rare -- are classified by k_node_any, launched
    // after this kernel on the same stream)
    if (COUNT) {
        h.flush_hot();
        __syncthreads();
        if constexpr (HALF) {  // two 16-bit cells per word: slots 2i and 2i + 1
            for (uint32_t i = threadIdx.x; i < (wn + 1u) / 2u; i += BS) {
                const uint32_t v = hist[i];
                if (v & 0xFFFFu) atomicAdd(&counters[2u * i], (unsigned long long)(v & 0xFFFFu));
                if ((v >> 16) && 2u * i + 1u < wn) atomicAdd(&counters[2u * i + 1u], (unsigned long long)(v >> 16));
            }
            return;
        }
        for (uint32_t i = threadIdx.x; has_hist && i <= wn + 1u; i += BS) {
            if (cache && i > wn) break;
            const uint32_t v = cache ? hist[wn + 1u + i] : hist[i];
            const uint32_t slot = cache ? hist[i] : (i < wn ? wbase + i : (i == wn ? xslot : xslot1));
#if !defined(PG_PROBE_NOFLUSH)  // measurement build only: the histogram is not flushed
            if (v) atomicAdd(&counters[slot], (unsigned long long)v);
#endif
        }
    }
}

// Stream probe (measurement): exactly the loads and the store of a k_classify launch over the
// same batch -- src, dport, proto (+ dst when DST, + sport when SP), P tuples per lane with
// 16/8/4-byte non-temporal loads, one 16-byte verdict store -- with a 1-instruction "verdict"
// instead of the classification. Its rate is the ceiling a classify launch of that byte mix
// can reach on this GPU (bench.py frac_of_stream_ceiling).
template <bool DST, bool SP, int BS>
__global__ __launch_bounds__(BS) void k_stream_probe(const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                                                     const uint16_t* __restrict__ sport,
                                                     const uint16_t* __restrict__ dport,
                                                     const uint8_t* __restrict__ proto, uint64_t n,
                                                     uint32_t* __restrict__ out) {
    constexpr int P = PG_TPL;
    const uint64_t stride = (uint64_t)gridDim.x * BS;
    const uint64_t first = (uint64_t)blockIdx.x * BS + threadIdx.x;
    const uint64_t nfull = n / P;
    for (uint64_t q = first; q < nfull; q += stride) {
        const uint64_t i0 = q * P;
        const Words<P> s = ld_words<P>(src + i0);
        const Words<P> d = DST ? ld_words<P>(dst + i0) : Words<P>{};
        const Words<P / 2> dp = ld_words<P / 2>(reinterpret_cast<const uint32_t*>(dport + i0));
        const Words<P / 2> sp = SP ? ld_words<P / 2>(reinterpret_cast<const uint32_t*>(sport + i0)) : Words<P / 2>{};
        const Words<P / 4> pr = ld_words<P / 4>(reinterpret_cast<const uint32_t*>(proto + i0));
        Words<P> o;
#pragma unroll
        for (int j = 0; j < P; j++)
            o.w[j] = s.w[j] ^ d.w[j] ^ ((dp.w[j / 2] >> (16 * (j & 1))) & 0xFFFFu) ^
                     ((sp.w[j / 2] >> (16 * (j & 1))) & 0xFFFFu) ^ ((pr.w[j / 4] >> (8 * (j & 3))) & 0xFFu);
        st_words<P>(o, out + i0);
    }
    for (uint64_t i = nfull * P + first; i < n; i += stride)
        out[i] = src[i] ^ (DST ? dst[i] : 0u) ^ dport[i] ^ (SP ? (uint32_t)sport[i] : 0u) ^ proto[i];
}

// K1: reference-shaped linear scan, one lane per tuple, rules wave-uniform
__global__ __launch_bounds__(kBlock) void k_linear(DevTableSet T, uint32_t t, const uint32_t* __restrict__ src,
                                                   const uint32_t* __restrict__ dst,
                                                   const uint16_t* __restrict__ dport,
                                                   const uint8_t* __restrict__ proto, uint64_t n,
                                                   uint32_t* __restrict__ out) {
    const DevTable hd = T.tabs[t];
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t base = (uint64_t)blockIdx.x * kBlock; base < n; base += stride) {
        const uint64_t i = base + threadIdx.x;
        const bool valid = i < n;
        uint32_t s = 0, d = 0, key = 0;
        if (valid) {
            s = src[i];
            d = dst[i];
            key = pkt_key(proto[i], dport[i]);
        }
        const bool any = key >= kKeyANY;
        bool done = !valid;
        uint32_t res = verdict(kActDeny, T.n_rules + t);
        for (uint32_t r = 0; r < hd.n_rules; r++) {
            if (__all(done)) break;
            const DevRule R = T.rules[hd.rule_base + r];
            if (!done && (s & R.smask) == R.snet && (d & R.dmask) == R.dnet) {
                uint32_t a = 4u;
                if (any) {
                    if ((R.act >> 4) != kActNever) a = (R.act >> 4) & 3u;
                } else if (key >= R.klo && key <= R.khi) {
                    a = R.act & 3u;
                }
                if (a < 4u) {
                    res = verdict(a, hd.rule_base + r);
                    done = true;
                }
            }
        }
        if (valid) out[i] = res;
    }
}

// ---- K5 generator ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t rnd(uint64_t seed, uint64_t i, uint32_t f) {
    return mix64(seed ^ mix64(i * 16ull + f));
}

__global__ __launch_bounds__(kBlock) void k_gen(DevTableSet T, GenParams g, uint64_t n, uint32_t* src, uint32_t* dst,
                                                uint16_t* sport, uint16_t* dport, uint8_t* proto) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t l = (uint64_t)blockIdx.x * kBlock + threadIdx.x; l < n; l += stride) {
        const uint64_t i = g.index_base + l;
        const uint64_t r0 = rnd(g.seed, i, 0), r1 = rnd(g.seed, i, 1), r2 = rnd(g.seed, i, 2);
        const uint64_t r3 = rnd(g.seed, i, 3), r4 = rnd(g.seed, i, 4), r5 = rnd(g.seed, i, 5);
        const uint32_t pct = (uint32_t)(r0 & 0xFFFFFFFFu) % 100u;
        uint32_t s, d, pr, dp;
        // protocol mix + ports (also the fallback for "inside" picks with an empty key range)
        const uint32_t pp = (uint32_t)(r3 & 0xFFFFFFFFu) % 100u;
        pr = pp < g.tcp_pct ? 0u : (pp < g.tcp_pct + g.udp_pct ? 1u : 2u);
        if (g.n_port_pool && (uint32_t)(r4 >> 32) % 100u < g.port_pool_pct)
            dp = g.port_pool[(uint32_t)(r4 & 0xFFFFFFFFu) % g.n_port_pool];
        else
            dp = (uint32_t)(r4 & 0xFFFFu);
        s = (g.n_ip_pool && (uint32_t)(r1 >> 32) % 100u < g.pool_pct) ? g.ip_pool[(uint32_t)r1 % g.n_ip_pool]
                                                                     : (uint32_t)r1;
        d = (g.n_ip_pool && (uint32_t)(r2 >> 32) % 100u < g.dst_pool_pct) ? g.ip_pool[(uint32_t)r2 % g.n_ip_pool]
                                                                         : (uint32_t)r2;
        if (g.table_id >= 0 && pct < g.inside_pct) {
            const DevTable hd = T.tabs[g.table_id];
            uint32_t k;
            const uint64_t r6 = rnd(g.seed, i, 6);
            if (g.zipf_cdf) {
                const uint32_t u = (uint32_t)(r6 >> 32);
                uint32_t lo = 0, hi = hd.n_rules - 1;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (u < g.zipf_cdf[mid]) hi = mid;
                    else lo = mid + 1;
                }
                k = lo;
            } else {
                k = (uint32_t)(r6 % hd.n_rules);
            }
            const DevRule R = T.rules[hd.rule_base + k];
            s = R.snet | ((uint32_t)r1 & ~R.smask);
            d = R.dnet | ((uint32_t)r2 & ~R.dmask);
            if (R.klo <= R.khi) {
                const uint32_t key = R.klo + (uint32_t)((r4 >> 16) % (uint64_t)(R.khi - R.klo + 1u));
                if (key < kKeyUDP) pr = 0u, dp = key;
                else if (key < kKeyOTHER) pr = 1u, dp = key & 0xFFFFu;
                else pr = 2u;
            }
        }
        if (pct >= 100u - g.nomatch_pct) s = 0xF0000000u | ((uint32_t)r1 & 0x0FFFFFFFu);
        src[l] = s;
        dst[l] = d;
        if (sport) sport[l] = (uint16_t)(r5 & 0xFFFFu);
        dport[l] = (uint16_t)dp;
        proto[l] = (uint8_t)pr;
    }
}

__global__ void k_conn_queries(DevTableSet T, const ConnQueryDev* q, uint32_t n, uint32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ConnQueryDev c = q[i];
    auto end = [&](int32_t ifc) {
        return ifc < 0 ? End{-1, -1, -1} : End{ifc, T.ifaces[2 * ifc], T.ifaces[2 * ifc + 1]};
    };
    const End es[1] = {end(c.src_if)}, ed[1] = {end(c.dst_if)};
    const uint32_t s1[1] = {c.src_ip}, d1[1] = {c.dst_ip}, ks[1] = {c.key_syn}, ka[1] = {c.key_synack};
    uint32_t o[1];
    const TabEval<1> ev{T, s1, d1, ks, ka};
    conn_q<1, false>(T, ev, es, ed, Hist{nullptr, nullptr}, o);
    out[i] = o[0];
}

// ---- launchers --------------------------------------------------------------------------------
// Launch knobs come from the calling context's Tuning (device.hpp): blocks_per_cu (0 = as many
// workgroups per CU as fit), stage_max_words (blobs up to 64 KiB staged in LDS),
// node_stage_max_words, stage_root_max_words (larger blobs: header + src root up to 2^14
// entries), node_path, node_common_lds_max (LDS bytes -- image + counter histogram -- up to
// which a node image's common-row section is staged: 80 KiB keeps two 512-thread workgroups
// per CU), block_stage (workgroup size of LDS-staged launches; 0 = per mode).
constexpr uint32_t kCommonStageExtraWords = 8192;  // the section may take the image past the base cap

// CUs of the current device (per device: contexts on different GPUs share the process)
static uint32_t num_cus() {
    constexpr int kMaxDev = 64;
    static std::atomic<uint32_t> cus[kMaxDev] = {};  // contexts on several threads may launch at once
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return 256;
    uint32_t c = cus[dev].load(std::memory_order_relaxed);
    if (!c) {
        hipDeviceProp_t p;
        c = (hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0) ? (uint32_t)p.multiProcessorCount
                                                                                       : 256u;
        cus[dev].store(c, std::memory_order_relaxed);
    }
    return c;
}

static int grid_for(uint64_t items, uint32_t blocks_per_cu = 0) {
    const uint32_t bpc = blocks_per_cu ? blocks_per_cu : 4u;
    uint64_t g = (items + kBlock - 1) / kBlock;
    return (int)std::max<uint64_t>(1, std::min<uint64_t>(g, (uint64_t)num_cus() * bpc));
}

// Grid of a grid-stride classify kernel: exactly the workgroups that are resident at once
// (registers / LDS of this instantiation), so no workgroup waits for another to finish, capped
// by the work and by blocks_per_cu when set.
template <class K>
static int grid_resident(K kernel, int bs, size_t lds, uint64_t items, uint32_t blocks_per_cu) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, bs, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    const int occ = per_cu;
    if (blocks_per_cu) per_cu = std::min<int>(per_cu, (int)blocks_per_cu);
    const uint64_t g = (items + bs - 1) / bs;
    const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(g, (uint64_t)num_cus() * per_cu));
    static const bool dbg = std::getenv("PG_DEBUG_LAUNCH") != nullptr;  // measurement aid: launch geometry
    if (dbg) std::fprintf(stderr, "pg launch: block %d, LDS %zu B, occupancy %d blocks/CU, grid %d\n", bs, lds, occ, grid);
    return grid;
}

template <int MODE, bool COUNT, bool VEC, int STAGE, bool NODE, int BS>
static void launch_bs(const DevTableSet& T, const Tuning& tu, int t, const uint32_t* src, const uint32_t* dst, const uint16_t* sport,
                      const uint16_t* dport, const uint8_t* proto, uint64_t n, uint32_t* out,
                      unsigned long long* counters, hipStream_t st, size_t hist, uint32_t cells, uint32_t stage,
                      uint64_t items) {
    auto k = k_classify<MODE, COUNT, VEC, STAGE, NODE, BS>;
    // SINGLE over an LDS-staged FD table without counters: two resident workgroups per CU, not
    // the three LDS would allow (A/B on MI355X, config 2: 541-546 vs 533-535 Gpps, repeated
    // three times; with counters no difference): fewer streams in flight per CU contend less
    const uint32_t bpc = tu.blocks_per_cu ? tu.blocks_per_cu : (MODE == 0 && (STAGE & 7) == 4 && !COUNT ? 2u : 0u);
    // (STAGE 6 with PG_CANDI_COMPACT: + 256 B of scratch per wave)
    const size_t lds = hist + (size_t)stage * 4 + (!NODE && (STAGE & 7) == 6 && PG_CANDI_COMPACT ? (size_t)BS * 4 : 0);
    // PERPOD / CONN over a uniform node: k_node_any after the classify kernel, for its deferred
    // ANY-protocol packets (PG_CONN_DEFER_ANY, PG_POD_DEFER_ANY; the launch's mark word and
    // number: dev_classify)
    constexpr bool defer = NODE && (STAGE & 32) && (STAGE & 64) && defer_any<MODE>();
    hipLaunchKernelGGL(k, dim3(grid_resident(k, BS, lds, items, bpc)), dim3(BS), lds, st, T, t, src, dst, sport, dport,
                       proto, n, out, counters, stage, cells);
    if constexpr (defer && !PG_PROBE_NOANYLAUNCH) {  // (measurement build: -DPG_PROBE_NOANYLAUNCH=1 skips it)
        auto ka = k_node_any<MODE, COUNT>;
        hipLaunchKernelGGL(ka, dim3(grid_for(n)), dim3(kBlock), 0, st, T, src, dst, proto, n, out, counters);
    }
}

// Workgroup size: a staged image is shared by the workgroup, so larger workgroups hold more
// waves per CU for the same LDS.
template <int MODE, bool COUNT, bool VEC, int STAGE, bool NODE>
static void launch_one(const DevTableSet& T, const Tuning& tu, int t, const uint32_t* src, const uint32_t* dst, const uint16_t* sport,
                       const uint16_t* dport, const uint8_t* proto, uint64_t n, uint32_t* out,
                       unsigned long long* counters, hipStream_t st, size_t hist, uint32_t cells, uint32_t stage,
                       uint64_t items) {
    if constexpr ((STAGE & 7) != 0) {
        // 512 (A/B on MI355X: SINGLE with counters +14 % over 1024 at config 2; without
        // counters +2.5 % since SINGLE classifies one tuple per chunk, v15; config 4 over its
        // 12-bit staged root 163 vs 132 Gpps at 1024)
        // 1024 for CONN (32 waves per CU at 64 registers) and for SINGLE over an LDS-staged FD
        // blob whose LDS (+ histogram) leaves room for fewer than three workgroups per CU: one
        // image copy then serves 16 waves (A/B on MI355X, the 10k-rule sweep table, 59.5 KB:
        // 393.8 -> 471.5 Gpps; config 2's 49 KB blob, three fit: 530 vs 475 at 1024)
        const size_t lds_bytes = hist + (size_t)stage * 4;
        // (wide-record node builds, STAGE + 128: the per-mode workgroup size only -- block_stage is
        // an A/B knob of the other builds, and every extra size is another set of kernels)
        // The wide sets' images are larger (config 9: 502 tables, 53.8 KB with the common rows),
        // so LDS holds two workgroups per CU where config 3's 41 KB holds three: 768-thread
        // workgroups keep the 24 waves per CU of three 512-thread ones (PG_NODE_WIDE_REC_BS)
        // (16-bit-cell histogram builds, STAGE + 256: likewise)
        if constexpr (NODE && (STAGE & (128 | 256))) {
            constexpr int BSW = node_wide<MODE, COUNT, NODE, STAGE>() ? PG_NODE_WIDE_BS : PG_NODE_WIDE_REC_BS;
            return launch_bs<MODE, COUNT, VEC, STAGE, NODE, BSW>(T, tu, t, src, dst, sport, dport, proto, n, out,
                                                                 counters, st, hist, cells, stage, items);
        }
        if constexpr (node_wide<MODE, COUNT, NODE, STAGE>() && PG_NODE_WIDE_BS != 1024)
            if (!tu.block_stage)
                return launch_bs<MODE, COUNT, VEC, STAGE, NODE, PG_NODE_WIDE_BS>(T, tu, t, src, dst, sport, dport, proto,
                                                                                n, out, counters, st, hist, cells, stage,
                                                                                items);
        const uint32_t bs = tu.block_stage ? tu.block_stage
                            : node_wide<MODE, COUNT, NODE, STAGE>()                                ? 1024u
                            : (MODE == 0 && (STAGE & 7) == 4 && lds_bytes > kLdsPerCU / 3 && PG_FD_BS1024) ? 1024u
                                                                                                     : 512u;
        if (bs == 1024u)
            return launch_bs<MODE, COUNT, VEC, STAGE, NODE, 1024>(T, tu, t, src, dst, sport, dport, proto, n, out,
                                                                  counters, st, hist, cells, stage, items);
        if (bs == 512u)
            return launch_bs<MODE, COUNT, VEC, STAGE, NODE, 512>(T, tu, t, src, dst, sport, dport, proto, n, out,
                                                                 counters, st, hist, cells, stage, items);
    }
    launch_bs<MODE, COUNT, VEC, STAGE, NODE, 256>(T, tu, t, src, dst, sport, dport, proto, n, out, counters, st, hist,
                                                  cells, stage, items);
}

// SINGLE over a non-FD table: the blob in LDS (STAGE 1), its root in LDS (2) or all in HBM (0);
// NODST = 8 for dst-free tables
template <int MODE, bool COUNT, bool VEC, int NODST>
static void launch_generic(const DevTableSet& T, const Tuning& tu, int t, const uint32_t* src, const uint32_t* dst,
                           const uint16_t* sport, const uint16_t* dport, const uint8_t* proto, uint64_t n,
                           uint32_t* out, unsigned long long* counters, hipStream_t st, size_t hist, uint32_t cells,
                           uint32_t words, uint32_t root_words, uint64_t items) {
    const DevTable& hd = T.host_tabs[t];
    if (!(hd.fsk & kFlagLinear) && words && words <= tu.stage_max_words)
        launch_one<MODE, COUNT, VEC, 1 + NODST, false>(T, tu, t, src, dst, sport, dport, proto, n, out, counters, st,
                                                       hist, cells, words, items);
    else if ((hd.fsk & kFlagCandI) && NODST && PG_CANDI_LEAN && root_words <= tu.stage_root_max_words)
        launch_one<MODE, COUNT, VEC, 6 + NODST, false>(T, tu, t, src, dst, sport, dport, proto, n, out, counters, st,
                                                       hist, cells, root_words, items);
    else if (!(hd.fsk & kFlagLinear) && words && root_words <= tu.stage_root_max_words)
        launch_one<MODE, COUNT, VEC, 2 + NODST, false>(T, tu, t, src, dst, sport, dport, proto, n, out, counters, st,
                                                       hist, cells, root_words, items);
    else
        launch_one<MODE, COUNT, VEC, 0 + NODST, false>(T, tu, t, src, dst, sport, dport, proto, n, out, counters, st,
                                                       hist, cells, 0, items);
}

template <int MODE, bool COUNT, bool VEC>
static void launch_classify(const DevTableSet& T, const Tuning& tu, int t, const uint32_t* src, const uint32_t* dst,
                            const uint16_t* sport, const uint16_t* dport, const uint8_t* proto, uint64_t n,
                            uint32_t* out, unsigned long long* counters, hipStream_t st) {
    // hit-counter LDS histogram (k_classify): every slot + 2 cells; or (more slots than fit) a
    // SINGLE table's window of hist_window cells + 2; or a node set's slot cache (node_hist_cells
    // rounded down to a power of two; 0 = global atomics only)
    const bool node = MODE != 0 && tu.node_path && T.node.img;
    uint32_t cells = 0;
    size_t hist = 0;
    // node sets counted into 16-bit cells (k_classify STAGE + 256): the uniform layout, every
    // slot in the histogram, and a 32-bit histogram that even beside the base image would exceed
    // the LDS budget of two workgroups per CU (node_common_lds_max)
    const bool half = PG_NODE_HALF && COUNT && node && PG_NODE_FULLH && T.node.uniform && T.n_slots <= kLdsHistMax - 2u &&
                      ((size_t)T.n_slots + 2u) * 4 + (size_t)T.node.img_words_base * 4 > tu.node_common_lds_max;
    if (COUNT) {
        if (half) {
            cells = T.n_slots;
            hist = ((size_t)(cells + 1u) / 2u + 1u) * 4;
        } else if (T.n_slots <= kLdsHistMax - 2u) {
            cells = T.n_slots;
            hist = ((size_t)cells + 2u) * 4;
        } else if (!node) {
            cells = std::min(tu.hist_window, kLdsHistMax - 2u);
            hist = ((size_t)cells + 2u) * 4;
        } else if (tu.node_hist_cells >= 16u) {  // the slot cache: 2^k cells of {key, count} + the hot cell
            cells = 1u << (31 - __builtin_clz(tu.node_hist_cells));
            hist = ((size_t)cells + 1u) * 8;
        }
    }
    const uint64_t items = VEC ? (n + tuples_per_lane<MODE>() - 1) / tuples_per_lane<MODE>() : n;
    if constexpr (MODE == 0) {
        const DevTable& hd = T.host_tabs[t];
        const uint32_t words = T.host_blob_words[t];
        const uint32_t root_words = blob_root_words(hd.fsk, hd.nkc);  // (CANDI: + its window)
        const uint32_t prefix = T.host_blob_prefix[t];
        if ((hd.fsk & kFlagFD) && words <= tu.stage_max_words)  // FD blob in LDS, no dst stream
            launch_one<MODE, COUNT, VEC, 4, false>(T, tu, t, src, dst, sport, dport, proto, n, out, counters, st, hist,
                                                   cells, words, items);
        else if ((hd.fsk & kFlagFD) && prefix <= tu.stage_root_max_words)  // its prefix in LDS, the rest in HBM
            launch_one<MODE, COUNT, VEC, 5, false>(T, tu, t, src, dst, sport, dport, proto, n, out, counters, st, hist,
                                                   cells, prefix, items);
        else if (hd.fsk & kFlagDstFree)  // no rule tests dst: the dst stream is not read
            launch_generic<MODE, COUNT, VEC, 8>(T, tu, t, src, dst, sport, dport, proto, n, out, counters, st, hist,
                                                cells, words, root_words, items);
        else
            launch_generic<MODE, COUNT, VEC, 0>(T, tu, t, src, dst, sport, dport, proto, n, out, counters, st, hist,
                                                cells, words, root_words, items);
    } else if (node) {
        // the image with its common-row section and dst records when that fits the LDS budget
        // next to the histogram, else without the records (the kernel then reads them from the
        // cross array: lrec cleared), else the base image (STAGE 1), else the image is read from
        // HBM / L2
        DevTableSet Tn = T;
        const uint32_t all = T.node.img_words, norec = T.node.lrec ? T.node.lrec : all;
        auto fits = [&](uint32_t w) {
            return hist + (size_t)w * 4 <= tu.node_common_lds_max && w <= tu.node_stage_max_words + kCommonStageExtraWords;
        };
        // (+ 16: counters in an LDS histogram of every slot, k_classify FULLH)
        const bool full = PG_NODE_FULLH && COUNT && T.n_slots <= kLdsHistMax - 2u;
        // (+ 32: the set has no PAIR tables, k_classify NOPAIR)
        const bool nopair = T.node.n_pair == 0 && PG_NODE_NOPAIR;
        // (+ 64: the uniform cross layout, k_classify UNIF)
        const bool unif = T.node.uniform != 0;  // (no PAIR tables either; its tries take the aligned encoding)
        const bool wide = unif && T.node.wide != 0;  // (+ 128: its wide class records, k_classify WIDE)
        auto go1 = [&](auto stage, const DevTableSet& Ts, uint32_t words) {
            constexpr int S = decltype(stage)::value;
            if constexpr (COUNT) {
                if constexpr ((S & 64) != 0 && PG_NODE_HALF) {
                    if (full && half)
                        return launch_one<MODE, COUNT, VEC, S + 16 + 256, true>(Ts, tu, t, src, dst, sport, dport, proto,
                                                                                n, out, counters, st, hist, cells, words,
                                                                                items);
                }
                if (full)
                    return launch_one<MODE, COUNT, VEC, S + 16, true>(Ts, tu, t, src, dst, sport, dport, proto, n, out,
                                                                      counters, st, hist, cells, words, items);
            }
            launch_one<MODE, COUNT, VEC, S, true>(Ts, tu, t, src, dst, sport, dport, proto, n, out, counters, st, hist,
                                                  cells, words, items);
        };
        auto go = [&](auto stage, const DevTableSet& Ts, uint32_t words) {
            constexpr int S = decltype(stage)::value;
            if (wide) return go1(std::integral_constant<int, S + 96 + 128>{}, Ts, words);
            if (unif) return go1(std::integral_constant<int, S + 96>{}, Ts, words);
            if (nopair) return go1(std::integral_constant<int, S + 32>{}, Ts, words);
            go1(stage, Ts, words);
        };
        if (T.node.cmap && (fits(all) || fits(norec))) {
            const uint32_t w = fits(all) ? all : norec;
            if (w < all) Tn.node.lrec = 0;
            go(std::integral_constant<int, 3>{}, Tn, w);
        } else if (T.node.img_words_base <= tu.node_stage_max_words) {
            // (without a common-row section the records follow the base image directly)
            const bool recs = !T.node.cmap && T.node.lrec && all <= tu.node_stage_max_words;
            if (!recs) Tn.node.lrec = 0;
            go(std::integral_constant<int, 1>{}, Tn, recs ? all : T.node.img_words_base);
        } else {
            go(std::integral_constant<int, 0>{}, T, 0u);
        }
    } else {
        launch_one<MODE, COUNT, VEC, 0, false>(T, tu, t, src, dst, sport, dport, proto, n, out, counters, st, hist,
                                               cells, 0, items);
    }
}

// A/B variant builds (make variant DEFS=-DPG_ONLY_MODE=1): only one mode's kernels are compiled
// (a fraction of the full build's time); other modes' launches fail with PG_EIO
#ifndef PG_ONLY_MODE
#define PG_ONLY_MODE -1
#endif
constexpr bool mode_built(int mode) { return PG_ONLY_MODE < 0 || PG_ONLY_MODE == mode; }
#ifndef PG_ONLY_NOCOUNT
#define PG_ONLY_NOCOUNT 0
#endif

template <int MODE>
static void dispatch_mode(bool count, bool vec, const DevTableSet& T, const Tuning& tu, int t, const uint32_t* src,
                          const uint32_t* dst, const uint16_t* sport, const uint16_t* dport, const uint8_t* proto,
                          uint64_t n, uint32_t* out, unsigned long long* counters, hipStream_t st) {
    if (count) {
        if constexpr (PG_ONLY_MODE < 0 || !PG_ONLY_NOCOUNT) {  // (A/B builds: -DPG_ONLY_NOCOUNT=1 leaves these out)
            if (vec) launch_classify<MODE, true, true>(T, tu, t, src, dst, sport, dport, proto, n, out, counters, st);
            else launch_classify<MODE, true, false>(T, tu, t, src, dst, sport, dport, proto, n, out, counters, st);
        }
    } else {
        if (vec) launch_classify<MODE, false, true>(T, tu, t, src, dst, sport, dport, proto, n, out, counters, st);
        else launch_classify<MODE, false, false>(T, tu, t, src, dst, sport, dport, proto, n, out, counters, st);
    }
}

int dev_classify(const DevTableSet& T, const Tuning& tu, int mode, int table_id, const uint32_t* src,
                 const uint32_t* dst, const uint16_t* sport, const uint16_t* dport, const uint8_t* proto, uint64_t n,
                 uint32_t* out, unsigned long long* counters, void* stream, std::string* err) {
    if (n == 0) return 0;
    // (PG_IDX32) pieces of at most kMaxLaunchTuples (or Tuning launch_max_tuples), in order on the stream
    const uint64_t cap = tu.launch_max_tuples ? std::min<uint64_t>(tu.launch_max_tuples, kMaxLaunchTuples)
                                              : kMaxLaunchTuples;
    if (n > cap) {
        for (uint64_t o = 0; o < n; o += cap) {
            const uint64_t k = std::min<uint64_t>(cap, n - o);
            const int rc = dev_classify(T, tu, mode, table_id, src + o, dst + o, sport ? sport + o : nullptr, dport + o,
                                        proto + o, k, out + o, counters, stream, err);
            if (rc != 0) return rc;
        }
        return 0;
    }
    if (mode != 0 && !T.any_mark) {  // (a node build may defer packets to k_node_any: dev_any_mark)
        if (err) *err = "PERPOD / CONN launch without a launch-mark word";
        return -1;
    }
    auto al = [](const void* p, uintptr_t a) { return ((uintptr_t)p & (a - 1)) == 0; };
    // the group loads: 4*P-byte src/dst/out (16-B pieces), 2*P-byte ports, P-byte protocols
    const uintptr_t P = mode == 2 ? tuples_per_lane<2>() : tuples_per_lane<0>();
    const uintptr_t kPort = 2 * P > 16 ? 16 : 2 * P, kProto = P > 16 ? 16 : P;
    const bool vec = al(src, 16) && al(dst, 16) && al(dport, kPort) && al(proto, kProto) && al(out, 16) &&
                     (mode != 2 || al(sport, kPort));
    hipStream_t st = (hipStream_t)stream;
    const bool count = counters != nullptr;
    if (!mode_built(mode)) {
        if (err) *err = "this build (PG_ONLY_MODE) has no kernels for mode " + std::to_string(mode);
        return -1;
    }
    if (mode == 0) {
        if constexpr (mode_built(0)) dispatch_mode<0>(count, vec, T, tu, table_id, src, dst, sport, dport, proto, n, out, counters, st);
    } else if (mode == 1) {
        if constexpr (mode_built(1)) dispatch_mode<1>(count, vec, T, tu, table_id, src, dst, sport, dport, proto, n, out, counters, st);
    } else {
        if constexpr (mode_built(2)) dispatch_mode<2>(count, vec, T, tu, table_id, src, dst, sport, dport, proto, n, out, counters, st);
    }
    HIPCHK(hipGetLastError());
    return 0;
}

int dev_classify_linear(const DevTableSet& T, int table_id, const uint32_t* src, const uint32_t* dst,
                        const uint16_t* dport, const uint8_t* proto, uint64_t n, uint32_t* out, void* stream,
                        std::string* err) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_linear, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, T, (uint32_t)table_id,
                       src, dst, dport, proto, n, out);
    HIPCHK(hipGetLastError());
    return 0;
}

template <bool DST, bool SP>
static void launch_probe(const Tuning& tu, const uint32_t* src, const uint32_t* dst, const uint16_t* sport,
                         const uint16_t* dport, const uint8_t* proto, uint64_t n, uint32_t* out, hipStream_t st) {
    auto k = k_stream_probe<DST, SP, 512>;
    hipLaunchKernelGGL(k, dim3(grid_resident(k, 512, 0, (n + PG_TPL - 1) / PG_TPL, tu.blocks_per_cu)), dim3(512), 0,
                       st, src, dst, sport, dport, proto, n, out);
}

int dev_stream_probe(const Tuning& tu, int fields, const uint32_t* src, const uint32_t* dst, const uint16_t* sport,
                     const uint16_t* dport, const uint8_t* proto, uint64_t n, uint32_t* out, void* stream,
                     std::string* err) {
    if (n == 0) return 0;
    auto al = [](const void* p, uintptr_t a) { return ((uintptr_t)p & (a - 1)) == 0; };
    constexpr uintptr_t kPort = 2 * PG_TPL > 16 ? 16 : 2 * PG_TPL, kProto = PG_TPL > 16 ? 16 : PG_TPL;
    if (!(al(src, 16) && al(dport, kPort) && al(proto, kProto) && al(out, 16) && (!(fields & 1) || al(dst, 16)) &&
          (!(fields & 2) || al(sport, kPort)))) {
        if (err) *err = "stream probe: tuple fields / output not vector-aligned";
        return -1;
    }
    hipStream_t st = (hipStream_t)stream;
    if (fields == 0) launch_probe<false, false>(tu, src, dst, sport, dport, proto, n, out, st);
    else if (fields == 1) launch_probe<true, false>(tu, src, dst, sport, dport, proto, n, out, st);
    else if (fields == 2) launch_probe<false, true>(tu, src, dst, sport, dport, proto, n, out, st);
    else launch_probe<true, true>(tu, src, dst, sport, dport, proto, n, out, st);
    HIPCHK(hipGetLastError());
    return 0;
}

int dev_gen(const DevTableSet& T, const GenParams& g, uint64_t n, uint32_t* src, uint32_t* dst, uint16_t* sport,
            uint16_t* dport, uint8_t* proto, void* stream, std::string* err) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_gen, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, T, g, n, src, dst, sport,
                       dport, proto);
    HIPCHK(hipGetLastError());
    return 0;
}

// hit counters carried into a recompiled set's slots (engine.cpp slot_remap)
__global__ __launch_bounds__(kBlock) void k_counter_remap(unsigned long long* __restrict__ dst,
                                                          const unsigned long long* __restrict__ src,
                                                          const uint32_t* __restrict__ map, uint32_t n) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) dst[i] = map[i] == 0xFFFFFFFFu ? 0ull : src[map[i]];
}

int dev_counters_remap(unsigned long long* dst, const unsigned long long* src, const uint32_t* map, size_t n,
                       std::string* err) {
    if (n == 0) return 0;
    uint32_t* m = nullptr;
    HIPCHK(hipMalloc(&m, n * 4));
    hipError_t e = hipMemcpy(m, map, n * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_counter_remap, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, 0, dst, src,
                           m, (uint32_t)n);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr);  // (m is freed next)
    (void)hipFree(m);
    if (e != hipSuccess) {
        if (err) *err = std::string("counter remap: ") + hipGetErrorString(e);
        return -1;
    }
    return 0;
}

int dev_conn_queries(const DevTableSet& T, const ConnQueryDev* q_host, size_t n, uint32_t* out_host,
                     std::string* err) {
    if (n == 0) return 0;
    ConnQueryDev* q = nullptr;
    uint32_t* o = nullptr;
    HIPCHK(hipMalloc(&q, n * sizeof(ConnQueryDev)));
    hipError_t e = hipMalloc(&o, n * 4);
    if (e != hipSuccess) {
        (void)hipFree(q);
        if (err) *err = hipGetErrorString(e);
        return -1;
    }
    e = hipMemcpy(q, q_host, n * sizeof(ConnQueryDev), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_conn_queries, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, T, q, (uint32_t)n, o);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out_host, o, n * 4, hipMemcpyDeviceToHost);
    (void)hipFree(q);
    (void)hipFree(o);
    if (e != hipSuccess) {
        if (err) *err = hipGetErrorString(e);
        return -1;
    }
    return 0;
}

}  // namespace pg
