// gfx950 kernels of the policy classification path.
//
//  K1 k_linear       reference-shaped first-match scan: one lane per tuple, rules read
//                    wave-uniformly (scalar loads), wave exits when every lane matched.
//  K2 k_classify     the production path for SINGLE / PERPOD / CONN modes: src-interval
//                    lookup (radix + short binary search) then a scan of that interval's
//                    candidate list (dst + L4 tests only); 4 tuples per lane with 16/8/4-byte
//                    coalesced SoA loads; per-rule hit counters kept in an LDS histogram
//                    and flushed once per workgroup with u64 atomics (K6).
//  K3 (inside K2)    CONN mode fuses testConnection's up-to-4 evalACL lookups
//                    (mock/aclengine/aclengine_mock.go:424-501).
//  K5 k_gen          counter-based (splitmix64) synthetic 5-tuple generator.
//
// Semantics of one evaluation == evalACL (aclengine_mock.go:503-652) over the ACL the table
// was compiled from (engine.cpp compile_acl_rule); the output word packs the ACLAction (or
// ConnAction) in bits 31-30 and the deciding counter slot in bits 29-0.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "blobwalk.hpp"
#include "device.hpp"

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
};

const DevTableSet& dev_view(const DeviceBuffers* b) { return b->view; }

int dev_set_device(int dev, std::string* err) {
    HIPCHK(hipSetDevice(dev));
    return 0;
}
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
int dev_sync(std::string* err) {
    HIPCHK(hipDeviceSynchronize());
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
    std::vector<uint8_t> img(off, 0);
    auto put = [&](size_t o, const void* p, size_t n) {
        if (n) std::memcpy(img.data() + o, p, n);
    };
    put(o_rules, h.rules.data(), h.rules.size() * sizeof(DevRule));
    put(o_tabs, h.tabs.data(), h.tabs.size() * sizeof(DevTable));
    put(o_blob, h.blobs.data(), h.blobs.size() * 4);
    put(o_if, h.ifaces.data(), h.ifaces.size() * 4);
    put(o_ip, h.iphash.data(), h.iphash.size() * 4);
    auto* b = new DeviceBuffers();
    b->blob = dev_alloc(off, err);
    if (!b->blob) {
        delete b;
        return nullptr;
    }
    if (dev_copy_h2d(b->blob, img.data(), off, err) != 0 || dev_sync(err) != 0) {
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
    v.n_rules = (uint32_t)h.rules.size();
    v.n_tables = (uint32_t)h.tabs.size();
    v.n_ifaces = (uint32_t)(h.ifaces.size() / 2);
    v.slot_noacl = v.n_rules + v.n_tables;
    v.slot_unresolved = v.slot_noacl + 1;
    v.n_slots = v.slot_unresolved + 1;
    b->host_tabs = h.tabs;
    v.host_tabs = b->host_tabs.data();
    return b;
}

void dev_free(DeviceBuffers* b) {
    if (!b) return;
    (void)hipDeviceSynchronize();
    dev_release(b->blob);
    delete b;
}

// ---------------------------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t pkt_key(uint32_t proto, uint32_t port) {
    return proto == 0u ? port : (proto == 1u ? (kKeyUDP | port) : (proto == 2u ? kKeyOTHER : kKeyANY));
}
__device__ __forceinline__ uint32_t verdict(uint32_t act, uint32_t slot) { return (act << 30) | slot; }

// Linear first-match over a table's compiled rules (fallback for tables whose candidate
// lists would exceed the budget; also the ANY-packet path).
__device__ __noinline__ uint32_t eval_linear_lane(const DevTableSet& T, uint32_t t, uint32_t src, uint32_t dst,
                                                  uint32_t key) {
    const DevTable hd = T.tabs[t];
    const bool any = key >= kKeyANY;
    for (uint32_t i = 0; i < hd.n_rules; i++) {
        const DevRule r = T.rules[hd.rule_base + i];
        if ((src & r.smask) != r.snet || (dst & r.dmask) != r.dnet) continue;
        if (any) {
            if ((r.act >> 4) != kActNever) return verdict((r.act >> 4) & 3u, hd.rule_base + i);
        } else if (key >= r.klo && key <= r.khi) {
            return verdict(r.act & 3u, hd.rule_base + i);
        }
    }
    return verdict(kActDeny, T.n_rules + t);
}

// ---- classification blob walk (layout: fastpath.cpp, walk: blobwalk.hpp) -----------------------
struct DevLoader {  // 16/8-byte loads; LDS or global depending on where the pointer came from
    const uint32_t* b;
    __device__ __forceinline__ uint32_t u32(uint32_t i) const { return b[i]; }
    __device__ __forceinline__ W2 u2(uint32_t i) const {
        const uint2 v = *reinterpret_cast<const uint2*>(b + i);
        return W2{v.x, v.y};
    }
    __device__ __forceinline__ W4 u4(uint32_t i) const {
        const uint4 v = *reinterpret_cast<const uint4*>(b + i);
        return W4{v.x, v.y, v.z, v.w};
    }
};
__device__ __forceinline__ BlobHdr load_hdr(const uint32_t* b) { return blob_hdr(DevLoader{b}); }
__device__ __forceinline__ uint32_t eval_blob(const uint32_t* b, const BlobHdr& h, uint32_t src, uint32_t dst,
                                              uint32_t key) {
    return blob_eval(DevLoader{b}, h, src, dst, key);
}

// evalACL(table t) -- t < 0: no ACL on the interface (PERMIT, aclengine_mock.go:506-508)
__device__ __forceinline__ uint32_t eval_table(const DevTableSet& T, int32_t t, uint32_t src, uint32_t dst,
                                               uint32_t key) {
    if (t < 0) return verdict(kActPermit, T.slot_noacl);
    const DevTable hd = T.tabs[t];
    if ((hd.flags & kFlagLinear) || key >= kKeyANY) return eval_linear_lane(T, (uint32_t)t, src, dst, key);
    const uint32_t* b = T.blobs + hd.blob_off;
    return eval_blob(b, load_hdr(b), src, dst, key);
}

__device__ __forceinline__ uint32_t hash_ip(uint32_t ip) {
    ip ^= ip >> 16;
    ip *= 0x7feb352du;
    ip ^= ip >> 15;
    ip *= 0x846ca68bu;
    ip ^= ip >> 16;
    return ip;
}
// IPv4 -> interface: local pod TAP, else the node-output interface (VXLAN BVI or main)
__device__ __forceinline__ int32_t iface_by_ip(const DevTableSet& T, uint32_t ip) {
    uint32_t s = hash_ip(ip) & T.iphash_mask;
    for (;;) {
        const uint2 e = reinterpret_cast<const uint2*>(T.iphash)[s];
        if (e.y == 0xFFFFFFFFu) return T.node_if;
        if (e.x == ip) return (int32_t)e.y;
        s = (s + 1u) & T.iphash_mask;
    }
}

struct Hist {
    uint32_t* lds;
    unsigned long long* glob;
    __device__ __forceinline__ void inc(uint32_t slot) const {
        if (lds) atomicAdd(&lds[slot], 1u);
        else if (glob) atomicAdd(&glob[slot], 1ull);
    }
};

// testConnection (aclengine_mock.go:424-501) on resolved interfaces
template <bool COUNT>
__device__ __forceinline__ uint32_t test_connection(const DevTableSet& T, int32_t sif, int32_t dif, uint32_t src,
                                                    uint32_t dst, uint32_t key_syn, uint32_t key_synack,
                                                    const Hist& h) {
    if (sif < 0 || dif < 0) {
        if (COUNT) h.inc(T.slot_unresolved);
        return verdict(3u, T.slot_unresolved);
    }
    const int2 si = reinterpret_cast<const int2*>(T.ifaces)[sif];
    const int2 di = reinterpret_cast<const int2*>(T.ifaces)[dif];
    const bool same = sif == dif;
    bool src_refl = false, dst_refl = false;
    uint32_t w = eval_table(T, si.x, src, dst, key_syn);  // SYN: src inbound
    if (COUNT) h.inc(w & 0x3FFFFFFFu);
    uint32_t a = w >> 30;
    if (a == kActFailure) return verdict(3u, w & 0x3FFFFFFFu);
    if (a == kActDeny) return verdict(0u, w & 0x3FFFFFFFu);
    if (a == kActReflect) {
        src_refl = true;
        if (same) dst_refl = true;
    }
    if (!dst_refl) {  // SYN: dst outbound
        w = eval_table(T, di.y, src, dst, key_syn);
        if (COUNT) h.inc(w & 0x3FFFFFFFu);
        a = w >> 30;
        if (a == kActFailure) return verdict(3u, w & 0x3FFFFFFFu);
        if (a == kActDeny) return verdict(0u, w & 0x3FFFFFFFu);
        if (a == kActReflect) {
            dst_refl = true;
            if (same) src_refl = true;
        }
    }
    if (!dst_refl) {  // SYN-ACK: dst inbound
        w = eval_table(T, di.x, dst, src, key_synack);
        if (COUNT) h.inc(w & 0x3FFFFFFFu);
        a = w >> 30;
        if (a == kActFailure) return verdict(3u, w & 0x3FFFFFFFu);
        if (a == kActDeny) return verdict(1u, w & 0x3FFFFFFFu);
    }
    if (!src_refl) {  // SYN-ACK: src outbound
        w = eval_table(T, si.y, dst, src, key_synack);
        if (COUNT) h.inc(w & 0x3FFFFFFFu);
        a = w >> 30;
        if (a == kActFailure) return verdict(3u, w & 0x3FFFFFFFu);
        if (a == kActDeny) return verdict(1u, w & 0x3FFFFFFFu);
    }
    return verdict(2u, w & 0x3FFFFFFFu);
}

// SINGLE mode: the table's blob (staged in LDS or read from HBM/L2) and its header
struct Single {
    const uint32_t* b;
    BlobHdr hdr;
    bool linear;
};

template <int MODE, bool COUNT>
__device__ __forceinline__ uint32_t classify_one(const DevTableSet& T, int32_t t, const Single& sg, uint32_t src,
                                                 uint32_t dst, uint32_t sport, uint32_t dport, uint32_t proto,
                                                 const Hist& h) {
    if (MODE == 0) {  // SINGLE
        const uint32_t key = pkt_key(proto, dport);
        const uint32_t w = (sg.linear || key >= kKeyANY) ? eval_linear_lane(T, (uint32_t)t, src, dst, key)
                                                         : eval_blob(sg.b, sg.hdr, src, dst, key);
        if (COUNT) h.inc(w & 0x3FFFFFFFu);
        return w;
    } else if (MODE == 1) {  // PERPOD: outbound ACL of the egress interface of dst
        const int32_t dif = iface_by_ip(T, dst);
        if (dif < 0) {
            if (COUNT) h.inc(T.slot_unresolved);
            return verdict(kActFailure, T.slot_unresolved);
        }
        const int32_t tt = reinterpret_cast<const int2*>(T.ifaces)[dif].y;
        const uint32_t w = eval_table(T, tt, src, dst, pkt_key(proto, dport));
        if (COUNT) h.inc(w & 0x3FFFFFFFu);
        return w;
    } else {  // CONN
        const int32_t sif = iface_by_ip(T, src), dif = iface_by_ip(T, dst);
        return test_connection<COUNT>(T, sif, dif, src, dst, pkt_key(proto, dport), pkt_key(proto, sport), h);
    }
}

constexpr int kBlock = 256;
constexpr uint32_t kLdsHistMax = 16384;  // slots kept in LDS (64 KiB)

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

// STAGE (SINGLE mode only): the table's blob (stage_words u32, multiple of 4) is copied into
// LDS once per workgroup and every lookup of the grid-stride loop reads it from there.
template <int MODE, bool COUNT, bool VEC, bool STAGE>
__global__ __launch_bounds__(kBlock) void k_classify(DevTableSet T, int32_t t, const uint32_t* __restrict__ src,
                                                     const uint32_t* __restrict__ dst,
                                                     const uint16_t* __restrict__ sport,
                                                     const uint16_t* __restrict__ dport,
                                                     const uint8_t* __restrict__ proto, uint64_t n,
                                                     uint32_t* __restrict__ out, unsigned long long* counters,
                                                     uint32_t stage_words) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t* hist = smem + (STAGE ? stage_words : 0u);
    Hist h{nullptr, counters};
    const bool use_lds = COUNT && T.n_slots <= kLdsHistMax;
    Single sg{nullptr, BlobHdr{}, true};
    if (MODE == 0) {
        const DevTable hd = T.tabs[t];
        sg.linear = (hd.flags & kFlagLinear) != 0u;
        if (STAGE) {
            const uint4* g = reinterpret_cast<const uint4*>(T.blobs + hd.blob_off);
            for (uint32_t i = threadIdx.x; i < stage_words / 4u; i += kBlock) reinterpret_cast<uint4*>(smem)[i] = g[i];
            sg.b = smem;
        } else {
            sg.b = T.blobs + hd.blob_off;
        }
    }
    if (COUNT && use_lds) {
        for (uint32_t i = threadIdx.x; i < T.n_slots; i += kBlock) hist[i] = 0;
        h.lds = hist;
    }
    if (STAGE || (COUNT && use_lds)) __syncthreads();
    if (MODE == 0 && !sg.linear) sg.hdr = load_hdr(sg.b);
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t first = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    // full quads: software-pipelined -- the next quad's 44 bytes are in flight while this
    // quad is classified (16-B src/dst, 8-B ports, 4-B protocols per lane, coalesced)
    const uint64_t nfull = VEC ? (n >> 2) : 0;
    struct Quad {
        v4u s, d;
        v2u dp, sp;
        uint32_t pr;
    };
    auto load = [&](uint64_t q) {
        Quad x;
        const uint64_t i0 = q << 2;
        x.s = stream_load(reinterpret_cast<const v4u*>(src + i0));
        x.d = stream_load(reinterpret_cast<const v4u*>(dst + i0));
        x.dp = stream_load(reinterpret_cast<const v2u*>(dport + i0));
        x.pr = stream_load(reinterpret_cast<const uint32_t*>(proto + i0));
        x.sp = MODE == 2 ? stream_load(reinterpret_cast<const v2u*>(sport + i0)) : v2u{0u, 0u};
        return x;
    };
    uint64_t q = first;
    Quad cur;
    if (q < nfull) cur = load(q);
    while (q < nfull) {
        const uint64_t qn = q + stride;
        Quad nxt = cur;
        if (qn < nfull) nxt = load(qn);
        v4u o;
        o.x = classify_one<MODE, COUNT>(T, t, sg, cur.s.x, cur.d.x, cur.sp.x & 0xFFFFu, cur.dp.x & 0xFFFFu,
                                        cur.pr & 0xFFu, h);
        o.y = classify_one<MODE, COUNT>(T, t, sg, cur.s.y, cur.d.y, cur.sp.x >> 16, cur.dp.x >> 16,
                                        (cur.pr >> 8) & 0xFFu, h);
        o.z = classify_one<MODE, COUNT>(T, t, sg, cur.s.z, cur.d.z, cur.sp.y & 0xFFFFu, cur.dp.y & 0xFFFFu,
                                        (cur.pr >> 16) & 0xFFu, h);
        o.w = classify_one<MODE, COUNT>(T, t, sg, cur.s.w, cur.d.w, cur.sp.y >> 16, cur.dp.y >> 16, cur.pr >> 24, h);
        stream_store(o, reinterpret_cast<v4u*>(out + (q << 2)));
        cur = nxt;
        q = qn;
    }
    // remainder (or everything when the pointers are not vector-aligned): one tuple per lane
    for (uint64_t i = (nfull << 2) + first; i < n; i += stride)
        out[i] = classify_one<MODE, COUNT>(T, t, sg, src[i], dst[i], MODE == 2 ? sport[i] : 0u, dport[i], proto[i],
                                           h);
    if (COUNT && use_lds) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < T.n_slots; i += kBlock) {
            const uint32_t v = hist[i];
            if (v) atomicAdd(&counters[i], (unsigned long long)v);
        }
    }
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
    Hist h{nullptr, nullptr};
    out[i] = test_connection<false>(T, c.src_if, c.dst_if, c.src_ip, c.dst_ip, c.key_syn, c.key_synack, h);
}

// ---- launchers --------------------------------------------------------------------------------
static uint32_t g_blocks_per_cu = 4;        // grid = min(work, 256 CUs x this), grid-stride beyond
static uint32_t g_stage_max_words = 16384;  // blobs up to 64 KiB are staged in LDS

int dev_set_tuning(const std::string& key, int value) {
    if (key == "blocks_per_cu" && value > 0 && value <= 64) g_blocks_per_cu = (uint32_t)value;
    else if (key == "stage_max_words" && value >= 0 && value <= 36864) g_stage_max_words = (uint32_t)value;
    else return -1;
    return 0;
}

static int grid_for(uint64_t items) {
    uint64_t g = (items + kBlock - 1) / kBlock;
    return (int)std::max<uint64_t>(1, std::min<uint64_t>(g, 256ull * g_blocks_per_cu));
}

template <int MODE, bool COUNT, bool VEC>
static void launch_classify(const DevTableSet& T, int t, const uint32_t* src, const uint32_t* dst,
                            const uint16_t* sport, const uint16_t* dport, const uint8_t* proto, uint64_t n,
                            uint32_t* out, unsigned long long* counters, hipStream_t st) {
    const size_t hist = (COUNT && T.n_slots <= kLdsHistMax) ? T.n_slots * 4 : 0;
    uint32_t stage = 0;
    if (MODE == 0) {
        const DevTable& hd = T.host_tabs[t];
        if (!(hd.flags & kFlagLinear) && hd.blob_words <= g_stage_max_words) stage = hd.blob_words;
    }
    const dim3 grid(grid_for((n + 3) / 4));
    if (stage)
        hipLaunchKernelGGL((k_classify<MODE, COUNT, VEC, true>), grid, dim3(kBlock), hist + stage * 4, st, T, t, src,
                           dst, sport, dport, proto, n, out, counters, stage);
    else
        hipLaunchKernelGGL((k_classify<MODE, COUNT, VEC, false>), grid, dim3(kBlock), hist, st, T, t, src, dst, sport,
                           dport, proto, n, out, counters, 0u);
}

template <int MODE>
static void dispatch_mode(bool count, bool vec, const DevTableSet& T, int t, const uint32_t* src,
                          const uint32_t* dst, const uint16_t* sport, const uint16_t* dport, const uint8_t* proto,
                          uint64_t n, uint32_t* out, unsigned long long* counters, hipStream_t st) {
    if (count) {
        if (vec) launch_classify<MODE, true, true>(T, t, src, dst, sport, dport, proto, n, out, counters, st);
        else launch_classify<MODE, true, false>(T, t, src, dst, sport, dport, proto, n, out, counters, st);
    } else {
        if (vec) launch_classify<MODE, false, true>(T, t, src, dst, sport, dport, proto, n, out, counters, st);
        else launch_classify<MODE, false, false>(T, t, src, dst, sport, dport, proto, n, out, counters, st);
    }
}

int dev_classify(const DevTableSet& T, int mode, int table_id, const uint32_t* src, const uint32_t* dst,
                 const uint16_t* sport, const uint16_t* dport, const uint8_t* proto, uint64_t n, uint32_t* out,
                 unsigned long long* counters, void* stream, std::string* err) {
    if (n == 0) return 0;
    auto al = [](const void* p, uintptr_t a) { return ((uintptr_t)p & (a - 1)) == 0; };
    const bool vec = al(src, 16) && al(dst, 16) && al(dport, 8) && al(proto, 4) && al(out, 16) &&
                     (mode != 2 || al(sport, 8));
    hipStream_t st = (hipStream_t)stream;
    const bool count = counters != nullptr;
    if (mode == 0) dispatch_mode<0>(count, vec, T, table_id, src, dst, sport, dport, proto, n, out, counters, st);
    else if (mode == 1) dispatch_mode<1>(count, vec, T, table_id, src, dst, sport, dport, proto, n, out, counters, st);
    else dispatch_mode<2>(count, vec, T, table_id, src, dst, sport, dport, proto, n, out, counters, st);
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

int dev_gen(const DevTableSet& T, const GenParams& g, uint64_t n, uint32_t* src, uint32_t* dst, uint16_t* sport,
            uint16_t* dport, uint8_t* proto, void* stream, std::string* err) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_gen, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, T, g, n, src, dst, sport,
                       dport, proto);
    HIPCHK(hipGetLastError());
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
