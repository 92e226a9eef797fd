// The walk of a classification blob (layout: fastpath.cpp), written once for both sides:
// the HIP kernels instantiate it with a loader that issues 16/8-byte LDS or global loads,
// and pg_debug_walk_blob (tests only, never on the classify path) instantiates it with a
// host loader so the builder can be checked against the oracle without a GPU.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define PG_HD __host__ __device__ __forceinline__
#else
#define PG_HD inline
#endif

namespace pg {

constexpr uint32_t kFlagCross = 1u, kFlagLists = 2u, kFlagCand = 4u, kFlagLinear = 8u;

struct W2 {
    uint32_t x, y;
};
struct W4 {
    uint32_t x, y, z, w;
};

struct BlobHdr {
    uint32_t flags, dflt, sroot, s1, kroot, k1, xoff, nkc, loff, voff;
};

template <class L>
PG_HD BlobHdr blob_hdr(const L& ld) {
    const W4 a = ld.u4(0), c = ld.u4(4);
    const W2 d = ld.u2(8);
    return BlobHdr{a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w, d.x, d.y};
}

// multibit trie: root stride s1 over a W-bit value, then 8-bit strides; bit 31 marks a leaf
template <class L>
PG_HD uint32_t blob_trie(const L& ld, uint32_t root, uint32_t s1, uint32_t W, uint32_t x) {
    uint32_t shift = W - s1;
    uint32_t e = ld.u32(root + (x >> shift));
    while (!(e & 0x80000000u)) {
        const uint32_t st = shift < 8u ? shift : 8u;
        shift -= st;
        e = ld.u32(e + ((x >> shift) & ((1u << st) - 1u)));
    }
    return e & 0x7FFFFFFFu;
}

// evalACL over a table's blob for TCP/UDP/OTHER packets (key < 0x30000)
template <class L>
PG_HD uint32_t blob_eval(const L& ld, const BlobHdr& h, uint32_t src, uint32_t dst, uint32_t key) {
    const uint32_t sc = blob_trie(ld, h.sroot, h.s1, 32u, src);
    if (h.flags & kFlagCross) {
        const uint32_t kc = blob_trie(ld, h.kroot, h.k1, 18u, key);
        const uint32_t idx = sc * h.nkc + kc;
        if (!(h.flags & kFlagLists)) return ld.u32(h.xoff + idx);
        const W2 e = ld.u2(h.xoff + 2u * idx);
        const uint32_t cnt = e.y & 255u;
        for (uint32_t j = 0; j < cnt; j++) {
            const W4 l = ld.u4((e.y >> 8) + 4u * j);
            if ((dst & l.y) == l.x) return l.z;
        }
        return e.x;
    }
    const W2 c = ld.u2(h.xoff + 2u * sc);
    for (uint32_t j = 0; j < c.y; j++) {
        const W4 k = ld.u4(h.loff + 4u * (c.x + j));
        if ((dst & k.y) == k.x && key >= k.z && key <= k.w) return ld.u32(h.voff + c.x + j);
    }
    return h.dflt;
}

struct HostLoader {
    const uint32_t* b;
    uint32_t u32(uint32_t i) const { return b[i]; }
    W2 u2(uint32_t i) const { return W2{b[i], b[i + 1]}; }
    W4 u4(uint32_t i) const { return W4{b[i], b[i + 1], b[i + 2], b[i + 3]}; }
};

}  // namespace pg
