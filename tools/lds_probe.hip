// MEASUREMENT ONLY (not part of the library): LDS bank conflicts of random-address lookups --
// the access pattern of the node kernels' trie walks and class-record reads.
//   hipcc -O3 --offload-arch=gfx950 tools/lds_probe.hip -o build/lds_probe && build/lds_probe
//   rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv \
//       -d OUT -o run -- build/lds_probe
// Every variant: 512-thread workgroups, a 40 KB table in LDS, each lane makes ITER dependent
// reads (the next address depends on the value read). Variants (kernel name suffix):
//   rand32   ds_read_b32 at a uniformly random word of the table (a trie step's entry)
//   rec32    ds_read_b32 at word 1 of a random 16-byte record (the packed end point of a class)
//   rec64    ds_read_b64 at words 2-3 of a random 16-byte record (a class's common-row mask)
//   soa32    ds_read_b32 at a random word of a dense array of 1 word per record (records as SoA)
//   bcast32  ds_read_b32, every lane of a wave at the same random word (broadcast)
//   seq32    ds_read_b32, lane i at word (base + i) (conflict-free)
// Prints ns per wave-read; the PMC pass gives the conflict cycles per LDS-array cycle.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            return 1;                                                              \
        }                                                                          \
    } while (0)

constexpr uint32_t kWords = 10240;  // 40 KB
constexpr uint32_t kRecs = kWords / 4;
constexpr int kIter = 4096;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

template <int V>
__global__ __launch_bounds__(512) void k_lds(const uint32_t* tab, uint32_t* out, uint32_t seed) {
    __shared__ __attribute__((aligned(16))) uint32_t t[kWords];
    for (uint32_t i = threadIdx.x; i < kWords; i += blockDim.x) t[i] = tab[i];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t x = mix(seed ^ (blockIdx.x * 512u + threadIdx.x));
    uint32_t acc = 0;
    for (int it = 0; it < kIter; it++) {
        uint32_t v;
        if constexpr (V == 0) {  // rand32
            v = t[x % kWords];
        } else if constexpr (V == 1) {  // rec32
            v = t[(x % kRecs) * 4u + 1u];
        } else if constexpr (V == 2) {  // rec64
            const uint2 m = *reinterpret_cast<const uint2*>(&t[(x % kRecs) * 4u + 2u]);
            v = m.x ^ m.y;
        } else if constexpr (V == 3) {  // soa32
            v = t[x % kRecs];
        } else if constexpr (V == 4) {  // bcast32
            v = t[__builtin_amdgcn_readfirstlane(x) % kWords];
        } else {  // seq32
            v = t[(__builtin_amdgcn_readfirstlane(x) % (kWords - 64u)) + lane];
        }
        acc += v;
        x = mix(x ^ v);  // the next address depends on this read
    }
    if (acc == 0x12345678u) out[blockIdx.x * 8u + wave] = acc;  // keeps the reads
}

int main() {
    std::vector<uint32_t> h(kWords);
    for (uint32_t i = 0; i < kWords; i++) h[i] = i * 2654435761u;
    uint32_t *tab, *out;
    CK(hipMalloc(&tab, kWords * 4));
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMemcpy(tab, h.data(), kWords * 4, hipMemcpyHostToDevice));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int blocks = p.multiProcessorCount * 3;  // three 512-thread workgroups per CU (40 KB each)
    const char* names[] = {"rand32", "rec32", "rec64", "soa32", "bcast32", "seq32"};
    void (*ks[])(const uint32_t*, uint32_t*, uint32_t) = {k_lds<0>, k_lds<1>, k_lds<2>, k_lds<3>, k_lds<4>, k_lds<5>};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int v = 0; v < 6; v++) {
        for (int w = 0; w < 3; w++) hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(512), 0, 0, tab, out, 7u + w);
        CK(hipEventRecord(a));
        const int reps = 10;
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(512), 0, 0, tab, out, 11u + r);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        const double wave_reads = (double)blocks * 8 * kIter * reps;
        std::printf("%-8s %.3f ms/launch  %.3f ns per wave-read chip-wide  %.1f G lane-reads/s\n", names[v], ms / reps,
                    ms * 1e6 / wave_reads, wave_reads * 64 / (ms * 1e-3) / 1e9);
    }
    CK(hipDeviceSynchronize());
    return 0;
}
