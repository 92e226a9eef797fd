// MEASUREMENT ONLY (not part of the library): the rate of scattered global atomic increments on
// this GPU -- the cost a per-rule hit counter pays when no LDS cell holds its slot.
//   hipcc -O3 --offload-arch=gfx950 tools/atomic_probe.hip -o build/atomic_probe && build/atomic_probe
// Every variant adds 1 to counters[h(i) % slots] for i < n (h: a 32-bit mix, so the slots are
// uniform), with one or four increments per lane per loop trip; prints G increments/s and checks
// that the counters sum to n.
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

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

template <class T, int SCOPE>
__global__ __launch_bounds__(256) void k_inc(T* c, uint32_t slots, uint64_t n, uint32_t seed) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t s = mix((uint32_t)i ^ seed) % slots;
        if (SCOPE == 0) atomicAdd(&c[s], (T)1);
        else __hip_atomic_fetch_add(&c[s], (T)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// the same increments, aggregated per distinct slot over the wave first (the library's global
// fallback for the node kernels)
__global__ __launch_bounds__(256) void k_inc_agg(unsigned long long* c, uint32_t slots, uint64_t n, uint32_t seed) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t s = mix((uint32_t)i ^ seed) % slots;
        for (;;) {
            const uint32_t lead = __builtin_amdgcn_readfirstlane(s);
            const unsigned long long m = __ballot(s == lead);
            if (s == lead) {
                if (__lane_id() == (unsigned)(__ffsll((long long)m) - 1)) atomicAdd(&c[lead], (unsigned long long)__popcll(m));
                break;
            }
        }
    }
}

template <class T>
static double run(void (*k)(T*, uint32_t, uint64_t, uint32_t), T* c, uint32_t slots, uint64_t n, int grid,
                  const char* name) {
    hipMemset(c, 0, (size_t)slots * sizeof(T));
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, c, slots, n, 1u);  // warm
    hipDeviceSynchronize();
    hipMemset(c, 0, (size_t)slots * sizeof(T));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, c, slots, n, 2u + r);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    std::vector<T> h(slots);
    hipMemcpy(h.data(), c, (size_t)slots * sizeof(T), hipMemcpyDeviceToHost);
    unsigned long long sum = 0;
    for (T v : h) sum += (unsigned long long)v;
    const double g = (double)n * reps / (ms / reps * 1e-3 * reps) / 1e9;
    std::printf("{\"variant\": \"%s\", \"slots\": %u, \"n\": %llu, \"ms\": %.4f, \"G_inc_per_s\": %.2f, \"sum_ok\": %s}\n",
                name, slots, (unsigned long long)n, ms / reps, g, sum == n * reps ? "true" : "false");
    return g;
}

int main() {
    const uint64_t n = 64ull << 20;
    int cus = 256;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) == hipSuccess) cus = p.multiProcessorCount;
    const int grid = cus * 8;
    unsigned long long* c64 = nullptr;
    uint32_t* c32 = nullptr;
    CK(hipMalloc(&c64, (size_t)(1u << 22) * 8));
    CK(hipMalloc(&c32, (size_t)(1u << 22) * 4));
    for (uint32_t slots : {4096u, 100000u, 1000000u}) {
        run<unsigned long long>(k_inc<unsigned long long, 0>, c64, slots, n, grid, "u64_atomicAdd");
        run<unsigned long long>(k_inc<unsigned long long, 1>, c64, slots, n, grid, "u64_agent_relaxed");
        run<uint32_t>(k_inc<uint32_t, 0>, c32, slots, n, grid, "u32_atomicAdd");
        run<unsigned long long>(k_inc_agg, c64, slots, n, grid, "u64_wave_aggregated");
    }
    hipFree(c64);
    hipFree(c32);
    return 0;
}
