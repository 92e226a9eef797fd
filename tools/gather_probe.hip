// Measurement tool (not part of the library): throughput of random 4-B / 16-B gathers on
// gfx950 by table size and by the share of active lanes -- the cost model behind the
// HBM-resident table walks (DESIGN.md §5, config 4 and the large FD tables).
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/gather_probe tools/gather_probe.hip
//   tools/gather_probe            -> one line per (table KiB, load width, active lanes / 64)
//
// Each lane issues ITER independent gathers (8 in flight) at splitmix-hashed indices into a
// table of T bytes; lanes with (lane % 64) >= active skip the loads (exec-masked). Rate =
// lane-gathers of active lanes / kernel time, and wave-instructions / time.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#define CHK(x)                                                                             \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    return x ^ (x >> 16);
}

constexpr int ITER = 256;

template <int W>  // words per gather: 1 (4 B) or 4 (16 B)
__global__ __launch_bounds__(512) void k_gather(const uint32_t* __restrict__ t, uint32_t mask_elems, int active,
                                                uint32_t* __restrict__ out) {
    const uint32_t g = blockIdx.x * 512 + threadIdx.x;
    uint32_t acc = 0;
    if ((int)(threadIdx.x & 63) < active) {
        uint32_t s = hsh(g * 0x9E3779B9u + 1u);
#pragma unroll 8
        for (int i = 0; i < ITER; i++) {
            s = hsh(s + (uint32_t)i);
            const uint32_t e = s & mask_elems;
            if constexpr (W == 1) {
                acc += t[e];
            } else {
                const uint4 v = reinterpret_cast<const uint4*>(t)[e];
                acc += v.x ^ v.y ^ v.z ^ v.w;
            }
        }
    }
    out[g] = acc;
}

int main() {
    int cus = 256;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) == hipSuccess) cus = p.multiProcessorCount;
    const size_t max_bytes = 256ull << 20;
    uint32_t* t = nullptr;
    uint32_t* out = nullptr;
    CHK(hipMalloc(&t, max_bytes));
    CHK(hipMemset(t, 1, max_bytes));
    const int blocks = cus * 4;  // 2048 threads per CU resident (512-thread workgroups)
    CHK(hipMalloc(&out, (size_t)blocks * 512 * 4));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const size_t sizes_kib[] = {256, 1024, 3072, 6144, 16384, 262144};
    const int actives[] = {64, 32, 16, 8};
    std::printf("{\"cus\": %d, \"iter\": %d, \"threads\": %d}\n", cus, ITER, blocks * 512);
    for (size_t kib : sizes_kib) {
        for (int w : {1, 4}) {
            for (int a : actives) {
                const uint32_t elems = (uint32_t)(kib * 1024 / (4 * w));
                const uint32_t mask = elems - 1;
                auto run = [&]() {
                    if (w == 1) hipLaunchKernelGGL(k_gather<1>, dim3(blocks), dim3(512), 0, 0, t, mask, a, out);
                    else hipLaunchKernelGGL(k_gather<4>, dim3(blocks), dim3(512), 0, 0, t, mask, a, out);
                };
                for (int r = 0; r < 3; r++) run();
                CHK(hipDeviceSynchronize());
                float best = 1e30f;
                for (int r = 0; r < 5; r++) {
                    CHK(hipEventRecord(e0, 0));
                    run();
                    CHK(hipEventRecord(e1, 0));
                    CHK(hipEventSynchronize(e1));
                    float ms = 0;
                    CHK(hipEventElapsedTime(&ms, e0, e1));
                    if (ms < best) best = ms;
                }
                const double per_lane = ITER;
                const double lane_loads = (double)blocks * 512 / 64 * a * per_lane;
                const double wave_insts = (double)blocks * 512 / 64 * per_lane;
                std::printf("{\"table_kib\": %zu, \"bytes\": %d, \"active\": %d, \"ms\": %.4f, "
                            "\"G_lane_loads_s\": %.1f, \"G_wave_insts_s\": %.2f, \"lane_loads_per_cu_clk_at_2.3GHz\": %.3f}\n",
                            kib, 4 * w, a, best, lane_loads / best / 1e6, wave_insts / best / 1e6,
                            lane_loads / (best * 1e-3) / cus / 2.3e9);
                std::fflush(stdout);
            }
        }
    }
    CHK(hipFree(t));
    CHK(hipFree(out));
    return 0;
}
