// calib_fetch.hip — calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access patterns of the deps
// kernels (MI355X_MICROARCH.md §HBM: only wide coalesced streaming reads are calibrated, at 1/2). Each kernel moves a
// known number of requests of a known width over a 2 GiB table (beyond the 256 MiB Infinity Cache); the profile of
// this program divided by the request counts printed here gives the bytes each counter tallies per request.
//
//   hipcc -O3 --offload-arch=gfx950 tools/calib_fetch.hip -o tools/calib_fetch
//   rocprofv3 --pmc FETCH_SIZE -- tools/calib_fetch ; rocprofv3 --pmc WRITE_SIZE -- tools/calib_fetch
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// coalesced 16 B per lane
__global__ void k_stream_read(const uint4 *__restrict__ a, size_t n, uint32_t *__restrict__ sink)
{
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// random gathers of W bytes (W/4 consecutive u32, W-aligned) from a table of n_bytes
template <int W>
__global__ void k_gather(const uint32_t *__restrict__ t, uint64_t n_lines, uint64_t reqs, uint32_t *__restrict__ sink)
{
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < reqs; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t line = mix(i) % n_lines;
        const uint32_t *p = t + line * (W / 4);
        if constexpr (W == 4) acc ^= p[0];
        else if constexpr (W == 16) { const uint4 v = *reinterpret_cast<const uint4 *>(p); acc ^= v.x ^ v.w; }
        else {
#pragma unroll
            for (int q = 0; q < W / 16; ++q) { const uint4 v = reinterpret_cast<const uint4 *>(p)[q]; acc ^= v.x ^ v.w; }
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// random scatters of W bytes
template <int W>
__global__ void k_scatter(uint32_t *__restrict__ t, uint64_t n_lines, uint64_t reqs)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < reqs; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t line = mix(i ^ 0xABCDull) % n_lines;
        uint32_t *p = t + line * (W / 4);
        if constexpr (W == 4) p[0] = (uint32_t)i;
        else {
#pragma unroll
            for (int q = 0; q < W / 16; ++q) reinterpret_cast<uint4 *>(p)[q] = make_uint4((uint32_t)i, 1, 2, 3);
        }
    }
}

// coalesced 16 B per lane stores
__global__ void k_stream_write(uint4 *__restrict__ a, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_uint4((uint32_t)i, 0, 0, 0);
}

int main()
{
    const size_t bytes = 2ull << 30;
    void *buf;
    uint32_t *sink;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 1, bytes));
    const uint64_t reqs = 32ull << 20;   // 33.5M requests per gather / scatter kernel
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timed = [&](const char *name, double req_bytes, uint64_t nreq, auto &&launch) {
        launch();   // warm (page tables)
        hipEventRecord(e0);
        launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("{\"kernel\": \"%s\", \"requests\": %llu, \"bytes_requested\": %.0f, \"ms\": %.4f, \"launches\": 2}\n", name,
               (unsigned long long)nreq, req_bytes, ms);
    };
    const dim3 g(4096), b(256);
    timed("k_stream_read", (double)bytes, bytes / 16, [&] { hipLaunchKernelGGL(k_stream_read, g, b, 0, 0, (const uint4 *)buf, bytes / 16, sink); });
    timed("k_gather<4>", 4.0 * reqs, reqs, [&] { hipLaunchKernelGGL(k_gather<4>, g, b, 0, 0, (const uint32_t *)buf, (uint64_t)(bytes / 4), reqs, sink); });
    timed("k_gather<16>", 16.0 * reqs, reqs, [&] { hipLaunchKernelGGL(k_gather<16>, g, b, 0, 0, (const uint32_t *)buf, (uint64_t)(bytes / 16), reqs, sink); });
    timed("k_gather<32>", 32.0 * reqs, reqs, [&] { hipLaunchKernelGGL(k_gather<32>, g, b, 0, 0, (const uint32_t *)buf, (uint64_t)(bytes / 32), reqs, sink); });
    timed("k_gather<64>", 64.0 * reqs, reqs, [&] { hipLaunchKernelGGL(k_gather<64>, g, b, 0, 0, (const uint32_t *)buf, (uint64_t)(bytes / 64), reqs, sink); });
    timed("k_scatter<4>", 4.0 * reqs, reqs, [&] { hipLaunchKernelGGL(k_scatter<4>, g, b, 0, 0, (uint32_t *)buf, (uint64_t)(bytes / 4), reqs); });
    timed("k_scatter<16>", 16.0 * reqs, reqs, [&] { hipLaunchKernelGGL(k_scatter<16>, g, b, 0, 0, (uint32_t *)buf, (uint64_t)(bytes / 16), reqs); });
    timed("k_scatter<64>", 64.0 * reqs, reqs, [&] { hipLaunchKernelGGL(k_scatter<64>, g, b, 0, 0, (uint32_t *)buf, (uint64_t)(bytes / 64), reqs); });
    timed("k_stream_write", (double)bytes, bytes / 16, [&] { hipLaunchKernelGGL(k_stream_write, g, b, 0, 0, (uint4 *)buf, bytes / 16); });
    CK(hipDeviceSynchronize());
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}
