// Checks xor_lanes (prims.hpp: DPP / permlane-swap lane exchange) against the lane ^ m definition on the GPU, for
// 32- and 64-bit values. Build: hipcc -O3 --offload-arch=gfx950 -I cassandra-accord_amd/csrc tools/xor_lanes_check.hip
#include "prims.hpp"
#include <cstdio>

__global__ void k_xl(const uint64_t *in, uint64_t *o32, uint64_t *o64)
{
    const uint32_t l = threadIdx.x;
    const uint64_t x = in[blockIdx.x * 64 + l];
    uint64_t *a = o32 + (size_t)blockIdx.x * 6 * 64, *b = o64 + (size_t)blockIdx.x * 6 * 64;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        a[i * 64 + l] = acc::xor_lanes((uint32_t)x, 1 << i);
        b[i * 64 + l] = acc::xor_lanes(x, 1 << i);
    }
}

int main()
{
    const int nb = 64;
    std::vector<uint64_t> h(nb * 64);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (auto &v : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; v = s; }
    uint64_t *d, *o32, *o64;
    (void)hipMalloc(&d, h.size() * 8); (void)hipMalloc(&o32, h.size() * 6 * 8); (void)hipMalloc(&o64, h.size() * 6 * 8);
    (void)hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    k_xl<<<nb, 64>>>(d, o32, o64);
    std::vector<uint64_t> r32(h.size() * 6), r64(h.size() * 6);
    if (hipMemcpy(r32.data(), o32, r32.size() * 8, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(r64.data(), o64, r64.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) { printf("hip error\n"); return 2; }
    int bad = 0;
    for (int b = 0; b < nb; ++b)
        for (int i = 0; i < 6; ++i)
            for (int l = 0; l < 64; ++l) {
                const uint64_t want = h[b * 64 + (l ^ (1 << i))];
                if (r32[(b * 6 + i) * 64 + l] != (uint32_t)want || r64[(b * 6 + i) * 64 + l] != want) {
                    if (bad++ < 8) printf("mismatch m=%d lane=%d\n", 1 << i, l);
                }
            }
    printf("xor_lanes: %s (%d mismatches)\n", bad ? "FAIL" : "ok", bad);
    return bad ? 1 : 0;
}
