// lds_atomic_order.hip -- does one wave's ds_add_rtn_u32 to a shared LDS word hand the lanes
// their old values in lane order?  (If so, a radix-sort scatter can take a lane's stable rank
// among the lanes of its digit from one returning LDS atomic instead of a ballot per digit bit.)
//   hipcc --offload-arch=gfx950 -O3 scripts/micro/lds_atomic_order.hip -o /tmp/lds_order && /tmp/lds_order
// Each wave runs many trials: lanes pick digits from a small, skewed alphabet (packed two u16
// counters per dword, as the sort's table is), add 1 to their digit's counter and keep the
// returned count; the host checks every digit's lanes got consecutive counts in lane order.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int kTrials = 4096, kWaves = 4, kBlocks = 1024;

__global__ void __launch_bounds__(256) order_kernel(uint16_t *out, uint32_t seed) {
    __shared__ uint32_t tab[kWaves][128];
    const int w = threadIdx.x / 64, l = threadIdx.x & 63;
    for (int t = 0; t < kTrials; t++) {
        for (int k = l; k < 128; k += 64) tab[w][k] = 0;
        __builtin_amdgcn_wave_barrier();
        uint32_t x = (seed ^ (uint32_t)(blockIdx.x * 7919 + w * 104729 + t * 31)) * 2654435761u + (uint32_t)l * 40503u;
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        // alphabets of 1..256 digits, skewed toward small ones
        const uint32_t alpha = 1u + ((uint32_t)(t * 37 + blockIdx.x) % 7 == 0 ? 255u : (uint32_t)(t % 9));
        const uint32_t d = (x % alpha) & 255u;
        const uint32_t old = __atomic_fetch_add(&tab[w][d >> 1], 1u << (16 * (d & 1)), __ATOMIC_RELAXED);
        const uint32_t r = (old >> (16 * (d & 1))) & 0xffffu;
        const size_t o = (((size_t)blockIdx.x * kWaves + w) * kTrials + t) * 64 + l;
        out[o] = (uint16_t)(d << 8 | (r & 255));
        __builtin_amdgcn_wave_barrier();
    }
}

int main() {
    const size_t n = (size_t)kBlocks * kWaves * kTrials * 64;
    uint16_t *d = nullptr;
    if (hipMalloc(&d, n * 2) != hipSuccess) return 2;
    hipLaunchKernelGGL(order_kernel, dim3(kBlocks), dim3(256), 0, 0, d, 12345u);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    std::vector<uint16_t> h(n);
    hipMemcpy(h.data(), d, n * 2, hipMemcpyDeviceToHost);
    size_t bad = 0, trials = 0, conflicts = 0;
    for (size_t base = 0; base < n; base += 64) {
        int next[256];
        for (int k = 0; k < 256; k++) next[k] = 0;
        bool ok = true;
        for (int l = 0; l < 64; l++) {
            const int dg = h[base + l] >> 8, r = h[base + l] & 255;
            if (r != next[dg]) ok = false;
            if (next[dg]) conflicts++;
            next[dg]++;
        }
        bad += !ok;
        trials++;
    }
    printf("trials %zu  same-address lanes %zu  out-of-lane-order trials %zu\n", trials, conflicts, bad);
    hipFree(d);
    return bad ? 1 : 0;
}
