// Semantics check of two cross-lane primitives on gfx950 (prints one line each):
//   wave_shl:1 DPP (which neighbour a lane reads, what the last lane gets with bound_ctrl off)
//   ds_permute_b32 with only some lanes active (what non-targeted lanes receive)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *o) {
    const unsigned l = threadIdx.x, v = l * 3 + 1;
    o[l] = (unsigned)__builtin_amdgcn_update_dpp(777, (int)v, 0x130, 0xf, 0xf, false);
    unsigned r = 999;
    if (l % 4 == 0) r = 0;
    // lanes 0, 8, 16, .. send l+100 to lane l/2; every lane receives
    r = (unsigned)__builtin_amdgcn_ds_permute((int)((l % 8 == 0 ? l / 2 : 63) * 4), (int)(l % 8 == 0 ? l + 100 : 5000 + l));
    o[64 + l] = r;
}
int main() {
    unsigned *d, h[128];
    hipMalloc(&d, 512);
    k<<<1, 64>>>(d);
    hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
    printf("wave_shl1:");
    for (int i = 0; i < 64; i++) printf(" %u", h[i]);
    printf("\npermute:");
    for (int i = 0; i < 64; i++) printf(" %u", h[64 + i]);
    printf("\n");
    return 0;
}
