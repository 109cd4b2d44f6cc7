// Issue-rate microbenchmark (diagnostic): SALU vs VALU throughput per CU as a function of
// waves per CU, to decide whether scalar (uniform) control work is a shared-CU bottleneck.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

template <int KIND>
__global__ void __launch_bounds__(64) bench(int iters, unsigned *out) {
    unsigned a0 = threadIdx.x, a1 = 1, a2 = 2, a3 = 3, a4 = 4, a5 = 5, a6 = 6, a7 = 7;
    unsigned s0 = __builtin_amdgcn_readfirstlane(blockIdx.x), s1 = 1, s2 = 2, s3 = 3, s4 = 4, s5 = 5, s6 = 6, s7 = 7;
    for (int i = 0; i < iters; i++) {
        if (KIND == 0 || KIND == 2) {
            asm volatile(
                "s_add_u32 %0, %0, %8\n s_add_u32 %1, %1, %8\n s_add_u32 %2, %2, %8\n s_add_u32 %3, %3, %8\n"
                "s_add_u32 %4, %4, %8\n s_add_u32 %5, %5, %8\n s_add_u32 %6, %6, %8\n s_add_u32 %7, %7, %8\n"
                "s_add_u32 %0, %0, %8\n s_add_u32 %1, %1, %8\n s_add_u32 %2, %2, %8\n s_add_u32 %3, %3, %8\n"
                "s_add_u32 %4, %4, %8\n s_add_u32 %5, %5, %8\n s_add_u32 %6, %6, %8\n s_add_u32 %7, %7, %8\n"
                : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7)
                : "s"(iters)
                : "scc");
        }
        if (KIND == 1 || KIND == 2) {
            asm volatile(
                "v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
                "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"
                "v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
                "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                : "v"(a0 >> 20)
                :);
        }
        if (KIND == 3) { // dependent SALU chain: latency
            asm volatile(
                "s_add_u32 %0, %0, %1\n s_add_u32 %0, %0, %1\n s_add_u32 %0, %0, %1\n s_add_u32 %0, %0, %1\n"
                "s_add_u32 %0, %0, %1\n s_add_u32 %0, %0, %1\n s_add_u32 %0, %0, %1\n s_add_u32 %0, %0, %1\n"
                "s_add_u32 %0, %0, %1\n s_add_u32 %0, %0, %1\n s_add_u32 %0, %0, %1\n s_add_u32 %0, %0, %1\n"
                "s_add_u32 %0, %0, %1\n s_add_u32 %0, %0, %1\n s_add_u32 %0, %0, %1\n s_add_u32 %0, %0, %1\n"
                : "+s"(s0) : "s"(iters) : "scc");
        }
        if (KIND == 4) { // v_readlane -> SALU dependency chain
            asm volatile(
                "v_readlane_b32 %0, %1, %0\n s_and_b32 %0, %0, 63\n"
                "v_readlane_b32 %0, %1, %0\n s_and_b32 %0, %0, 63\n"
                "v_readlane_b32 %0, %1, %0\n s_and_b32 %0, %0, 63\n"
                "v_readlane_b32 %0, %1, %0\n s_and_b32 %0, %0, 63\n"
                "v_readlane_b32 %0, %1, %0\n s_and_b32 %0, %0, 63\n"
                "v_readlane_b32 %0, %1, %0\n s_and_b32 %0, %0, 63\n"
                "v_readlane_b32 %0, %1, %0\n s_and_b32 %0, %0, 63\n"
                "v_readlane_b32 %0, %1, %0\n s_and_b32 %0, %0, 63\n"
                : "+s"(s0) : "v"(a0) : "scc");
        }
    }
    if (threadIdx.x == 0) out[blockIdx.x] = s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7 + a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    unsigned *out;
    hipMalloc(&out, 1 << 24);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 20000;
    const char *names[] = {"SALU indep", "VALU indep", "SALU+VALU", "SALU dep chain", "readlane->SALU chain"};
    for (int kind = 0; kind < 5; kind++) {
        for (int wpc : {1, 4, 8, 16, 32}) {
            const int blocks = cus * wpc;
            auto launch = [&] {
                switch (kind) {
                case 0: hipLaunchKernelGGL(bench<0>, dim3(blocks), dim3(64), 0, 0, iters, out); break;
                case 1: hipLaunchKernelGGL(bench<1>, dim3(blocks), dim3(64), 0, 0, iters, out); break;
                case 2: hipLaunchKernelGGL(bench<2>, dim3(blocks), dim3(64), 0, 0, iters, out); break;
                case 3: hipLaunchKernelGGL(bench<3>, dim3(blocks), dim3(64), 0, 0, iters, out); break;
                case 4: hipLaunchKernelGGL(bench<4>, dim3(blocks), dim3(64), 0, 0, iters, out); break;
                }
            };
            launch();
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            double per_wave = (kind == 4 ? 16.0 : 16.0) * iters;
            double clk = 2.4e9;
            // instructions (of the measured type) per CU-cycle
            double ipc = per_wave * wpc / (ms * 1e-3 * clk);
            // cycles per instruction for one wave
            double cpi = (ms * 1e-3 * clk) / per_wave;
            printf("%-22s waves/CU %2d: %.3f ms  instr/CU-cycle %.2f  wave cycles/instr %.2f\n", names[kind], wpc, ms,
                   ipc, cpi);
        }
    }
    return 0;
}
