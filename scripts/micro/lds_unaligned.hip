// LDS loads at unaligned byte addresses on gfx950: does a 4/8/16-byte LDS load at any byte offset return
// the bytes at that offset, and what does it cost against the dword loads + v_alignbyte it would replace?
// (The front's load16 reads 16 bytes at a byte position as five dword loads and four alignbytes.)
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/lds_unaligned scripts/micro/lds_unaligned.hip && /tmp/lds_unaligned
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));

// correctness: lane l reads at byte offset base + l * stride (all 16 residues covered over the launches)
__global__ void check(const uint32_t *in, uint32_t *out, uint32_t base, uint32_t stride) {
    __shared__ __attribute__((aligned(16))) uint8_t b[8192];
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) ((uint32_t *)b)[i] = in[i];
    __syncthreads();
    const uint32_t q = base + threadIdx.x * stride;
    v4u x16;
    v2u x8;
    uint32_t x4;
    __builtin_memcpy(&x16, b + q, 16);
    __builtin_memcpy(&x8, b + q + 1, 8);
    __builtin_memcpy(&x4, b + q + 2, 4);
    uint32_t *o = out + threadIdx.x * 7;
    o[0] = x16.x, o[1] = x16.y, o[2] = x16.z, o[3] = x16.w, o[4] = x8.x, o[5] = x8.y, o[6] = x4;
}

// cost: a chain of dependent 16-byte reads at byte addresses derived from the previous result
template <int MODE>
__global__ void chain(const uint32_t *in, uint32_t *out, int iters) {
    __shared__ __attribute__((aligned(16))) uint8_t b[8192 + 64];
    for (int i = threadIdx.x; i < 2048 + 16; i += blockDim.x) ((uint32_t *)b)[i] = in[i & 2047];
    __syncthreads();
    uint32_t p = (threadIdx.x * 37) & 4095, acc = 0;
    for (int it = 0; it < iters; it++) {
        v4u x;
        if (MODE == 0) { // one 16-byte load at a byte address
            __builtin_memcpy(&x, b + p, 16);
        } else if (MODE == 1) { // five dword loads + alignbyte (the product's load16)
            const uint32_t w = p >> 2, sh = p & 3;
            const uint32_t *bw = (const uint32_t *)b;
            const uint32_t w0 = bw[w], w1 = bw[w + 1], w2 = bw[w + 2], w3 = bw[w + 3], w4 = bw[w + 4];
            x = v4u{__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                    __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh)};
        } else if (MODE == 2) { // aligned 16-byte load (reference point)
            __builtin_memcpy(&x, b + (p & ~15u), 16);
        } else if (MODE == 3) { // one 16-byte load at the dword address + one dword, four alignbytes
            // (inline asm: for a known dword-aligned address the compiler splits the load into ds_read2_b32)
            const uint32_t sh = p & 3;
            v4u y;
            uint32_t w4;
            const uint32_t la = (uint32_t)(uintptr_t)(b + (p & ~3u));
            asm volatile("ds_read_b128 %0, %2\n\tds_read_b32 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
                         : "=v"(y), "=v"(w4)
                         : "v"(la));
            x = v4u{__builtin_amdgcn_alignbyte(y.y, y.x, sh), __builtin_amdgcn_alignbyte(y.z, y.y, sh),
                    __builtin_amdgcn_alignbyte(y.w, y.z, sh), __builtin_amdgcn_alignbyte(w4, y.w, sh)};
        } else if (MODE == 4) { // two 8-byte loads at byte addresses
            v2u y0, y1;
            __builtin_memcpy(&y0, b + p, 8);
            __builtin_memcpy(&y1, b + p + 8, 8);
            x = v4u{y0.x, y0.y, y1.x, y1.y};
        } else { // 8-byte loads at dword addresses: b64 + b64 + b32, four alignbytes
            const uint32_t sh = p & 3;
            v2u y0, y1;
            __builtin_memcpy(&y0, b + (p & ~3u), 8);
            __builtin_memcpy(&y1, b + (p & ~3u) + 8, 8);
            const uint32_t w4 = *(const uint32_t *)(b + (p & ~3u) + 16);
            x = v4u{__builtin_amdgcn_alignbyte(y0.y, y0.x, sh), __builtin_amdgcn_alignbyte(y1.x, y0.y, sh),
                    __builtin_amdgcn_alignbyte(y1.y, y1.x, sh), __builtin_amdgcn_alignbyte(w4, y1.y, sh)};
        }
        acc += x.x ^ x.y ^ x.z ^ x.w;
        p = (p + 13 + (acc & 7)) & 4095;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
    std::vector<uint32_t> h(2048);
    for (int i = 0; i < 2048; i++) h[i] = 0x9e3779b9u * (i + 1) ^ (i << 7);
    const uint8_t *hb = (const uint8_t *)h.data();
    uint32_t *din, *dout;
    hipMalloc(&din, 2048 * 4);
    hipMalloc(&dout, 1 << 24);
    hipMemcpy(din, h.data(), 2048 * 4, hipMemcpyHostToDevice);
    long bad = 0, tot = 0;
    std::vector<uint32_t> o(64 * 7);
    for (uint32_t stride = 1; stride <= 17; stride += 2)
        for (uint32_t base = 0; base < 64; base++) {
            hipLaunchKernelGGL(check, dim3(1), dim3(64), 0, 0, din, dout, base, stride);
            hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost);
            for (uint32_t l = 0; l < 64; l++) {
                const uint32_t q = base + l * stride;
                uint32_t e[7];
                __builtin_memcpy(e, hb + q, 16);
                __builtin_memcpy(e + 4, hb + q + 1, 8);
                __builtin_memcpy(e + 6, hb + q + 2, 4);
                for (int k = 0; k < 7; k++) {
                    tot++;
                    if (o[l * 7 + k] != e[k]) bad++;
                }
            }
        }
    printf("unaligned LDS loads: %ld of %ld words wrong\n", bad, tot);
    const int iters = 4096, blocks = 256 * 8, threads = 256;
    hipEvent_t a, z;
    hipEventCreate(&a);
    hipEventCreate(&z);
    const char *names[6] = {"b128 at byte address", "5 x b32 + alignbyte", "b128 aligned", "b128+b32 at dword addr",
                            "2 x b64 at byte address", "2 x b64+b32 dword addr"};
    for (int rep = 0; rep < 2; rep++)
        for (int m = 0; m < 6; m++) {
            hipEventRecord(a);
            if (m == 0) hipLaunchKernelGGL(chain<0>, dim3(blocks), dim3(threads), 0, 0, din, dout, iters);
            if (m == 1) hipLaunchKernelGGL(chain<1>, dim3(blocks), dim3(threads), 0, 0, din, dout, iters);
            if (m == 2) hipLaunchKernelGGL(chain<2>, dim3(blocks), dim3(threads), 0, 0, din, dout, iters);
            if (m == 3) hipLaunchKernelGGL(chain<3>, dim3(blocks), dim3(threads), 0, 0, din, dout, iters);
            if (m == 4) hipLaunchKernelGGL(chain<4>, dim3(blocks), dim3(threads), 0, 0, din, dout, iters);
            if (m == 5) hipLaunchKernelGGL(chain<5>, dim3(blocks), dim3(threads), 0, 0, din, dout, iters);
            hipEventRecord(z);
            hipEventSynchronize(z);
            float ms = 0;
            hipEventElapsedTime(&ms, a, z);
            const double reads = (double)blocks * threads / 64 * iters; // wave-level 16-byte reads
            printf("%-24s %8.3f ms  %.2f ns per wave read (whole chip)\n", names[m], ms, ms * 1e6 / reads);
        }
    return bad ? 1 : 0;
}
