// Does a ds_read_b32 / ds_read_b64 at an unaligned LDS byte address return the bytes at that address (unaligned
// access mode) or the aligned word (low address bits ignored)?  Development probe, not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k(uint32_t *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t buf[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) buf[i] = (uint8_t)i;
    __syncthreads();
    const int t = threadIdx.x;
    if (t < 8) {
        uint32_t a = (uint32_t)(uintptr_t)buf + 16 + t;
        uint32_t v32;
        uint64_t v64;
        asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v32) : "v"(a) : "memory");
        asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v64) : "v"(a) : "memory");
        out[3 * t] = v32;
        out[3 * t + 1] = (uint32_t)v64;
        out[3 * t + 2] = (uint32_t)(v64 >> 32);
        if (t == 0) out[24] = buf[t + 40];
    }
}

int main()
{
    uint32_t *d, h[25];
    hipMalloc(&d, sizeof(h));
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int t = 0; t < 8; ++t) printf("addr %d: b32 %08x b64 %08x %08x\n", 16 + t, h[3 * t], h[3 * t + 2], h[3 * t + 1]);
    return 0;
}
