// Does LDS run in unaligned mode on this box: ds_read_b32 / b64 / b128 and ds_write_b128 at byte addresses that are
// not multiples of their size.  Development probe, not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ void k(uint32_t *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t buf[512];
    for (int i = threadIdx.x; i < 512; i += blockDim.x) buf[i] = (uint8_t)i;
    __syncthreads();
    const int t = threadIdx.x;
    if (t < 8) {
        uint32_t a = (uint32_t)(uintptr_t)buf + 16 + t;
        uint32_t v32;
        uint64_t v64;
        v4u v128;
        asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v32) : "v"(a) : "memory");
        asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v64) : "v"(a) : "memory");
        asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v128) : "v"(a) : "memory");
        out[8 * t] = v32;
        out[8 * t + 1] = (uint32_t)v64;
        out[8 * t + 2] = (uint32_t)(v64 >> 32);
        for (int i = 0; i < 4; ++i) out[8 * t + 3 + i] = v128[i];
    }
    __syncthreads();
    // unaligned 16-byte writes: lane t writes 0xA0+t x16 at byte 256 + 17 t
    if (t < 8) {
        uint32_t a = (uint32_t)(uintptr_t)buf + 256 + 17 * t;
        const uint32_t x = 0x01010101u * (0xA0u + t);
        v4u w = {x, x, x, x};
        asm volatile("ds_write_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : : "v"(a), "v"(w) : "memory");
    }
    __syncthreads();
    if (t == 0)
        for (int i = 0; i < 40; ++i) out[64 + i] = ((const uint32_t *)(buf + 256))[i];
}

int main()
{
    uint32_t *d, h[104];
    hipMalloc(&d, sizeof(h));
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int t = 0; t < 8; ++t)
        printf("addr %d: b32 %08x b64 %08x%08x b128 %08x %08x %08x %08x\n", 16 + t, h[8 * t], h[8 * t + 2], h[8 * t + 1],
               h[8 * t + 3], h[8 * t + 4], h[8 * t + 5], h[8 * t + 6]);
    printf("writes:");
    for (int i = 0; i < 40; ++i) printf(" %08x", h[64 + i]);
    printf("\n");
    return 0;
}
