// LDS atomic-add ceiling micro-benchmark for the sparse tile kernel's
// counter updates (ds_add_u32 into a 128 x 128 int32 tile of counters,
// 1024-thread workgroups, two per CU as the kernel runs). Variants:
//   rand   : ds_add_u32 at pseudo-random counters (the kernel's pattern)
//   seq    : ds_add_u32 at lane-consecutive counters (no bank conflicts)
//   write  : plain ds_write_b32 at the random counters (no read-modify-write)
//   rmw    : ds_read_b32 + ds_write_b32 at the random counters (racy, timing only)
// Prints lane-operations per second chip-wide.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int SB = 128;

template <int MODE>
__global__ __launch_bounds__(1024, 2) void kern(int iters, int* out) {
    __shared__ int cnt[SB * SB];
    for (int t = threadIdx.x; t < SB * SB; t += 1024) cnt[t] = 0;
    __syncthreads();
    unsigned x = 0x9E3779B9u * (blockIdx.x * 1024 + threadIdx.x + 1);
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            x ^= x << 13; x ^= x >> 17; x ^= x << 5;
            const int idx = MODE == 1 ? ((threadIdx.x + i * 8 + u) & (SB * SB - 1)) : (int)(x & (SB * SB - 1));
            if (MODE == 0 || MODE == 1) atomicAdd(&cnt[idx], 1);
            else if (MODE == 2) cnt[idx] = (int)x;
            else cnt[idx] += 1;
        }
    }
    __syncthreads();
    int s = 0;
    for (int t = threadIdx.x; t < SB * SB; t += 1024) s += cnt[t];
    if (s == 0x7fffffff) out[blockIdx.x] = s;
}

template <class K>
double run(K k, int iters) {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int* out;
    hipMalloc(&out, 1 << 20);
    const int grid = cus * 2;
    k<<<grid, 1024>>>(iters / 10, out);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    k<<<grid, 1024>>>(iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    hipFree(out);
    return (double)grid * 1024 * iters * 8 / (ms * 1e-3);
}

int main() {
    const int iters = 4000;
    printf("lane-ops/s chip-wide (2 x 1024-thread workgroups per CU, 64 KiB counters each)\n");
    printf("rand ds_add_u32   %.3e\n", run(kern<0>, iters));
    printf("seq  ds_add_u32   %.3e\n", run(kern<1>, iters));
    printf("rand ds_write_b32 %.3e\n", run(kern<2>, iters));
    printf("rand read+write   %.3e\n", run(kern<3>, iters));
    return 0;
}
