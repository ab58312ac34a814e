// Calibration of rocprofv3's FETCH_SIZE (and the TCC_EA0_RDREQ request
// counters) on gfx950 for the load shapes of this repo's kernels, against
// known byte counts. MI355X_MICROARCH.md (HBM section) establishes that
// FETCH_SIZE reports half the bytes of a 16 B/lane coalesced streaming read
// and leaves other widths uncalibrated; the sparse tile kernel reads 12-byte
// records at data-dependent positions and the rare walk reads 16 bytes at
// arbitrary 4-byte-aligned positions of a list array.
//
// Every kernel reads from its own 512 MiB table (twice the Infinity Cache, so
// no kernel's lines are resident from an earlier one; each table is written
// once, in order, by the first kernel) and writes one word per thread:
//   stream16   each lane reads 16 B, consecutive (known: 512 MiB of lines)
//   rec12      each lane reads one 12-byte record (dwordx3) of a 16-byte slot,
//              slots visited in a random permutation, every slot once
//              (known: 512 MiB of lines, 384 MiB of useful bytes)
//   gather16   each lane reads 16 B at a random 4-byte-aligned position
//              (known: the loads x 16 B useful; distinct 128-B lines below)
//   gather4    each lane reads 4 B at a random position (known: loads x 4 B)
// Prints per kernel: loads, useful bytes, distinct 64-B sectors and 128-B
// lines touched (computed on the host from the same positions).
//   build: hipcc -O3 --offload-arch=gfx950 fetch_calib.hip -o fetch_calib
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <numeric>
#include <random>
#include <unordered_set>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } \
    } while (0)

__global__ void fill_kernel(uint4* p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((uint32_t)i, (uint32_t)(i >> 32) ^ 0x9E37u, (uint32_t)i * 3u, 7u);
}

__global__ void stream16(const uint4* __restrict__ t, int64_t n, uint32_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 v = t[i];
    out[i] = v.x ^ v.y ^ v.z ^ v.w;
}

struct R3 { uint32_t a, b, c; };
__global__ void rec12(const uint4* __restrict__ t, const uint32_t* __restrict__ perm, int64_t n,
                      uint32_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const R3 r = *reinterpret_cast<const R3*>(t + perm[i]);
    out[i] = r.a ^ r.b ^ r.c;
}

__global__ void gather16(const uint32_t* __restrict__ t, const uint32_t* __restrict__ pos, int64_t n,
                         uint32_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint4 v;
    __builtin_memcpy(&v, t + pos[i], 16);
    out[i] = v.x ^ v.y ^ v.z ^ v.w;
}

__global__ void gather4(const uint32_t* __restrict__ t, const uint32_t* __restrict__ pos, int64_t n,
                        uint32_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = t[pos[i]];
}

static void touched(const std::vector<uint32_t>& pos, int64_t elem, int64_t bytes, const char* name, int64_t useful) {
    std::unordered_set<int64_t> s64, s128;
    for (uint32_t p : pos) {
        const int64_t b0 = (int64_t)p * elem, b1 = b0 + bytes - 1;
        for (int64_t b = b0 >> 6; b <= b1 >> 6; b++) s64.insert(b);
        for (int64_t b = b0 >> 7; b <= b1 >> 7; b++) s128.insert(b);
    }
    printf("%-9s loads %zu useful_bytes %lld sectors64 %zu (%lld B) lines128 %zu (%lld B)\n", name, pos.size(),
           (long long)useful, s64.size(), (long long)s64.size() * 64, s128.size(), (long long)s128.size() * 128);
}

int main() {
    const int64_t bytes = int64_t(512) << 20;        // per table: twice the 256 MiB Infinity Cache
    const int64_t n16 = bytes / 16;                  // 16-byte slots
    uint4 *t1, *t2, *t3, *t4;
    uint32_t *out, *dperm, *dpos16, *dpos4;
    CK(hipMalloc(&t1, bytes)); CK(hipMalloc(&t2, bytes)); CK(hipMalloc(&t3, bytes)); CK(hipMalloc(&t4, bytes));
    CK(hipMalloc(&out, n16 * 4));
    for (uint4* t : {t1, t2, t3, t4}) fill_kernel<<<4096, 256>>>(t, n16);
    CK(hipDeviceSynchronize());
    std::mt19937_64 rng(12345);
    // rec12: every slot once, random order
    std::vector<uint32_t> perm(n16);
    std::iota(perm.begin(), perm.end(), 0u);
    std::shuffle(perm.begin(), perm.end(), rng);
    // gather16 / gather4: 4 M loads at random dword positions
    const int64_t ng = int64_t(4) << 20;
    std::vector<uint32_t> p16(ng), p4(ng);
    const uint32_t ndw = (uint32_t)(bytes / 4);
    for (auto& p : p16) p = (uint32_t)(rng() % (ndw - 4));
    for (auto& p : p4) p = (uint32_t)(rng() % ndw);
    CK(hipMalloc(&dperm, n16 * 4)); CK(hipMalloc(&dpos16, ng * 4)); CK(hipMalloc(&dpos4, ng * 4));
    CK(hipMemcpy(dperm, perm.data(), n16 * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dpos16, p16.data(), ng * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dpos4, p4.data(), ng * 4, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    stream16<<<(unsigned)((n16 + 255) / 256), 256>>>(t1, n16, out);
    CK(hipDeviceSynchronize());
    rec12<<<(unsigned)((n16 + 255) / 256), 256>>>(t2, dperm, n16, out);
    CK(hipDeviceSynchronize());
    gather16<<<(unsigned)((ng + 255) / 256), 256>>>(reinterpret_cast<const uint32_t*>(t3), dpos16, ng, out);
    CK(hipDeviceSynchronize());
    gather4<<<(unsigned)((ng + 255) / 256), 256>>>(reinterpret_cast<const uint32_t*>(t4), dpos4, ng, out);
    CK(hipDeviceSynchronize());
    printf("stream16  loads %lld useful_bytes %lld lines128 %lld (%lld B)\n", (long long)n16, (long long)bytes,
           (long long)(bytes / 128), (long long)bytes);
    printf("rec12     loads %lld useful_bytes %lld lines128 %lld (%lld B) (+ the permutation: %lld B streamed)\n",
           (long long)n16, (long long)(n16 * 12), (long long)(bytes / 128), (long long)bytes, (long long)(n16 * 4));
    touched(p16, 4, 16, "gather16", ng * 16);
    touched(p4, 4, 4, "gather4", ng * 4);
    printf("(every kernel also streams its index array: 4 B per load, and writes 4 B per thread)\n");
    return 0;
}
