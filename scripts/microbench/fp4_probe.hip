// Probe of the block-scaled MFMA v_mfma_scale_f32_32x32x64_f8f6f4 with FP4
// (e2m1) operands as a bit-matrix product: 0/1 bits as the e2m1 codes 0x0 /
// 0x2 (= 1.0), so D[m][n] = sum_k A[m][k] B[n][k] = popcount(a_m & b_n) over
// 64 bits, exact in f32. Assumed operand map (checked here against the CPU):
// lane l = r + 32 h holds row r's bits [32 h, 32 h + 32) as 32 nibbles
// (element j in nibble j of the 16 bytes, low nibble first) for A, and
// column r's for B; D: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5).
//   build: hipcc -O3 --offload-arch=gfx950 fp4_probe.hip -o fp4_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <random>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t nib8(uint32_t byte) {   // 8 bits -> 8 nibbles 0x0 / 0x2
    uint32_t t = (byte & 0x0Fu) | ((byte & 0xF0u) << 12);
    t = (t | (t << 6)) & 0x03030303u;
    t = (t | (t << 3)) & 0x11111111u;
    return t << 1;
}

template <int SCALE>
__global__ void probe(const unsigned long long* a, const unsigned long long* b, float* d) {
    const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
    const uint32_t abits = (uint32_t)(a[r] >> (32 * h)), bbits = (uint32_t)(b[r] >> (32 * h));
    v8i av = {0, 0, 0, 0, 0, 0, 0, 0}, bv = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int q = 0; q < 4; q++) {
        av[q] = (int)nib8((abits >> (8 * q)) & 0xFF);
        bv[q] = (int)nib8((bbits >> (8 * q)) & 0xFF);
    }
    v16f acc;
    for (int i = 0; i < 16; i++) acc[i] = 0.0f;
    acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc, 4, 4, 0, SCALE, 0, SCALE);
    for (int reg = 0; reg < 16; reg++) {
        const int row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5), col = lane & 31;
        d[row * 32 + col] = acc[reg];
    }
}

int main() {
    std::mt19937_64 rng(7);
    unsigned long long ha[32], hb[32];
    for (int i = 0; i < 32; i++) { ha[i] = rng(); hb[i] = rng() & rng(); }
    unsigned long long *da, *db;
    float* dd;
    hipMalloc(&da, 256); hipMalloc(&db, 256); hipMalloc(&dd, 32 * 32 * 4);
    hipMemcpy(da, ha, 256, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, 256, hipMemcpyHostToDevice);
    float hd[1024];
    for (int pass = 0; pass < 2; pass++) {
        hipMemset(dd, 0, 4096);
        if (pass == 0) probe<0><<<1, 64>>>(da, db, dd);
        else probe<127><<<1, 64>>>(da, db, dd);
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
        hipMemcpy(hd, dd, 4096, hipMemcpyDeviceToHost);
        int bad = 0, bad_t = 0;
        double ratio = 0;
        for (int m = 0; m < 32; m++)
            for (int n = 0; n < 32; n++) {
                const float want = (float)__builtin_popcountll(ha[m] & hb[n]);
                const float want_t = (float)__builtin_popcountll(ha[n] & hb[m]);
                bad += hd[m * 32 + n] != want;
                bad_t += hd[m * 32 + n] != want_t;
                if (want > 0) ratio = hd[m * 32 + n] / want;
            }
        printf("scale %d: mismatches %d (transposed %d), d[0]=%g want %d, last ratio %g\n", pass ? 127 : 0, bad,
               bad_t, hd[0], __builtin_popcountll(ha[0] & hb[0]), ratio);
    }
    return 0;
}
