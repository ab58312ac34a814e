// VALU ceiling micro-benchmark for the bitset inner step (and + bcnt).
// Each variant runs an unrolled register-only stream with explicit VGPRs so
// operand banks (register index mod 4) are controlled. Prints wave-instr/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define REP8(x) x x x x x x x x
// A: and with same-bank sources (v0,v4 ...), bcnt(temp, acc) — the pattern hipcc emits
#define BODY_A \
  "v_and_b32 v40, v0, v4\n v_bcnt_u32_b32 v20, v40, v20\n" \
  "v_and_b32 v41, v1, v5\n v_bcnt_u32_b32 v21, v41, v21\n" \
  "v_and_b32 v42, v2, v6\n v_bcnt_u32_b32 v22, v42, v22\n" \
  "v_and_b32 v43, v3, v7\n v_bcnt_u32_b32 v23, v43, v23\n" \
  "v_and_b32 v44, v8, v12\n v_bcnt_u32_b32 v24, v44, v24\n" \
  "v_and_b32 v45, v9, v13\n v_bcnt_u32_b32 v25, v45, v25\n" \
  "v_and_b32 v46, v10, v14\n v_bcnt_u32_b32 v26, v46, v26\n" \
  "v_and_b32 v47, v11, v15\n v_bcnt_u32_b32 v27, v47, v27\n"
// B: and with different-bank sources (v0,v5), temp/acc banks differ too
#define BODY_B \
  "v_and_b32 v40, v0, v5\n v_bcnt_u32_b32 v21, v40, v21\n" \
  "v_and_b32 v41, v1, v6\n v_bcnt_u32_b32 v22, v41, v22\n" \
  "v_and_b32 v42, v2, v7\n v_bcnt_u32_b32 v23, v42, v23\n" \
  "v_and_b32 v43, v3, v4\n v_bcnt_u32_b32 v20, v43, v20\n" \
  "v_and_b32 v44, v8, v13\n v_bcnt_u32_b32 v25, v44, v25\n" \
  "v_and_b32 v45, v9, v14\n v_bcnt_u32_b32 v26, v45, v26\n" \
  "v_and_b32 v46, v10, v15\n v_bcnt_u32_b32 v27, v46, v27\n" \
  "v_and_b32 v47, v11, v12\n v_bcnt_u32_b32 v24, v47, v24\n"
// C: all and first then all bcnt (no back-to-back dependency), different banks
#define BODY_C \
  "v_and_b32 v40, v0, v5\n v_and_b32 v41, v1, v6\n v_and_b32 v42, v2, v7\n v_and_b32 v43, v3, v4\n" \
  "v_and_b32 v44, v8, v13\n v_and_b32 v45, v9, v14\n v_and_b32 v46, v10, v15\n v_and_b32 v47, v11, v12\n" \
  "v_bcnt_u32_b32 v21, v40, v21\n v_bcnt_u32_b32 v22, v41, v22\n v_bcnt_u32_b32 v23, v42, v23\n v_bcnt_u32_b32 v20, v43, v20\n" \
  "v_bcnt_u32_b32 v25, v44, v25\n v_bcnt_u32_b32 v26, v45, v26\n v_bcnt_u32_b32 v27, v46, v27\n v_bcnt_u32_b32 v24, v47, v24\n"
// D: and only; E: bcnt only
#define BODY_D \
  "v_and_b32 v40, v0, v5\n v_and_b32 v41, v1, v6\n v_and_b32 v42, v2, v7\n v_and_b32 v43, v3, v4\n" \
  "v_and_b32 v44, v8, v13\n v_and_b32 v45, v9, v14\n v_and_b32 v46, v10, v15\n v_and_b32 v47, v11, v12\n"
#define BODY_E \
  "v_bcnt_u32_b32 v21, v40, v21\n v_bcnt_u32_b32 v22, v41, v22\n v_bcnt_u32_b32 v23, v42, v23\n v_bcnt_u32_b32 v20, v43, v20\n" \
  "v_bcnt_u32_b32 v25, v44, v25\n v_bcnt_u32_b32 v26, v45, v26\n v_bcnt_u32_b32 v27, v46, v27\n v_bcnt_u32_b32 v24, v47, v24\n"
// F: same as C with same-bank and sources
#define BODY_F \
  "v_and_b32 v40, v0, v4\n v_and_b32 v41, v1, v5\n v_and_b32 v42, v2, v6\n v_and_b32 v43, v3, v7\n" \
  "v_and_b32 v44, v8, v12\n v_and_b32 v45, v9, v13\n v_and_b32 v46, v10, v14\n v_and_b32 v47, v11, v15\n" \
  "v_bcnt_u32_b32 v20, v40, v20\n v_bcnt_u32_b32 v21, v41, v21\n v_bcnt_u32_b32 v22, v42, v22\n v_bcnt_u32_b32 v23, v43, v23\n" \
  "v_bcnt_u32_b32 v24, v44, v24\n v_bcnt_u32_b32 v25, v45, v25\n v_bcnt_u32_b32 v26, v46, v26\n v_bcnt_u32_b32 v27, v47, v27\n"

#define CLOB "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15", \
  "v20","v21","v22","v23","v24","v25","v26","v27","v40","v41","v42","v43","v44","v45","v46","v47"

#define KERNEL(NAME, BODY, NINSTR)                                                     \
__global__ __launch_bounds__(256) void NAME(int iters, unsigned* out) {               \
    for (int i = 0; i < iters; i++) asm volatile(REP8(BODY) ::: CLOB);                 \
    unsigned r;                                                                        \
    asm volatile("v_mov_b32 %0, v20" : "=v"(r) :: "v20");                              \
    if (r == 0xdeadbeef) out[threadIdx.x] = r;                                         \
}                                                                                      \
static const int NAME##_n = NINSTR;

KERNEL(kA, BODY_A, 16 * 8)
KERNEL(kB, BODY_B, 16 * 8)
KERNEL(kC, BODY_C, 16 * 8)
KERNEL(kD, BODY_D, 8 * 8)
KERNEL(kE, BODY_E, 8 * 8)
KERNEL(kF, BODY_F, 16 * 8)

template <class K>
double run(K k, int ninstr, int wg_per_cu, int iters) {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned* out;
    hipMalloc(&out, 4096);
    int grid = cus * wg_per_cu;
    k<<<grid, 256>>>(iters / 10, out);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    k<<<grid, 256>>>(iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    hipFree(out);
    double waves = (double)grid * 4;
    return waves * iters * (double)ninstr / (ms * 1e-3);   // wave-instructions per second
}

int main() {
    const int iters = 20000;
    printf("peak (2 cyc/wave-instr @2.4GHz): %.3e wave-instr/s\n", 256.0 * 4 * 2.4e9 / 2);
    for (int occ : {1, 2, 4, 8}) {
        printf("waves/SIMD %d: A(same-bank,dep) %.3e  B(diff-bank,dep) %.3e  C(diff,indep) %.3e  D(and) %.3e  E(bcnt) %.3e  F(same,indep) %.3e\n",
               occ, run(kA, kA_n, occ, iters), run(kB, kB_n, occ, iters), run(kC, kC_n, occ, iters),
               run(kD, kD_n, occ, iters), run(kE, kE_n, occ, iters), run(kF, kF_n, occ, iters));
    }
    return 0;
}
