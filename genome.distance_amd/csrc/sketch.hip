// sketch.hip — MinHash bottom-s sketches and the all-pairs sketch distance.
//
// sketch_build replaces SequenceKmers.hashSet(width) (SketchProcessor.java:88,
// WidthProcessor.java:178): the `width` smallest distinct murmur3_x86_32
// (seed 0) hashes, in Java signed-int order, of the set's kmer strings.
// sketch_matrix replaces Sketch.distance over all pairs
// (WidthProcessor.java:183-185, TuningProcessor.java:131-133). The
// reference's hash function and sketch formula live in the un-vendored
// org.theseed:sequence module: this contract is the restatement of
// SURVEY App. B Q6 (parity unpinned), mirrored by oracle/.
//
// Build: hash every code of a chunk of sets, radix-sort 64-bit keys
// (set id << 32 | biased hash), keep the first `width` distinct hashes of
// each set. Matrix: sketch_ring_kernel (default) — a workgroup owns a
// 32 x 32 tile of sketch pairs, one lane per pair, the 64 sketches streaming
// through interleaved LDS rings in step-synchronised phases; the
// whole-sketch kernels (option sketch_phase = 0) stage whole sketches in LDS.
#include <cstring>
#include <rocprim/rocprim.hpp>

#include <algorithm>

#include "gdist_internal.hpp"

namespace gdist {
namespace {

inline int grid_for(int64_t n, int block = 256, int64_t cap = 256 * 32) {
    int64_t g = ceil_div(n, block);
    return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// kmer string byte t of code (first char most significant), decoded per spec
__device__ __forceinline__ uint32_t kmer_byte(uint64_t code, int t, int k, int bits, int dna_mode) {
    const uint32_t s = (uint32_t)((code >> (bits * (k - 1 - t))) & ((1u << bits) - 1));
    if (dna_mode == 2) return "ACGT"[s & 3];
    if (dna_mode == 3) return "ACGNRTY"[s < 7 ? s : 3];
    if (bits == 8) return s;
    return s == 0 ? (uint32_t)'*' : (uint32_t)('A' + s - 1);
}

__device__ uint32_t murmur3_kmer(uint64_t code, int k, int bits, int dna_mode) {
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    uint32_t h = 0;
    int t = 0;
    for (; t + 4 <= k; t += 4) {
        uint32_t kk = kmer_byte(code, t, k, bits, dna_mode) | (kmer_byte(code, t + 1, k, bits, dna_mode) << 8) |
                      (kmer_byte(code, t + 2, k, bits, dna_mode) << 16) |
                      (kmer_byte(code, t + 3, k, bits, dna_mode) << 24);
        kk *= c1; kk = rotl32(kk, 15); kk *= c2;
        h ^= kk; h = rotl32(h, 13); h = h * 5 + 0xe6546b64u;
    }
    uint32_t k1 = 0;
    const int tail = k - t;
    if (tail >= 3) k1 ^= kmer_byte(code, t + 2, k, bits, dna_mode) << 16;
    if (tail >= 2) k1 ^= kmer_byte(code, t + 1, k, bits, dna_mode) << 8;
    if (tail >= 1) {
        k1 ^= kmer_byte(code, t, k, bits, dna_mode);
        k1 *= c1; k1 = rotl32(k1, 15); k1 *= c2; h ^= k1;
    }
    h ^= (uint32_t)k;
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}

// key = (local set id << 32) | (hash ^ 0x80000000): unsigned order == (set, signed hash)
__global__ void hash_keys_kernel(const uint64_t* __restrict__ codes, const int64_t* __restrict__ off,
                                 int64_t s0, int64_t ns, int k, int bits, int dna_mode,
                                 uint64_t* __restrict__ keys) {
    const int64_t base = off[s0];
    const int64_t n = off[s0 + ns] - base;
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
        const int64_t g = base + e;
        int64_t lo = s0, hi = s0 + ns;
        while (hi - lo > 1) {
            int64_t mid = (lo + hi) >> 1;
            if (off[mid] <= g) lo = mid; else hi = mid;
        }
        const uint32_t h = murmur3_kmer(codes[g], k, bits, dna_mode);
        keys[e] = ((uint64_t)(lo - s0) << 32) | (uint64_t)(h ^ 0x80000000u);
    }
}

__global__ void head_flags_kernel(const uint64_t* __restrict__ keys, int64_t n, int32_t* __restrict__ flag) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        flag[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
}

// per local set: first index (lower_bound of set<<32) and distinct count
__global__ void set_starts_kernel(const uint64_t* __restrict__ keys, const int64_t* __restrict__ pos,
                                  const int32_t* __restrict__ flag, int64_t n, int64_t ns,
                                  int64_t* __restrict__ ustart) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s > ns) return;
    const uint64_t v = (uint64_t)s << 32;
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (keys[mid] < v) lo = mid + 1; else hi = mid;
    }
    const int64_t total = n ? pos[n - 1] + flag[n - 1] : 0;
    ustart[s] = lo < n ? pos[lo] : total;
}

__global__ void emit_sig_kernel(const uint64_t* __restrict__ keys, const int32_t* __restrict__ flag,
                                const int64_t* __restrict__ pos, const int64_t* __restrict__ ustart,
                                const int64_t* __restrict__ out_off, int64_t n, int width,
                                int32_t* __restrict__ sig) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (!flag[i]) continue;
        const int64_t s = (int64_t)(keys[i] >> 32);
        const int64_t r = pos[i] - ustart[s];
        if (r < width) sig[out_off[s] + r] = (int32_t)((uint32_t)keys[i] ^ 0x80000000u);
    }
}

constexpr int LDS_SK_MAX = 160 * 1024;      // whole CU LDS: one workgroup per CU at width ~1000
constexpr int LDS_SK_SLACK = 64;            // phase-1 reads stop at n-1, slack only guards rounding

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

// LDS row stride (dwords): odd, so the R+C rows of a tile start on distinct
// banks (ds_read2_b32 banks by dword mod 32). Measured against the even
// stride it made no difference (lanes' merge positions spread the banks
// anyway: DESIGN.md §4); kept as the conflict-neutral choice.
inline int sketch_stride(int width) { return width | 1; }

// One workgroup = an R x C tile of sketch pairs, one lane per pair
// (R*C threads).  16x24 at width <= ~1000 puts 40 sketches (160,000 B) in LDS
// and 6 waves on the CU; 16x16 covers wider sketches (and the global-memory
// variant, LDS=false, anything wider still).
//
// Fill (LDS variant): the R+C sketches of the tile are DMA'd global->LDS with
// global_load_lds, one 64-dword row segment per wave instruction, all issued
// before a single vmcnt(0) wait.  Lanes past a sketch's length are masked off
// (exec), so rows sit at the odd stride sketch_stride(width) with no padding.
//
// Merge (Sketch.distance, WidthProcessor.java:185; restated in
// oracle/pyref.py:sketch_distance).  Sketches are strictly increasing
// (built that way; uploads are validated), so:
//   phase 1 - while both sides have elements (and, for Mash, fewer than
//             `width` union elements were taken): load both heads, advance by
//             the <=/>= masks.  Branch-free, one LDS latency per step.
//             common = ia + ib - steps (a common element advances both).
//   phase 2 - closed form: the rest of the non-exhausted side are distinct
//             union elements with no common ones.
//
// V2 (round 3): lanes of a 32-lane LDS group cover a 4 x 8 block of pairs
// (4 row sketches, 8 column sketches) instead of one and a third rows of 24
// columns, so a group's reads fall on 4 (rows) or 8 (columns) sketches at
// similar positions, not 24 scattered ones; each LDS row carries two INT_MAX
// sentinels past its last hash, so while fewer than max(ina, inb) steps are
// taken (one side still has elements) the two-step rounds run without bounds
// checks. A pair whose sketch ends in INT_MAX (a real hash the sentinel
// would equal) takes the checked loop.
template <int R, int C, bool LDS, int KW, bool V2 = false>
__global__ __launch_bounds__(R * C) void sketch_tile_kernel(const int32_t* __restrict__ sig,
                                                            const int64_t* __restrict__ off, int width, int sw,
                                                            int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                                                            int64_t tile0, int tiles_c, int upper, int jaccard,
                                                            int empty_nan,
                                                            int32_t* __restrict__ common_out,
                                                            double* __restrict__ D, int64_t ld) {
#pragma clang fp contract(off)
    constexpr int NT = R * C, NW = NT / 64, NS = R + C;
    extern __shared__ int32_t sm[];   // [R+C][sketch_stride(width)] (+ slack)
    __shared__ int64_t s_base[NS];
    __shared__ int32_t s_n[NS];
    constexpr int GR = 4, GC = 8;
    static_assert(!V2 || (R % GR == 0 && C % GC == 0 && LDS && KW == 2), "V2: GR x GC lane groups, LDS, K = 2");
    const int64_t bt = tile0 + blockIdx.x;
    const int tr = (int)(bt / tiles_c), tcb = (int)(bt % tiles_c);
    const int64_t row0 = r0 + (int64_t)tr * R, col0 = c0 + (int64_t)tcb * C;
    int ty, tx;
    if (V2) {
        const int g = threadIdx.x >> 5, l = threadIdx.x & 31;
        ty = (g / (C / GC)) * GR + l / GC;
        tx = (g % (C / GC)) * GC + l % GC;
    } else {
        ty = threadIdx.x / C;
        tx = threadIdx.x - ty * C;
    }
    if (upper && col0 + C - 1 <= row0) return;
    if (LDS) {
        if (threadIdx.x < NS) {
            const int s = threadIdx.x;
            const int64_t g = s < R ? row0 + s : col0 + (s - R);
            const bool ok = s < R ? g < r1 : g < c1;
            s_base[s] = ok ? off[g] : 0;
            s_n[s] = ok ? (int32_t)(off[g + 1] - off[g]) : 0;
        }
        __syncthreads();
        const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
        for (int s = wave; s < NS; s += NW) {
            const int n = __builtin_amdgcn_readfirstlane(s_n[s]);
            const int32_t* src = sig + s_base[s];
            if (V2 && lane < 2) sm[s * sw + n + lane] = 0x7FFFFFFF;      // sentinels past the hashes
            for (int t = 0; t < n; t += 64) {
                if (t + lane < n)
                    __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + t + lane),
                                                     (lds_void_t*)(sm + s * sw + t), 4, 0, 0);
            }
        }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    const int64_t i = row0 + ty, j = col0 + tx;
    if (i >= r1 || j >= c1 || (upper && j <= i)) return;
    const int ina = LDS ? s_n[ty] : (int)(off[i + 1] - off[i]);
    const int inb = LDS ? s_n[R + tx] : (int)(off[j + 1] - off[j]);
    const int32_t* A = LDS ? sm + ty * sw : sig + off[i];
    const int32_t* B = LDS ? sm + (R + tx) * sw : sig + off[j];
    const int lim = jaccard ? ina + inb : width;
    int ia = 0, ib = 0, steps = 0;
    if (V2) {
        const bool imax = (ina > 0 && A[ina - 1] == 0x7FFFFFFF) || (inb > 0 && B[inb - 1] == 0x7FFFFFFF);
        // one unchecked two-step round of a merge at (pa, pb): the rows'
        // sentinels stand in for an exhausted side
        auto round2 = [&](int& pa, int& pb) {
            const int32_t a0 = A[pa], a1 = A[pa + 1], b0 = B[pb], b1 = B[pb + 1];
            const bool le = a0 <= b0, ge = b0 <= a0;
            const int32_t x = le ? a1 : a0, y = ge ? b1 : b0;
            pa += le;
            pb += ge;
            pa += x <= y;
            pb += y <= x;
        };
        // unchecked rounds while steps < max(ina, inb) (and < lim): one side
        // still has hashes, the other reads its sentinels
        const int ns = imax ? 0 : min(lim, max(ina, inb));
        const int nr = ns > steps ? (ns - steps) >> 1 : 0;
        for (int r = 0; r < nr; r++) round2(ia, ib);
        steps += 2 * nr;
    }
    if (KW > 1) {
        // steady state: both sides have >= KW elements left and >= KW steps
        // remain, so KW steps run unchecked on a KW-element window per side
        // (one LDS round trip); a step shifts the window of the side(s) it
        // advances.  Boundary rounds fall through to the one-step loop.
        while (ina - ia >= KW && inb - ib >= KW && lim - steps >= KW) {
            int32_t a[KW], b[KW];
#pragma unroll
            for (int u = 0; u < KW; u++) { a[u] = A[ia + u]; b[u] = B[ib + u]; }
#pragma unroll
            for (int s = 0; s < KW; s++) {
                const bool le = a[0] <= b[0], ge = b[0] <= a[0];
                ia += le;
                ib += ge;
#pragma unroll
                for (int u = 0; u + 1 < KW - s; u++) {
                    a[u] = le ? a[u + 1] : a[u];
                    b[u] = ge ? b[u + 1] : b[u];
                }
            }
            steps += KW;
        }
    }
    while (ia < ina && ib < inb && steps < lim) {
        const int32_t va = A[ia], vb = B[ib];
        ia += va <= vb;
        ib += vb <= va;
        steps++;
    }
    const int common = ia + ib - steps;
    const int taken = steps + min((ina - ia) + (inb - ib), width - steps);
    const int64_t na = ina, nb = inb;
    double d;
    if (jaccard) {
        if (common > 0) d = 1.0 - (double)common / (double)(na + nb - common);
        else d = (empty_nan && na + nb == 0) ? __builtin_nan("") : 1.0;
    } else {
        if (common > 0) d = 1.0 - (double)common / (double)taken;
        else d = (empty_nan && taken == 0) ? __builtin_nan("") : 1.0;
    }
    const int64_t o = (i - r0) * ld + (j - c0);
    if (common_out) common_out[o] = (int32_t)common;
    if (D) D[o] = d;
}

constexpr int kSkTile = 32;                 // rows = columns = LDS banks of ds_read_b32
constexpr int kSkLanes = 2 * kSkTile;       // interleave stride (dwords) = sketches per tile
typedef int32_t i32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

// Ring kernel (round 3, default; option sketch_phase = 0 keeps the
// whole-sketch kernels above). Those are bound by LDS bank conflicts: their
// lanes read their sketches at data-dependent positions, so a 32-lane
// group's ds_read hits random banks (68 % of LDS cycles are conflict cycles,
// profiles/r03/sketch/pmc_v2.txt). Here the tile is 32 row x 32 column
// sketches and LDS is interleaved: slot q of sketch s (rows 0..31, columns
// 32..63) sits at dword 64 q + s, so its bank is s mod 32 whatever q is. Lane
// l of 32-lane group g merges row l with column (l + g) mod 32: the 32 lanes
// of a group read 32 distinct rows and 32 distinct columns — conflict-free at
// any merge positions (SQ_LDS_BANK_CONFLICT = 0, profiles/r03/sketch2/).
//
// 64 whole sketches do not fit LDS interleaved, so each sketch streams
// through a ring of RS slots (RS a power of two, slot = position & (RS - 1),
// plus one mirror row RS = row 0 so the head pair (q, q + 1) is one
// ds_read2st64 at any slot) in step-synchronised phases: every open pair
// takes (up to) the same budget K of merge steps per phase. (Value-range
// phases — every sketch's hashes below a common bound per phase — were
// measured first: a pair's merge per phase is then the union of its two
// windows, twice as many steps for a dissimilar pair as for a near-identical
// one, and C5's waves ran ~1.45x their lanes' mean steps: 368 vs 320 ms.
// Unmasked slot indexes with kmax + 1 mirror rows cut 2 VALU per round, but
// the larger LDS leaves one workgroup per CU: 389 ms.)
// Each phase: s_min[s] = the least position of the open pairs reading s;
// the ring is topped up to top_s = min(n_s + 2, s_min[s] + RS) (positions
// n_s, n_s + 1 are INT_MAX sentinels; positions below s_min are never read
// again and not loaded; every slot a load overwrites held a position <
// s_min[s]); a pair at (pa, pb) may take K = min(kmax, lim - steps,
// top_a - pa, top_b - pb) steps, since a round starting after j <= K - 2
// steps reads positions <= p + K - 1. Within K the unchecked rounds run in
// batches bounded by the remaining real union (>= the longer remainder, as
// above), then at most one checked step. A pair with no room (it leads a
// sketch by a whole ring over that sketch's slowest pair) takes up to kmax
// checked steps straight from global memory, so every phase advances
// (option sketch_wait = 1: such a pair waits for the slower ones instead,
// and reads global memory only after a phase in which no pair advanced —
// C5: 430 vs 336 ms with a 448-slot ring, the waiting pairs add phases). Positions, steps and the
// closed form are the merge's: results are identical
// (test_sketch_merge_edges_vs_oracle runs rings of 16..448 slots).
typedef __attribute__((address_space(3))) const int32_t lds_i32;   // an LDS dword
__global__ __launch_bounds__(kSkTile * kSkTile) void sketch_ring_kernel(
    const int32_t* __restrict__ sig, const int64_t* __restrict__ off, int width, int RS, int kmax, int64_t r0,
    int64_t r1, int64_t c0, int64_t c1, int64_t tile0, int tiles_c, int upper, int jaccard, int empty_nan,
    int32_t* __restrict__ common_out, double* __restrict__ D, int64_t ld, int fallback, int tri, int sperm) {
#pragma clang fp contract(off)
    constexpr int R = kSkTile, C = kSkTile, NT = R * C, NW = NT / 64, NS = kSkLanes;
    // [RS + 1][64]: ring slot q of sketch s at 64 q + s, row RS = row 0; then
    // the sketches' metadata and three flag words (round 6: no static LDS, so
    // the ring starts at LDS address 0 and a slot's byte offset is its LDS
    // address: the 256-slot walk's one-v_perm addresses need no add)
    extern __shared__ __attribute__((aligned(16))) int32_t sm[];
    int64_t* s_base = reinterpret_cast<int64_t*>(sm + (RS + 1) * NS);     // 8-byte aligned: 256 B a ring row
    int32_t* s_n = reinterpret_cast<int32_t*>(s_base + NS);
    int32_t* s_top = s_n + NS;
    int32_t* s_min = s_top + NS;
    int32_t* s_imax = s_min + NS;
    int32_t* s_or = s_imax + NS;                                           // block_or's three flag words
    // the ring's LDS byte address (0: the kernel declares no static LDS)
    const uint32_t ring0 = (uint32_t)(size_t)(const lds_i32*)sm;
    const int64_t bt = tile0 + blockIdx.x;
    int tr, tcb;
    if (tri) {
        // a square upper triangle launches only its tiles tr <= tcb:
        // bt = tcb (tcb + 1) / 2 + tr
        int64_t a = (int64_t)((__builtin_sqrt(8.0 * (double)bt + 1.0) - 1.0) * 0.5);
        while (a * (a + 1) / 2 > bt) a--;
        while ((a + 1) * (a + 2) / 2 <= bt) a++;
        tcb = (int)a;
        tr = (int)(bt - a * (a + 1) / 2);
    } else {
        tr = (int)(bt / tiles_c);
        tcb = (int)(bt % tiles_c);
    }
    const int64_t row0 = r0 + (int64_t)tr * R, col0 = c0 + (int64_t)tcb * C;
    const int g = threadIdx.x >> 5, l = threadIdx.x & 31;
    const int ty = l, tx = (l + g) & (C - 1);
    if (upper && col0 + C - 1 <= row0) return;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (threadIdx.x < NS) {
        const int s = threadIdx.x;
        const int64_t gi = s < R ? row0 + s : col0 + (s - R);
        const bool ok = s < R ? gi < r1 : gi < c1;
        const int64_t b = ok ? off[gi] : 0;
        const int n = ok ? (int)(off[gi + 1] - b) : 0;
        s_base[s] = b;
        s_n[s] = n;
        s_top[s] = 0;
        s_imax[s] = n > 0 && sig[b + n - 1] == 0x7FFFFFFF;
        if (s < 3) s_or[s] = 0;
    }
    __syncthreads();
    // __syncthreads_or without its own LDS: use k ORs into flag k mod 3 (zeroed
    // by use k - 2, whose readers all passed use k - 1's barrier) and zeroes
    // flag (k + 1) mod 3, whose last readers (use k - 2) passed this use's
    // writes' barrier; one barrier a use
    int orc = 0;
    auto block_or = [&](bool v) -> bool {
        const int k = orc % 3;
        if (v) s_or[k] = 1;
        if (threadIdx.x == 0) s_or[k == 2 ? 0 : k + 1] = 0;
        __syncthreads();
        const bool r = s_or[k] != 0;
        orc++;
        return r;
    };
    const int64_t i = row0 + ty, j = col0 + tx;
    const bool valid = i < r1 && j < c1 && !(upper && j <= i);
    const int ina = s_n[ty], inb = s_n[R + tx];
    const bool imax = s_imax[ty] || s_imax[R + tx];
    const int lim = jaccard ? ina + inb : width;
    int ia = 0, ib = 0, steps = 0, extra = 0;
    bool open = valid;
    if (open && (ina == 0 || inb == 0 || lim == 0)) {
        extra = min(ina + inb, lim);
        open = false;
    }
    const int32_t* Arow = sm + ty;
    const int32_t* Brow = sm + R + tx;
    const int32_t* gA = sig + s_base[ty];
    const int32_t* gB = sig + s_base[R + tx];
    bool stalled = false;
    for (;;) {
        // 1. the least position of the open pairs on every sketch
        if (threadIdx.x < NS) s_min[threadIdx.x] = 0x7FFFFFFF;
        __syncthreads();
        if (open) {
            atomicMin(&s_min[ty], ia);
            atomicMin(&s_min[R + tx], ib);
        }
        __syncthreads();
        // 2. top the rings up: positions [max(top, least), min(n + 2, least +
        // RS)), the sentinels past n; thread (s = lane, q = wave) moves 4
        // positions per step, the 32 lanes of a group store to 32 distinct banks
        {
            const int s = lane;
            const int n = s_n[s], least = s_min[s];
            const int lo = least == 0x7FFFFFFF ? 0 : max(s_top[s], least);
            const int hi = least == 0x7FFFFFFF ? 0 : min(n + 2, least + RS);
            const int32_t* src = sig + s_base[s];
            const int M = RS - 1;                   // RS: a power of two
            int q = (lo + wave * 4) & M;
            for (int t = lo + wave * 4; t < hi; t += NW * 4) {
                i32x4_a4 v;
                if (t + 4 <= n) {
                    v = *reinterpret_cast<const i32x4_a4*>(src + t);
                } else {
                    v.x = t < n ? src[t] : 0x7FFFFFFF;
                    v.y = t + 1 < n ? src[t + 1] : 0x7FFFFFFF;
                    v.z = t + 2 < n ? src[t + 2] : 0x7FFFFFFF;
                    v.w = 0x7FFFFFFF;
                }
                const int32_t vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    if (t + u < hi) {
                        const int qu = (q + u) & M;
                        sm[qu * NS + s] = vv[u];
                        if (qu == 0) sm[RS * NS + s] = vv[u];
                    }
                }
                q = (q + NW * 4) & M;
            }
        }
        __syncthreads();
        if (threadIdx.x < NS && s_min[threadIdx.x] != 0x7FFFFFFF)
            s_top[threadIdx.x] = min(s_n[threadIdx.x] + 2, s_min[threadIdx.x] + RS);
        // 3. K steps per open pair
        int done = 0;
        if (open) {
            const int roomA = min(s_n[ty] + 2, s_min[ty] + RS) - ia;
            const int roomB = min(s_n[R + tx] + 2, s_min[R + tx] + RS) - ib;
            const int K = min(min(kmax, lim - steps), min(roomA, roomB));
            if (K > 0) {
                const int mask = RS - 1;
                int pa = ia, pb = ib;
                while (!imax) {
                    const int ns = min(K - done, max(ina - pa, inb - pb));
                    if (ns < 2) break;
                    const int nr = ns >> 1;
                    if (RS == 256 && sperm && ring0 == 0) {
                        // 256-slot rings (the default): a slot's byte offset in
                        // the ring is (p & 255) << 8 | the sketch's 4 s < 256,
                        // one v_perm_b32 (byte 1 = p's low byte, byte 0 = 4 s)
                        // instead of an AND and a shift-add, used as the LDS
                        // address itself (the ring starts at 0; round 6)
                        const uint32_t ra = 4u * (uint32_t)ty, rb = 4u * (uint32_t)(R + tx);
                        for (int r = 0; r < nr; r++) {
                            const lds_i32* pA = (const lds_i32*)(size_t)__builtin_amdgcn_perm((uint32_t)pa, ra, 0x0C0C0400u);
                            const lds_i32* pB = (const lds_i32*)(size_t)__builtin_amdgcn_perm((uint32_t)pb, rb, 0x0C0C0400u);
                            const int32_t a0 = pA[0], a1 = pA[NS], b0 = pB[0], b1 = pB[NS];
                            const bool le = a0 <= b0, ge = b0 <= a0;
                            const int32_t x = le ? a1 : a0, y = ge ? b1 : b0;
                            pa += le;
                            pb += ge;
                            pa += x <= y;
                            pb += y <= x;
                        }
                    } else {
                        for (int r = 0; r < nr; r++) {
                            const int32_t* pA = Arow + (pa & mask) * NS;      // slot RS - 1: pA[NS] is the mirror row
                            const int32_t* pB = Brow + (pb & mask) * NS;
                            const int32_t a0 = pA[0], a1 = pA[NS], b0 = pB[0], b1 = pB[NS];
                            const bool le = a0 <= b0, ge = b0 <= a0;
                            const int32_t x = le ? a1 : a0, y = ge ? b1 : b0;
                            pa += le;
                            pb += ge;
                            pa += x <= y;
                            pb += y <= x;
                        }
                    }
                    done += 2 * nr;
                }
                while (done < K && pa < ina && pb < inb) {            // checked steps inside the rings
                    const int32_t va = Arow[(pa & mask) * NS], vb = Brow[(pb & mask) * NS];
                    pa += va <= vb;
                    pb += vb <= va;
                    done++;
                }
                ia = pa;
                ib = pb;
            } else if (stalled || fallback) {
                // no room in a ring: checked steps from global memory (option
                // sketch_wait = 1: only after a phase with no progress anywhere)
                const int Kg = min(kmax, lim - steps);
                while (done < Kg && ia < ina && ib < inb) {
                    const int32_t va = gA[ia], vb = gB[ib];
                    ia += va <= vb;
                    ib += vb <= va;
                    done++;
                }
            }
            steps += done;
            if (steps >= lim) open = false;
            else if (ia == ina || ib == inb) {     // a side ended: the rest are union-only
                extra = min((ina - ia) + (inb - ib), lim - steps);
                open = false;
            }
        }
        stalled = !block_or(done > 0);
        if (!block_or(open)) break;
    }
    if (!valid) return;
    const int common = ia + ib - steps;
    const int taken = steps + extra;
    const int64_t na = ina, nb = inb;
    double d;
    if (jaccard) {
        if (common > 0) d = 1.0 - (double)common / (double)(na + nb - common);
        else d = (empty_nan && na + nb == 0) ? __builtin_nan("") : 1.0;
    } else {
        if (common > 0) d = 1.0 - (double)common / (double)taken;
        else d = (empty_nan && taken == 0) ? __builtin_nan("") : 1.0;
    }
    const int64_t o = (i - r0) * ld + (j - c0);
    if (common_out) common_out[o] = (int32_t)common;
    if (D) D[o] = d;
}

template <int R, int C>
constexpr size_t sketch_meta_bytes() { return (size_t)(R + C) * (sizeof(int64_t) + sizeof(int32_t)); }

// ring kernel LDS: RS ring rows + the mirror row, 64 dwords each, then the
// metadata (int64 base + four int32 per sketch) and three flag words
inline size_t sketch_ring_lds(int rs) { return (size_t)(rs + 1) * kSkLanes * 4 + (size_t)kSkLanes * 24 + 16; }

int launch_sketch_ring(hipStream_t st, const gdist_sets* sk, int width, int rs, int kmax, int64_t r0, int64_t r1,
                        int64_t c0, int64_t c1, bool upper, int jac, int en, int32_t* d_common, double* d_D,
                        int64_t ld, bool fallback, bool sperm) {
    const size_t lds = sketch_ring_lds(rs);
    GD_REQUIRE(rs >= 16 && (rs & (rs - 1)) == 0 && kmax >= 2 && kmax < rs,
               "sketch ring: a power of two >= 16 slots, 2 <= steps per phase < slots");
    GD_REQUIRE(lds + 64 <= (size_t)LDS_SK_MAX, "sketch ring exceeds LDS");
    const int tr = (int)ceil_div(r1 - r0, kSkTile), tc = (int)ceil_div(c1 - c0, kSkTile);
    // a square upper triangle (the all-pairs call) launches only tiles on or
    // above the diagonal instead of exiting the lower half's workgroups
    const bool tri = upper && r0 == c0 && r1 == c1;
    const int64_t grid = tri ? (int64_t)tc * (tc + 1) / 2 : (int64_t)tr * tc;
    const int threads = kSkTile * kSkTile;
    const int64_t per = (int64_t(1) << 31) / threads;     // a dispatch holds < 2^32 work-items
    auto kern = &sketch_ring_kernel;
    GD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds));
    int launches = 0;
    for (int64_t t0 = 0; t0 < grid; t0 += per, launches++)
        kern<<<(unsigned)std::min(per, grid - t0), threads, lds, st>>>(
            sk->codes.as<int32_t>(), sk->off.as<int64_t>(), width, rs, kmax, r0, r1, c0, c1, t0, tc, upper, jac, en,
            d_common, d_D, ld, fallback ? 1 : 0, tri ? 1 : 0, sperm ? 1 : 0);
    GD_HIP(hipGetLastError());
    return launches;
}

// launches made (0: the tile does not fit LDS and no global fallback was asked)
template <int R, int C>
int launch_sketch_tiles(hipStream_t st, const gdist_sets* sk, int width, int64_t r0, int64_t r1, int64_t c0,
                         int64_t c1, bool upper, int jac, int en, int32_t* d_common, double* d_D, int64_t ld,
                         bool force_global, int64_t kw_opt, bool v2_opt) {
    // option sketch_k selects the merge window (1, 2, 4, 6; A/B measurements)
    const int kw = (int)kw_opt;
    const bool v2 = kw == 2 && v2_opt;
    const int sw = v2 ? ((width + 2) | 1) : sketch_stride(width);
    const size_t lds = (size_t)(R + C) * sw * 4 + LDS_SK_SLACK;
    const bool use_lds = !force_global && lds + sketch_meta_bytes<R, C>() <= (size_t)LDS_SK_MAX;
    if (!use_lds && !force_global) return 0;
    const int tr = (int)ceil_div(r1 - r0, R), tc = (int)ceil_div(c1 - c0, C);
    const int64_t grid = (int64_t)tr * tc;
    const int launches = (int)ceil_div(grid, (int64_t(1) << 31) / (R * C));
    // a dispatch holds < 2^32 work-items: launches of at most 2^31 threads
    const int threads = R * C;
    const int64_t per = (int64_t(1) << 31) / threads;

    const int32_t* sig = sk->codes.as<int32_t>();
    const int64_t* off = sk->off.as<int64_t>();
    if (!use_lds) {
        for (int64_t t0 = 0; t0 < grid; t0 += per)
            sketch_tile_kernel<R, C, false, 1><<<(unsigned)std::min(per, grid - t0), R * C, 0, st>>>(
                sig, off, width, sw, r0, r1, c0, c1, t0, tc, upper, jac, en, d_common, d_D, ld);
    } else {
        auto go = [&](auto kern) {
            GD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       LDS_SK_MAX - (int)sketch_meta_bytes<R, C>()));
            for (int64_t t0 = 0; t0 < grid; t0 += per)
                kern<<<(unsigned)std::min(per, grid - t0), threads, lds, st>>>(sig, off, width, sw, r0, r1, c0, c1, t0, tc,
                                                                            upper, jac, en, d_common, d_D, ld);
        };
        switch (kw) {
            case 1: go(&sketch_tile_kernel<R, C, true, 1>); break;
            case 4:
                go(&sketch_tile_kernel<R, C, true, 4>);
                break;
            case 6: go(&sketch_tile_kernel<R, C, true, 6>); break;
            default:
                if (v2) go(&sketch_tile_kernel<R, C, true, 2, true>);
                else go(&sketch_tile_kernel<R, C, true, 2>);
                break;
        }
    }
    GD_HIP(hipGetLastError());
    return launches;
}

}  // namespace

void sketch_build(gdist_ctx* ctx, const gdist_sets* s, int width, gdist_sets* out) {
    hipStream_t st = ctx->stream;
    GD_REQUIRE(width > 0, "sketch width must be positive");
    GD_REQUIRE(s->kind == GDIST_DNA || s->kind == GDIST_PROT, "sketches are built from kmer sets");
    const int k = s->k;
    const unsigned am = s->flags & GDIST_AMBIG_MASK;
    int bits, dna_mode = 0;
    if (s->kind == GDIST_DNA) {
        const bool keep = am == GDIST_AMBIG_KEEP;
        bits = keep ? 3 : 2;
        dna_mode = keep ? 3 : 2;
    } else {
        bits = k <= 8 ? 8 : 5;
    }
    const int64_t nsets = s->nsets;
    std::vector<int64_t> h_out(nsets + 1, 0);
    std::vector<DevBuf> parts;
    std::vector<int64_t> part_n;
    DevBuf d_out_off((nsets + 1) * 8, st);
    const int64_t kChunk = int64_t(1) << 29;
    // chunks of whole sets of at most kChunk codes (or one larger set); the
    // work buffers are sized once for the largest chunk and reused
    std::vector<std::pair<int64_t, int64_t>> chunks;
    int64_t nmax = 0, nsmax = 0;
    for (int64_t a = 0; a < nsets;) {
        int64_t b = a + 1;
        while (b < nsets && s->h_off[b + 1] - s->h_off[a] <= kChunk) b++;
        chunks.push_back({a, b});
        nmax = std::max(nmax, s->h_off[b] - s->h_off[a]);
        nsmax = std::max(nsmax, b - a);
        a = b;
    }
    DevBuf kA(nmax * 8 + 8, st), kB(nmax * 8 + 8, st), flag(nmax * 4 + 4, st), pos(nmax * 8 + 8, st),
        us((nsmax + 1) * 8, st);
    for (const auto& ch : chunks) {
        const int64_t s0 = ch.first, s1 = ch.second;
        const int64_t ns = s1 - s0;
        const int64_t n = s->h_off[s1] - s->h_off[s0];
        if (n) {
            hash_keys_kernel<<<grid_for(n), 256, 0, st>>>(s->codes.as<uint64_t>(), s->off.as<int64_t>(), s0, ns, k,
                                                         bits, dna_mode, kA.as<uint64_t>());
            GD_HIP(hipGetLastError());
        }
        uint64_t* keys = kA.as<uint64_t>(); uint64_t* alt = kB.as<uint64_t>();
        int idbits = 1;
        while ((int64_t(1) << idbits) <= ns) idbits++;
        sort_keys_u64(ctx, keys, alt, (size_t)n, 0, 32 + idbits);
        if (n) {
            head_flags_kernel<<<grid_for(n), 256, 0, st>>>(keys, n, flag.as<int32_t>());
            GD_HIP(hipGetLastError());
            exclusive_scan_i32_to_i64(ctx, flag.as<int32_t>(), pos.as<int64_t>(), (size_t)n);
        }
        set_starts_kernel<<<(int)ceil_div(ns + 1, 256), 256, 0, st>>>(keys, pos.as<int64_t>(), flag.as<int32_t>(), n,
                                                                       ns, us.as<int64_t>());
        GD_HIP(hipGetLastError());
        std::vector<int64_t> hus(ns + 1);
        d2h(hus.data(), us.p, (ns + 1) * 8, st);
        GD_HIP(hipStreamSynchronize(st));
        std::vector<int64_t> loc(ns + 1, 0);
        for (int64_t t = 0; t < ns; t++) {
            const int64_t cnt = std::min<int64_t>(width, hus[t + 1] - hus[t]);
            loc[t + 1] = loc[t] + cnt;
            h_out[s0 + t + 1] = h_out[s0 + t] + cnt;
        }
        DevBuf dloc((ns + 1) * 8, st), sig(loc[ns] * 4 + 4, st);
        h2d(dloc.p, loc.data(), (ns + 1) * 8, st);
        if (n) {
            emit_sig_kernel<<<grid_for(n), 256, 0, st>>>(keys, flag.as<int32_t>(), pos.as<int64_t>(), us.as<int64_t>(),
                                                         dloc.as<int64_t>(), n, width, sig.as<int32_t>());
            GD_HIP(hipGetLastError());
        }
        parts.push_back(std::move(sig));
        part_n.push_back(loc[ns]);
    }
    out->kind = GDIST_SKETCH;
    out->k = s->k;
    out->flags = s->flags;
    out->width = width;
    out->nsets = nsets;
    out->total = h_out[nsets];
    out->h_off = h_out;
    h2d(d_out_off.p, h_out.data(), (nsets + 1) * 8, st);
    out->off = std::move(d_out_off);
    out->codes.alloc(out->total * 4 + 4, st);
    int64_t at = 0;
    for (size_t p = 0; p < parts.size(); p++) {
        if (part_n[p])
            GD_HIP(hipMemcpyAsync(out->codes.as<int32_t>() + at, parts[p].p, part_n[p] * 4, hipMemcpyDeviceToDevice,
                                  st));
        at += part_n[p];
    }
    GD_HIP(hipStreamSynchronize(st));
}

void sketch_matrix(gdist_ctx* ctx, const gdist_sets* sk, int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                   unsigned flags, int32_t* d_common, double* d_D, int64_t ld) {
    hipStream_t st = ctx->stream;
    if (r1 - r0 <= 0 || c1 - c0 <= 0) return;
    const bool upper = (flags & GDIST_UPPER_TRIANGLE) != 0;
    const int jac = (flags & GDIST_SKETCH_JACCARD) ? 1 : 0, en = (flags & GDIST_EMPTY_NAN) ? 1 : 0;
    const int width = std::max(1, sk->width);
    // option sketch_tile = 16 forces the 16x16 tile (A/B measurements)
    const bool only16 = ctx->option(OPT_SKETCH_TILE, 0) == 16;
    const int64_t kw = ctx->option(OPT_SKETCH_K, 2);
    const bool v2 = ctx->option(OPT_SKETCH_V2, 1) != 0;
    // option sketch_phase = 0 keeps whole sketches in LDS (the V2 / window
    // kernels); sketch_cap sets the ring kernel's steps per phase and
    // sketch_ring its slots per sketch
    const bool ring = ctx->option(OPT_SKETCH_PHASE, 1) != 0 && !only16 && kw == 2;
    GD_HIP(hipEventRecord(ctx->ev_k0, st));
    int launches = 0;
    if (ring) {
        // default 160 steps per phase, 256 slots: 257 rows of 256 B = 66 KB,
        // two workgroups per CU
        const int kmax = (int)std::max<int64_t>(2, std::min<int64_t>(ctx->option(OPT_SKETCH_CAP, 160), 1 << 20));
        const int rs = (int)std::max<int64_t>(16, std::min<int64_t>(ctx->option(OPT_SKETCH_RING, 256), 1 << 20));
        launches = launch_sketch_ring(st, sk, width, rs, std::min(kmax, rs - 1), r0, r1, c0, c1, upper, jac, en,
                                      d_common, d_D, ld, ctx->option(OPT_SKETCH_WAIT, 0) == 0,
                                      ctx->option(OPT_SKETCH_PERM, 1) != 0);
    } else {
        if (!only16)
            launches = launch_sketch_tiles<16, 24>(st, sk, width, r0, r1, c0, c1, upper, jac, en, d_common, d_D, ld,
                                                   false, kw, v2);
        if (!launches)
            launches = launch_sketch_tiles<16, 16>(st, sk, width, r0, r1, c0, c1, upper, jac, en, d_common, d_D, ld,
                                                   false, kw, v2);
        if (!launches)
            launches = launch_sketch_tiles<16, 16>(st, sk, width, r0, r1, c0, c1, upper, jac, en, d_common, d_D, ld,
                                                   true, kw, v2);
    }
    GD_HIP(hipEventRecord(ctx->ev_k1, st));
    ctx->last.launches = launches;
}

}  // namespace gdist
