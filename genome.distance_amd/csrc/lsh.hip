// lsh.hip — LSH bucket query over MinHash sketches: getClosest(kmers, n, maxDist)
// of the reference's LSHMemSeqHash / LSHDiskSeqHash (MashProcessor.java:110,130,150,
// FindProcessor.java:110).
//
// The LSH classes live in the un-vendored org.theseed:sequence module, so the
// hashing is restated (parity unpinned): an index of `stages`
// independent MinHash functions over each set's bottom-s signature. Stage t
// keys a sketch by min over its signature values x of mix(x ^ salt_t)
// (splitmix64 finaliser; salt_t = splitmix64 stream of the index seed), and
// files it in bucket key mod `buckets` of that stage. Two sketches meet in a
// stage with probability = the Jaccard index of their signatures, so close
// genomes share buckets. getClosest: every set sharing a bucket with the
// query in any stage is a candidate; candidates at sketch distance <= maxDist
// (Mash bottom-s of the union, as gdist_sketch_matrix) are returned nearest
// first (ties by index), at most n.
//
// Device work: keys of every (set, stage) (a workgroup per set, one min
// reduction per stage), the bucket CSR (radix sort of (stage, bucket) keys),
// per query the candidate (query, set) keys gathered from its buckets and
// made unique by one radix sort, then one lane per candidate pair merges the
// two signatures from HBM.
#include <algorithm>
#include <cmath>

#include "gdist_internal.hpp"


namespace gdist {
namespace {

constexpr int kMaxStages = 64;

__host__ __device__ inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

inline int grid_for(int64_t n, int block = 256, int64_t cap = 256 * 32) {
    int64_t g = ceil_div(n, block);
    return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

// bucket[set * S + t] = (min over the signature of mix(x ^ salt_t)) mod B
__global__ __launch_bounds__(256) void lsh_keys_kernel(const int32_t* __restrict__ sig, const int64_t* __restrict__ off,
                                                       int64_t nsets, int S, int B, const uint64_t* __restrict__ salts,
                                                       int32_t* __restrict__ bucket) {
    __shared__ unsigned long long red[256 / 64];
    const int64_t set = blockIdx.x;
    if (set >= nsets) return;
    const int64_t b0 = off[set], b1 = off[set + 1];
    for (int t = 0; t < S; t++) {
        const uint64_t salt = salts[t];
        unsigned long long m = ~0ull;
        for (int64_t e = b0 + threadIdx.x; e < b1; e += 256) {
            const unsigned long long h = mix64((uint64_t)(uint32_t)sig[e] ^ salt);
            m = h < m ? h : m;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long v = __shfl_xor(m, o, 64);
            m = v < m ? v : m;
        }
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long r = red[0];
            for (int w = 1; w < 256 / 64; w++) r = red[w] < r ? red[w] : r;
            bucket[set * S + t] = (int32_t)(r % (unsigned long long)B);
        }
        __syncthreads();
    }
}

__global__ void lsh_entry_keys_kernel(const int32_t* __restrict__ bucket, int64_t nsets, int S, int B,
                                      uint64_t* __restrict__ key, int32_t* __restrict__ val,
                                      int32_t* __restrict__ count) {
    const int64_t n = nsets * S;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
        const int64_t set = e / S, t = e - set * S;
        const int64_t k = t * B + bucket[e];
        key[e] = (uint64_t)k;
        val[e] = (int32_t)set;
        atomicAdd(count + k, 1);
    }
}

// candidates of each query: every member of its buckets (duplicates included)
__global__ void lsh_cand_count_kernel(const int32_t* __restrict__ qbucket, int64_t nq, int S, int B,
                                      const int64_t* __restrict__ boff, int64_t* __restrict__ cnt) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += stride) {
        int64_t c = 0;
        for (int t = 0; t < S; t++) {
            const int64_t k = (int64_t)t * B + qbucket[q * S + t];
            c += boff[k + 1] - boff[k];
        }
        cnt[q] = c;
    }
}

__global__ __launch_bounds__(256) void lsh_gather_kernel(const int32_t* __restrict__ qbucket, int64_t nq, int S, int B,
                                                         const int64_t* __restrict__ boff,
                                                         const int32_t* __restrict__ members,
                                                         const int64_t* __restrict__ qpos, uint64_t* __restrict__ out) {
    const int64_t q = blockIdx.x;
    if (q >= nq) return;
    int64_t at = qpos[q];
    for (int t = 0; t < S; t++) {
        const int64_t k = (int64_t)t * B + qbucket[q * S + t];
        const int64_t m0 = boff[k], m1 = boff[k + 1];
        for (int64_t e = m0 + threadIdx.x; e < m1; e += 256) out[at + (e - m0)] = ((uint64_t)q << 32) | (uint32_t)members[e];
        at += m1 - m0;
    }
}

__global__ void head_flags_kernel(const uint64_t* __restrict__ k, int64_t n, int32_t* __restrict__ flag) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        flag[i] = (i == 0 || k[i] != k[i - 1]) ? 1 : 0;
}

__global__ void compact_heads_kernel(const uint64_t* __restrict__ k, const int32_t* __restrict__ flag,
                                     const int64_t* __restrict__ pos, int64_t n, uint64_t* __restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        if (flag[i]) out[pos[i]] = k[i];
}

// Mash bottom-s of the union (gdist_sketch_matrix's distance, default flags)
__global__ void lsh_pair_distance_kernel(const uint64_t* __restrict__ pairs, int64_t n,
                                         const int32_t* __restrict__ qsig, const int64_t* __restrict__ qoff,
                                         const int32_t* __restrict__ ssig, const int64_t* __restrict__ soff,
                                         int width, double* __restrict__ dist) {
#pragma clang fp contract(off)
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += stride) {
        const int64_t q = (int64_t)(pairs[p] >> 32), c = (int64_t)(pairs[p] & 0xFFFFFFFFull);
        const int32_t* a = qsig + qoff[q];
        const int32_t* b = ssig + soff[c];
        const int64_t na = qoff[q + 1] - qoff[q], nb = soff[c + 1] - soff[c];
        int64_t i = 0, j = 0, common = 0, taken = 0;
        while (taken < width && (i < na || j < nb)) {
            if (j >= nb || (i < na && a[i] < b[j])) i++;
            else if (i >= na || b[j] < a[i]) j++;
            else { common++; i++; j++; }
            taken++;
        }
        dist[p] = common > 0 ? 1.0 - (double)common / (double)taken : 1.0;
    }
}

}  // namespace
}  // namespace gdist

using namespace gdist;

static void lsh_keys(gdist_ctx* ctx, const gdist_sets* sk, int S, int B, const uint64_t* salts, DevBuf& out) {
    hipStream_t st = ctx->stream;
    out.alloc((size_t)sk->nsets * S * 4 + 4, st);
    if (sk->nsets == 0) return;
    GD_REQUIRE(sk->nsets < (int64_t(1) << 31), "too many sketches for one launch");
    lsh_keys_kernel<<<(unsigned)sk->nsets, 256, 0, st>>>(sk->codes.as<int32_t>(), sk->off.as<int64_t>(), sk->nsets, S,
                                                         B, salts, out.as<int32_t>());
    GD_HIP(hipGetLastError());
}

namespace gdist {
void lsh_build(gdist_ctx* ctx, const gdist_sets* sk, int stages, int buckets, uint64_t seed, gdist_lsh* L) {
    GD_REQUIRE(sk->kind == GDIST_SKETCH, "the LSH index is built over sketches (gdist_sketch_build)");
    GD_REQUIRE(stages >= 1 && stages <= kMaxStages, "stages must be 1..64");
    GD_REQUIRE(buckets >= 1, "buckets must be >= 1");
    GD_REQUIRE(sk->nsets < (int64_t(1) << 31), "too many sketches");
    hipStream_t st = ctx->stream;
    L->ctx = ctx; L->sk = sk; L->stages = stages; L->buckets = buckets; L->seed = seed;
    std::vector<uint64_t> salts(stages);
    for (int t = 0; t < stages; t++) salts[t] = mix64(seed + 0x9E3779B97F4A7C15ull * (uint64_t)(t + 1));
    L->salts.alloc(stages * 8, st);
    h2d(L->salts.p, salts.data(), stages * 8, st);
    DevBuf bucket;
    lsh_keys(ctx, sk, stages, buckets, L->salts.as<uint64_t>(), bucket);
    const int64_t n = sk->nsets * stages, nk = (int64_t)stages * buckets;
    DevBuf kA(n * 8 + 8, st), kB(n * 8 + 8, st), vA(n * 4 + 4, st), vB(n * 4 + 4, st), cnt(nk * 4 + 4, st);
    GD_HIP(hipMemsetAsync(cnt.p, 0, nk * 4 + 4, st));
    if (n) {
        lsh_entry_keys_kernel<<<grid_for(n), 256, 0, st>>>(bucket.as<int32_t>(), sk->nsets, stages, buckets,
                                                           kA.as<uint64_t>(), vA.as<int32_t>(), cnt.as<int32_t>());
        GD_HIP(hipGetLastError());
    }
    uint64_t* k = kA.as<uint64_t>(); uint64_t* ka = kB.as<uint64_t>();
    int32_t* v = vA.as<int32_t>(); int32_t* va = vB.as<int32_t>();
    int bits = 1;
    while ((int64_t(1) << bits) <= nk) bits++;
    sort_pairs_u64_i32(ctx, k, ka, v, va, (size_t)n, 0, bits);   // stable: members ascend within a bucket
    L->off.alloc((nk + 1) * 8, st);
    exclusive_scan_i32_to_i64(ctx, cnt.as<int32_t>(), L->off.as<int64_t>(), (size_t)(nk + 1));
    L->members.alloc(n * 4 + 4, st);
    if (n) GD_HIP(hipMemcpyAsync(L->members.p, v, n * 4, hipMemcpyDeviceToDevice, st));
    GD_HIP(hipStreamSynchronize(st));
}

void lsh_closest(gdist_ctx* ctx, const gdist_lsh* L, const gdist_sets* qs, int nbest, double max_dist,
                 int64_t* idx_out, double* d_out, int32_t* count_out) {
    GD_REQUIRE(qs->kind == GDIST_SKETCH, "queries are sketches (gdist_sketch_build)");
    GD_REQUIRE(nbest >= 0, "n must be >= 0");
    hipStream_t st = ctx->stream;
    const int64_t nq = qs->nsets;
    GD_REQUIRE(nq < (int64_t(1) << 31), "too many queries");
    std::fill(count_out, count_out + nq, 0);
    if (nq == 0 || nbest == 0 || L->sk->nsets == 0) return;
    DevBuf qb;
    lsh_keys(ctx, qs, L->stages, L->buckets, L->salts.as<uint64_t>(), qb);
    DevBuf qc(nq * 8, st), qpos(nq * 8 + 8, st);
    lsh_cand_count_kernel<<<grid_for(nq), 256, 0, st>>>(qb.as<int32_t>(), nq, L->stages, L->buckets,
                                                       L->off.as<int64_t>(), qc.as<int64_t>());
    GD_HIP(hipGetLastError());
    exclusive_scan_i64(ctx, qc.as<int64_t>(), qpos.as<int64_t>(), (size_t)nq);
    int64_t last = 0, lc = 0;
    d2h(&last, qpos.as<int64_t>() + nq - 1, 8, st);
    d2h(&lc, qc.as<int64_t>() + nq - 1, 8, st);
    const int64_t total = last + lc;
    if (total == 0) return;
    DevBuf cA(total * 8, st), cB(total * 8, st);
    lsh_gather_kernel<<<(unsigned)nq, 256, 0, st>>>(qb.as<int32_t>(), nq, L->stages, L->buckets,
                                                    L->off.as<int64_t>(), L->members.as<int32_t>(),
                                                    qpos.as<int64_t>(), cA.as<uint64_t>());
    GD_HIP(hipGetLastError());
    uint64_t* k = cA.as<uint64_t>(); uint64_t* ka = cB.as<uint64_t>();
    int qbits = 1;
    while ((int64_t(1) << qbits) <= nq) qbits++;
    sort_keys_u64(ctx, k, ka, (size_t)total, 0, 32 + qbits);
    DevBuf flag(total * 4, st), pos(total * 8, st);
    head_flags_kernel<<<grid_for(total), 256, 0, st>>>(k, total, flag.as<int32_t>());
    GD_HIP(hipGetLastError());
    exclusive_scan_i32_to_i64(ctx, flag.as<int32_t>(), pos.as<int64_t>(), (size_t)total);
    int64_t lp = 0;
    int32_t lf = 0;
    d2h(&lp, pos.as<int64_t>() + total - 1, 8, st);
    d2h(&lf, flag.as<int32_t>() + total - 1, 4, st);
    const int64_t nu = lp + lf;
    DevBuf up(nu * 8, st), dd(nu * 8, st);
    compact_heads_kernel<<<grid_for(total), 256, 0, st>>>(k, flag.as<int32_t>(), pos.as<int64_t>(), total,
                                                          up.as<uint64_t>());
    lsh_pair_distance_kernel<<<grid_for(nu), 256, 0, st>>>(up.as<uint64_t>(), nu, qs->codes.as<int32_t>(),
                                                           qs->off.as<int64_t>(), L->sk->codes.as<int32_t>(),
                                                           L->sk->off.as<int64_t>(), std::max(1, L->sk->width),
                                                           dd.as<double>());
    GD_HIP(hipGetLastError());
    std::vector<uint64_t> hp(nu);
    std::vector<double> hd(nu);
    d2h(hp.data(), up.p, nu * 8, st);
    d2h(hd.data(), dd.p, nu * 8, st);
    // per query (pairs are sorted by query): d <= max_dist, nearest first, ties by index
    std::vector<std::pair<double, int64_t>> best;
    for (int64_t a = 0; a < nu;) {
        const int64_t q = (int64_t)(hp[a] >> 32);
        int64_t b = a;
        best.clear();
        for (; b < nu && (int64_t)(hp[b] >> 32) == q; b++)
            if (hd[b] <= max_dist) best.emplace_back(hd[b], (int64_t)(hp[b] & 0xFFFFFFFFull));
        std::sort(best.begin(), best.end());
        const int m = (int)std::min<size_t>(best.size(), (size_t)nbest);
        for (int r = 0; r < m; r++) {
            idx_out[q * nbest + r] = best[r].second;
            d_out[q * nbest + r] = best[r].first;
        }
        count_out[q] = m;
        a = b;
    }
}
}  // namespace gdist
