// reps.hip — greedy representative selection on the device.
//
// Pass 1 (DistanceRepsProcessor.java:185-200, FastaDistanceRepsProcessor.java:
// 117-144): sets in index order; set k becomes a representative unless an
// earlier representative r has d(k, r) <= max_dist. Blocked: for rows
// [b0, b1) the distances to every earlier set are computed at once (the
// matrix kernels + the fp64 epilogue, so d is the reference's double);
// cover_kernel flags the rows an earlier block's representative already
// covers, and the host resolves the in-block order from the B x B tile.
//
// Pass 2 (DistanceRepsProcessor.java:227-237): for every set the closest
// representative, reduce(NULL_RESULT, merge) with merge = "left wins ties",
// i.e. the minimum of (d, tie rank) over representatives with d < 1.0 (the
// NULL_RESULT identity, d = 1.0, wins ties at 1.0). Representatives map to
// themselves at 0.0. The tie rank is the caller's (the reference iterates a
// HashMap: gdist.processors derives Java's bucket order), index by default.
#include <algorithm>
#include <cstring>

#include "gdist_internal.hpp"

namespace gdist {
namespace {

// cov[k] = 1 if some r in [c0, c1) with is_rep[r] has D[k][r - c0] <= t (one wave per row)
__global__ __launch_bounds__(256) void cover_kernel(const double* __restrict__ D, int64_t ldD, int64_t nrows,
                                                    int64_t c0, int64_t c1, const int32_t* __restrict__ is_rep,
                                                    double t, int32_t* __restrict__ cov) {
    const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (k >= nrows) return;
    const double* row = D + k * ldD - c0;
    bool hit = false;
    for (int64_t r = c0 + lane; r < c1 && !hit; r += 64) hit = is_rep[r] && row[r] <= t;
    const unsigned long long any = __ballot(hit);
    if (lane == 0) cov[k] = any != 0ull;
}

// closest representative of each row: min (d, rank) over columns with
// is_rep and d < 1.0; -1 / 1.0 when none (one wave per row)
// (columns [c0, c1), D's column 0 is c0; best_rk: the winner's tie rank)
__global__ __launch_bounds__(256) void closest_rep_kernel(const double* __restrict__ D, int64_t ldD, int64_t nrows,
                                                          int64_t c0, int64_t c1, const int32_t* __restrict__ is_rep,
                                                          const int64_t* __restrict__ rank, int64_t* __restrict__ best,
                                                          double* __restrict__ best_d, int64_t* __restrict__ best_rk) {
    const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (k >= nrows) return;
    const double* row = D + k * ldD - c0;
    double bd = 1.0;
    int64_t br = INT64_MAX, bi = -1;
    for (int64_t c = c0 + lane; c < c1; c += 64) {
        if (!is_rep[c]) continue;
        const double d = row[c];
        const int64_t rk = rank ? rank[c] : c;
        if (d < bd || (d == bd && d < 1.0 && rk < br)) { bd = d; br = rk; bi = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double od = __shfl_xor(bd, o, 64);
        const int64_t orr = __shfl_xor(br, o, 64), oi = __shfl_xor(bi, o, 64);
        if (od < bd || (od == bd && orr < br)) { bd = od; br = orr; bi = oi; }
    }
    if (lane == 0) {
        best[k] = bi;
        best_d[k] = bi < 0 ? 1.0 : bd;
        if (best_rk) best_rk[k] = bi < 0 ? INT64_MAX : br;
    }
}

// distances of rows [b0, b1) x columns [c0, c1) into D (device, ld = ldD)
void distance_rows(gdist_ctx* ctx, gdist_sets* s, int method, int64_t b0, int64_t b1, int64_t c0, int64_t c1,
                   int32_t* dI, double* dD, int64_t ldD) {
    if (c1 <= c0 || b1 <= b0) return;
    if (method == GDIST_METHOD_BITSET) {
        zero_counts(ctx, b0, b1, c0, c1, false, dI, ldD);
        bitset_matrix(ctx, s, b0, b1, c0, c1, false, dI, ldD);
    } else {
        sorted_matrix(ctx, s, b0, b1, c0, c1, false, dI, ldD);
    }
    distance_epilogue(ctx, s, b0, b1, c0, c1, false, 0, dI, ldD, dD, ldD);
}

}  // namespace

// A gathered collection on R ranks: the columns are sharded.
// Every rank computes a block's distances to its 1/R of the columns (pass 1:
// of the earlier sets; pass 2: of all sets); the cover flags (any: OR) and
// the closest representatives (min (d, tie rank)) of the block's rows are
// combined through one all-gather per block, so every rank takes the same
// decisions. The in-block tile (B x B) is computed on every rank.
void greedy_reps(gdist_ctx* ctx, gdist_sets* s, int method, double t, const int64_t* tie_rank, int32_t* is_rep,
                 int64_t* rep_of, double* rep_dist, int64_t* nreps) {
    hipStream_t st = ctx->stream;
    const int64_t n = s->nsets;
    std::fill(is_rep, is_rep + n, 0);
    if (nreps) *nreps = 0;
    if (n == 0) return;
    const bool split = s->replicated && comm_active(ctx) && ctx->option(OPT_REPS_SPLIT, 1) != 0;
    const int R = split ? ctx->nranks : 1, me = split ? ctx->rank : 0;
    // row block: B x N counts + distances within ~1.5 GiB, a multiple of 128 rows
    int64_t B = std::max<int64_t>(128, std::min<int64_t>(4096, ((int64_t(1) << 27) / n) / 128 * 128));
    B = std::min<int64_t>(B, ceil_div(n, 128) * 128);
    if (ctx->has_option(OPT_REPS_BLOCK)) B = std::max<int64_t>(1, ctx->option(OPT_REPS_BLOCK, B));   // tests: several blocks
    DevBuf dI((size_t)B * n * 4 + 4, st), dD((size_t)B * n * 8 + 8, st), drep(n * 4 + 4, st), dcov(B * 4 + 4, st);
    GD_HIP(hipMemsetAsync(drep.p, 0, n * 4, st));
    std::vector<int32_t> cov(B);
    std::vector<double> tile((size_t)B * B);
    DevBuf gcov(split ? (size_t)R * B * 4 + 4 : 4, st);
    std::vector<int32_t> hcov(split ? (size_t)R * B : 1);
    int64_t count = 0;
    for (int64_t b0 = 0; b0 < n; b0 += B) {
        const int64_t b1 = std::min(n, b0 + B), nb = b1 - b0;
        std::fill(cov.begin(), cov.begin() + nb, 0);
        if (!split) {
            distance_rows(ctx, s, method, b0, b1, 0, b1, dI.as<int32_t>(), dD.as<double>(), b1);
            if (b0 > 0) {
                cover_kernel<<<(unsigned)ceil_div(nb, 4), 256, 0, st>>>(dD.as<double>(), b1, nb, 0, b0,
                                                                        drep.as<int32_t>(), t, dcov.as<int32_t>());
                GD_HIP(hipGetLastError());
                d2h(cov.data(), dcov.p, nb * 4, st);
            }
            // the in-block tile D[b0..b1) x [b0..b1)
            GD_HIP(hipStreamSynchronize(st));
            GD_HIP(hipMemcpy2DAsync(tile.data(), nb * 8, dD.as<double>() + b0, b1 * 8, nb * 8, nb,
                                    hipMemcpyDeviceToHost, st));
            GD_HIP(hipStreamSynchronize(st));
        } else {
            distance_rows(ctx, s, method, b0, b1, b0, b1, dI.as<int32_t>(), dD.as<double>(), nb);
            GD_HIP(hipStreamSynchronize(st));
            d2h(tile.data(), dD.p, (size_t)nb * nb * 8, st);
            // this rank's share of the earlier columns, then OR over ranks
            const int64_t lo = b0 * me / R, hi = b0 * (me + 1) / R;
            GD_HIP(hipMemsetAsync(dcov.p, 0, B * 4, st));
            if (hi > lo) {
                distance_rows(ctx, s, method, b0, b1, lo, hi, dI.as<int32_t>(), dD.as<double>(), hi - lo);
                cover_kernel<<<(unsigned)ceil_div(nb, 4), 256, 0, st>>>(dD.as<double>(), hi - lo, nb, lo, hi,
                                                                        drep.as<int32_t>(), t, dcov.as<int32_t>());
                GD_HIP(hipGetLastError());
            }
            if (b0 > 0) {
                comm_allgather(ctx, dcov.p, gcov.p, (size_t)B * 4);
                d2h(hcov.data(), gcov.p, (size_t)R * B * 4, st);
                for (int r = 0; r < R; r++)
                    for (int64_t k = 0; k < nb; k++) cov[k] |= hcov[(size_t)r * B + k];
            }
        }
        for (int64_t k = 0; k < nb; k++) {
            bool covered = cov[k] != 0;
            for (int64_t j = 0; j < k && !covered; j++)
                covered = is_rep[b0 + j] && tile[(size_t)k * nb + j] <= t;
            if (!covered) { is_rep[b0 + k] = 1; count++; }
        }
        h2d(drep.as<int32_t>() + b0, is_rep + b0, nb * 4, st);
    }
    if (nreps) *nreps = count;
    if (!rep_of && !rep_dist) return;
    DevBuf drank, dbest(B * 8 + 8, st), dbd(B * 8 + 8, st), dbr(B * 8 + 8, st);
    if (tie_rank) {
        drank.alloc(n * 8, st);
        h2d(drank.p, tie_rank, n * 8, st);
    }
    // pass 2: columns [lo, hi) of this rank (all of them on one rank)
    const int64_t lo = n * me / R, hi = n * (me + 1) / R;
    DevBuf pack(split ? (size_t)B * 24 + 8 : 8, st), gpack(split ? (size_t)R * (B * 24 + 8) : 8, st);
    std::vector<char> hpack(split ? (size_t)R * (B * 24 + 8) : 1);
    std::vector<int64_t> hb(B), hr(B);
    std::vector<double> hd(B);
    for (int64_t b0 = 0; b0 < n; b0 += B) {
        const int64_t b1 = std::min(n, b0 + B), nb = b1 - b0;
        if (hi > lo) {
            distance_rows(ctx, s, method, b0, b1, lo, hi, dI.as<int32_t>(), dD.as<double>(), hi - lo);
            closest_rep_kernel<<<(unsigned)ceil_div(nb, 4), 256, 0, st>>>(
                dD.as<double>(), hi - lo, nb, lo, hi, drep.as<int32_t>(), tie_rank ? drank.as<int64_t>() : nullptr,
                dbest.as<int64_t>(), dbd.as<double>(), dbr.as<int64_t>());
            GD_HIP(hipGetLastError());
        } else {
            std::vector<int64_t> none(nb, -1), inf(nb, INT64_MAX);
            std::vector<double> one(nb, 1.0);
            h2d(dbest.p, none.data(), nb * 8, st);
            h2d(dbd.p, one.data(), nb * 8, st);
            h2d(dbr.p, inf.data(), nb * 8, st);
        }
        if (!split) {
            d2h(hb.data(), dbest.p, nb * 8, st);
            d2h(hd.data(), dbd.p, nb * 8, st);
        } else {
            // every rank's (index, d, tie rank) of the block's rows; the
            // least d wins, equal d < 1.0 the lower tie rank (the kernel's rule)
            const size_t per = (size_t)B * 24 + 8;
            GD_HIP(hipMemcpyAsync(pack.p, dbest.p, B * 8, hipMemcpyDeviceToDevice, st));
            GD_HIP(hipMemcpyAsync(static_cast<char*>(pack.p) + B * 8, dbd.p, B * 8, hipMemcpyDeviceToDevice, st));
            GD_HIP(hipMemcpyAsync(static_cast<char*>(pack.p) + B * 16, dbr.p, B * 8, hipMemcpyDeviceToDevice, st));
            comm_allgather(ctx, pack.p, gpack.p, per);
            d2h(hpack.data(), gpack.p, per * R, st);
            for (int64_t k = 0; k < nb; k++) {
                int64_t bi = -1, br = INT64_MAX;
                double bd = 1.0;
                for (int r = 0; r < R; r++) {
                    const char* base = hpack.data() + per * r;
                    int64_t ci, crk;
                    double cd;
                    memcpy(&ci, base + k * 8, 8);
                    memcpy(&cd, base + B * 8 + k * 8, 8);
                    memcpy(&crk, base + B * 16 + k * 8, 8);
                    if (ci < 0) continue;
                    if (cd < bd || (cd == bd && cd < 1.0 && crk < br)) { bd = cd; br = crk; bi = ci; }
                }
                hb[k] = bi;
                hd[k] = bi < 0 ? 1.0 : bd;
            }
        }
        GD_HIP(hipStreamSynchronize(st));
        for (int64_t k = 0; k < nb; k++) {
            const int64_t g = b0 + k;
            const bool self = is_rep[g] != 0;
            if (rep_of) rep_of[g] = self ? g : hb[k];
            if (rep_dist) rep_dist[g] = self ? 0.0 : hd[k];
        }
    }
}

}  // namespace gdist
