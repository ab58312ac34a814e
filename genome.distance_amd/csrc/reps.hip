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

// cov[k] = 1 if some r < b0 with is_rep[r] has D[k][r] <= t (one wave per row)
__global__ __launch_bounds__(256) void cover_kernel(const double* __restrict__ D, int64_t ldD, int64_t nrows,
                                                    int64_t b0, const int32_t* __restrict__ is_rep, double t,
                                                    int32_t* __restrict__ cov) {
    const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (k >= nrows) return;
    const double* row = D + k * ldD;
    bool hit = false;
    for (int64_t r = lane; r < b0 && !hit; r += 64) hit = is_rep[r] && row[r] <= t;
    const unsigned long long any = __ballot(hit);
    if (lane == 0) cov[k] = any != 0ull;
}

// closest representative of each row: min (d, rank) over columns with
// is_rep and d < 1.0; -1 / 1.0 when none (one wave per row)
__global__ __launch_bounds__(256) void closest_rep_kernel(const double* __restrict__ D, int64_t ldD, int64_t nrows,
                                                          int64_t ncols, const int32_t* __restrict__ is_rep,
                                                          const int64_t* __restrict__ rank, int64_t* __restrict__ best,
                                                          double* __restrict__ best_d) {
    const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (k >= nrows) return;
    const double* row = D + k * ldD;
    double bd = 1.0;
    int64_t br = INT64_MAX, bi = -1;
    for (int64_t c = lane; c < ncols; c += 64) {
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
    }
}

// distances of rows [b0, b1) x columns [0, nc) into D (device, ld = ldD)
void distance_rows(gdist_ctx* ctx, gdist_sets* s, int method, int64_t b0, int64_t b1, int64_t nc, int32_t* dI,
                   double* dD, int64_t ldD) {
    if (method == GDIST_METHOD_BITSET) {
        zero_counts(ctx, b0, b1, 0, nc, false, dI, ldD);
        bitset_matrix(ctx, s, b0, b1, 0, nc, false, dI, ldD);
    } else {
        sorted_matrix(ctx, s, b0, b1, 0, nc, false, dI, ldD);
    }
    distance_epilogue(ctx, s, b0, b1, 0, nc, false, 0, dI, ldD, dD, ldD);
}

}  // namespace

void greedy_reps(gdist_ctx* ctx, gdist_sets* s, int method, double t, const int64_t* tie_rank, int32_t* is_rep,
                 int64_t* rep_of, double* rep_dist, int64_t* nreps) {
    hipStream_t st = ctx->stream;
    const int64_t n = s->nsets;
    std::fill(is_rep, is_rep + n, 0);
    if (nreps) *nreps = 0;
    if (n == 0) return;
    // row block: B x N counts + distances within ~1.5 GiB, a multiple of 128 rows
    int64_t B = std::max<int64_t>(128, std::min<int64_t>(4096, ((int64_t(1) << 27) / n) / 128 * 128));
    B = std::min<int64_t>(B, ceil_div(n, 128) * 128);
    if (ctx->has_option(OPT_REPS_BLOCK)) B = std::max<int64_t>(1, ctx->option(OPT_REPS_BLOCK, B));   // tests: several blocks
    DevBuf dI((size_t)B * n * 4 + 4, st), dD((size_t)B * n * 8 + 8, st), drep(n * 4 + 4, st), dcov(B * 4 + 4, st);
    GD_HIP(hipMemsetAsync(drep.p, 0, n * 4, st));
    std::vector<int32_t> cov(B);
    std::vector<double> tile((size_t)B * B);
    int64_t count = 0;
    for (int64_t b0 = 0; b0 < n; b0 += B) {
        const int64_t b1 = std::min(n, b0 + B), nb = b1 - b0;
        distance_rows(ctx, s, method, b0, b1, b1, dI.as<int32_t>(), dD.as<double>(), b1);
        if (b0 > 0) {
            cover_kernel<<<(unsigned)ceil_div(nb, 4), 256, 0, st>>>(dD.as<double>(), b1, nb, b0, drep.as<int32_t>(), t,
                                                                    dcov.as<int32_t>());
            GD_HIP(hipGetLastError());
            d2h(cov.data(), dcov.p, nb * 4, st);
        } else {
            std::fill(cov.begin(), cov.begin() + nb, 0);
        }
        // the in-block tile D[b0..b1) x [b0..b1)
        GD_HIP(hipStreamSynchronize(st));
        GD_HIP(hipMemcpy2DAsync(tile.data(), nb * 8, dD.as<double>() + b0, b1 * 8, nb * 8, nb, hipMemcpyDeviceToHost,
                                st));
        GD_HIP(hipStreamSynchronize(st));
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
    DevBuf drank, dbest(B * 8 + 8, st), dbd(B * 8 + 8, st);
    if (tie_rank) {
        drank.alloc(n * 8, st);
        h2d(drank.p, tie_rank, n * 8, st);
    }
    std::vector<int64_t> hb(B);
    std::vector<double> hd(B);
    for (int64_t b0 = 0; b0 < n; b0 += B) {
        const int64_t b1 = std::min(n, b0 + B), nb = b1 - b0;
        distance_rows(ctx, s, method, b0, b1, n, dI.as<int32_t>(), dD.as<double>(), n);
        closest_rep_kernel<<<(unsigned)ceil_div(nb, 4), 256, 0, st>>>(dD.as<double>(), n, nb, n, drep.as<int32_t>(),
                                                                       tie_rank ? drank.as<int64_t>() : nullptr,
                                                                       dbest.as<int64_t>(), dbd.as<double>());
        GD_HIP(hipGetLastError());
        d2h(hb.data(), dbest.p, nb * 8, st);
        d2h(hd.data(), dbd.p, nb * 8, st);
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
