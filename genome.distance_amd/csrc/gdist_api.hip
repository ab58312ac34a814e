// gdist_api.hip — the C-ABI of libgdist.so (declared in include/gdist.h).
//
// Thin host layer: argument checking with the reference's error behaviour
// (bad parameters -> GDIST_EINVAL, which the JNI shim maps to
// IllegalArgumentException, like ParseFailureException at
// FastaDistanceProcessor.java:98-102), context/stream management, H2D/D2H,
// dispatch to the device paths in pack/bitset/sorted/sketch.hip, and the
// RCCL communicator for row-sharded multi-GPU runs.
#include <cstring>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <thread>
#include <cmath>
#include <cstring>
#include <new>

#include "gdist_internal.hpp"

namespace gdist {

const char* const kOptNames[OPT_COUNT] = {
#define GDIST_OPT_NAME(id, name) name,
    GDIST_OPTIONS(GDIST_OPT_NAME)
#undef GDIST_OPT_NAME
};

static int option_index(const char* name) {
    GD_REQUIRE(name != nullptr, "null option name");
    for (int i = 0; i < OPT_COUNT; i++)
        if (strcmp(kOptNames[i], name) == 0) return i;
    throw Error(GDIST_EINVAL, std::string("unknown option: ") + name);
}

static thread_local std::string g_last_error;

void set_last_error(const std::string& msg) { g_last_error = msg; }

// ---------------------------------------------------------------------------
// caching device allocator (see DevBuf)
namespace {
constexpr int kMaxDevices = 64;
struct BlockCache {
    std::mutex mu;
    std::multimap<size_t, void*> free_blocks[kMaxDevices];
};
BlockCache& block_cache() {
    static BlockCache* c = new BlockCache();   // never destroyed: blocks outlive static teardown
    return *c;
}
// size classes: 256 B granules up to 1 MiB, then 8 classes per power of two
// (<= 12.5 % rounding)
size_t size_class(size_t n) {
    if (n <= (size_t(1) << 20)) return (n + 255) & ~size_t(255);
    size_t p = size_t(1) << (63 - __builtin_clzll((unsigned long long)n));
    const size_t step = p >> 3;
    return (n + step - 1) / step * step;
}
}  // namespace

// fresh device memory is slow to get (hipMalloc maps it: ~5 GB/s, C4's
// build spent seconds there), so a request takes a cached block of its class,
// else the smallest cached block of up to twice its class (the block keeps its
// own class and returns to that list), and only then a fresh one; out of
// memory, any larger cached block before the cache is trimmed
void* cache_alloc(int device, size_t bytes, size_t* cls_out) {
    GD_REQUIRE(device >= 0 && device < kMaxDevices, "device index out of range");
    const size_t cls = size_class(bytes);
    auto& c = block_cache();
    auto take = [&](size_t limit) -> void* {
        std::lock_guard<std::mutex> lk(c.mu);
        auto it = c.free_blocks[device].lower_bound(cls);
        if (it == c.free_blocks[device].end() || it->first > limit) return nullptr;
        void* p = it->second;
        *cls_out = it->first;
        c.free_blocks[device].erase(it);
        return p;
    };
    if (void* p = take(cls <= (size_t(1) << 20) ? cls : 2 * cls)) return p;
    *cls_out = cls;
    void* p = nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t e = hipMalloc(&p, cls);
    if (e == hipErrorOutOfMemory) {
        (void)hipGetLastError();
        if (void* q = take(~size_t(0))) return q;
        cache_trim(device);
        alloc_stats().trims++;
        e = hipMalloc(&p, cls);
    }
    GD_HIP(e);
    auto& st = alloc_stats();
    st.fresh++;
    st.fresh_bytes += cls;
    st.fresh_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return p;
}

AllocStats& alloc_stats() {
    static AllocStats s;
    return s;
}

void cache_free(int device, void* p, size_t cls) {
    auto& c = block_cache();
    std::lock_guard<std::mutex> lk(c.mu);
    c.free_blocks[device].emplace(cls, p);
}

void cache_trim(int device) {
    auto& c = block_cache();
    std::multimap<size_t, void*> blocks;
    {
        std::lock_guard<std::mutex> lk(c.mu);
        blocks.swap(c.free_blocks[device]);
    }
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(device);
    for (auto& b : blocks) (void)hipFree(b.second);
    (void)hipSetDevice(cur);
}

template <class F>
static int guard(F&& f) {
    try {
        f();
        return GDIST_OK;
    } catch (const Error& e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc&) {
        set_last_error("host allocation failed");
        return GDIST_ENOMEM;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return GDIST_EDEVICE;
    } catch (...) {
        set_last_error("unknown failure");
        return GDIST_EDEVICE;
    }
}

#define GD_NCCL(x)                                                                                    \
    do {                                                                                              \
        ncclResult_t r_ = (x);                                                                        \
        if (r_ != ncclSuccess) throw ::gdist::Error(GDIST_ECOMM, std::string(#x) + ": " + ncclGetErrorString(r_)); \
    } while (0)

static void use_device(gdist_ctx* ctx) {
    GD_REQUIRE(ctx != nullptr, "null context");
    GD_HIP(hipSetDevice(ctx->device));
}

static bool has_comm(const gdist_ctx* ctx) { return ctx->comm != nullptr || ctx->host_ag != nullptr; }

// The one collective the data path needs: every rank's `bytes` at d_send,
// gathered in rank order into d_recv (nranks * bytes), stream-ordered on
// ctx->stream. RCCL over xGMI, or staged through host memory and the
// caller's all-gather (gdist_comm_init_host).
static void allgather(gdist_ctx* ctx, const void* d_send, void* d_recv, size_t bytes) {
    hipStream_t st = ctx->stream;
    if (ctx->comm) {
        GD_NCCL(ncclAllGather(d_send, d_recv, bytes, ncclUint8, ctx->comm, st));
        return;
    }
    if (!ctx->host_ag) throw ::gdist::Error(GDIST_ECOMM, "communicator not initialised (gdist_comm_init)");
    std::vector<char> hs(bytes + 1), hr((size_t)ctx->nranks * bytes + 1);
    if (bytes) d2h(hs.data(), d_send, bytes, st);
    if (ctx->host_ag(hs.data(), hr.data(), (int64_t)bytes, ctx->host_user) != 0)
        throw ::gdist::Error(GDIST_ECOMM, "host all-gather callback failed");
    if (bytes) h2d(d_recv, hr.data(), (size_t)ctx->nranks * bytes, st);
}

// In place: this rank's `bytes` already sit at d_buf + rank * bytes.
static void allgather_inplace(gdist_ctx* ctx, void* d_buf, size_t bytes) {
    hipStream_t st = ctx->stream;
    char* mine = static_cast<char*>(d_buf) + bytes * ctx->rank;
    if (ctx->comm) {
        GD_NCCL(ncclAllGather(mine, d_buf, bytes, ncclUint8, ctx->comm, st));
        return;
    }
    if (!ctx->host_ag) throw ::gdist::Error(GDIST_ECOMM, "communicator not initialised (gdist_comm_init)");
    std::vector<char> hs(bytes + 1), hr((size_t)ctx->nranks * bytes + 1);
    if (bytes) d2h(hs.data(), mine, bytes, st);
    if (ctx->host_ag(hs.data(), hr.data(), (int64_t)bytes, ctx->host_user) != 0)
        throw ::gdist::Error(GDIST_ECOMM, "host all-gather callback failed");
    if (bytes) h2d(d_buf, hr.data(), (size_t)ctx->nranks * bytes, st);
}


static void check_sets(const gdist_sets* s) { GD_REQUIRE(s != nullptr && s->ctx != nullptr, "null sets handle"); }
// entry points that read the codes (or signatures) themselves
static void check_codes(const gdist_sets* s) {
    check_sets(s);
    GD_REQUIRE(s->has_codes, "the collection holds no codes (bitset-only, or consumed by an all-gather)");
}

// The call's kernel-time events: the next pair of the ring.
static void begin_timing(gdist_ctx* ctx) {
    const int slot = (int)(ctx->ring_n % gdist_ctx::kTimingRing);
    ctx->ev_k0 = ctx->ring0[slot];
    ctx->ev_k1 = ctx->ring1[slot];
}

// Reads the last call's times (waits for it).
static void settle_timing(gdist_ctx* ctx) {
    if (!ctx->pending) return;
    ctx->pending = false;
    GD_HIP(hipEventSynchronize(ctx->ev_call1));
    float ms = 0.f;
    GD_HIP(hipEventElapsedTime(&ms, ctx->ev_call0, ctx->ev_call1));
    ctx->last.call_ms = ms;
    ctx->last.kernel_ms = __builtin_nan("");
    if (ctx->last_kernel) {
        float km = 0.f;
        GD_HIP(hipEventElapsedTime(&km, ctx->ev_k0, ctx->ev_k1));
        ctx->last.kernel_ms = km;
    }
}

// async: the call's outputs are device buffers and it returns once its work
// is queued (gdist.h, GDIST_OUT_DEVICE); the times are read on demand
static void finish_timing(gdist_ctx* ctx, bool kernel_recorded, bool async = false) {
    GD_HIP(hipEventRecord(ctx->ev_call1, ctx->stream));
    ctx->last_kernel = kernel_recorded;
    if (kernel_recorded) ctx->ring_n++;
    ctx->pending = true;
    if (!async) settle_timing(ctx);
}

bool comm_active(const gdist_ctx* ctx) { return has_comm(ctx) && ctx->nranks > 1; }

void comm_allgather_inplace(gdist_ctx* ctx, void* d_buf, size_t bytes) { allgather_inplace(ctx, d_buf, bytes); }

void comm_allgather(gdist_ctx* ctx, const void* d_send, void* d_recv, size_t bytes) { allgather(ctx, d_send, d_recv, bytes); }

int64_t allgather_concat(gdist_ctx* ctx, DevBuf& buf, int64_t n, size_t es) {
    hipStream_t st = ctx->stream;
    const int R = ctx->nranks, me = ctx->rank;
    std::vector<int64_t> hn(R);
    {
        DevBuf mine(8, st), all(8 * R, st);
        h2d(mine.p, &n, 8, st);
        allgather(ctx, mine.p, all.p, 8);
        d2h(hn.data(), all.p, 8 * R, st);
    }
    int64_t mx = 0, tot = 0;
    for (int64_t v : hn) { mx = std::max(mx, v); tot += v; }
    const size_t slot = (size_t)mx * es;
    DevBuf g(slot * R + 8, st);
    if (n) GD_HIP(hipMemcpyAsync(static_cast<char*>(g.p) + slot * me, buf.p, (size_t)n * es, hipMemcpyDeviceToDevice, st));
    buf.release();
    if (slot) allgather_inplace(ctx, g.p, slot);
    // slot r's elements move down to the sum of the earlier counts (staged
    // when source and destination overlap)
    DevBuf stage;
    int64_t at = 0;
    for (int r = 0; r < R; r++) {
        char* src = static_cast<char*>(g.p) + slot * r;
        char* dst = static_cast<char*>(g.p) + (size_t)at * es;
        const size_t b = (size_t)hn[r] * es;
        if (b && src != dst) {
            if (dst + b <= src) {
                GD_HIP(hipMemcpyAsync(dst, src, b, hipMemcpyDeviceToDevice, st));
            } else {
                if (!stage.p) stage.alloc(slot + 8, st);
                GD_HIP(hipMemcpyAsync(stage.p, src, b, hipMemcpyDeviceToDevice, st));
                GD_HIP(hipMemcpyAsync(dst, stage.p, b, hipMemcpyDeviceToDevice, st));
            }
        }
        at += hn[r];
    }
    GD_HIP(hipStreamSynchronize(st));
    buf = std::move(g);
    return tot;
}

BuildSplit build_split(const gdist_ctx* ctx, const gdist_sets* s) {
    BuildSplit sp;
    const int64_t opt = ctx->option(OPT_SPLIT_BUILD, -1);
    if (opt != 0 && s->replicated && comm_active(ctx)) {
        sp.R = ctx->nranks;
        sp.me = ctx->rank;
        sp.real = true;
    } else if (opt >= 2 && !comm_active(ctx)) {
        sp.R = (int)std::min<int64_t>(opt, 1024);
    }
    sp.share_ms.assign(sp.R, 0.0);
    return sp;
}

// one flag over the communicator: true when any rank's is
static bool comm_any(gdist_ctx* ctx, bool v) {
    hipStream_t st = ctx->stream;
    const int R = ctx->nranks;
    int32_t h = v ? 1 : 0;
    DevBuf d(4, st), all(4 * R, st);
    h2d(d.p, &h, 4, st);
    allgather(ctx, d.p, all.p, 4);
    std::vector<int32_t> hv(R);
    d2h(hv.data(), all.p, 4 * R, st);
    GD_HIP(hipStreamSynchronize(st));
    for (int32_t x : hv)
        if (x) return true;
    return false;
}

}  // namespace gdist

using namespace gdist;

extern "C" {

const char* gdist_version(void) { return "gdist 0.1.0 (gfx950)"; }
int gdist_abi_version(void) { return GDIST_ABI_VERSION; }
const char* gdist_last_error(void) { return g_last_error.c_str(); }

int gdist_device_count(int* n) {
    return guard([&] {
        GD_REQUIRE(n, "null output");
        GD_HIP(hipGetDeviceCount(n));
    });
}

// Timing-only events: no system-scope release / acquire when they are
// recorded. With the default flags every record wrote back and invalidated
// the caches: 18 us between two C2 steps (0.167 vs 0.148 ms per step,
// profiles/r02/sparse6/events.txt). Completion that the host relies on goes
// through stream synchronisation or the staging events (default flags).
static constexpr unsigned kTimingEventFlags = hipEventDisableSystemFence;

int gdist_ctx_create(int device, gdist_ctx** out) {
    return guard([&] {
        GD_REQUIRE(out, "null output");
        int n = 0;
        GD_HIP(hipGetDeviceCount(&n));
        GD_REQUIRE(device >= 0 && device < n, "device index out of range");
        GD_HIP(hipSetDevice(device));
        auto* c = new gdist_ctx();
        c->device = device;
        GD_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        GD_HIP(hipEventCreateWithFlags(&c->ev_call0, kTimingEventFlags));
        GD_HIP(hipEventCreateWithFlags(&c->ev_call1, kTimingEventFlags));
        for (int i = 0; i < gdist_ctx::kTimingRing; i++) {
            GD_HIP(hipEventCreateWithFlags(&c->ring0[i], kTimingEventFlags));
            GD_HIP(hipEventCreateWithFlags(&c->ring1[i], kTimingEventFlags));
        }
        c->ev_k0 = c->ring0[0];
        c->ev_k1 = c->ring1[0];
        GD_HIP(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
        GD_HIP(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
        GD_HIP(hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
        for (int f = 0; f < gdist_ctx::kFamilies; f++) {
            GD_HIP(hipEventCreateWithFlags(&c->ev_kf0[f], kTimingEventFlags));
            GD_HIP(hipEventCreateWithFlags(&c->ev_kf1[f], kTimingEventFlags));
        }
        GD_HIP(hipEventCreateWithFlags(&c->ev_stage[0], hipEventDisableTiming));
        GD_HIP(hipEventCreateWithFlags(&c->ev_stage[1], hipEventDisableTiming));
        GD_HIP(hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device));
        *out = c;
    });
}

int gdist_ctx_destroy(gdist_ctx* ctx) {
    return guard([&] {
        if (!ctx) return;
        (void)hipSetDevice(ctx->device);
        (void)hipStreamSynchronize(ctx->stream);
        if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
        (void)hipEventDestroy(ctx->ev_call0);
        (void)hipEventDestroy(ctx->ev_call1);
        for (int i = 0; i < gdist_ctx::kTimingRing; i++) {
            (void)hipEventDestroy(ctx->ring0[i]);
            (void)hipEventDestroy(ctx->ring1[i]);
        }
        (void)hipStreamSynchronize(ctx->side);
        (void)hipEventDestroy(ctx->ev_fork);
        (void)hipEventDestroy(ctx->ev_join);
        for (int f = 0; f < gdist_ctx::kFamilies; f++) {
            (void)hipEventDestroy(ctx->ev_kf0[f]);
            (void)hipEventDestroy(ctx->ev_kf1[f]);
        }
        (void)hipStreamDestroy(ctx->side);
        (void)hipEventDestroy(ctx->ev_stage[0]);
        (void)hipEventDestroy(ctx->ev_stage[1]);
        if (ctx->pinned) (void)hipHostFree(ctx->pinned);
        (void)hipStreamDestroy(ctx->stream);
        gdist::cache_trim(ctx->device);
        delete ctx;
    });
}

int gdist_ctx_synchronize(gdist_ctx* ctx) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        GD_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int gdist_ctx_set_option(gdist_ctx* ctx, const char* name, int64_t value) {
    return guard([&] {
        GD_REQUIRE(ctx, "null context");
        const int i = option_index(name);
        std::lock_guard<std::recursive_mutex> lk(ctx->mu);
        ctx->opt[i] = value == GDIST_OPTION_DEFAULT ? kOptUnset : value;
        // launch plans cache per-call choices: drop none here (their keys
        // carry the options they depend on), sets built later see the value
    });
}

int gdist_ctx_get_option(gdist_ctx* ctx, const char* name, int64_t* value, int* is_set) {
    return guard([&] {
        GD_REQUIRE(ctx && value, "null argument");
        const int i = option_index(name);
        std::lock_guard<std::recursive_mutex> lk(ctx->mu);      // set_option writes under the lock
        *value = ctx->opt[i] == kOptUnset ? GDIST_OPTION_DEFAULT : ctx->opt[i];
        if (is_set) *is_set = ctx->opt[i] != kOptUnset;
    });
}

int gdist_ctx_option_name(int index, const char** name) {
    return guard([&] {
        GD_REQUIRE(name, "null output");
        GD_REQUIRE(index >= 0 && index < OPT_COUNT, "option index out of range");
        *name = kOptNames[index];
    });
}

int gdist_ctx_recent_timings(gdist_ctx* ctx, int max, double* kernel_ms, int* count) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        GD_REQUIRE(count && (max <= 0 || kernel_ms), "null output");
        gdist::settle_timing(ctx);
        const int64_t n = std::min<int64_t>({(int64_t)std::max(max, 0), ctx->ring_n, (int64_t)gdist_ctx::kTimingRing});
        for (int64_t i = 0; i < n; i++) {     // oldest first
            const int slot = (int)((ctx->ring_n - n + i) % gdist_ctx::kTimingRing);
            GD_HIP(hipEventSynchronize(ctx->ring1[slot]));
            float km = 0.f;
            GD_HIP(hipEventElapsedTime(&km, ctx->ring0[slot], ctx->ring1[slot]));
            kernel_ms[i] = km;
        }
        *count = (int)n;
    });
}

int gdist_ctx_kernel_ms(gdist_ctx* ctx, int family, double* ms) {
    return guard([&] {
        GD_REQUIRE(ctx && ms, "null argument");
        GD_REQUIRE(family >= 0 && family < gdist_ctx::kFamilies, "unknown kernel family");
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        *ms = -1.0;
        if (!ctx->kf_timed[family]) return;
        GD_HIP(hipEventSynchronize(ctx->ev_kf1[family]));
        float t = 0.f;
        GD_HIP(hipEventElapsedTime(&t, ctx->ev_kf0[family], ctx->ev_kf1[family]));
        *ms = t;
    });
}

int gdist_ctx_last_timing(gdist_ctx* ctx, double* kernel_ms, double* call_ms, int64_t* launches) {
    return guard([&] {
        GD_REQUIRE(ctx, "null context");
        {
            std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
            use_device(ctx);
            gdist::settle_timing(ctx);
        }
        if (kernel_ms) *kernel_ms = ctx->last.kernel_ms;
        if (call_ms) *call_ms = ctx->last.call_ms;
        if (launches) *launches = ctx->last.launches;
    });
}

int gdist_dev_alloc(gdist_ctx* ctx, int64_t bytes, void** dptr) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        GD_REQUIRE(dptr && bytes >= 0, "bad allocation request");
        *dptr = nullptr;
        if (!bytes) return;
        hipError_t e = hipMalloc(dptr, (size_t)bytes);
        if (e == hipErrorOutOfMemory) {          // the library's cached blocks may hold the memory
            (void)hipGetLastError();
            gdist::cache_trim(ctx->device);
            e = hipMalloc(dptr, (size_t)bytes);
        }
        GD_HIP(e);
    });
}

int gdist_dev_free(gdist_ctx* ctx, void* dptr) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        GD_HIP(hipStreamSynchronize(ctx->stream));
        if (dptr) GD_HIP(hipFree(dptr));
    });
}

int gdist_memcpy_d2h(gdist_ctx* ctx, void* dst, const void* src, int64_t bytes) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        if (bytes <= 0) return;
        d2h(dst, src, (size_t)bytes, ctx->stream);
        GD_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int gdist_memcpy_h2d(gdist_ctx* ctx, void* dst, const void* src, int64_t bytes) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        if (bytes <= 0) return;
        h2d(dst, src, (size_t)bytes, ctx->stream);
        GD_HIP(hipStreamSynchronize(ctx->stream));
    });
}

// ---------------------------------------------------------------------------
int gdist_host_alloc(int64_t bytes, void** hptr) {
    return guard([&] {
        GD_REQUIRE(hptr && bytes >= 0, "bad host allocation arguments");
        *hptr = nullptr;
        GD_HIP(hipHostMalloc(hptr, (size_t)std::max<int64_t>(1, bytes), hipHostMallocDefault));
    });
}

int gdist_release_cache(int device) {
    // the caller's current device is restored on every exit (as use_device)
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    const int rc = guard([&] {
        GD_HIP(hipSetDevice(device));
        GD_HIP(hipDeviceSynchronize());
        gdist::cache_trim(device);
    });
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
    return rc;
}

int gdist_host_free(void* hptr) {
    return guard([&] {
        if (hptr) GD_HIP(hipHostFree(hptr));
    });
}

int gdist_sets_pack(gdist_ctx* ctx, int kind, int k, unsigned flags, const char* seqs, const int64_t* seq_off,
                    int64_t nseqs, gdist_sets** out) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk(ctx->mu);
        GD_REQUIRE(out && nseqs >= 0 && (nseqs == 0 || (seqs && seq_off)), "bad pack arguments");
        *out = nullptr;
        std::vector<int64_t> h(nseqs + 1, 0);
        const int64_t base = nseqs ? seq_off[0] : 0;
        for (int64_t s = 0; s <= nseqs; s++) h[s] = (nseqs ? seq_off[s] : 0) - base;
        for (int64_t s = 0; s < nseqs; s++) GD_REQUIRE(h[s + 1] >= h[s], "sequence offsets must be non-decreasing");
        const int64_t bytes = h[nseqs];
        Trace tr(ctx->stream, ctx->trace());
        DevBuf dseq(bytes + 1, ctx->stream), doff((nseqs + 1) * 8, ctx->stream);
        h2d(doff.p, h.data(), (nseqs + 1) * 8, ctx->stream);
        tr.mark("pack: byte buffer");
        auto* s = new gdist_sets();
        s->ctx = ctx;
        try {
            // the bytes move to dseq during the pack, chunk by chunk
            pack_sets(ctx, kind, k, flags, dseq.as<char>(), doff.as<int64_t>(), h, s, seqs + base);
        } catch (...) {
            delete s;
            throw;
        }
        *out = s;
    });
}

int gdist_sets_append(gdist_ctx* ctx, gdist_sets* sets, const char* seqs, const int64_t* seq_off, int64_t nseqs,
                      int64_t* first) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk(ctx->mu);
        check_codes(sets);
        GD_REQUIRE(sets->ctx == ctx, "sets belong to another context");
        GD_REQUIRE(sets->kind != GDIST_SKETCH, "sketch collections are built, not appended to");
        GD_REQUIRE(nseqs >= 0 && (nseqs == 0 || (seqs && seq_off)), "bad append arguments");
        if (first) *first = sets->nsets;
        if (nseqs == 0) return;
        std::vector<int64_t> h(nseqs + 1, 0);
        const int64_t base = seq_off[0];
        for (int64_t i = 0; i <= nseqs; i++) h[i] = seq_off[i] - base;
        for (int64_t i = 0; i < nseqs; i++) GD_REQUIRE(h[i + 1] >= h[i], "sequence offsets must be non-decreasing");
        hipStream_t st = ctx->stream;
        gdist_sets add;                        // the new sequences, packed with the collection's kmer spec
        add.ctx = ctx;
        {
            DevBuf dseq(h[nseqs] + 1, st), doff((nseqs + 1) * 8, st);
            h2d(doff.p, h.data(), (nseqs + 1) * 8, st);
            pack_sets(ctx, sets->kind, sets->k, sets->flags, dseq.as<char>(), doff.as<int64_t>(), h, &add, seqs + base);
        }
        // every representation derived from the old sets is stale (dictionary,
        // tiers, plans, captured steps, the pack summaries the dictionary
        // merges) — except the sorted join's segment index, which is extended
        // below with the new sets' rows (round 6)
        free_bitsets(sets);
        const int64_t n_old = sets->nsets;
        const bool extend_seg = sets->segoff.p && sets->nseg >= 1 && (sets->nseg == 1 || sets->seg_split.p);
        if (!extend_seg) {
            sets->segoff.release();
            sets->seg_split.release();
            sets->nseg = 0;
            sets->max_seg = 0;
        }
        sets->auto_sorted = false;
        sets->pack_sum.clear();
        sets->replicated = false;             // this rank's sets only from here
        // codes: in place while the buffer's size class has room, else a
        // buffer of twice the need (n appends copy O(n) codes in all)
        const int64_t total = sets->total + add.total;
        if ((size_t)(total * 8 + 8) > sets->codes.cls) {
            DevBuf grown((size_t)total * 16 + 8, st);
            if (sets->total)
                GD_HIP(hipMemcpyAsync(grown.p, sets->codes.p, sets->total * 8, hipMemcpyDeviceToDevice, st));
            sets->codes = std::move(grown);
        } else {
            sets->codes.bytes = std::max(sets->codes.bytes, (size_t)(total * 8 + 8));
        }
        if (add.total)
            GD_HIP(hipMemcpyAsync(sets->codes.as<uint64_t>() + sets->total, add.codes.p, add.total * 8,
                                  hipMemcpyDeviceToDevice, st));
        for (int64_t i = 1; i <= add.nsets; i++) sets->h_off.push_back(add.h_off[i] + sets->total);
        sets->nsets += add.nsets;
        sets->total = total;
        sets->off.alloc((sets->nsets + 1) * 8, st);
        h2d(sets->off.p, sets->h_off.data(), (sets->nsets + 1) * 8, st);
        // locus guides: the collection's first sequences (the new ones only
        // when it had none)
        if (sets->n_guide == 0 && add.n_guide) {
            sets->guide_codes = std::move(add.guide_codes);
            sets->guide_keys = std::move(add.guide_keys);
            sets->n_guide = add.n_guide;
        }
        if (extend_seg) extend_segments(ctx, sets, n_old);
        GD_HIP(hipStreamSynchronize(st));
    });
}

int gdist_sets_pack_device(gdist_ctx* ctx, int kind, int k, unsigned flags, const char* d_seqs,
                           const int64_t* d_seq_off, int64_t nseqs, int64_t total_bytes, gdist_sets** out) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk(ctx->mu);
        GD_REQUIRE(out && nseqs >= 0 && d_seq_off, "bad pack arguments");
        *out = nullptr;
        std::vector<int64_t> h(nseqs + 1, 0);
        d2h(h.data(), d_seq_off, (nseqs + 1) * 8, ctx->stream);
        GD_HIP(hipStreamSynchronize(ctx->stream));
        for (int64_t s = 0; s < nseqs; s++) GD_REQUIRE(h[s + 1] >= h[s], "sequence offsets must be non-decreasing");
        GD_REQUIRE(h[0] >= 0 && h[nseqs] <= total_bytes, "sequence offsets exceed the byte buffer");
        auto* s = new gdist_sets();
        s->ctx = ctx;
        try {
            pack_sets(ctx, kind, k, flags, d_seqs, d_seq_off, h, s);
        } catch (...) {
            delete s;
            throw;
        }
        *out = s;
    });
}

int gdist_sets_upload(gdist_ctx* ctx, int kind, int k, int64_t nsets, const int64_t* offsets, const uint64_t* codes,
                      gdist_sets** out) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk(ctx->mu);
        GD_REQUIRE(out && nsets >= 0 && offsets, "bad upload arguments");
        GD_REQUIRE(kind == GDIST_DNA || kind == GDIST_PROT, "kind must be GDIST_DNA or GDIST_PROT");
        *out = nullptr;
        GD_REQUIRE(offsets[0] == 0, "offsets[0] must be 0");
        for (int64_t s = 0; s < nsets; s++) {
            GD_REQUIRE(offsets[s + 1] >= offsets[s], "offsets must be non-decreasing");
            for (int64_t e = offsets[s] + 1; e < offsets[s + 1]; e++)
                GD_REQUIRE(codes[e - 1] < codes[e], "codes of each set must be sorted and unique");
        }
        const int64_t total = offsets[nsets];
        auto* s = new gdist_sets();
        s->ctx = ctx; s->kind = kind; s->k = k; s->nsets = nsets; s->total = total;
        s->h_off.assign(offsets, offsets + nsets + 1);
        s->off.alloc((nsets + 1) * 8, ctx->stream);
        s->codes.alloc(total * 8 + 8, ctx->stream);
        h2d(s->off.p, offsets, (nsets + 1) * 8, ctx->stream);
        if (total) h2d(s->codes.p, codes, total * 8, ctx->stream);
        GD_HIP(hipStreamSynchronize(ctx->stream));
        *out = s;
    });
}

int gdist_sets_free(gdist_sets* s) {
    return guard([&] {
        if (!s) return;
        gdist_ctx* ctx = s->ctx;
        (void)hipSetDevice(ctx->device);
        (void)hipStreamSynchronize(ctx->stream);
        delete s;   // stream-ordered frees
        (void)hipStreamSynchronize(ctx->stream);
    });
}

int gdist_sets_info(const gdist_sets* s, int* kind, int* k, int64_t* nsets, int64_t* total) {
    return guard([&] {
        check_sets(s);
        if (kind) *kind = s->kind;
        if (k) *k = s->kind == GDIST_SKETCH ? s->width : s->k;
        if (nsets) *nsets = s->nsets;
        if (total) *total = s->total;
    });
}

int gdist_sets_sizes(const gdist_sets* s, int64_t* sizes) {
    return guard([&] {
        check_sets(s);
        GD_REQUIRE(sizes, "null output");
        for (int64_t i = 0; i < s->nsets; i++) sizes[i] = s->h_off[i + 1] - s->h_off[i];
    });
}

int gdist_sets_download(const gdist_sets* s, int64_t* offsets, uint64_t* codes) {
    return guard([&] {
        check_codes(s);
        GD_REQUIRE(s->kind != GDIST_SKETCH, "use gdist_sketch_download for sketches");
        use_device(s->ctx);
        std::lock_guard<std::recursive_mutex> lk_(s->ctx->mu);
        if (offsets) std::memcpy(offsets, s->h_off.data(), (s->nsets + 1) * 8);
        if (codes && s->total)
            d2h(codes, s->codes.p, s->total * 8, s->ctx->stream);
        GD_HIP(hipStreamSynchronize(s->ctx->stream));
    });
}

int gdist_sets_build_bitsets(gdist_sets* s, unsigned flags) { return gdist_sets_build_bitsets_ex(s, flags, -1); }

int gdist_sets_build_bitsets_ex(gdist_sets* s, unsigned flags, int64_t rare_threshold) {
    return guard([&] {
        check_sets(s);
        GD_REQUIRE(s->kind != GDIST_SKETCH && s->has_codes, "bitsets are built from kmer sets");
        use_device(s->ctx);
        std::lock_guard<std::recursive_mutex> lk(s->ctx->mu);
        build_bitsets(s->ctx, s, flags, rare_threshold);
    });
}

int gdist_sets_release_codes(gdist_sets* s) {
    return guard([&] {
        check_sets(s);
        GD_REQUIRE(s->kind != GDIST_SKETCH, "sketch collections hold signatures, not codes");
        GD_REQUIRE(s->bits.p, "the collection holds no bitsets: its codes are its only representation");
        use_device(s->ctx);
        std::lock_guard<std::recursive_mutex> lk(s->ctx->mu);
        GD_HIP(hipStreamSynchronize(s->ctx->stream));
        s->codes.release();
        s->segoff.release();
        s->seg_split.release();
        s->nseg = 0;
        s->max_seg = 0;
        s->pack_sum.clear();
        s->has_codes = false;
        gdist::cache_trim(s->ctx->device);
    });
}

int gdist_sets_build_timing(const gdist_sets* s, double* build_ms, double* split_ms, double* share_max_ms,
                            int* shares) {
    return guard([&] {
        check_sets(s);
        if (build_ms) *build_ms = s->build_ms;
        if (split_ms) *split_ms = s->build_split_ms;
        if (share_max_ms) *share_max_ms = s->build_share_max_ms;
        if (shares) *shares = s->build_shares;
    });
}

int gdist_sets_rare_info(const gdist_sets* s, int64_t* threshold, int64_t* lists, int64_t* records) {
    return guard([&] {
        check_sets(s);
        if (threshold) *threshold = s->rare_T;
        if (lists) *lists = s->n_rare;
        if (records) *records = s->rare_records;
    });
}

int gdist_sets_sparse_info(const gdist_sets* s, int64_t* sparse_words, int64_t* dense_words, int64_t* entries) {
    return guard([&] {
        check_sets(s);
        if (sparse_words) *sparse_words = s->sparse ? s->Ws : 0;
        if (dense_words) *dense_words = s->sparse ? s->Wd : s->W;
        if (entries) *entries = s->sparse ? s->sp_entries : 0;
    });
}

int gdist_sets_variant_info(const gdist_sets* s, int64_t* kmers, int64_t* words, int64_t* entries, double* products) {
    return guard([&] {
        check_sets(s);
        if (kmers) *kmers = s->variant ? s->vw_kmers : 0;
        if (words) *words = s->variant ? s->vw_words : 0;
        if (entries) *entries = s->variant ? s->vw_entries : 0;
        if (products) *products = s->variant ? s->vw_products : 0.0;
    });
}

int gdist_sets_variant_layout(const gdist_sets* s, int* word_kmers, int* member_bytes, int64_t* row_weight_max) {
    return guard([&] {
        check_sets(s);
        if (word_kmers) *word_kmers = s->variant ? s->vw_bits : 0;
        if (member_bytes) *member_bytes = !s->variant ? 0 : s->vw_pack.p ? 4 : s->vw_pk64.p ? 8 : 12;
        if (row_weight_max) *row_weight_max = s->variant ? s->vw_row_wmax : 0;
    });
}

int gdist_sets_sparse_pairs(const gdist_sets* s, double* pairs) {
    return guard([&] {
        check_sets(s);
        if (pairs) *pairs = s->sparse ? s->sp_pairs : 0.0;
    });
}

int gdist_sets_sparse_sides(const gdist_sets* s, int64_t* complement_words, int64_t* positive_words) {
    return guard([&] {
        check_sets(s);
        if (complement_words) *complement_words = s->sparse ? s->Ws - s->sp_pos_words : 0;
        if (positive_words) *positive_words = s->sparse ? s->sp_pos_words : 0;
    });
}

int gdist_sets_group_info(const gdist_sets* s, int64_t* groups, int64_t* grouped_words) {
    return guard([&] {
        check_sets(s);
        if (groups) *groups = s->sparse ? s->sp_groups : 0;
        if (grouped_words) *grouped_words = s->sparse ? s->sp_group_words : 0;
    });
}

int gdist_sets_rare_kmers(const gdist_sets* s, int64_t* kmers) {
    return guard([&] {
        check_sets(s);
        if (kmers) *kmers = s->rare_kmers;
    });
}

int gdist_sets_rare_stats(const gdist_sets* s, int64_t* pair_incs, int64_t* max_list) {
    return guard([&] {
        check_sets(s);
        if (pair_incs) *pair_incs = s->rare_incs;
        if (max_list) *max_list = s->rare_max_list;
    });
}

int gdist_sets_bitset_info(const gdist_sets* s, int64_t* dict_size, int64_t* words_per_set) {
    return guard([&] {
        check_sets(s);
        if (dict_size) *dict_size = s->bits.p ? s->dict_size : -1;
        if (words_per_set) *words_per_set = s->bits.p ? s->W : 0;
    });
}

int gdist_sets_bitset_download(const gdist_sets* s, uint64_t* bits) {
    return guard([&] {
        check_sets(s);
        GD_REQUIRE(s->bits.p, "no bitsets built");
        GD_REQUIRE(bits, "null output");
        use_device(s->ctx);
        std::lock_guard<std::recursive_mutex> lk_(s->ctx->mu);
        d2h(bits, s->bits.p, (size_t)s->nsets * s->W * 8, s->ctx->stream);
        GD_HIP(hipStreamSynchronize(s->ctx->stream));
    });
}

int gdist_sets_concat(const gdist_sets* a, const gdist_sets* b, gdist_sets** out) {
    return guard([&] {
        check_codes(a);
        check_codes(b);
        GD_REQUIRE(out, "null output");
        GD_REQUIRE(a->ctx == b->ctx, "sets belong to different contexts");
        GD_REQUIRE(a->kind == b->kind && a->k == b->k && a->width == b->width &&
                       (a->flags & ~GDIST_NO_CASE_FOLD) == (b->flags & ~GDIST_NO_CASE_FOLD),
                   "sets were packed with different kmer specs");
        gdist_ctx* ctx = a->ctx;
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk(ctx->mu);
        const size_t es = a->kind == GDIST_SKETCH ? 4 : 8;
        auto* s = new gdist_sets();
        s->ctx = ctx; s->kind = a->kind; s->k = a->k; s->flags = a->flags; s->width = a->width;
        s->nsets = a->nsets + b->nsets;
        s->total = a->total + b->total;
        s->h_off = a->h_off;
        for (int64_t i = 1; i <= b->nsets; i++) s->h_off.push_back(b->h_off[i] + a->total);
        s->off.alloc((s->nsets + 1) * 8, ctx->stream);
        h2d(s->off.p, s->h_off.data(), (s->nsets + 1) * 8, ctx->stream);
        s->codes.alloc(s->total * es + 8, ctx->stream);
        if (a->total)
            GD_HIP(hipMemcpyAsync(s->codes.p, a->codes.p, a->total * es, hipMemcpyDeviceToDevice, ctx->stream));
        if (b->total)
            GD_HIP(hipMemcpyAsync((char*)s->codes.p + a->total * es, b->codes.p, b->total * es,
                                  hipMemcpyDeviceToDevice, ctx->stream));
        // locus guides: the first collection's (its sets come first), else the second's
        const gdist_sets* g = a->n_guide ? a : b;
        if (g->n_guide) {
            s->guide_codes.alloc(g->n_guide * 8, ctx->stream);
            s->guide_keys.alloc(g->n_guide * 8, ctx->stream);
            GD_HIP(hipMemcpyAsync(s->guide_codes.p, g->guide_codes.p, g->n_guide * 8, hipMemcpyDeviceToDevice,
                                  ctx->stream));
            GD_HIP(hipMemcpyAsync(s->guide_keys.p, g->guide_keys.p, g->n_guide * 8, hipMemcpyDeviceToDevice,
                                  ctx->stream));
            s->n_guide = g->n_guide;
        }
        GD_HIP(hipStreamSynchronize(ctx->stream));
        *out = s;
    });
}

// ---------------------------------------------------------------------------
// Method resolution (shared by gdist_intersect_matrix and gdist_sets_prepare).
// AUTO: bitsets when built; otherwise, when the sorted join would take more
// than ~20 ms on the region (small regions of small sets stay on the join
// without building anything), build the two-tier dictionary and keep it
// only when its cost estimate beats the sorted join's.
static int resolve_method(gdist_ctx* ctx, gdist_sets* s, int method, double pairs) {
    int m = method;
    if (m == GDIST_METHOD_AUTO) {
        bool want = !s->bits.p && !s->auto_sorted && !s->segoff.p && s->has_codes && sorted_cost_s(s, pairs) >= 0.02;
        // a gathered collection's build is collective (split by rank): every
        // rank builds when any rank's region asks for it
        const bool collective =
            s->replicated && comm_active(ctx) && ctx->option(OPT_SPLIT_BUILD, -1) != 0 && !s->bits.p && s->has_codes;
        if (collective) want = comm_any(ctx, want);
        if (want) {
            try {
                build_bitsets(ctx, s, 0);
            } catch (const Error& e) {
                if (e.code != GDIST_ENOMEM) throw;
                // the dictionary does not fit next to the codes: the join needs no more memory
                (void)hipGetLastError();
                free_bitsets(s);
                gdist::cache_trim(ctx->device);
            }
            bool keep = s->bits.p && bitset_cost_s(s, pairs) <= sorted_cost_s(s, pairs);
            if (collective) {
                // one verdict for every rank: the estimates differ
                // per rank (each prices its own region) and an ENOMEM strikes
                // one rank, so a per-rank verdict would leave some ranks with
                // the bits and the next collective build (AUTO or BITSET)
                // entered by the others only. Keep them when every rank holds
                // them and some rank's region prefers them (the build is paid).
                const bool missing = comm_any(ctx, !s->bits.p);
                keep = !missing && comm_any(ctx, keep);
            }
            if (!keep) {
                free_bitsets(s);
                s->auto_sorted = true;
            }
        }
        m = s->bits.p ? GDIST_METHOD_BITSET : GDIST_METHOD_SORTED;
    }
    GD_REQUIRE(m == GDIST_METHOD_BITSET || s->has_codes, "this collection holds bitsets only");
    // a shard consumed by the code all-gather holds neither codes nor bitsets
    GD_REQUIRE(s->has_codes || s->bits.p, "the collection holds no codes (consumed by an all-gather)");
    if (m == GDIST_METHOD_BITSET && !s->bits.p) build_bitsets(ctx, s, 0);
    if (m == GDIST_METHOD_SORTED && !s->segoff.p) build_segments(ctx, s);
    return m;
}

int gdist_sets_prepare(gdist_ctx* ctx, gdist_sets* sets, int method, double pairs, int* chosen,
                       double* cost_bitset_s, double* cost_sorted_s) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        check_sets(sets);
        GD_REQUIRE(sets->ctx == ctx, "sets belong to another context");
        GD_REQUIRE(sets->kind != GDIST_SKETCH, "sketch collections have one method");
        GD_REQUIRE(method >= GDIST_METHOD_AUTO && method <= GDIST_METHOD_BITSET, "unknown method");
        std::lock_guard<std::recursive_mutex> lk(ctx->mu);
        if (pairs < 0) pairs = 0.5 * (double)sets->nsets * (double)(sets->nsets - 1);
        const int m = resolve_method(ctx, sets, method, pairs);
        if (chosen) *chosen = m;
        if (cost_bitset_s) *cost_bitset_s = sets->bits.p ? bitset_cost_s(sets, pairs) : -1.0;
        if (cost_sorted_s) *cost_sorted_s = sorted_cost_s(sets, pairs);
    });
}

// Device region (nr x nc, element `elem` bytes, device row stride nc) into a
// host matrix with row stride ld, through double-buffered pinned staging in
// row blocks; each row lands with one memcpy per contiguous span (rows of a
// block split over a few host threads). With `upper` only the entries with
// global column > global row are written: the others stay the caller's
// (gdist.h, GDIST_UPPER_TRIANGLE).
static void copy_out_rows(gdist_ctx* ctx, const void* dsrc, size_t elem, int64_t nr, int64_t nc, int64_t r0,
                          int64_t c0, bool upper, void* hdst, int64_t ld) {
    if (nr <= 0 || nc <= 0) return;
    hipStream_t st = ctx->stream;
    const size_t row_bytes = (size_t)nc * elem;
    const size_t half = std::max(row_bytes, (size_t)64 << 20);
    if (ctx->pinned_bytes < 2 * half) {
        if (ctx->pinned) GD_HIP(hipHostFree(ctx->pinned));
        ctx->pinned = nullptr;
        ctx->pinned_bytes = 0;
        GD_HIP(hipHostMalloc(&ctx->pinned, 2 * half, hipHostMallocDefault));
        ctx->pinned_bytes = 2 * half;
    }
    const int64_t rows_per = (int64_t)(half / row_bytes);
    char* stage[2] = {static_cast<char*>(ctx->pinned), static_cast<char*>(ctx->pinned) + half};
    const char* src = static_cast<const char*>(dsrc);
    char* dst = static_cast<char*>(hdst);
    auto issue = [&](int64_t a0, int b) {
        const int64_t a1 = std::min(nr, a0 + rows_per);
        GD_HIP(hipMemcpyAsync(stage[b], src + (size_t)a0 * row_bytes, (size_t)(a1 - a0) * row_bytes,
                              hipMemcpyDeviceToHost, st));
        GD_HIP(hipEventRecord(ctx->ev_stage[b], st));
    };
    const int nthreads = (int)std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    issue(0, 0);
    int b = 0;
    for (int64_t a0 = 0; a0 < nr; a0 += rows_per, b ^= 1) {
        GD_HIP(hipEventSynchronize(ctx->ev_stage[b]));
        if (a0 + rows_per < nr) issue(a0 + rows_per, b ^ 1);
        const int64_t a1 = std::min(nr, a0 + rows_per);
        auto rows = [&](int64_t lo, int64_t hi) {
            for (int64_t a = lo; a < hi; a++) {
                const int64_t first = upper ? std::max<int64_t>(0, r0 + a + 1 - c0) : 0;
                if (first >= nc) continue;
                std::memcpy(dst + ((size_t)a * ld + first) * elem, stage[b] + ((size_t)(a - a0) * nc + first) * elem,
                            (size_t)(nc - first) * elem);
            }
        };
        const int64_t nrows = a1 - a0;
        if (nthreads == 1 || nrows * (int64_t)row_bytes < (int64_t(4) << 20)) {
            rows(a0, a1);
        } else {
            std::vector<std::thread> pool;
            const int64_t per = ceil_div(nrows, (int64_t)nthreads);
            for (int t = 0; t < nthreads; t++) {
                const int64_t lo = a0 + t * per, hi = std::min(a1, lo + per);
                if (lo < hi) pool.emplace_back(rows, lo, hi);
            }
            for (auto& th : pool) th.join();
        }
    }
}

// ---------------------------------------------------------------------------
int gdist_intersect_matrix(gdist_ctx* ctx, const gdist_sets* sets, int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                           int method, unsigned flags, int32_t* I_out, double* D_out, int64_t ld) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        check_sets(sets);
        GD_REQUIRE(sets->ctx == ctx, "sets belong to another context");
        GD_REQUIRE(sets->kind != GDIST_SKETCH, "use gdist_sketch_matrix for sketches");
        GD_REQUIRE(0 <= r0 && r0 <= r1 && r1 <= sets->nsets && 0 <= c0 && c0 <= c1 && c1 <= sets->nsets,
                   "row/column range outside the set collection");
        const int64_t nr = r1 - r0, nc = c1 - c0;
        GD_REQUIRE(ld >= nc, "leading dimension smaller than the column range");
        GD_REQUIRE(method >= GDIST_METHOD_AUTO && method <= GDIST_METHOD_BITSET, "unknown method");
        std::lock_guard<std::recursive_mutex> lk(ctx->mu);
        auto* s = const_cast<gdist_sets*>(sets);
        const int m = resolve_method(ctx, s, method,
                                     (double)nr * (double)nc * (flags & GDIST_UPPER_TRIANGLE ? 0.5 : 1.0));
        const bool upper = (flags & GDIST_UPPER_TRIANGLE) != 0;
        const bool dev = (flags & GDIST_OUT_DEVICE) != 0;
        hipStream_t st = ctx->stream;
        ctx->pending = false;          // an unread previous call's times are dropped, not waited for
        ctx->last = Timing{};
        for (bool& f : ctx->kf_timed) f = false;
        // Graph-replayed steps record no timing events unless option
        // step_timing = 1: four event records (call and kernel span) cost
        // 13 us between two C2 steps even without the system fence (0.161
        // vs 0.148 ms, profiles/r02/sparse6/events.txt). Such calls leave
        // last_timing empty and are not in recent_timings.
        const bool quiet = dev && I_out && m == GDIST_METHOD_BITSET && ctx->option(OPT_GRAPH, 1) != 0 &&
                           ctx->option(OPT_STEP_TIMING, 0) == 0 && ctx->option(OPT_TIME_KERNELS, 0) == 0;
        bool timing_started = false;
        auto start_timing = [&] {
            if (timing_started) return;
            gdist::begin_timing(ctx);
            GD_HIP(hipEventRecord(ctx->ev_call0, st));
            timing_started = true;
        };
        if (!quiet) start_timing();
        if (nr == 0 || nc == 0) {
            start_timing();
            gdist::finish_timing(ctx, false);
            return;
        }
        // intersection counts: caller's device buffer or a temporary
        DevBuf tI;
        int32_t* dI;
        int64_t ldI;
        if (dev && I_out) {
            dI = I_out; ldI = ld;
        } else {
            tI.alloc((size_t)nr * nc * 4, st);
            dI = tI.as<int32_t>(); ldI = nc;
        }
        // Repeated calls over one region into the same device outputs (the
        // bench steps, a processor's row-block loop) replay the step as one
        // hipGraph: the launches of both streams, the fork / join and the
        // epilogue without host round trips between them. The first call
        // runs uncaptured (it builds the launch plans), the second is
        // captured; a refused capture leaves the key uncaptured.
        if (dev && I_out && m == GDIST_METHOD_BITSET && ctx->option(OPT_GRAPH, 1) != 0 &&
            ctx->option(OPT_TIME_KERNELS, 0) == 0) {
            std::vector<int64_t> key{r0, r1, c0, c1, (int64_t)flags, (int64_t)(intptr_t)I_out,
                                     (int64_t)(intptr_t)D_out, ld};
            key.insert(key.end(), ctx->opt, ctx->opt + OPT_COUNT);
            auto it = s->graphs.find(key);
            if (it == s->graphs.end()) {
                if (s->graphs.size() >= 8) s->graphs.clear();
                it = s->graphs.emplace(key, std::make_unique<StepGraph>()).first;
            }
            StepGraph& g = *it->second;
            if (!g.exec && !g.failed && g.calls >= 1) {
                hipGraph_t graph = nullptr;
                GD_HIP(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
                ctx->capturing = true;
                bool ok = true;
                try {
                    if (!bitset_matrix_fused(ctx, s, r0, r1, c0, c1, upper, flags, dI, ldI, D_out, ld)) {
                        zero_counts(ctx, r0, r1, c0, c1, upper, dI, ldI);
                        bitset_matrix(ctx, s, r0, r1, c0, c1, upper, dI, ldI);
                        if (D_out) distance_epilogue(ctx, s, r0, r1, c0, c1, upper, flags, dI, ldI, D_out, ld);
                    }
                } catch (...) {
                    ok = false;
                }
                ctx->capturing = false;
                const hipError_t ce = hipStreamEndCapture(st, &graph);
                if (ok && ce == hipSuccess && graph) {
                    if (hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0) != hipSuccess) g.exec = nullptr;
                }
                if (graph) (void)hipGraphDestroy(graph);
                (void)hipGetLastError();
                if (!g.exec) g.failed = true;
            }
            if (g.exec) {
                if (quiet) {
                    GD_HIP(hipGraphLaunch(g.exec, st));
                    ctx->last.launches = 1;
                    return;
                }
                GD_HIP(hipEventRecord(ctx->ev_k0, st));
                GD_HIP(hipGraphLaunch(g.exec, st));
                GD_HIP(hipEventRecord(ctx->ev_k1, st));
                ctx->last.launches = 1;
                gdist::finish_timing(ctx, true, true);
                return;
            }
            g.calls++;
        }
        start_timing();
        DevBuf tD;
        double* dD = nullptr;
        int64_t ldD = 0;
        if (D_out) {
            if (dev) { dD = D_out; ldD = ld; }
            else { tD.alloc((size_t)nr * nc * 8, st); dD = tD.as<double>(); ldD = nc; }
        }
        // the fused sparse step writes I and D itself (bitset.hip)
        const bool fused = m == GDIST_METHOD_BITSET && dD &&
                           bitset_matrix_fused(ctx, s, r0, r1, c0, c1, upper, flags, dI, ldI, dD, ldD);
        if (!fused) {
            if (m == GDIST_METHOD_BITSET)   // accumulated with atomics
                zero_counts(ctx, r0, r1, c0, c1, upper && dev, dI, ldI);
            if (m == GDIST_METHOD_BITSET) bitset_matrix(ctx, s, r0, r1, c0, c1, upper, dI, ldI);
            else sorted_matrix(ctx, s, r0, r1, c0, c1, upper, dI, ldI);
            if (D_out) distance_epilogue(ctx, s, r0, r1, c0, c1, upper, flags, dI, ldI, dD, ldD);
        }
        if (D_out && !dev) copy_out_rows(ctx, dD, 8, nr, nc, r0, c0, upper, D_out, ld);
        if (I_out && !dev) copy_out_rows(ctx, dI, 4, nr, nc, r0, c0, upper, I_out, ld);
        gdist::finish_timing(ctx, true, dev);
    });
}

int gdist_greedy_reps(gdist_ctx* ctx, const gdist_sets* sets, int method, double max_dist, const int64_t* tie_rank,
                      int32_t* is_rep, int64_t* rep_of, double* rep_dist, int64_t* nreps) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        check_sets(sets);
        GD_REQUIRE(sets->ctx == ctx, "sets belong to another context");
        GD_REQUIRE(sets->kind != GDIST_SKETCH, "representatives are chosen on kmer sets");
        GD_REQUIRE(is_rep != nullptr, "is_rep is required");
        GD_REQUIRE(method >= GDIST_METHOD_AUTO && method <= GDIST_METHOD_BITSET, "unknown method");
        std::lock_guard<std::recursive_mutex> lk(ctx->mu);
        auto* s = const_cast<gdist_sets*>(sets);
        const int64_t n = s->nsets;
        const int m = resolve_method(ctx, s, method, (double)n * (double)n);
        ctx->last = Timing{};
        greedy_reps(ctx, s, m, max_dist, tie_rank, is_rep, rep_of, rep_dist, nreps);
    });
}

int gdist_row_query(gdist_ctx* ctx, const gdist_sets* sets, int64_t q, const int64_t* cols, int64_t ncols, int mode,
                    double t, double* D_out, int32_t* hit, int64_t* best_idx, double* best_d) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        check_sets(sets);
        GD_REQUIRE(sets->ctx == ctx, "sets belong to another context");
        GD_REQUIRE(sets->kind != GDIST_SKETCH, "row queries run on kmer sets");
        GD_REQUIRE(q >= 0 && q < sets->nsets, "query index out of range");
        GD_REQUIRE(ncols >= 0 && (ncols == 0 || cols), "bad column list");
        GD_REQUIRE(mode >= GDIST_QUERY_ALL && mode <= GDIST_QUERY_ARGMIN, "unknown query mode");
        for (int64_t c = 0; c < ncols; c++) GD_REQUIRE(cols[c] >= 0 && cols[c] < sets->nsets, "column index out of range");
        std::lock_guard<std::recursive_mutex> lk(ctx->mu);
        auto* s = const_cast<gdist_sets*>(sets);
        GD_REQUIRE(s->bits.p || s->has_codes, "this collection holds bitsets only");
        hipStream_t st = ctx->stream;
        std::vector<double> d(ncols);
        if (ncols) {
            DevBuf dc(ncols * 8, st), dI(ncols * 4, st), dD(ncols * 8, st);
            h2d(dc.p, cols, ncols * 8, st);
            if (s->bits.p) {
                bitset_row(ctx, s, q, dc.as<int64_t>(), ncols, dI.as<int32_t>());
            } else {
                if (!s->segoff.p) build_segments(ctx, s);
                sorted_row(ctx, s, q, dc.as<int64_t>(), ncols, dI.as<int32_t>());
            }
            row_epilogue(ctx, s, q, dc.as<int64_t>(), ncols, 0, dI.as<int32_t>(), dD.as<double>());
            d2h(d.data(), dD.p, ncols * 8, st);
            GD_HIP(hipStreamSynchronize(st));
        }
        if (D_out) std::memcpy(D_out, d.data(), ncols * 8);
        if (mode == GDIST_QUERY_ANY_LE && hit) {
            // anyMatch(x -> x.distance(kmers) <= maxDist), DistanceRepsProcessor.java:190
            int32_t h = 0;
            for (int64_t c = 0; c < ncols; c++) if (d[c] <= t) { h = 1; break; }
            *hit = h;
        }
        if (mode == GDIST_QUERY_ARGMIN) {
            // reduce(NULL_RESULT, (x,y) -> x.distance <= y.distance ? x : y),
            // DistanceRepsProcessor.java:108-122,238-239: the 1.0 identity wins ties at 1.0
            int64_t bi = -1;
            double bd = 1.0;
            for (int64_t c = 0; c < ncols; c++) if (d[c] < bd) { bd = d[c]; bi = c; }
            if (best_idx) *best_idx = bi;
            if (best_d) *best_d = bd;
        }
    });
}

// ---------------------------------------------------------------------------
int gdist_sketch_build(gdist_ctx* ctx, const gdist_sets* sets, int width, gdist_sets** out) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        check_codes(sets);
        GD_REQUIRE(out, "null output");
        *out = nullptr;
        std::lock_guard<std::recursive_mutex> lk(ctx->mu);
        auto* s = new gdist_sets();
        s->ctx = ctx;
        try {
            sketch_build(ctx, sets, width, s);
        } catch (...) {
            delete s;
            throw;
        }
        *out = s;
    });
}

int gdist_sketch_upload(gdist_ctx* ctx, int width, int64_t nsets, const int64_t* offsets, const int32_t* sigs,
                        gdist_sets** out) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        GD_REQUIRE(out && nsets >= 0 && offsets && width > 0, "bad sketch upload arguments");
        *out = nullptr;
        GD_REQUIRE(offsets[0] == 0, "offsets[0] must be 0");
        for (int64_t s = 0; s < nsets; s++) {
            GD_REQUIRE(offsets[s + 1] >= offsets[s] && offsets[s + 1] - offsets[s] <= width,
                       "each signature holds at most `width` hashes");
            for (int64_t e = offsets[s] + 1; e < offsets[s + 1]; e++)
                GD_REQUIRE(sigs[e - 1] < sigs[e], "signatures must be sorted ascending and unique");
        }
        std::lock_guard<std::recursive_mutex> lk(ctx->mu);
        const int64_t total = offsets[nsets];
        auto* s = new gdist_sets();
        s->ctx = ctx; s->kind = GDIST_SKETCH; s->width = width; s->nsets = nsets; s->total = total;
        s->h_off.assign(offsets, offsets + nsets + 1);
        s->off.alloc((nsets + 1) * 8, ctx->stream);
        s->codes.alloc(total * 4 + 4, ctx->stream);
        h2d(s->off.p, offsets, (nsets + 1) * 8, ctx->stream);
        if (total) h2d(s->codes.p, sigs, total * 4, ctx->stream);
        GD_HIP(hipStreamSynchronize(ctx->stream));
        *out = s;
    });
}

int gdist_sketch_download(const gdist_sets* sk, int64_t* offsets, int32_t* sigs) {
    return guard([&] {
        check_codes(sk);
        GD_REQUIRE(sk->kind == GDIST_SKETCH, "not a sketch collection");
        use_device(sk->ctx);
        std::lock_guard<std::recursive_mutex> lk_(sk->ctx->mu);
        if (offsets) std::memcpy(offsets, sk->h_off.data(), (sk->nsets + 1) * 8);
        if (sigs && sk->total)
            d2h(sigs, sk->codes.p, sk->total * 4, sk->ctx->stream);
        GD_HIP(hipStreamSynchronize(sk->ctx->stream));
    });
}

int gdist_sketch_matrix(gdist_ctx* ctx, const gdist_sets* sk, int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                        unsigned flags, int32_t* common_out, double* D_out, int64_t ld) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        check_codes(sk);
        GD_REQUIRE(sk->ctx == ctx, "sketches belong to another context");
        GD_REQUIRE(sk->kind == GDIST_SKETCH, "not a sketch collection");
        GD_REQUIRE(0 <= r0 && r0 <= r1 && r1 <= sk->nsets && 0 <= c0 && c0 <= c1 && c1 <= sk->nsets,
                   "row/column range outside the sketch collection");
        const int64_t nr = r1 - r0, nc = c1 - c0;
        GD_REQUIRE(ld >= nc, "leading dimension smaller than the column range");
        std::lock_guard<std::recursive_mutex> lk(ctx->mu);
        hipStream_t st = ctx->stream;
        ctx->pending = false;          // an unread previous call's times are dropped, not waited for
        ctx->last = Timing{};
        gdist::begin_timing(ctx);
        GD_HIP(hipEventRecord(ctx->ev_call0, st));
        if (nr == 0 || nc == 0) {
            gdist::finish_timing(ctx, false);
            return;
        }
        const bool dev = (flags & GDIST_OUT_DEVICE) != 0;
        const bool upper = (flags & GDIST_UPPER_TRIANGLE) != 0;
        DevBuf tC, tD;
        int32_t* dC = nullptr;
        double* dD = nullptr;
        int64_t ldo = ld;
        if (dev) {
            dC = common_out; dD = D_out;
        } else {
            ldo = nc;
            if (common_out) { tC.alloc((size_t)nr * nc * 4, st); dC = tC.as<int32_t>(); }
            if (D_out) { tD.alloc((size_t)nr * nc * 8, st); dD = tD.as<double>(); }
        }
        sketch_matrix(ctx, sk, r0, r1, c0, c1, flags, dC, dD, ldo);
        if (!dev) {
            if (dC) copy_out_rows(ctx, dC, 4, nr, nc, r0, c0, upper, common_out, ld);
            if (dD) copy_out_rows(ctx, dD, 8, nr, nc, r0, c0, upper, D_out, ld);
        }
        gdist::finish_timing(ctx, true, dev);
    });
}

// ---------------------------------------------------------------------------
int gdist_lsh_build(gdist_ctx* ctx, const gdist_sets* sketches, int stages, int buckets, uint64_t seed,
                    gdist_lsh** out) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        check_codes(sketches);
        GD_REQUIRE(out, "null output");
        *out = nullptr;
        auto* L = new gdist_lsh();
        try {
            gdist::lsh_build(ctx, sketches, stages, buckets, seed, L);
        } catch (...) {
            delete L;
            throw;
        }
        *out = L;
    });
}

int gdist_lsh_free(gdist_lsh* lsh) {
    return guard([&] {
        if (!lsh) return;
        (void)hipSetDevice(lsh->ctx->device);
        delete lsh;
    });
}

int gdist_lsh_closest(gdist_ctx* ctx, const gdist_lsh* lsh, const gdist_sets* queries, int n, double max_dist,
                      int64_t* idx_out, double* d_out, int32_t* count_out) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        GD_REQUIRE(lsh && lsh->ctx == ctx, "index of another context");
        check_codes(queries);
        GD_REQUIRE(count_out && (n == 0 || (idx_out && d_out)), "null output");
        gdist::lsh_closest(ctx, lsh, queries, n, max_dist, idx_out, d_out, count_out);
    });
}

int gdist_comm_unique_id(char id[GDIST_UNIQUE_ID_BYTES]) {
    return guard([&] {
        static_assert(sizeof(ncclUniqueId) <= GDIST_UNIQUE_ID_BYTES, "unique id size");
        ncclUniqueId u;
        GD_NCCL(ncclGetUniqueId(&u));
        std::memset(id, 0, GDIST_UNIQUE_ID_BYTES);
        std::memcpy(id, &u, sizeof(u));
    });
}

int gdist_comm_init(gdist_ctx* ctx, const char id[GDIST_UNIQUE_ID_BYTES], int nranks, int rank) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        GD_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank / world size");
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        if (ctx->comm) { (void)ncclCommDestroy(ctx->comm); ctx->comm = nullptr; }
        ctx->host_ag = nullptr;
        GD_NCCL(ncclCommInitRank(&ctx->comm, nranks, u, rank));
        ctx->nranks = nranks;
        ctx->rank = rank;
    });
}

int gdist_comm_init_host(gdist_ctx* ctx, int nranks, int rank, gdist_allgather_fn fn, void* user) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        GD_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank / world size");
        GD_REQUIRE(fn != nullptr, "null all-gather callback");
        if (ctx->comm) { (void)ncclCommDestroy(ctx->comm); ctx->comm = nullptr; }
        ctx->host_ag = fn;
        ctx->host_user = user;
        ctx->nranks = nranks;
        ctx->rank = rank;
    });
}

int gdist_comm_destroy(gdist_ctx* ctx) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        if (ctx->comm) GD_NCCL(ncclCommDestroy(ctx->comm));
        ctx->comm = nullptr;
        ctx->host_ag = nullptr;
        ctx->host_user = nullptr;
        ctx->nranks = 1;
        ctx->rank = 0;
    });
}

// The code all-gather (one all-gather of the packed sets). Each
// rank places its codes in its slot of one padded receive buffer and the
// gather runs in place (RCCL: sendbuff = recvbuff + rank * count), so no send
// copy exists; with GDIST_ALLGATHER_CONSUME the local codes are released as
// soon as they sit in that slot. The padded slots are then compacted in rank
// order through one staging buffer of the largest shard. Peak device bytes
// per rank: R x the largest shard (the gather) + one shard (staging or the
// local codes), e.g. C4 on 8 GPUs: 160 + 20 GB.
int gdist_sets_allgather_ex(gdist_ctx* ctx, gdist_sets* local, unsigned flags, gdist_sets** out) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        check_sets(local);
        GD_REQUIRE(out, "null output");
        GD_REQUIRE(local->has_codes, "the local collection holds no codes (bitset-only, or consumed by an all-gather)");
        GD_REQUIRE((flags & ~GDIST_ALLGATHER_CONSUME) == 0, "unknown all-gather flags");
        if (!has_comm(ctx)) throw ::gdist::Error(GDIST_ECOMM, "communicator not initialised (gdist_comm_init)");
        hipStream_t st = ctx->stream;
        const int R = ctx->nranks, me = ctx->rank;
        const size_t es = local->kind == GDIST_SKETCH ? 4 : 8;
        // 1. (nsets, total) of every rank
        DevBuf mine(16, st), all(16 * R, st);
        int64_t h2[2] = {local->nsets, local->total};
        h2d(mine.p, h2, 16, st);
        allgather(ctx, mine.p, all.p, 16);
        std::vector<int64_t> hall(2 * R);
        d2h(hall.data(), all.p, 16 * R, st);
        int64_t mxs = 0, mxt = 0, ns = 0, nt = 0;
        for (int r = 0; r < R; r++) {
            mxs = std::max(mxs, hall[2 * r]); mxt = std::max(mxt, hall[2 * r + 1]);
            ns += hall[2 * r]; nt += hall[2 * r + 1];
        }
        // 2. offsets (small: a send copy) and codes (in place), padded to the largest shard
        const size_t ob = (size_t)(mxs + 1) * 8, cb = (size_t)mxt * es + 8;
        std::vector<int64_t> hoff((mxs + 1) * R);
        {
            DevBuf so(ob, st), ao(ob * R, st);
            GD_HIP(hipMemcpyAsync(so.p, local->off.p, (local->nsets + 1) * 8, hipMemcpyDeviceToDevice, st));
            allgather(ctx, so.p, ao.p, ob);
            d2h(hoff.data(), ao.p, ob * R, st);
        }
        // rank 0's locus guides (pack time: the first sequences' windows) travel
        // with the gathered collection: the bitset build's locus order and the
        // variant tier's substitution keys read them (one small all-gather of
        // every rank's guides, padded; slot 0 kept)
        int64_t g0 = 0;
        DevBuf gcodes, gkeys;
        if (local->kind != GDIST_SKETCH) {
            DevBuf mg(8, st), ag(8 * R, st);
            h2d(mg.p, &local->n_guide, 8, st);
            allgather(ctx, mg.p, ag.p, 8);
            std::vector<int64_t> hg(R);
            d2h(hg.data(), ag.p, 8 * R, st);
            int64_t mx = 0;
            for (int64_t v : hg) mx = std::max(mx, v);
            g0 = hg[0];
            if (mx > 0) {
                const size_t gb = (size_t)mx * 16;
                DevBuf sg(gb, st), all(gb * R, st);
                GD_HIP(hipMemsetAsync(sg.p, 0, gb, st));
                if (local->n_guide) {
                    GD_HIP(hipMemcpyAsync(sg.p, local->guide_codes.p, local->n_guide * 8, hipMemcpyDeviceToDevice, st));
                    GD_HIP(hipMemcpyAsync(static_cast<char*>(sg.p) + mx * 8, local->guide_keys.p, local->n_guide * 8,
                                          hipMemcpyDeviceToDevice, st));
                }
                allgather(ctx, sg.p, all.p, gb);
                gcodes.alloc(g0 * 8 + 8, st);
                gkeys.alloc(g0 * 8 + 8, st);
                if (g0) {
                    GD_HIP(hipMemcpyAsync(gcodes.p, all.p, g0 * 8, hipMemcpyDeviceToDevice, st));
                    GD_HIP(hipMemcpyAsync(gkeys.p, static_cast<char*>(all.p) + mx * 8, g0 * 8, hipMemcpyDeviceToDevice,
                                          st));
                }
                GD_HIP(hipStreamSynchronize(st));
            }
        }
        const bool consume = (flags & GDIST_ALLGATHER_CONSUME) != 0;
        DevBuf ac;
        if (consume && R == 1 && local->codes.bytes >= cb) {
            ac = std::move(local->codes);            // one rank: the gather buffer is the shard itself
        } else {
            ac.alloc(cb * R, st);
            char* slot = static_cast<char*>(ac.p) + cb * me;
            if (local->total)
                GD_HIP(hipMemcpyAsync(slot, local->codes.p, local->total * es, hipMemcpyDeviceToDevice, st));
        }
        if (consume) {
            // the local collection keeps its sizes (h_off) but no device data
            GD_HIP(hipStreamSynchronize(st));
            free_bitsets(local);
            local->codes.release();
            local->segoff.release();
            local->guide_codes.release();
            local->guide_keys.release();
            local->pack_sum.clear();
            local->has_codes = false;
            gdist::cache_trim(ctx->device);           // the gather buffer may need that memory back
        }
        allgather_inplace(ctx, ac.p, cb);
        // 3. compact the slots in rank order: slot r's codes move down to the
        // sum of the earlier ranks' totals (staged: source and destination overlap)
        auto* s = new gdist_sets();
        std::unique_ptr<gdist_sets> guard_s(s);
        s->ctx = ctx; s->kind = local->kind; s->k = local->k; s->flags = local->flags; s->width = local->width;
        s->nsets = ns; s->total = nt;
        s->h_off.assign(1, 0);
        int64_t at = 0;
        {
            DevBuf stage(R > 1 ? mxt * es + 8 : 8, st);
            for (int r = 0; r < R; r++) {
                const int64_t rn = hall[2 * r], rt = hall[2 * r + 1];
                for (int64_t i = 1; i <= rn; i++) s->h_off.push_back(at + hoff[(mxs + 1) * r + i]);
                char* src = static_cast<char*>(ac.p) + cb * r;
                char* dst = static_cast<char*>(ac.p) + at * es;
                if (rt && src != dst) {
                    GD_HIP(hipMemcpyAsync(stage.p, src, rt * es, hipMemcpyDeviceToDevice, st));
                    GD_HIP(hipMemcpyAsync(dst, stage.p, rt * es, hipMemcpyDeviceToDevice, st));
                }
                at += rt;
            }
            GD_HIP(hipStreamSynchronize(st));
        }
        s->codes = std::move(ac);                     // R x cb bytes; the compacted codes first
        s->replicated = true;                         // the same collection on every rank
        s->guide_codes = std::move(gcodes);
        s->guide_keys = std::move(gkeys);
        s->n_guide = g0;
        s->off.alloc((ns + 1) * 8, st);
        h2d(s->off.p, s->h_off.data(), (ns + 1) * 8, st);
        GD_HIP(hipStreamSynchronize(st));
        *out = guard_s.release();
    });
}

int gdist_sets_allgather(gdist_ctx* ctx, const gdist_sets* local, gdist_sets** out) {
    return gdist_sets_allgather_ex(ctx, const_cast<gdist_sets*>(local), 0, out);
}

// Per-rank peak device bytes of the two exchanges (estimates) and the choice.
// Collective: one all-gather of (nsets, codes, summary bound) per rank, then
// the same arithmetic on every rank.
int gdist_sets_exchange_plan(gdist_ctx* ctx, const gdist_sets* local, int method, int* chosen, double* bytes_bitsets,
                             double* bytes_codes) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        check_sets(local);
        GD_REQUIRE(chosen, "null output");
        GD_REQUIRE(method >= GDIST_METHOD_AUTO && method <= GDIST_METHOD_BITSET, "unknown method");
        GD_REQUIRE(local->has_codes, "the local collection holds no codes");
        hipStream_t st = ctx->stream;
        const int R = has_comm(ctx) ? ctx->nranks : 1;
        // the dictionary summary's length is at most the sum of the pack
        // chunks' summaries when the pack kept them, else the codes themselves
        int64_t sum_n = 0;
        for (const auto& p : local->pack_sum) sum_n += p.n;
        if (local->pack_sum.empty()) sum_n = local->total;
        std::vector<int64_t> h(3 * R);
        h[0] = local->nsets; h[1] = local->total; h[2] = sum_n;
        if (R > 1) {
            DevBuf mine(24, st), all(24 * R, st);
            h2d(mine.p, h.data(), 24, st);
            allgather(ctx, mine.p, all.p, 24);
            d2h(h.data(), all.p, 24 * R, st);
        }
        double mxt = 0, mxn = 0;
        for (int r = 0; r < R; r++) { mxt = std::max(mxt, (double)h[3 * r + 1]); mxn = std::max(mxn, (double)h[3 * r + 2]); }
        const double es = local->kind == GDIST_SKETCH ? 4.0 : 8.0;
        // codes (the local shard consumed, GDIST_ALLGATHER_CONSUME): the padded
        // gather + one shard (the local codes while they are copied into their
        // slot, then the compaction's staging); one rank adopts its own buffer
        const double b_codes = R == 1 ? mxt * es : ((double)R + 1.0) * mxt * es;
        // bitsets: the local codes + the gathered summaries (12 B per
        // distinct code) + the merge's workspace (~2x them) + the bitsets the
        // exchange allocates: every set's words (N_total x W) and the R x
        // (largest shard) x W gather buffer, W bounded by the distinct codes
        // (min(R x largest summary, sum of summaries) / 64)
        double n_total = 0, mxs = 0, sum_all = 0;
        for (int r = 0; r < R; r++) {
            n_total += (double)h[3 * r];
            mxs = std::max(mxs, (double)h[3 * r]);
            sum_all += (double)h[3 * r + 2];
        }
        const double w_bound = std::ceil(std::min((double)R * mxn, sum_all) / 64.0);
        const double b_bits = local->kind == GDIST_SKETCH
                                  ? INFINITY
                                  : mxt * 8.0 + 3.0 * (double)R * mxn * 12.0 +
                                        (n_total + (double)R * mxs) * w_bound * 8.0;
        hipDeviceProp_t prop;
        GD_HIP(hipGetDeviceProperties(&prop, ctx->device));
        const double budget = ctx->has_option(OPT_EXCHANGE_BUDGET) ? (double)ctx->option(OPT_EXCHANGE_BUDGET, 0)
                                                                    : 0.8 * (double)prop.totalGlobalMem;
        int m = method;
        if (m == GDIST_METHOD_AUTO) m = b_bits <= budget ? GDIST_METHOD_BITSET : GDIST_METHOD_SORTED;
        if (local->kind == GDIST_SKETCH) m = GDIST_METHOD_SORTED;
        if (ctx->trace())
            fprintf(stderr, "gdist: exchange plan: bitsets ~%.1f GB, codes ~%.1f GB per rank, budget %.1f GB -> %s\n",
                    b_bits / 1e9, b_codes / 1e9, budget / 1e9, m == GDIST_METHOD_BITSET ? "bitsets" : "codes");
        if (m == GDIST_METHOD_SORTED && b_codes > budget)
            throw Error(GDIST_ENOMEM, "neither exchange fits the device memory budget (option exchange_budget)");
        *chosen = m;
        if (bytes_bitsets) *bytes_bitsets = b_bits;
        if (bytes_codes) *bytes_codes = b_codes;
    });
}

int gdist_sets_allgather_bitsets(gdist_ctx* ctx, const gdist_sets* local, unsigned flags, gdist_sets** out) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        check_sets(local);
        GD_REQUIRE(out, "null output");
        GD_REQUIRE(local->kind != GDIST_SKETCH && local->has_codes, "local kmer sets with codes required");
        std::lock_guard<std::recursive_mutex> lk(ctx->mu);
        hipStream_t st = ctx->stream;
        const int R = has_comm(ctx) ? ctx->nranks : 1;
        // every exchange runs when there are peers, or on a one-rank
        // communicator with option force_exchange (runs the RCCL calls on a
        // one-GPU box; the result must equal the local build)
        const bool xchg = R > 1 || (has_comm(ctx) && ctx->option(OPT_FORCE_EXCHANGE, 0) != 0);
        const bool keep = (flags & GDIST_BITSET_KEEP_SINGLETONS) != 0;
        // 1. local dictionary summary
        Summary sum;
        local_summary(ctx, local, sum);
        // 2. every rank's (nsets, summary length)
        std::vector<int64_t> hall(2 * R);
        hall[0] = local->nsets; hall[1] = sum.n;
        if (xchg) {
            DevBuf mine(16, st), all(16 * R, st);
            h2d(mine.p, hall.data(), 16, st);
            allgather(ctx, mine.p, all.p, 16);
            d2h(hall.data(), all.p, 16 * R, st);
            GD_HIP(hipStreamSynchronize(st));
        }
        int64_t mxs = 0, mxn = 0, N = 0;
        for (int r = 0; r < R; r++) { mxs = std::max(mxs, hall[2 * r]); mxn = std::max(mxn, hall[2 * r + 1]); N += hall[2 * r]; }
        // 3. all-gather the summaries (padded), merge into the global dictionary
        DevBuf gc, gn;
        std::vector<SummaryView> parts;
        if (xchg) {
            DevBuf sc(mxn * 8 + 8, st), sn(mxn * 4 + 4, st);
            if (sum.n) {
                GD_HIP(hipMemcpyAsync(sc.p, sum.codes.p, sum.n * 8, hipMemcpyDeviceToDevice, st));
                GD_HIP(hipMemcpyAsync(sn.p, sum.counts.p, sum.n * 4, hipMemcpyDeviceToDevice, st));
            }
            gc.alloc((mxn * 8 + 8) * R, st);
            gn.alloc((mxn * 4 + 4) * R, st);
            allgather(ctx, sc.p, gc.p, mxn * 8 + 8);
            allgather(ctx, sn.p, gn.p, mxn * 4 + 4);
            for (int r = 0; r < R; r++)
                parts.push_back({reinterpret_cast<const uint64_t*>((char*)gc.p + (mxn * 8 + 8) * r),
                                 reinterpret_cast<const uint32_t*>((char*)gn.p + (mxn * 4 + 4) * r), hall[2 * r + 1]});
        } else {
            parts.push_back({sum.codes.as<uint64_t>(), sum.counts.as<uint32_t>(), sum.n});
        }
        DevBuf dict, rare, dcnt;
        int64_t U = 0, Ur = 0, mass_all = 0;
        int64_t T = keep ? 0 : -1;                 // cost-optimal from the global count histogram
        dictionary_from(ctx, parts, keep, T, N, dict, U, rare, Ur, mass_all, &dcnt);
        gc.release(); gn.release();
        const int64_t W = bitset_words(U);
        // 4. local bitsets (padded to the largest shard) + local rare-tier records
        int64_t id_base = 0;
        for (int r = 0; r < ctx->rank && xchg; r++) id_base += hall[2 * r];
        const int64_t cap = local_rare_mass(ctx, sum, rare.as<uint64_t>(), Ur);
        // locus order of the dense ranks: every rank keys them by its own
        // guides (tagged with the rank, so rank 0's guides come first), one
        // all-gather, the minimum over ranks -> the same permutation everywhere
        DevBuf perm;
        if (locus_order_enabled(ctx)) {
            DevBuf key;
            locus_keys(ctx, local, dict.as<uint64_t>(), dcnt.as<uint32_t>(), U, (uint64_t)ctx->rank << 40, key);
            if (xchg) {
                DevBuf allk((U * 8 + 8) * R, st);
                allgather(ctx, key.p, allk.p, U * 8 + 8);
                locus_keys_min(ctx, allk.as<uint64_t>(), U, U + 1, R, key);
            }
            locus_perm(ctx, key, U, perm);
        }
        DevBuf lb((size_t)mxs * W * 8 + 8, st), lrec(cap * 8 + 8, st);
        int64_t written = 0;
        if (local->nsets)
            fill_bits(ctx, local, dict.as<uint64_t>(), U, W, lb.as<unsigned long long>(), rare.as<uint64_t>(), Ur,
                      id_base, lrec.as<unsigned long long>(), cap, &written, perm.as<uint32_t>());
        auto* s = new gdist_sets();
        s->ctx = ctx; s->kind = local->kind; s->k = local->k; s->flags = local->flags;
        s->nsets = N; s->has_codes = false;
        s->fp4.release();                    // the MFMA operand expanded the old bits
        s->fp4_W = 0;
        s->bits.alloc((size_t)N * W * 8 + 8, st);
        if (xchg) {
            DevBuf gb((size_t)mxs * W * 8 * R + 8, st);
            allgather(ctx, lb.p, gb.p, (size_t)mxs * W * 8);
            int64_t at = 0;
            for (int r = 0; r < R; r++) {
                if (hall[2 * r])
                    GD_HIP(hipMemcpyAsync(s->bits.as<uint64_t>() + at * W, gb.as<uint64_t>() + (size_t)mxs * W * r,
                                          (size_t)hall[2 * r] * W * 8, hipMemcpyDeviceToDevice, st));
                at += hall[2 * r];
            }
            GD_HIP(hipStreamSynchronize(st));
        } else if (N) {
            GD_HIP(hipMemcpyAsync(s->bits.p, lb.p, (size_t)N * W * 8, hipMemcpyDeviceToDevice, st));
        }
        // 5. set sizes of all ranks (one all-gather of the padded size arrays)
        std::vector<int64_t> sizes(mxs + 1, 0), allsz((mxs + 1) * R, 0);
        for (int64_t i = 0; i < local->nsets; i++) sizes[i] = local->h_off[i + 1] - local->h_off[i];
        if (xchg) {
            DevBuf ds((mxs + 1) * 8, st), da((mxs + 1) * 8 * R, st);
            h2d(ds.p, sizes.data(), (mxs + 1) * 8, st);
            allgather(ctx, ds.p, da.p, (mxs + 1) * 8);
            d2h(allsz.data(), da.p, (mxs + 1) * 8 * R, st);
            GD_HIP(hipStreamSynchronize(st));
        } else {
            allsz = sizes;
        }
        s->h_off.assign(1, 0);
        for (int r = 0; r < R; r++)
            for (int64_t i = 0; i < hall[2 * r]; i++) s->h_off.push_back(s->h_off.back() + allsz[(mxs + 1) * r + i]);
        s->total = s->h_off.back();
        s->off.alloc((N + 1) * 8, st);
        h2d(s->off.p, s->h_off.data(), (N + 1) * 8, st);
        s->codes.alloc(8, st);
        s->W = W; s->dict_size = U; s->bits_keep_singletons = keep;
        // 6. rare-tier records of every rank (one all-gather), posting lists
        std::vector<int64_t> wr(R, 0);
        wr[0] = written;
        int64_t mxw = written, totw = written;
        if (xchg) {
            DevBuf mw(8, st), aw(8 * R, st);
            h2d(mw.p, &written, 8, st);
            allgather(ctx, mw.p, aw.p, 8);
            d2h(wr.data(), aw.p, 8 * R, st);
            mxw = 0; totw = 0;
            for (int r = 0; r < R; r++) { mxw = std::max(mxw, wr[r]); totw += wr[r]; }
            DevBuf ga((size_t)(mxw + 1) * 8 * R, st), allrec(totw * 8 + 8, st);
            DevBuf pad((mxw + 1) * 8, st);
            if (written) GD_HIP(hipMemcpyAsync(pad.p, lrec.p, written * 8, hipMemcpyDeviceToDevice, st));
            allgather(ctx, pad.p, ga.p, (mxw + 1) * 8);
            int64_t at = 0;
            for (int r = 0; r < R; r++) {
                if (wr[r])
                    GD_HIP(hipMemcpyAsync(allrec.as<uint64_t>() + at, ga.as<uint64_t>() + (mxw + 1) * r, wr[r] * 8,
                                          hipMemcpyDeviceToDevice, st));
                at += wr[r];
            }
            build_postings(ctx, s, allrec.as<unsigned long long>(), totw, Ur);
        } else {
            build_postings(ctx, s, lrec.as<unsigned long long>(), written, Ur);
        }
        s->rare_T = T;
        build_sparse_words(ctx, s);
        GD_HIP(hipStreamSynchronize(st));
        *out = s;
    });
}

int gdist_comm_allreduce_max(gdist_ctx* ctx, double* value) {
    return guard([&] {
        use_device(ctx);
        std::lock_guard<std::recursive_mutex> lk_(ctx->mu);
        GD_REQUIRE(value, "null value");
        if (!has_comm(ctx)) return;
        DevBuf d(8, ctx->stream), all(8 * ctx->nranks, ctx->stream);
        h2d(d.p, value, 8, ctx->stream);
        allgather(ctx, d.p, all.p, 8);
        std::vector<double> h(ctx->nranks);
        d2h(h.data(), all.p, 8 * ctx->nranks, ctx->stream);
        GD_HIP(hipStreamSynchronize(ctx->stream));
        *value = *std::max_element(h.begin(), h.end());
    });
}

int gdist_sets_block_cost(const gdist_sets* sets, int64_t r0, int64_t r1, int64_t c0, int64_t c1, int upper,
                          double* seconds, int* rare_kernel) {
    return guard([&] {
        check_sets(sets);
        GD_REQUIRE(0 <= r0 && r0 <= r1 && r1 <= sets->nsets && 0 <= c0 && c0 <= c1 && c1 <= sets->nsets,
                   "block out of range");
        int rk = -1;
        double t;
        if (sets->bits.p) {
            bool row_major = false;
            t = bitset_block_cost_s(sets, r0, r1, c0, c1, upper != 0, &row_major);
            if (sets->n_rare > 0) rk = row_major ? 1 : 0;
        } else {
            t = sorted_cost_s(sets, block_pairs(r0, r1, c0, c1, upper != 0));
        }
        if (seconds) *seconds = t;
        if (rare_kernel) *rare_kernel = rk;
    });
}

int gdist_triangle_partition(int64_t n, int nparts, int64_t align, int64_t* bounds) {
    return guard([&] {
        GD_REQUIRE(n >= 0 && nparts >= 1 && align >= 1 && bounds, "bad partition arguments");
        bounds[0] = 0;
        for (int g = 1; g < nparts; g++) {
            const double r = (double)n * (1.0 - std::sqrt(1.0 - (double)g / (double)nparts));
            int64_t b = (int64_t)std::llround(r / (double)align) * align;
            b = std::min<int64_t>(n, std::max<int64_t>(bounds[g - 1], b));
            bounds[g] = b;
        }
        bounds[nparts] = n;
    });
}

}  // extern "C"
