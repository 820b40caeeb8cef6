// C ABI of libfdfs_gpu (include/fdfs_gpu.h): context, workspace and argument
// checking around the kernels.  No CPU compute path exists: every result
// comes from a gfx950 kernel, and a missing/failed device is an error.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/fdfs_gpu.h"
#include "fdfs_device.hpp"
#include "fdfs_kernels.hpp"

struct fdfs_gpu_ctx {
    int device = 0;
    unsigned flags = 0;
    bool sar = true;
    fdfs::DevTables *d_tabs = nullptr;
    uint32_t lat_files = 0;  // lane batches up to one wave per SIMD (BigCrcWs::lat_files)
    uint32_t ncu = 0;        // the device's CU count, read once at open (BigCrcWs::ncu)
    uint64_t lane_err_seen = 0;  // lane-path error count already reported (lane_err_check)
    uint32_t lane_err_next = 0;  // the next launch's slot of the error-count ring (lane_err_note)
    void *ws = nullptr;
    size_t ws_bytes = 0;
    char err[256] = {0};
    // kernel timing (fdfs_gpu_set_timing)
    bool timing = false;
    struct Rec {
        hipEvent_t a, b;
        int kernel;
    };
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;
    double acc_ms[4] = {0, 0, 0, 0};
    uint64_t acc_n[4] = {0, 0, 0, 0};
    // One call at a time per context (host threads serialise here; entry
    // points that call other entry points re-enter on the same thread).
    std::recursive_mutex mu;
    // The workspace is shared by every call: ws_ev is recorded on the stream
    // of the last call that used it, and a call on another stream waits for
    // it first, so calls on different streams never overlap on ws.
    hipEvent_t ws_ev = nullptr;
    hipStream_t ws_st = nullptr;
    bool ws_rec = false;
    // fdfs_gpu_dedup_global: exchange buffers (ordered like ws), and the
    // announcement words every rank all-gathers before the row exchange
    // (device: this rank's, then all ranks'; host: tail staging, all ranks',
    // the agreement flag), allocated at open so that no rank can fail before
    // its first collective
    void *xa = nullptr, *xb = nullptr;
    size_t xa_bytes = 0, xb_bytes = 0;
    uint64_t *dann = nullptr, *hann = nullptr;
    // lane_err_note's per-slot events: a slot is reused only once the copy
    // that last wrote it has landed
    hipEvent_t err_ev[64] = {};
    bool err_ev_rec[64] = {};
    // bytes the last dedup_global(_local) call moved between ranks: rows,
    // answers (fdfs_gpu_dedup_global_stats)
    uint64_t x_row_bytes = 0, x_ans_bytes = 0;
};

namespace {

struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess)
            prev = -1;
        ok = (prev == dev) || (hipSetDevice(dev) == hipSuccess);
    }
    ~DeviceGuard()
    {
        if (prev >= 0)
            (void)hipSetDevice(prev);
    }
};

int fail(fdfs_gpu_ctx *ctx, hipError_t e, const char *where)
{
    if (ctx)
        std::snprintf(ctx->err, sizeof(ctx->err), "%s: %s", where, hipGetErrorString(e));
    return EIO;
}

constexpr size_t kAlign = 256;
size_t align_up(size_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

// Bump allocator over the context workspace.
struct Carve {
    char *base;
    size_t off = 0;
    template <typename T>
    T *take(size_t count)
    {
        T *p = reinterpret_cast<T *>(base + off);
        off += align_up(count * sizeof(T));
        return p;
    }
};

// CRC-only batches above this many waves per SIMD take the lane path.
#ifndef FDFS_CRC_LANE_MIN_FILL
#define FDFS_CRC_LANE_MIN_FILL 3
#endif
constexpr uint32_t kCrcLaneMinFill = FDFS_CRC_LANE_MIN_FILL;

size_t sig_ws_bytes(uint64_t n)
{
    size_t lane = align_up(sizeof(uint32_t) * fdfs::kLaneWsDwords) + align_up(sizeof(uint32_t) * n) +
                  align_up(sizeof(uint32_t)) + 2 * align_up(sizeof(uint64_t) * n) +
                  align_up(sizeof(uint64_t) * (n + 1)) + align_up(sizeof(uint32_t) * n) +
                  align_up(2 * sizeof(uint32_t) * n) + align_up(sizeof(uint64_t));  // + BigCrcWs
    size_t seg = align_up(sizeof(uint64_t) * 2 * n) + align_up(sizeof(uint64_t) * 2 * (n + 1)) +
                 align_up(sizeof(uint64_t) * 2 * fdfs::scan_workspace_elems(n));  // launch_crc_seg's two lists
    return lane > seg ? lane : seg;  // one path per call
}

// The big-file offload lists of the HASH lane path (sig_ws_bytes counts them).
fdfs::BigCrcWs carve_big(const fdfs_gpu_ctx *ctx, Carve &cv, uint32_t n)
{
    fdfs::BigCrcWs big;
    big.nbig = cv.take<uint32_t>(1);
    big.offs = cv.take<uint64_t>(n);
    big.sizes = cv.take<uint64_t>(n);
    big.seg_first = cv.take<uint64_t>((size_t)n + 1);
    big.crc = cv.take<uint32_t>(n);
    big.poly = cv.take<uint32_t>(2 * (size_t)n);
    big.big_min = cv.take<uint64_t>(1);
    big.lat_files = ctx->lat_files;
    big.ncu = ctx->ncu;
    return big;
}

size_t dedup_ws_bytes(uint64_t n) { return fdfs::dedup_ws_bytes(n) + align_up(8 * 64); }

// fdfs_gpu_dedup_global announcement: rank p's row count per owner (nranks
// words), then kAnnTail words {owner-side room, workspace room, errno, the
// capacity of each owner region of its send order (0: exact prefix layout)}.
constexpr int kAnnTail = 4;
constexpr size_t kAnnMax = 64 + kAnnTail;                   // words of one announcement
constexpr size_t kErrRing = 64;  // lane_err_note's per-launch slots
// fdfs_gpu_dedup_global's answer counts: every owner's sink-record count
// per segment (64 x u32 per rank), all-gathered, at the end of both areas
constexpr size_t kAnsAllWords = 64 * 64 / 2;
constexpr size_t kAnnDevWords = kAnnMax + 64 * kAnnMax + 8 + kErrRing + kAnsAllWords;  // own, all ranks', flag, ring, counts
constexpr size_t kAnnHostWords = 64 * kAnnTail + 64 * kAnnMax + 8 + kErrRing + kAnsAllWords;  // tails, all ranks', flag, ring, counts
constexpr size_t kAnsAllDev = kAnnMax + 64 * kAnnMax + 8 + kErrRing;
constexpr size_t kAnsAllHost = 64 * kAnnTail + 64 * kAnnMax + 8 + kErrRing;

bool capturing(hipStream_t st)
{
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

// Workspace ordering across streams (see fdfs_gpu_ctx::ws_ev).  Inside a
// stream capture nothing is recorded or waited on: a captured sequence must
// use one stream (include/fdfs_gpu.h).
void ws_enter(fdfs_gpu_ctx *ctx, hipStream_t st)
{
    if (ctx->ws_rec && ctx->ws_st != st && !capturing(st))
        (void)hipStreamWaitEvent(st, ctx->ws_ev, 0);
}

void ws_leave(fdfs_gpu_ctx *ctx, hipStream_t st)
{
    if (!capturing(st) && hipEventRecord(ctx->ws_ev, st) == hipSuccess) {
        ctx->ws_st = st;
        ctx->ws_rec = true;
    }
}

struct WsScope {
    fdfs_gpu_ctx *ctx;
    hipStream_t st;
    WsScope(fdfs_gpu_ctx *c, hipStream_t s) : ctx(c), st(s) { ws_enter(c, s); }
    ~WsScope() { ws_leave(ctx, st); }
};

// The lane path's device error word (fdfs::kLaneErrWord, zeroed with the
// histogram at every launch) feeds a per-context error COUNT: after each lane
// launch a one-thread kernel adds 1 to a device counter (a device-scope
// atomic: a context may be called on several streams) when the launch's word
// is set, and writes the new count to the launch's own slot of a ring, which
// is copied to the same slot of a pinned host ring.  The count only grows and
// every launch has its own slot, so no copy can erase another launch's count
// (one shared host word could go back: two calls on two streams, the older
// count's copy landing after the newer one).  The context's next call whose
// check sees a count (the ring's maximum) above the last one it reported
// fails with EIO.  Device: dann[kAnnErrCount] and the ring at
// dann[kAnnErrRing]; host ring: hann[kHannErrRing].
constexpr size_t kAnnErrCount = kAnnMax + 64 * kAnnMax + 6;
constexpr size_t kAnnErrRing = kAnnMax + 64 * kAnnMax + 8;
constexpr size_t kHannErrRing = 64 * kAnnTail + 64 * kAnnMax + 8;

hipError_t lane_err_note(fdfs_gpu_ctx *ctx, const uint32_t *hist, hipStream_t st)
{
    const uint32_t k = ctx->lane_err_next++ % kErrRing;  // under the context's mutex
    // Slot k was last written by the copy of launch k - 64, possibly on
    // another stream: wait for it before enqueueing this one, so that an
    // older count can never land after a newer one (almost
    // always long done).  Inside a stream capture nothing is recorded or
    // waited on: a captured graph replays into the one slot it captured.
    const bool cap = capturing(st);
    if (!cap && ctx->err_ev_rec[k]) {
        hipError_t e = hipEventSynchronize(ctx->err_ev[k]);
        if (e != hipSuccess)
            return e;
    }
    hipError_t e = fdfs::launch_lane_err_count(hist ? hist + fdfs::kLaneErrWord : nullptr, ctx->dann + kAnnErrCount,
                                               ctx->dann + kAnnErrRing + k, st);
    if (e == hipSuccess)
        e = hipMemcpyAsync(ctx->hann + kHannErrRing + k, ctx->dann + kAnnErrRing + k, 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess && !cap) {
        if (!ctx->err_ev[k])
            e = hipEventCreateWithFlags(&ctx->err_ev[k], hipEventDisableTiming);
        if (e == hipSuccess)
            e = hipEventRecord(ctx->err_ev[k], st);
        ctx->err_ev_rec[k] = e == hipSuccess;
    }
    return e;
}

int lane_err_check(fdfs_gpu_ctx *ctx)
{
    uint64_t v = 0;
    for (size_t k = 0; k < kErrRing; k++) {
        const uint64_t x = __atomic_load_n(ctx->hann + kHannErrRing + k, __ATOMIC_ACQUIRE);
        v = x > v ? x : v;
    }
    if (v <= ctx->lane_err_seen)
        return 0;
    ctx->lane_err_seen = v;
    std::snprintf(ctx->err, sizeof(ctx->err),
                  "an earlier signature call on this context found its size binning inconsistent "
                  "(%llu launch(es) so far): its outputs are invalid", (unsigned long long)v);
    return EIO;
}

// Grow a context-owned device buffer (like ensure_ws: the last call that
// used the context's buffers must be done before the old one is freed).
int ensure_buf(fdfs_gpu_ctx *ctx, void **buf, size_t *have, size_t bytes, hipStream_t st)
{
    if (bytes <= *have)
        return 0;
    if (capturing(st)) {
        std::snprintf(ctx->err, sizeof(ctx->err), "exchange buffer growth during stream capture");
        return ENOMEM;
    }
    if (*buf) {
        hipError_t e = ctx->ws_rec ? hipEventSynchronize(ctx->ws_ev) : hipSuccess;
        if (e == hipSuccess)
            e = hipStreamSynchronize(st);
        if (e != hipSuccess)
            return fail(ctx, e, "buffer growth sync");
        (void)hipFree(*buf);
        *buf = nullptr;
        *have = 0;
    }
    const size_t sz = bytes + bytes / 4;
    hipError_t e = hipMalloc(buf, sz);
    if (e != hipSuccess) {
        std::snprintf(ctx->err, sizeof(ctx->err), "hipMalloc(%zu): %s", sz, hipGetErrorString(e));
        return ENOMEM;
    }
    *have = sz;
    return 0;
}

int ensure_ws(fdfs_gpu_ctx *ctx, size_t bytes, hipStream_t st)
{
    if (bytes <= ctx->ws_bytes)
        return 0;
    if (capturing(st)) {
        std::snprintf(ctx->err, sizeof(ctx->err),
                      "workspace growth needed during stream capture; call fdfs_gpu_reserve first");
        return ENOMEM;
    }
    if (ctx->ws) {
        // the last call that used ws (on any stream) must be done with it
        hipError_t e = ctx->ws_rec ? hipEventSynchronize(ctx->ws_ev) : hipSuccess;
        if (e == hipSuccess)
            e = hipStreamSynchronize(st);
        if (e != hipSuccess)
            return fail(ctx, e, "workspace growth sync");
        (void)hipFree(ctx->ws);
        ctx->ws = nullptr;
        ctx->ws_bytes = 0;
    }
    size_t sz = bytes + bytes / 4;
    hipError_t e = hipMalloc(&ctx->ws, sz);
    if (e != hipSuccess) {
        std::snprintf(ctx->err, sizeof(ctx->err), "hipMalloc(%zu): %s", sz, hipGetErrorString(e));
        return ENOMEM;
    }
    ctx->ws_bytes = sz;
    return 0;
}

// Event pair for one main-kernel launch when timing is on, else nulls.
void timing_pair(fdfs_gpu_ctx *ctx, int kernel, hipEvent_t &a, hipEvent_t &b)
{
    a = b = nullptr;
    if (!ctx->timing)
        return;
    hipEvent_t ev[2] = {nullptr, nullptr};
    for (auto &e : ev) {
        if (!ctx->pool.empty()) {
            e = ctx->pool.back();
            ctx->pool.pop_back();
        } else if (hipEventCreate(&e) != hipSuccess) {
            e = nullptr;
        }
    }
    if (!ev[0] || !ev[1]) {
        for (auto e : ev)
            if (e)
                ctx->pool.push_back(e);
        return;
    }
    a = ev[0];
    b = ev[1];
    ctx->recs.push_back({a, b, kernel});
}

}  // namespace

extern "C" {

int fdfs_gpu_abi_version(void) { return FDFS_GPU_ABI_VERSION; }

int fdfs_gpu_open(int device, unsigned flags, fdfs_gpu_ctx **out)
{
    if (!out)
        return EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev)
        return ENODEV;
    fdfs_gpu_ctx *ctx = new (std::nothrow) fdfs_gpu_ctx;
    if (!ctx)
        return ENOMEM;
    ctx->device = device;
    ctx->flags = flags;
    ctx->sar = (flags & FDFS_GPU_FLAG_UNSIGNED_HASH) == 0;
    DeviceGuard g(device);
    if (!g.ok) {
        delete ctx;
        return ENODEV;
    }
    auto *h = new (std::nothrow) fdfs::DevTables;
    if (!h) {
        delete ctx;
        return ENOMEM;
    }
    if (!fdfs::build_crc_tables(h->t, ctx->sar)) {
        delete h;
        delete ctx;
        return EINVAL;
    }
    for (int p = 0; p < 16; p++)
        for (int x = 0; x < 256; x++)
            h->Dc[p][x] = h->t.D[p][x ^ 0xFF];
    fdfs::build_poly_mfma_tables(h->pm);
    hipError_t e = hipEventCreateWithFlags(&ctx->ws_ev, hipEventDisableTiming);
    if (e == hipSuccess)
        e = hipMalloc(&ctx->d_tabs, sizeof(fdfs::DevTables));
    if (e == hipSuccess)
        e = hipMemcpy(ctx->d_tabs, h, sizeof(fdfs::DevTables), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMalloc(reinterpret_cast<void **>(&ctx->dann), 8 * kAnnDevWords);
    if (e == hipSuccess)
        e = hipHostMalloc(reinterpret_cast<void **>(&ctx->hann), 8 * kAnnHostWords, 0);
    if (e == hipSuccess) {  // zeroed on a private stream: waits for nothing else on the device
        hipStream_t zs = nullptr;
        e = hipStreamCreateWithFlags(&zs, hipStreamNonBlocking);
        if (e == hipSuccess)
            e = hipMemsetAsync(ctx->dann, 0, 8 * kAnnDevWords, zs);
        if (e == hipSuccess)
            e = hipStreamSynchronize(zs);
        if (zs)
            (void)hipStreamDestroy(zs);
    }
    if (e == hipSuccess)
        std::memset(ctx->hann, 0, 8 * kAnnHostWords);
    delete h;
    if (e != hipSuccess) {
        if (ctx->d_tabs)
            (void)hipFree(ctx->d_tabs);
        if (ctx->dann)
            (void)hipFree(ctx->dann);
        if (ctx->hann)
            (void)hipHostFree(ctx->hann);
        if (ctx->ws_ev)
            (void)hipEventDestroy(ctx->ws_ev);
        delete ctx;
        return EIO;
    }
    hipDeviceProp_t prop;
    int ncu = 256;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        ncu = prop.multiProcessorCount;
    ctx->lat_files = (uint32_t)ncu * 4 * 64;
    ctx->ncu = (uint32_t)ncu;
    *out = ctx;
    return 0;
}

int fdfs_gpu_close(fdfs_gpu_ctx *ctx)
{
    if (!ctx)
        return EINVAL;
    DeviceGuard g(ctx->device);
    (void)hipDeviceSynchronize();
    if (ctx->ws)
        (void)hipFree(ctx->ws);
    if (ctx->xa)
        (void)hipFree(ctx->xa);
    if (ctx->xb)
        (void)hipFree(ctx->xb);
    if (ctx->dann)
        (void)hipFree(ctx->dann);
    if (ctx->hann)
        (void)hipHostFree(ctx->hann);
    for (auto &r : ctx->recs) {
        (void)hipEventDestroy(r.a);
        (void)hipEventDestroy(r.b);
    }
    for (auto e : ctx->pool)
        (void)hipEventDestroy(e);
    if (ctx->d_tabs)
        (void)hipFree(ctx->d_tabs);
    if (ctx->ws_ev)
        (void)hipEventDestroy(ctx->ws_ev);
    for (hipEvent_t e : ctx->err_ev)
        if (e)
            (void)hipEventDestroy(e);
    delete ctx;
    return 0;
}

int fdfs_gpu_reserve(fdfs_gpu_ctx *ctx, uint64_t max_files, uint64_t max_records)
{
    if (!ctx)
        return EINVAL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    size_t a = sig_ws_bytes(max_files), b = dedup_ws_bytes(max_records);
    return ensure_ws(ctx, a > b ? a : b, nullptr);
}

const char *fdfs_gpu_last_error(fdfs_gpu_ctx *ctx) { return ctx ? ctx->err : "null context"; }

#ifdef FDFS_TEST_HOOKS  // the test build only (make test-hooks): not in the shipped library
#include "fdfs_test_hooks.h"

int fdfs_gpu_inject_error(fdfs_gpu_ctx *ctx, void *stream)
{
    if (!ctx)
        return EINVAL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    const hipError_t e = lane_err_note(ctx, nullptr, reinterpret_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : fail(ctx, e, "inject_error");
}
#endif

int fdfs_gpu_set_timing(fdfs_gpu_ctx *ctx, int enable)
{
    if (!ctx)
        return EINVAL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    ctx->timing = enable != 0;
    return 0;
}

int fdfs_gpu_crc_lane_min_files(fdfs_gpu_ctx *ctx, uint64_t *min_files)
{
    if (!ctx || !min_files)
        return EINVAL;
    *min_files = (uint64_t)kCrcLaneMinFill * ctx->lat_files;
    return 0;
}

int fdfs_gpu_read_timing(fdfs_gpu_ctx *ctx, int kernel, double *ms_out, uint64_t *launches_out)
{
    if (!ctx || kernel < 0 || kernel > 3)
        return EINVAL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    for (auto &r : ctx->recs) {
        float ms = 0.f;
        hipError_t e = hipEventSynchronize(r.b);
        if (e == hipSuccess)
            e = hipEventElapsedTime(&ms, r.a, r.b);
        if (e != hipSuccess)
            return fail(ctx, e, "fdfs_gpu_read_timing");
        ctx->acc_ms[r.kernel] += ms;
        ctx->acc_n[r.kernel] += 1;
        ctx->pool.push_back(r.a);
        ctx->pool.push_back(r.b);
    }
    ctx->recs.clear();
    if (ms_out)
        *ms_out = ctx->acc_ms[kernel];
    if (launches_out)
        *launches_out = ctx->acc_n[kernel];
    ctx->acc_ms[kernel] = 0;
    ctx->acc_n[kernel] = 0;
    return 0;
}

int fdfs_gpu_sig_batch(fdfs_gpu_ctx *ctx, const fdfs_gpu_batch *batch, int method,
                       uint32_t *crc_out, uint8_t *sig_out, int32_t *codes_out, void *stream)
{
    if (!ctx || !batch)
        return EINVAL;
    if (method != FDFS_SIG_CRC_ONLY && method != FDFS_SIG_HASH && method != FDFS_SIG_MD5)
        return EINVAL;
    const uint32_t n = batch->n;
    if (n == 0)
        return 0;
    if (!batch->base || !batch->offset || !batch->size || !crc_out)
        return EINVAL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    if (int rc0 = lane_err_check(ctx))
        return rc0;
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int rc = ensure_ws(ctx, sig_ws_bytes(n), st);
    if (rc)
        return rc;
    WsScope wsc(ctx, st);
    Carve cv{static_cast<char *>(ctx->ws)};
    const uint8_t *base = static_cast<const uint8_t *>(batch->base);
    hipError_t e;
    // CRC only: batches of up to kCrcLaneMinFill waves per SIMD keep a wave
    // per file (crc_tab_kernel) or per run (the sparse fold); larger ones
    // hash their files below kFoldMinBytes one lane per file in the size
    // order (crc_lane_kernel, the lane fold), the rest by the sparse fold.
    const bool crc_lanes = method == FDFS_SIG_CRC_ONLY && ctx->lat_files &&
                           (uint64_t)n > (uint64_t)kCrcLaneMinFill * ctx->lat_files;
    if (method == FDFS_SIG_CRC_ONLY && !crc_lanes) {
        uint64_t *nseg = cv.take<uint64_t>(2 * (size_t)n);
        uint64_t *first = cv.take<uint64_t>(2 * ((size_t)n + 1));
        uint64_t *bsum = cv.take<uint64_t>(2 * fdfs::scan_workspace_elems(n));
        hipEvent_t a, b;
        timing_pair(ctx, FDFS_KERNEL_CRC_SEG, a, b);
        e = fdfs::launch_crc_seg(ctx->sar, base, batch->offset, batch->size, n, nseg, first, bsum,
                                 ctx->d_tabs, crc_out, ctx->ncu, st, a, b);
    } else {
        uint32_t *hist = cv.take<uint32_t>(fdfs::kLaneWsDwords);
        uint32_t *order = cv.take<uint32_t>(n);
        const fdfs::BigCrcWs big = carve_big(ctx, cv, n);
        hipEvent_t a, b;
        timing_pair(ctx, crc_lanes ? FDFS_KERNEL_CRC_SEG : FDFS_KERNEL_SIG_LANE, a, b);
        e = fdfs::launch_sig_lane(ctx->sar, method, base, batch->offset, batch->size, n, hist,
                                  order, &big, ctx->d_tabs, crc_out, crc_lanes ? nullptr : sig_out,
                                  crc_lanes ? nullptr : codes_out, nullptr, nullptr, ctx->ncu, st, a, b);
        if (e == hipSuccess)
            e = lane_err_note(ctx, hist, st);
    }
    return e == hipSuccess ? 0 : fail(ctx, e, "sig_batch launch");
}

// ---- chunked (state-carrying) form ------------------------------------------

int fdfs_gpu_state_init(fdfs_gpu_ctx *ctx, fdfs_gpu_file_state *states, uint32_t n, void *stream)
{
    if (!ctx)
        return EINVAL;
    if (n == 0)
        return 0;
    if (!states)
        return EINVAL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipError_t e = fdfs::launch_state_init(states, n, reinterpret_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : fail(ctx, e, "state_init launch");
}

// check: the public entry's duplicate-state_idx check (one small kernel and
// a host synchronisation); sig_batch_host's windows are unique by plan.
static int update_batch(fdfs_gpu_ctx *ctx, const fdfs_gpu_batch *chunks, const uint32_t *state_idx, int method,
                        fdfs_gpu_file_state *states, void *stream, bool check)
{
    if (!ctx || !chunks)
        return EINVAL;
    if (method != FDFS_SIG_CRC_ONLY && method != FDFS_SIG_HASH && method != FDFS_SIG_MD5)
        return EINVAL;
    const uint32_t n = chunks->n;
    if (n == 0)
        return 0;
    if (!chunks->base || !chunks->offset || !chunks->size || !states)
        return EINVAL;
    if (reinterpret_cast<uintptr_t>(states) & 15)
        return EINVAL;
    // the duplicate check's open-addressing table holds 2n slots, at most 2^31
    if (check && state_idx && n > (1u << 30))
        return EINVAL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    if (int rc0 = lane_err_check(ctx))
        return rc0;
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const size_t tbytes = check && state_idx ? align_up(4ull * fdfs::sidx_table_size(n)) : 0;
    int rc = ensure_ws(ctx, std::max(sig_ws_bytes(n) + align_up(4ull * n), tbytes), st);
    if (rc)
        return rc;
    WsScope wsc(ctx, st);
    hipError_t e;
    if (tbytes && !capturing(st)) {
        // the contract (a state at most once per call) checked before any
        // state is touched: the table is scratch in the workspace the
        // kernels below then overwrite
        uint32_t *dflag = reinterpret_cast<uint32_t *>(ctx->dann + kAnnMax + 64 * kAnnMax + 1);
        volatile uint32_t *hflag = reinterpret_cast<uint32_t *>(ctx->hann + 64 * kAnnTail + 64 * kAnnMax + 1);
        if ((e = fdfs::launch_sidx_check(state_idx, n, static_cast<uint32_t *>(ctx->ws), dflag, st)) != hipSuccess ||
            (e = hipMemcpyAsync(const_cast<uint32_t *>(hflag), dflag, 4, hipMemcpyDeviceToHost, st)) != hipSuccess ||
            (e = hipStreamSynchronize(st)) != hipSuccess)
            return fail(ctx, e, "update_batch state_idx check");
        if (*hflag) {
            std::snprintf(ctx->err, sizeof(ctx->err), "update_batch: %s",
                          (*hflag & 1) ? "a state index appears more than once in one call"
                                       : "state index 0xFFFFFFFF");
            return EINVAL;
        }
    }
    Carve cv{static_cast<char *>(ctx->ws)};
    const uint8_t *base = static_cast<const uint8_t *>(chunks->base);
    if (method == FDFS_SIG_CRC_ONLY) {
        // per-chunk CRC by the segmented kernel, then carried onto the state
        uint32_t *tmp = cv.take<uint32_t>(n);
        uint64_t *nseg = cv.take<uint64_t>(2 * (size_t)n);
        uint64_t *first = cv.take<uint64_t>(2 * ((size_t)n + 1));
        uint64_t *bsum = cv.take<uint64_t>(2 * fdfs::scan_workspace_elems(n));
        hipEvent_t a, b;
        timing_pair(ctx, FDFS_KERNEL_CRC_SEG, a, b);
        e = fdfs::launch_crc_seg(ctx->sar, base, chunks->offset, chunks->size, n, nseg, first, bsum,
                                 ctx->d_tabs, tmp, ctx->ncu, st, a, b);
        if (e == hipSuccess)
            e = fdfs::launch_crc_carry(tmp, chunks->size, n, state_idx, states, ctx->d_tabs, st);
    } else {
        uint32_t *hist = cv.take<uint32_t>(fdfs::kLaneWsDwords);
        uint32_t *order = cv.take<uint32_t>(n);
        const fdfs::BigCrcWs big = carve_big(ctx, cv, n);
        hipEvent_t a, b;
        timing_pair(ctx, FDFS_KERNEL_SIG_LANE, a, b);
        e = fdfs::launch_sig_lane(ctx->sar, method, base, chunks->offset, chunks->size, n, hist, order, &big,
                                  ctx->d_tabs, nullptr, nullptr, nullptr, states, state_idx, ctx->ncu,
                                  st, a, b);
        if (e == hipSuccess)
            e = lane_err_note(ctx, hist, st);
    }
    return e == hipSuccess ? 0 : fail(ctx, e, "update_batch launch");
}

int fdfs_gpu_update_batch(fdfs_gpu_ctx *ctx, const fdfs_gpu_batch *chunks, const uint32_t *state_idx,
                          int method, fdfs_gpu_file_state *states, void *stream)
{
    return update_batch(ctx, chunks, state_idx, method, states, stream, true);
}

int fdfs_gpu_final_batch(fdfs_gpu_ctx *ctx, const fdfs_gpu_file_state *states,
                         const uint32_t *state_idx, uint32_t n, int method, uint32_t *crc_out,
                         uint8_t *sig_out, int32_t *codes_out, void *stream)
{
    if (!ctx)
        return EINVAL;
    if (method != FDFS_SIG_CRC_ONLY && method != FDFS_SIG_HASH && method != FDFS_SIG_MD5)
        return EINVAL;
    if (n == 0)
        return 0;
    if (!states || !crc_out)
        return EINVAL;
    if ((reinterpret_cast<uintptr_t>(states) | reinterpret_cast<uintptr_t>(sig_out)) & 3 ||
        reinterpret_cast<uintptr_t>(codes_out) & 15)
        return EINVAL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    if (int rc0 = lane_err_check(ctx))
        return rc0;
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipError_t e = fdfs::launch_final(method, states, state_idx, n, crc_out, sig_out, codes_out,
                                      reinterpret_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : fail(ctx, e, "final_batch launch");
}

int fdfs_gpu_crc_combine(fdfs_gpu_ctx *ctx, const uint32_t *crc_a, const uint32_t *crc_b,
                         const uint64_t *len_b, uint32_t n, uint32_t *out, void *stream)
{
    if (!ctx)
        return EINVAL;
    if (n == 0)
        return 0;
    if (!crc_a || !crc_b || !len_b || !out)
        return EINVAL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipError_t e = fdfs::launch_crc_combine(crc_a, crc_b, len_b, n, out, ctx->d_tabs,
                                            reinterpret_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : fail(ctx, e, "crc_combine launch");
}

// ---- host-resident batches: windows of chunks through the chunked path -----

extern "C++" {
namespace {

struct HostPiece {
    uint32_t file;
    uint64_t at, len;  // host byte range of this piece of the file
};

struct HostWindow {
    uint64_t lo, hi;   // host bytes copied for the window
    size_t p0, p1;     // its pieces
};

// Windows of at most `chunk` host bytes, each holding at most one piece of
// any file (the update contract): files are taken in order, a file larger
// than the space left is cut and continues in the next window, so every
// window fits its slot whatever the file sizes.  Packed batches (increasing
// offsets) copy each byte once; a file that starts before the window does
// opens a new one.  Empty files get no piece (init + final is their result).
void plan_host_windows(const uint64_t *off, const uint64_t *sz, uint32_t n, uint64_t chunk,
                       uint32_t max_pieces, std::vector<HostPiece> &pieces, std::vector<HostWindow> &wins)
{
    uint32_t i = 0;
    uint64_t a = 0;  // bytes of file i already placed
    while (i < n) {
        if (sz[i] == 0) {
            i++;
            continue;
        }
        HostWindow w{off[i] + a, off[i] + a, pieces.size(), pieces.size()};
        while (i < n && w.p1 - w.p0 < max_pieces) {
            if (sz[i] == 0) {
                i++;
                a = 0;
                continue;
            }
            const uint64_t s = off[i] + a;
            if (s < w.lo || s >= w.lo + chunk)
                break;
            const uint64_t take = std::min(sz[i] - a, w.lo + chunk - s);
            pieces.push_back({i, s, take});
            w.p1++;
            w.hi = std::max(w.hi, s + take);
            a += take;
            if (a < sz[i])
                break;  // the window is full: the file continues in the next one
            i++;
            a = 0;
        }
        wins.push_back(w);
    }
}

}  // namespace
}  // extern "C++"

int fdfs_gpu_sig_batch_host(fdfs_gpu_ctx *ctx, const fdfs_gpu_batch *hb, int method,
                            uint32_t *crc_out, uint8_t *sig_out, int32_t *codes_out,
                            uint64_t chunk_bytes)
{
    if (!ctx || !hb)
        return EINVAL;
    if (method != FDFS_SIG_CRC_ONLY && method != FDFS_SIG_HASH && method != FDFS_SIG_MD5)
        return EINVAL;
    const uint32_t n = hb->n;
    if (n == 0)
        return 0;
    if (!hb->base || !hb->offset || !hb->size || !crc_out)
        return EINVAL;
    if (chunk_bytes == 0)
        chunk_bytes = 256ull << 20;
    constexpr uint32_t kMaxPieces = 1u << 20;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    std::vector<HostPiece> pieces;
    std::vector<HostWindow> wins;
    plan_host_windows(hb->offset, hb->size, n, chunk_bytes, kMaxPieces, pieces, wins);
    uint64_t win = 16;
    uint32_t maxp = 1;
    for (const auto &w : wins) {
        win = std::max(win, w.hi - w.lo);
        maxp = std::max(maxp, (uint32_t)(w.p1 - w.p0));
    }
    const bool want_sig = method != FDFS_SIG_CRC_ONLY && sig_out;
    const bool want_codes = method != FDFS_SIG_CRC_ONLY && codes_out;
    // device: the n file states and results, and two window slots (bytes,
    // then offsets / sizes / state indices of its pieces)
    const size_t meta = 2 * align_up(8ull * maxp) + align_up(4ull * maxp);
    const size_t slot = align_up(win + 16) + meta;
    const size_t res = align_up(128ull * n) + align_up(4ull * n) + align_up(24ull * n) + align_up(16ull * n);
    int rc = ensure_ws(ctx, sig_ws_bytes(maxp) + align_up(4ull * maxp), nullptr);
    if (rc)
        return rc;
    char *dmem = nullptr, *hmeta = nullptr;
    hipStream_t cp = nullptr, cs = nullptr;
    hipEvent_t copied[2] = {nullptr, nullptr}, done[2] = {nullptr, nullptr};
    hipError_t e = hipMalloc(&dmem, res + 2 * slot);
    if (e == hipSuccess)
        e = hipHostMalloc(reinterpret_cast<void **>(&hmeta), 2 * meta, 0);
    if (e == hipSuccess)
        e = hipStreamCreateWithFlags(&cp, hipStreamNonBlocking);
    if (e == hipSuccess)
        e = hipStreamCreateWithFlags(&cs, hipStreamNonBlocking);
    for (int k = 0; k < 2 && e == hipSuccess; k++) {
        e = hipEventCreateWithFlags(&copied[k], hipEventDisableTiming);
        if (e == hipSuccess)
            e = hipEventCreateWithFlags(&done[k], hipEventDisableTiming);
    }
    auto *states = reinterpret_cast<fdfs_gpu_file_state *>(dmem);
    uint32_t *d_crc = reinterpret_cast<uint32_t *>(dmem + align_up(128ull * n));
    uint8_t *d_sig = reinterpret_cast<uint8_t *>(d_crc) + align_up(4ull * n);
    int32_t *d_codes = reinterpret_cast<int32_t *>(d_sig + align_up(24ull * n));
    if (e == hipSuccess)
        rc = fdfs_gpu_state_init(ctx, states, n, cs);
    const uint8_t *hbase = static_cast<const uint8_t *>(hb->base);
    for (size_t k = 0; k < wins.size() && e == hipSuccess && rc == 0; k++) {
        const HostWindow &w = wins[k];
        const uint32_t m = (uint32_t)(w.p1 - w.p0);
        char *sl = dmem + res + (k & 1) * slot;
        uint8_t *d_data = reinterpret_cast<uint8_t *>(sl);
        char *d_meta = sl + align_up(win + 16);
        char *h = hmeta + (k & 1) * meta;
        // the slot (and its pinned metadata) is free once window k - 2 is hashed
        if (k >= 2 && (e = hipEventSynchronize(done[k & 1])) != hipSuccess)
            break;
        auto *h_off = reinterpret_cast<uint64_t *>(h);
        auto *h_sz = reinterpret_cast<uint64_t *>(h + align_up(8ull * maxp));
        auto *h_idx = reinterpret_cast<uint32_t *>(h + 2 * align_up(8ull * maxp));
        for (uint32_t j = 0; j < m; j++) {
            const HostPiece &pc = pieces[w.p0 + j];
            h_off[j] = pc.at - w.lo;
            h_sz[j] = pc.len;
            h_idx[j] = pc.file;
        }
        if ((e = hipMemcpyAsync(d_data, hbase + w.lo, w.hi - w.lo, hipMemcpyHostToDevice, cp)) != hipSuccess ||
            (e = hipMemcpyAsync(d_meta, h, meta, hipMemcpyHostToDevice, cp)) != hipSuccess ||
            (e = hipEventRecord(copied[k & 1], cp)) != hipSuccess ||
            (e = hipStreamWaitEvent(cs, copied[k & 1], 0)) != hipSuccess)
            break;
        fdfs_gpu_batch b{d_data, reinterpret_cast<const uint64_t *>(d_meta),
                         reinterpret_cast<const uint64_t *>(d_meta + align_up(8ull * maxp)), m};
        rc = update_batch(ctx, &b, reinterpret_cast<const uint32_t *>(d_meta + 2 * align_up(8ull * maxp)), method,
                          states, cs, false);  // one piece per file per window by plan
        if (rc == 0)
            e = hipEventRecord(done[k & 1], cs);
    }
    if (e == hipSuccess && rc == 0)
        rc = fdfs_gpu_final_batch(ctx, states, nullptr, n, method, d_crc, want_sig ? d_sig : nullptr,
                                  want_codes ? d_codes : nullptr, cs);
    if (e == hipSuccess && rc == 0) {
        if ((e = hipMemcpyAsync(crc_out, d_crc, 4ull * n, hipMemcpyDeviceToHost, cs)) == hipSuccess && want_sig)
            e = hipMemcpyAsync(sig_out, d_sig, 24ull * n, hipMemcpyDeviceToHost, cs);
        if (e == hipSuccess && want_codes)
            e = hipMemcpyAsync(codes_out, d_codes, 16ull * n, hipMemcpyDeviceToHost, cs);
    }
    if (cs) {
        const hipError_t e2 = hipStreamSynchronize(cs);
        if (e == hipSuccess)
            e = e2;
    }
    if (cp)
        (void)hipStreamSynchronize(cp);
    for (int k = 0; k < 2; k++) {
        if (copied[k])
            (void)hipEventDestroy(copied[k]);
        if (done[k])
            (void)hipEventDestroy(done[k]);
    }
    if (cs)
        (void)hipStreamDestroy(cs);
    if (cp)
        (void)hipStreamDestroy(cp);
    if (hmeta)
        (void)hipHostFree(hmeta);
    if (dmem)
        (void)hipFree(dmem);
    if (rc)
        return rc;
    return e == hipSuccess ? 0 : fail(ctx, e, "sig_batch_host");
}

static int dedup_common(fdfs_gpu_ctx *ctx, const uint8_t *sig, uint32_t stride,
                        const uint64_t *gidx, uint32_t gstride, uint64_t n, uint64_t *rep_out,
                        uint32_t *ref_out, void *stream)
{
    if (!ctx)
        return EINVAL;
    if (n == 0)
        return 0;
    if (!sig || !rep_out || n >= 0xFFFFFFFFull)  // ref_out == nullptr: packed answers at rep_out
        return EINVAL;
    // records are read as u64 words, rep written as u64; packed answers are
    // written as one 16-byte store each
    if ((reinterpret_cast<uintptr_t>(sig) | reinterpret_cast<uintptr_t>(gidx) |
         reinterpret_cast<uintptr_t>(rep_out)) & 7)
        return EINVAL;
    if (!ref_out && (reinterpret_cast<uintptr_t>(rep_out) & 15))
        return EINVAL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    if (int rc0 = lane_err_check(ctx))
        return rc0;
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int rc = ensure_ws(ctx, dedup_ws_bytes(n), st);
    if (rc)
        return rc;
    WsScope wsc(ctx, st);
    hipEvent_t a, b;
    timing_pair(ctx, FDFS_KERNEL_DEDUP, a, b);
    hipError_t e = fdfs::launch_dedup_group(sig, stride, gidx, gstride, n, ctx->ws, rep_out, ref_out,
                                            ref_out == nullptr, st, a, b);
    return e == hipSuccess ? 0 : fail(ctx, e, "dedup launch");
}

int fdfs_gpu_dedup(fdfs_gpu_ctx *ctx, const uint8_t *sig, const uint64_t *gidx, uint64_t n,
                   uint64_t *rep_out, uint32_t *ref_out, void *stream)
{
    if (n && !ref_out)
        return EINVAL;
    return dedup_common(ctx, sig, 24, gidx, gidx ? 1 : 0, n, rep_out, ref_out, stream);
}

int fdfs_gpu_dedup_packed(fdfs_gpu_ctx *ctx, const uint8_t *sig, const uint64_t *gidx, uint64_t n,
                          fdfs_gpu_dedup_answer *out, void *stream)
{
    return dedup_common(ctx, sig, 24, gidx, gidx ? 1 : 0, n, reinterpret_cast<uint64_t *>(out), nullptr, stream);
}

int fdfs_gpu_dedup_group(fdfs_gpu_ctx *ctx, const uint8_t *records, uint64_t n, uint64_t *rep_out,
                         uint32_t *ref_out, void *stream)
{
    if (n && !ref_out)
        return EINVAL;
    // rows {sig[24], gidx}: gidx is the 4th uint64 of each 32-byte row
    return dedup_common(ctx, records, 32, records ? reinterpret_cast<const uint64_t *>(records + 24) : nullptr,
                        4, n, rep_out, ref_out, stream);
}

int fdfs_gpu_dedup_bucket(fdfs_gpu_ctx *ctx, const uint8_t *sig, const uint64_t *gidx, uint64_t n,
                          uint32_t nranks, uint8_t *records_out, uint64_t *counts_out,
                          uint64_t *row_of_out, void *stream)
{
    if (!ctx || nranks == 0 || nranks > 64 || !counts_out)
        return EINVAL;
    if (n && (!sig || !records_out))
        return EINVAL;
    if ((reinterpret_cast<uintptr_t>(sig) | reinterpret_cast<uintptr_t>(gidx) |
         reinterpret_cast<uintptr_t>(records_out) | reinterpret_cast<uintptr_t>(row_of_out)) & 7)
        return EINVAL;  // u64 words
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int rc = ensure_ws(ctx, align_up(8 * fdfs::bucket_ws_elems(n)), st);
    if (rc)
        return rc;
    WsScope wsc(ctx, st);
    uint64_t *bws = static_cast<uint64_t *>(ctx->ws);
    hipEvent_t a, b;
    timing_pair(ctx, FDFS_KERNEL_BUCKET, a, b);
    hipError_t e = fdfs::launch_dedup_bucket(sig, gidx, n, nranks, records_out, counts_out, bws,
                                             row_of_out, st, a, b);
    return e == hipSuccess ? 0 : fail(ctx, e, "dedup_bucket launch");
}

// ---- incremental dedup index ------------------------------------------------

struct fdfs_gpu_index {
    int device = 0;
    fdfs::IndexTable t{};
    void *mem = nullptr;
    uint64_t records = 0;  // records ingested so far (the implicit ingest index base)
    uint64_t bound = 0;    // upper bound of the classes in the table (exact after a read-back)
    hipEvent_t ev = nullptr;
    bool used = false;
    // ingest, stats and destroy of one index are serialised here (after the
    // calling context's mutex, never before it)
    std::mutex mu;
};

// The table keeps load <= 3/4.
static uint64_t index_capacity(uint64_t slots) { return slots / 4 * 3; }

static size_t index_bytes(uint64_t slots)
{
    return align_up(24 * slots) + align_up(8 * slots) + align_up(4 * slots) + align_up(4 * slots) + align_up(8 * 4);
}

static void index_carve(fdfs::IndexTable &t, void *mem, uint64_t slots)
{
    Carve cv{static_cast<char *>(mem)};
    t.slots = slots;
    t.keys = cv.take<uint8_t>(24 * slots);
    t.rep = cv.take<uint64_t>(slots);
    t.ref = cv.take<uint32_t>(slots);
    t.state = cv.take<uint32_t>(slots);
    t.counters = cv.take<uint64_t>(4);
}

int fdfs_gpu_index_create(fdfs_gpu_ctx *ctx, uint64_t max_classes, fdfs_gpu_index **out)
{
    if (!ctx || !out || max_classes > (1ull << 40))
        return EINVAL;
    *out = nullptr;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    uint64_t slots = 1024;
    while (index_capacity(slots) < max_classes)
        slots <<= 1;
    auto *ix = new (std::nothrow) fdfs_gpu_index;
    if (!ix)
        return ENOMEM;
    ix->device = ctx->device;
    const size_t bytes = index_bytes(slots);
    hipError_t e = hipMalloc(&ix->mem, bytes);
    if (e != hipSuccess) {
        delete ix;
        std::snprintf(ctx->err, sizeof(ctx->err), "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
        return ENOMEM;
    }
    index_carve(ix->t, ix->mem, slots);
    if ((e = hipEventCreateWithFlags(&ix->ev, hipEventDisableTiming)) == hipSuccess &&
        (e = hipMemset(ix->t.counters, 0, 32)) == hipSuccess &&
        (e = fdfs::launch_index_clear(ix->t.state, slots, nullptr)) == hipSuccess)
        e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        (void)hipFree(ix->mem);
        if (ix->ev)
            (void)hipEventDestroy(ix->ev);
        delete ix;
        return fail(ctx, e, "index_create");
    }
    *out = ix;
    return 0;
}

int fdfs_gpu_index_destroy(fdfs_gpu_index *ix)
{
    if (!ix)
        return EINVAL;
    {
        std::lock_guard<std::mutex> lk(ix->mu);  // waits for an ingest in progress
        DeviceGuard g(ix->device);
        if (ix->used)
            (void)hipEventSynchronize(ix->ev);
        (void)hipFree(ix->mem);
        (void)hipEventDestroy(ix->ev);
    }
    delete ix;
    return 0;
}

// Make room for `n` more classes: read back the exact class count (a sync
// on the index's last ingest) when the running bound says the batch might
// not fit, and if it still might, grow the table (twice the slots until it
// fits) and rehash every class into it.  On failure the index is unchanged.
static int index_make_room(fdfs_gpu_ctx *ctx, fdfs_gpu_index *ix, uint64_t n, hipStream_t st)
{
    if (ix->bound + n <= index_capacity(ix->t.slots))
        return 0;
    if (capturing(st)) {
        std::snprintf(ctx->err, sizeof(ctx->err), "index growth needed during stream capture");
        return ENOSPC;
    }
    uint64_t c[4] = {0, 0, 0, 0};
    hipError_t e = ix->used ? hipEventSynchronize(ix->ev) : hipSuccess;
    if (e == hipSuccess)
        e = hipMemcpy(c, ix->t.counters, sizeof(c), hipMemcpyDeviceToHost);
    if (e != hipSuccess)
        return fail(ctx, e, "index class count");
    ix->bound = c[0];
    if (ix->bound + n <= index_capacity(ix->t.slots))
        return 0;
    uint64_t slots = ix->t.slots;
    while (index_capacity(slots) < ix->bound + n) {
        if (slots >= (1ull << 41))
            return ENOMEM;
        slots <<= 1;
    }
    void *mem = nullptr;
    const size_t bytes = index_bytes(slots);
    if ((e = hipMalloc(&mem, bytes)) != hipSuccess) {
        std::snprintf(ctx->err, sizeof(ctx->err), "index growth to %llu slots: hipMalloc(%zu): %s",
                      (unsigned long long)slots, bytes, hipGetErrorString(e));
        return ENOMEM;
    }
    fdfs::IndexTable t{};
    index_carve(t, mem, slots);
    if ((e = fdfs::launch_index_clear(t.state, slots, st)) == hipSuccess &&
        (e = hipMemcpyAsync(t.counters, ix->t.counters, 32, hipMemcpyDeviceToDevice, st)) == hipSuccess &&
        (e = fdfs::launch_index_rehash(ix->t, t, st)) == hipSuccess)
        e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        (void)hipStreamSynchronize(st);
        (void)hipFree(mem);
        return fail(ctx, e, "index growth");
    }
    (void)hipFree(ix->mem);
    ix->mem = mem;
    ix->t = t;
    return 0;
}

int fdfs_gpu_index_ingest(fdfs_gpu_ctx *ctx, fdfs_gpu_index *ix, const uint8_t *sig, const uint64_t *gidx,
                          uint64_t n, uint64_t *rep_out, uint32_t *ref_out, void *stream)
{
    if (!ctx || !ix || ix->device != ctx->device || n >= 0xFFFFFFFFull)
        return EINVAL;
    if (n == 0)
        return 0;
    if (!sig || !rep_out || !ref_out)
        return EINVAL;
    if ((reinterpret_cast<uintptr_t>(sig) | reinterpret_cast<uintptr_t>(gidx) |
         reinterpret_cast<uintptr_t>(rep_out)) & 7)
        return EINVAL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    std::lock_guard<std::mutex> lki(ix->mu);
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const size_t dws = dedup_ws_bytes(n);
    int rc = ensure_ws(ctx, dws + 2 * align_up(8 * n) + 2 * align_up(4 * n), st);
    if (rc)
        return rc;
    WsScope wsc(ctx, st);
    // successive ingests into one index are ordered whatever their streams
    if (ix->used && !capturing(st))
        (void)hipStreamWaitEvent(st, ix->ev, 0);
    // every class of the batch finds a slot: the table grows first if needed
    if ((rc = index_make_room(ctx, ix, n, st)))
        return rc;
    Carve cv{static_cast<char *>(ctx->ws) + dws};
    uint64_t *rep_pos = cv.take<uint64_t>(n);
    uint32_t *ref_b = cv.take<uint32_t>(n);
    uint64_t *res_rep = cv.take<uint64_t>(n);
    uint32_t *res_ref = cv.take<uint32_t>(n);
    hipEvent_t a, b;
    timing_pair(ctx, FDFS_KERNEL_DEDUP, a, b);
    // 1. the batch on its own (record positions as the ingest order)
    hipError_t e = fdfs::launch_dedup_group(sig, 24, nullptr, 0, n, ctx->ws, rep_pos, ref_b, false, st, a, b);
    // 2. its classes against the index, 3. every record's answer
    if (e == hipSuccess)
        e = fdfs::launch_index_ingest(sig, gidx, ix->records, n, rep_pos, ref_b, ix->t, res_rep, res_ref,
                                      rep_out, ref_out, st);
    if (e != hipSuccess)
        return fail(ctx, e, "index_ingest");
    ix->records += n;
    ix->bound += n;
    if (!capturing(st) && hipEventRecord(ix->ev, st) == hipSuccess)
        ix->used = true;
    return 0;
}

int fdfs_gpu_index_stats(fdfs_gpu_index *ix, uint64_t *classes, uint64_t *records, uint64_t *unplaced)
{
    if (!ix)
        return EINVAL;
    std::lock_guard<std::mutex> lk(ix->mu);
    DeviceGuard g(ix->device);
    uint64_t c[4] = {0, 0, 0, 0};
    if (ix->used && hipEventSynchronize(ix->ev) != hipSuccess)
        return EIO;
    if (hipMemcpy(c, ix->t.counters, sizeof(c), hipMemcpyDeviceToHost) != hipSuccess)
        return EIO;
    ix->bound = c[0];
    if (classes)
        *classes = c[0];
    if (records)
        *records = ix->records;
    if (unplaced)
        *unplaced = c[2];
    return 0;
}

int fdfs_gpu_index_slots(fdfs_gpu_index *ix, uint64_t *slots)
{
    if (!ix || !slots)
        return EINVAL;
    std::lock_guard<std::mutex> lk(ix->mu);
    *slots = ix->t.slots;
    return 0;
}

// ---- multi-GPU dedup over RCCL ---------------------------------------------

static int nccl_fail(fdfs_gpu_ctx *ctx, ncclResult_t r, const char *where)
{
    if (ctx)
        std::snprintf(ctx->err, sizeof(ctx->err), "%s: %s", where, ncclGetErrorString(r));
    return EIO;
}

int fdfs_gpu_comm_unique_id(uint8_t *id_out)
{
    if (!id_out)
        return EINVAL;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess)
        return EIO;
    std::memcpy(id_out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return 0;
}

int fdfs_gpu_comm_init(fdfs_gpu_ctx *ctx, const uint8_t *id, int nranks, int rank, void **comm_out)
{
    if (!ctx || !id || !comm_out || nranks < 1 || nranks > 64 || rank < 0 || rank >= nranks)
        return EINVAL;
    *comm_out = nullptr;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
    ncclComm_t c = nullptr;
    const ncclResult_t r = ncclCommInitRank(&c, nranks, uid, rank);
    if (r != ncclSuccess)
        return nccl_fail(ctx, r, "ncclCommInitRank");
    *comm_out = c;
    return 0;
}

int fdfs_gpu_comm_destroy(void *comm)
{
    if (!comm)
        return EINVAL;
    return ncclCommDestroy(static_cast<ncclComm_t>(comm)) == ncclSuccess ? 0 : EIO;
}

// fdfs_gpu_dedup_global is two parts, so that its multi-rank logic also runs
// on one GPU (fdfs_gpu_dedup_global_local):
//  * the exchange plan (DgPlan), derived identically on every rank from all
//    ranks' announcements, all-gathered in one collective: each rank's row
//    count per owner, the room of its owner-side buffers and any local error.
//    From it every (src, dst) segment's count and its offsets on both sides,
//    each owner's row count, and the common outcome: an error on any rank is
//    every rank's error, returned before any row moves, so no rank is left
//    waiting in a send or receive;
//  * the transport: one rank of an RCCL communicator (ncclAllGather, grouped
//    ncclSend / ncclRecv), or N virtual ranks in one process on one device
//    (every segment a hipMemcpyAsync).
// Round 6: the bucket pass writes the rank's own rows
// straight into the front of its owner-side buffer (no self copy over the
// RCCL transport) and pre-fills every record's singleton answer; the owner
// answers only the rows of multi-member classes, as 16-byte sink records
// {sender row, ref, rep} per source segment (fdfs_dedup.hip DpSink), whose
// counts one small all-gather tells every rank before the way back; the
// sender applies them over its pre-filled answers.  Bucket, group, sink and
// apply are the same kernels for both transports.

extern "C++" {

struct DgPlan {
    int nranks = 0;
    uint64_t cnt[64][64];  // cnt[p][q]: rows rank p sends to owner q
    uint64_t m[64];        // rows owner q groups
    uint64_t cap[64];      // rank p's owner-region capacity (launch_bucket_place), 0: exact layout
    int err = 0, err_rank = -1;
    bool grow = false;     // an owner's buffers must grow: the ranks agree on the outcome first
    bool over = false;     // some rank's owner count exceeds its cap: every rank buckets again exactly
    // where p's rows for owner q start among p's rows in send order (the
    // sender row its answers name)
    uint64_t soff(int p, int q) const
    {
        if (cap[p])
            return (uint64_t)q * cap[p];
        uint64_t s = 0;
        for (int k = 0; k < q; k++)
            s += cnt[p][k];
        return s;
    }
    // after an over-capacity owner: every rank's exact prefix layout
    void exact()
    {
        for (int p = 0; p < nranks; p++)
            cap[p] = 0;
        over = false;
    }
    // where p's rows start among owner q's received rows: q's own rows
    // first, then the other ranks' in rank order (fdfs::dg_seg_src; the
    // device's sink_plan_kernel derives the same table)
    uint64_t roff(int q, int p) const
    {
        if (p == q)
            return 0;
        uint64_t s = cnt[q][q];
        for (int k = 0; k < p; k++)
            if (k != q)
                s += cnt[k][q];
        return s;
    }
};

// Sink-record counts after the owners' groups: a[q][p] = records owner q
// returns to rank p, from each owner's per-segment counters (all-gathered).
struct DgAns {
    uint64_t a[64][64];
    void load(const uint32_t *all, int nranks)
    {
        for (int q = 0; q < nranks; q++)
            for (int k = 0; k < nranks; k++)
                a[q][fdfs::dg_seg_src((uint32_t)q, (uint32_t)k)] = all[(size_t)q * nranks + k];
    }
    // where owner q's records start in rank p's receive buffer (the other
    // owners' records, in owner order)
    uint64_t boff(int p, int q) const
    {
        uint64_t s = 0;
        for (int k = 0; k < q; k++)
            if (k != p)
                s += a[k][p];
        return s;
    }
    uint64_t recv_total(int p, int nranks) const { return boff(p, nranks); }
};

// send-order slots of a rank's rows: the fixed-capacity owner regions of
// launch_bucket_place (nranks x cap, a little over n), or n
static uint64_t dg_slots(uint64_t n, int nranks)
{
    return std::max<uint64_t>(n, (uint64_t)nranks * fdfs::bucket_cap(n, (uint32_t)nranks));
}

static size_t dg_a_bytes(uint64_t n, int nranks)
{
    const uint64_t sl = dg_slots(n, nranks);
    return align_up(32 * sl) + align_up(4 * sl) + align_up(16 * n) + align_up(8 * fdfs::bucket_ws_elems(n));
}

static size_t dg_b_bytes(uint64_t m)
{
    return align_up(32 * m) + align_up(16 * m) + align_up(8 * fdfs::kSinkSegWords) + align_up(4 * 64);
}

// ann: nranks announcements of nranks + kAnnTail words, rank p's at p.
static void dg_plan(const uint64_t *ann, int nranks, DgPlan &pl)
{
    const size_t w = (size_t)nranks + kAnnTail;
    pl.nranks = nranks;
    for (int q = 0; q < nranks; q++)
        pl.m[q] = 0;
    for (int p = 0; p < nranks; p++) {
        const uint64_t *a = ann + p * w;
        pl.cap[p] = a[nranks + 3];
        for (int q = 0; q < nranks; q++) {
            pl.cnt[p][q] = a[q];
            pl.m[q] += a[q];
            if (pl.cap[p] && a[q] > pl.cap[p])
                pl.over = true;
        }
        if (a[nranks + 2] && !pl.err) {
            pl.err = (int)a[nranks + 2];
            pl.err_rank = p;
        }
    }
    for (int q = 0; q < nranks && !pl.err; q++)
        if (pl.m[q] >= 0xFFFFFFFFull) {  // the owner's group takes a uint32 record count
            pl.err = EINVAL;
            pl.err_rank = q;
        }
    for (int q = 0; q < nranks && !pl.err; q++) {
        const uint64_t *a = ann + q * w;
        if (dg_b_bytes(pl.m[q]) > a[nranks] || dedup_ws_bytes(pl.m[q]) > a[nranks + 1])
            pl.grow = true;
    }
}

// One rank's side: its records and the buffers of both directions.
struct DgSide {
    const uint8_t *sig = nullptr;
    const uint64_t *gidx = nullptr;
    uint64_t n = 0;
    uint64_t *rep_out = nullptr;
    uint32_t *ref_out = nullptr;
    uint8_t *rows = nullptr;      // [n] 32-byte rows in send order, grouped by owner
    uint32_t *rec_of = nullptr;   // [n] record of each send position
    uint8_t *back = nullptr;      // [n] 16-byte sink records from the other owners
    uint64_t *bws = nullptr;      // the bucket's tile counts and their scan (bucket_ws_elems)
    uint64_t m = 0;               // rows this rank groups as owner
    uint8_t *rows_in = nullptr;   // [m] received rows, own segment first (always at the buffer's start)
    uint8_t *ans = nullptr;       // [m] sink records, segment k's from ans + 16 seg_start[k]
    uint64_t *seg = nullptr;      // [kSinkSegWords] the segment table (launch_sink_plan)
    uint32_t *cntr = nullptr;     // [64] sink records per segment
};

static void dg_carve_a(DgSide &s, void *mem, int nranks)
{
    Carve c{static_cast<char *>(mem)};
    const uint64_t sl = dg_slots(s.n, nranks);
    s.rows = c.take<uint8_t>(32 * sl);
    s.rec_of = c.take<uint32_t>(sl);
    s.back = c.take<uint8_t>(16 * s.n);
    s.bws = c.take<uint64_t>(fdfs::bucket_ws_elems(s.n));
}

static void dg_carve_b(DgSide &s, void *mem, uint64_t m)
{
    Carve c{static_cast<char *>(mem)};
    s.m = m;
    s.rows_in = c.take<uint8_t>(32 * m);
    s.ans = c.take<uint8_t>(16 * m);
    s.seg = c.take<uint64_t>(fdfs::kSinkSegWords);
    s.cntr = c.take<uint32_t>(64);
}

// Argument check of one rank's share (0 or EINVAL).
static int dg_check(const uint8_t *sig, const uint64_t *gidx, uint64_t n, const uint64_t *rep_out,
                    const uint32_t *ref_out, int nranks)
{
    if (n >= 0xFFFFFFFFull)
        return EINVAL;
    if (n && (!sig || !rep_out || !ref_out))
        return EINVAL;
    // without ingest indices every rank would number its records 0..n-1 and
    // the owners' class minimum would mix records of different ranks
    if (n && !gidx && nranks > 1)
        return EINVAL;
    if ((reinterpret_cast<uintptr_t>(sig) | reinterpret_cast<uintptr_t>(gidx) |
         reinterpret_cast<uintptr_t>(rep_out)) & 7)
        return EINVAL;
    return 0;
}

// Phase 1: rows by owner (the counts are the first nranks words of `ann`),
// the record of each send position, every record's singleton answer; rank
// `me`'s own rows to `self_rows` when given (the RCCL form: the front of its
// owner-side buffer), else to their send slots (the local form copies them).
// cap > 0: the one-pass fixed-capacity form (launch_bucket_place); 0: the
// exact two-pass form (after a plan found an owner over some rank's cap).
static hipError_t dg_bucket(fdfs_gpu_ctx *ctx, DgSide &s, int nranks, int me, uint8_t *self_rows, uint64_t *ann,
                            uint64_t cap, hipStream_t st)
{
    hipEvent_t a, b;
    timing_pair(ctx, FDFS_KERNEL_BUCKET, a, b);
    const fdfs::BucketExtra x{(uint32_t)me, self_rows, s.rec_of, s.rep_out, s.ref_out};
    if (cap)
        return fdfs::launch_bucket_place(s.sig, s.gidx, s.n, (uint32_t)nranks, cap, s.rows, ann, x, st, a, b);
    return fdfs::launch_dedup_bucket(s.sig, s.gidx, s.n, (uint32_t)nranks, s.rows, ann, s.bws, nullptr, st, a, b,
                                     &x);
}

// The announcement's tail {owner-side room, workspace room, errno, cap},
// staged in pinned memory (`h`, untouched until the stream has copied it).
static hipError_t dg_announce(uint64_t *ann_tail, uint64_t *h, uint64_t b_room, uint64_t ws_room, int err,
                              uint64_t cap, hipStream_t st)
{
    h[0] = b_room;
    h[1] = ws_room;
    h[2] = (uint64_t)err;
    h[3] = cap;
    return hipMemcpyAsync(ann_tail, h, 8 * kAnnTail, hipMemcpyHostToDevice, st);
}

// Phase 3: owner q's segment table from the announcements (`all`, w words
// each), then its group of the received rows (min gidx from the rows' own
// word 3) into sink records.
static hipError_t dg_group(fdfs_gpu_ctx *ctx, DgSide &s, const uint64_t *all, size_t w, int nranks, int q,
                           bool exact, hipStream_t st)
{
    hipError_t e = fdfs::launch_sink_plan(all, (uint32_t)w, (uint32_t)nranks, (uint32_t)q, exact, s.seg, s.cntr, st);
    if (e != hipSuccess)
        return e;
    hipEvent_t a, b;
    timing_pair(ctx, FDFS_KERNEL_DEDUP, a, b);
    const fdfs::DedupSink xs{s.ans, s.cntr, s.seg, (uint32_t)nranks};
    return fdfs::launch_dedup_group(s.rows_in, 32, reinterpret_cast<const uint64_t *>(s.rows_in + 24), 4, s.m,
                                    ctx->ws, nullptr, nullptr, true, st, a, b, &xs);
}

// Phase 5: the sink records over the pre-filled answers: the rank's own
// owner's (segment 0 of its owner side, counted on the device) and `nb`
// received from the other owners.
static hipError_t dg_apply(DgSide &s, uint64_t self_rows, uint64_t nb, hipStream_t st)
{
    return fdfs::launch_answer_apply(s.ans, s.cntr, self_rows, s.back, nb, s.rec_of, s.rep_out, s.ref_out, st);
}

// One point-to-point move of an exchange.
struct DgMove {
    int peer;
    char *ptr;  // send: source, receive: destination
    size_t bytes;
};

// RCCL transport of one exchange: one group of sends and receives.
static int dg_nccl_group(fdfs_gpu_ctx *ctx, ncclComm_t c, const std::vector<DgMove> &sends,
                         const std::vector<DgMove> &recvs, hipStream_t st)
{
    if (sends.empty() && recvs.empty())
        return 0;
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess)
        return nccl_fail(ctx, r, "ncclGroupStart");
    for (const DgMove &g : sends)
        if (r == ncclSuccess)
            r = ncclSend(g.ptr, g.bytes, ncclUint8, g.peer, c, st);
    for (const DgMove &g : recvs)
        if (r == ncclSuccess)
            r = ncclRecv(g.ptr, g.bytes, ncclUint8, g.peer, c, st);
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
        return nccl_fail(ctx, r != ncclSuccess ? r : r2, "exchange");
    return 0;
}

static int dg_plan_error(fdfs_gpu_ctx *ctx, const DgPlan &pl, int me)
{
    if (pl.err_rank != me || pl.err == EINVAL)
        std::snprintf(ctx->err, sizeof(ctx->err), "dedup_global: rank %d failed: %s", pl.err_rank,
                      pl.err == EINVAL ? "invalid arguments or over 2^32-2 rows for one owner"
                                       : pl.err == ENOMEM ? "out of memory" : "HIP error");
    return pl.err;
}

// Grow the owner-side buffer keeping its first `keep` bytes (the own rows the
// bucket pass wrote there).
static int grow_keep(fdfs_gpu_ctx *ctx, void **buf, size_t *have, size_t bytes, size_t keep, hipStream_t st)
{
    if (bytes <= *have)
        return 0;
    void *nb = nullptr;
    const size_t sz = bytes + bytes / 4;
    hipError_t e = hipMalloc(&nb, sz);
    if (e != hipSuccess) {
        std::snprintf(ctx->err, sizeof(ctx->err), "hipMalloc(%zu): %s", sz, hipGetErrorString(e));
        return ENOMEM;
    }
    if (keep && (e = hipMemcpyAsync(nb, *buf, keep, hipMemcpyDeviceToDevice, st)) != hipSuccess) {
        (void)hipFree(nb);
        return fail(ctx, e, "exchange buffer growth copy");
    }
    if ((e = hipStreamSynchronize(st)) != hipSuccess) {
        (void)hipFree(nb);
        return fail(ctx, e, "exchange buffer growth sync");
    }
    (void)hipFree(*buf);
    *buf = nb;
    *have = sz;
    return 0;
}

}  // extern "C++"

int fdfs_gpu_dedup_global(fdfs_gpu_ctx *ctx, void *comm, const uint8_t *sig, const uint64_t *gidx,
                          uint64_t n, uint64_t *rep_out, uint32_t *ref_out, void *stream)
{
    if (!ctx || !comm)
        return EINVAL;
    ncclComm_t c = static_cast<ncclComm_t>(comm);
    int nranks = 0, me = 0;
    if (ncclCommCount(c, &nranks) != ncclSuccess || ncclCommUserRank(c, &me) != ncclSuccess ||
        nranks < 1 || nranks > 64)
        return EINVAL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    // A local error is announced, not returned: every rank takes part in the
    // all-gather and all of them return it together.
    // It synchronises on the announcements, so it cannot be captured.  Inside
    // a capture no collective would execute (not even one announcing the
    // error: it would only be recorded), so a capturing rank returns EINVAL
    // at once, before any collective is enqueued; that every rank calls
    // outside a capture is the caller's contract (include/fdfs_gpu.h).
    if (capturing(st)) {
        std::snprintf(ctx->err, sizeof(ctx->err), "dedup_global synchronises; not capturable");
        return EINVAL;
    }
    ctx->x_row_bytes = ctx->x_ans_bytes = 0;
    // the host-side plan and answer-count matrices (64 KB together: heap,
    // not a daemon thread's stack), before any collective, so that a failed
    // allocation is announced like any local error
    std::unique_ptr<DgPlan> plp(new (std::nothrow) DgPlan);
    std::unique_ptr<DgAns> anp(new (std::nothrow) DgAns);
    int err = dg_check(sig, gidx, n, rep_out, ref_out, nranks);
    if (!err && (!plp || !anp)) {
        std::snprintf(ctx->err, sizeof(ctx->err), "dedup_global: host allocation");
        err = ENOMEM;
    }
    if (!err)
        err = ensure_buf(ctx, &ctx->xa, &ctx->xa_bytes, dg_a_bytes(n, nranks), st);
    // room for the own rows the bucket pass writes in place (<= n of them)
    if (!err)
        err = ensure_buf(ctx, &ctx->xb, &ctx->xb_bytes, dg_b_bytes(n), st);
    WsScope wsc(ctx, st);
    const size_t w = (size_t)nranks + kAnnTail;
    uint64_t *ann = ctx->dann, *all = ctx->dann + kAnnMax, *dflag = ctx->dann + kAnnMax + 64 * kAnnMax;
    uint64_t *htail = ctx->hann, *hall = ctx->hann + 64 * kAnnTail, *hflag = hall + 64 * kAnnMax;
    uint32_t *dans = reinterpret_cast<uint32_t *>(ctx->dann + kAnsAllDev);
    uint32_t *hans = reinterpret_cast<uint32_t *>(ctx->hann + kAnsAllHost);
    DgSide s;
    s.sig = sig;
    s.gidx = gidx;
    s.n = n;
    s.rep_out = rep_out;
    s.ref_out = ref_out;
    hipError_t e;
    const uint64_t cap = fdfs::bucket_cap(n, (uint32_t)nranks);
    if (!err) {
        dg_carve_a(s, ctx->xa, nranks);
        if ((e = dg_bucket(ctx, s, nranks, me, static_cast<uint8_t *>(ctx->xb), ann, cap, st)) != hipSuccess)
            err = fail(ctx, e, "dedup_global bucket");
    }
    if (err && (e = fdfs::launch_zero_u32(ann, 2ull * nranks, st)) != hipSuccess)
        return fail(ctx, e, "dedup_global announce");  // the device is gone; so is the exchange
    if ((e = dg_announce(ann + nranks, htail, ctx->xb_bytes, ctx->ws_bytes, err, cap, st)) != hipSuccess)
        return fail(ctx, e, "dedup_global announce");
    // 1. every rank's announcement to every rank, then to the host (the row
    //    exchange is sized by it)
    ncclResult_t r = ncclAllGather(ann, all, w, ncclUint64, c, st);
    if (r != ncclSuccess)
        return nccl_fail(ctx, r, "ncclAllGather announcements");
    if ((e = hipMemcpyAsync(hall, all, 8 * w * nranks, hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return fail(ctx, e, "dedup_global announcements");
    if (!plp)
        return ENOMEM;  // announced above: every rank returns
    DgPlan &pl = *plp;
    dg_plan(hall, nranks, pl);
    if (pl.err)
        return dg_plan_error(ctx, pl, me);
    const bool exact = pl.over;
    if (pl.over) {
        // an owner over some rank's cap (skewed owners): every rank sees it
        // in the same counts and buckets again in the exact layout; the
        // counts do not change, so nothing is announced again
        pl.exact();
        if ((e = dg_bucket(ctx, s, nranks, me, static_cast<uint8_t *>(ctx->xb), ann, 0, st)) != hipSuccess)
            return fail(ctx, e, "dedup_global bucket");
    }
    if (pl.grow) {
        // some owner must grow its buffers: each grows its own (keeping the
        // own rows at the front), and the ranks agree on the outcome (max over
        // ranks) before any row moves
        int gerr = grow_keep(ctx, &ctx->xb, &ctx->xb_bytes, dg_b_bytes(pl.m[me]), 32 * pl.cnt[me][me], st);
        if (!gerr)
            gerr = ensure_ws(ctx, dedup_ws_bytes(pl.m[me]), st);
        hflag[0] = (uint64_t)gerr;
        if ((e = hipMemcpyAsync(dflag, hflag, 8, hipMemcpyHostToDevice, st)) != hipSuccess)
            return fail(ctx, e, "dedup_global agreement");
        if ((r = ncclAllReduce(dflag, dflag, 1, ncclUint64, ncclMax, c, st)) != ncclSuccess)
            return nccl_fail(ctx, r, "ncclAllReduce agreement");
        if ((e = hipMemcpyAsync(hflag, dflag, 8, hipMemcpyDeviceToHost, st)) != hipSuccess ||
            (e = hipStreamSynchronize(st)) != hipSuccess)
            return fail(ctx, e, "dedup_global agreement");
        if (hflag[0]) {
            if (!gerr)
                std::snprintf(ctx->err, sizeof(ctx->err), "dedup_global: another rank could not grow its buffers");
            return gerr ? gerr : (int)hflag[0];
        }
    }
    dg_carve_b(s, ctx->xb, pl.m[me]);
    // 2. rows to their owners over xGMI (the own rows are already in place)
    std::vector<DgMove> sends, recvs;
    for (int q = 0; q < nranks; q++)
        if (q != me && pl.cnt[me][q]) {
            sends.push_back({q, reinterpret_cast<char *>(s.rows) + 32 * pl.soff(me, q), 32 * pl.cnt[me][q]});
            ctx->x_row_bytes += 32 * pl.cnt[me][q];
        }
    for (int p = 0; p < nranks; p++)
        if (p != me && pl.cnt[p][me])
            recvs.push_back({p, reinterpret_cast<char *>(s.rows_in) + 32 * pl.roff(me, p), 32 * pl.cnt[p][me]});
    int rc;
    if ((rc = dg_nccl_group(ctx, c, sends, recvs, st)))
        return rc;
    // 3. the owner's group: sink records for the rows of multi-member classes
    if ((e = dg_group(ctx, s, all, w, nranks, me, exact, st)) != hipSuccess)
        return fail(ctx, e, "dedup_global group");
    uint64_t nb = 0;
    if (nranks > 1) {
        // 4. every owner's record count per segment to every rank (the way
        //    back is sized by it), then the records to their senders
        if ((r = ncclAllGather(s.cntr, dans, (size_t)nranks, ncclUint32, c, st)) != ncclSuccess)
            return nccl_fail(ctx, r, "ncclAllGather answer counts");
        if ((e = hipMemcpyAsync(hans, dans, 4 * (size_t)nranks * nranks, hipMemcpyDeviceToHost, st)) != hipSuccess ||
            (e = hipStreamSynchronize(st)) != hipSuccess)
            return fail(ctx, e, "dedup_global answer counts");
        DgAns *an = anp.get();
        an->load(hans, nranks);
        sends.clear();
        recvs.clear();
        for (int p = 0; p < nranks; p++)
            if (p != me && an->a[me][p]) {
                sends.push_back({p, reinterpret_cast<char *>(s.ans) + 16 * pl.roff(me, p), 16 * an->a[me][p]});
                ctx->x_ans_bytes += 16 * an->a[me][p];
            }
        for (int q = 0; q < nranks; q++)
            if (q != me && an->a[q][me])
                recvs.push_back({q, reinterpret_cast<char *>(s.back) + 16 * an->boff(me, q), 16 * an->a[q][me]});
        nb = an->recv_total(me, nranks);
        if ((rc = dg_nccl_group(ctx, c, sends, recvs, st)))
            return rc;
    }
    // 5. the records over the pre-filled singleton answers
    e = dg_apply(s, pl.cnt[me][me], nb, st);
    return e == hipSuccess ? 0 : fail(ctx, e, "dedup_global apply");
}

int fdfs_gpu_dedup_global_local(fdfs_gpu_ctx *ctx, int nranks, const uint8_t *const *sig,
                                const uint64_t *const *gidx, const uint64_t *n, uint64_t *const *rep_out,
                                uint32_t *const *ref_out, void *stream)
{
    if (!ctx || nranks < 1 || nranks > 64 || !sig || !n || !rep_out || !ref_out || (nranks > 1 && !gidx))
        return EINVAL;
    for (int p = 0; p < nranks; p++)
        if (dg_check(sig[p], gidx ? gidx[p] : nullptr, n[p], rep_out[p], ref_out[p], nranks))
            return EINVAL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (capturing(st)) {
        std::snprintf(ctx->err, sizeof(ctx->err), "dedup_global_local synchronises; not capturable");
        return EINVAL;
    }
    ctx->x_row_bytes = ctx->x_ans_bytes = 0;
    WsScope wsc(ctx, st);
    const size_t w = (size_t)nranks + kAnnTail;
    uint64_t *all = ctx->dann + kAnnMax;
    uint64_t *htail = ctx->hann, *hall = ctx->hann + 64 * kAnnTail;
    uint32_t *hans = reinterpret_cast<uint32_t *>(ctx->hann + kAnsAllHost);
    std::vector<DgSide> s(nranks);
    size_t abytes = 0;
    for (int p = 0; p < nranks; p++)
        abytes += dg_a_bytes(n[p], nranks);
    void *amem = nullptr, *bmem = nullptr;
    hipError_t e = hipMalloc(&amem, abytes);
    if (e != hipSuccess) {
        std::snprintf(ctx->err, sizeof(ctx->err), "hipMalloc(%zu): %s", abytes, hipGetErrorString(e));
        return ENOMEM;
    }
    int rc = 0;
    DgPlan *pl = new (std::nothrow) DgPlan;
    DgAns *an = new (std::nothrow) DgAns;
    if (!pl || !an)
        rc = ENOMEM;
    size_t done = 0;
    for (int p = 0; p < nranks && !rc; p++) {
        s[p].sig = sig[p];
        s[p].gidx = gidx ? gidx[p] : nullptr;
        s[p].n = n[p];
        s[p].rep_out = rep_out[p];
        s[p].ref_out = ref_out[p];
        dg_carve_a(s[p], static_cast<char *>(amem) + done, nranks);
        done += dg_a_bytes(n[p], nranks);
        // 1. every virtual rank's bucket (its own rows to their send slots:
        //    this transport copies every segment) and announcement (no
        //    owner-side buffers yet: room 0, so the plan always grows them)
        const uint64_t cap = fdfs::bucket_cap(n[p], (uint32_t)nranks);
        if ((e = dg_bucket(ctx, s[p], nranks, p, nullptr, all + p * w, cap, st)) != hipSuccess ||
            (e = dg_announce(all + p * w + nranks, htail + kAnnTail * p, 0, ctx->ws_bytes, 0, cap, st)) != hipSuccess)
            rc = fail(ctx, e, "dedup_global_local bucket");
    }
    if (!rc && ((e = hipMemcpyAsync(hall, all, 8 * w * nranks, hipMemcpyDeviceToHost, st)) != hipSuccess ||
                (e = hipStreamSynchronize(st)) != hipSuccess))
        rc = fail(ctx, e, "dedup_global_local announcements");
    if (!rc) {
        dg_plan(hall, nranks, *pl);
        rc = pl->err ? dg_plan_error(ctx, *pl, -1) : 0;
    }
    const bool exact = !rc && pl->over;
    if (exact) {  // an owner over some rank's cap: every rank's exact layout
        pl->exact();
        for (int p = 0; p < nranks && !rc; p++)
            if ((e = dg_bucket(ctx, s[p], nranks, p, nullptr, all + p * w, 0, st)) != hipSuccess)
                rc = fail(ctx, e, "dedup_global_local bucket");
    }
    size_t bbytes = 0, wsb = 0;
    for (int q = 0; q < nranks && !rc; q++) {
        bbytes += dg_b_bytes(pl->m[q]);
        wsb = std::max(wsb, dedup_ws_bytes(pl->m[q]));
    }
    if (!rc && (e = hipMalloc(&bmem, bbytes)) != hipSuccess) {
        std::snprintf(ctx->err, sizeof(ctx->err), "hipMalloc(%zu): %s", bbytes, hipGetErrorString(e));
        rc = ENOMEM;
    }
    if (!rc)
        rc = ensure_ws(ctx, wsb, st);
    if (!rc) {
        done = 0;
        for (int q = 0; q < nranks; q++) {
            dg_carve_b(s[q], static_cast<char *>(bmem) + done, pl->m[q]);
            done += dg_b_bytes(pl->m[q]);
        }
        // 2. rows to their owners (every segment a device copy), 3. each
        //    owner's group (one workspace, stream-ordered)
        for (int p = 0; p < nranks && !rc; p++)
            for (int q = 0; q < nranks && !rc; q++)
                if (pl->cnt[p][q]) {
                    if ((e = hipMemcpyAsync(s[q].rows_in + 32 * pl->roff(q, p), s[p].rows + 32 * pl->soff(p, q),
                                            32 * pl->cnt[p][q], hipMemcpyDeviceToDevice, st)) != hipSuccess)
                        rc = fail(ctx, e, "dedup_global_local row copy");
                    if (p != q)
                        ctx->x_row_bytes += 32 * pl->cnt[p][q];
                }
        for (int q = 0; q < nranks && !rc; q++)
            if ((e = dg_group(ctx, s[q], all, w, nranks, q, exact, st)) != hipSuccess)
                rc = fail(ctx, e, "dedup_global_local group");
        // 4. the owners' record counts, then the records back to the senders
        for (int q = 0; q < nranks && !rc; q++)
            if ((e = hipMemcpyAsync(hans + (size_t)q * nranks, s[q].cntr, 4 * (size_t)nranks,
                                    hipMemcpyDeviceToHost, st)) != hipSuccess)
                rc = fail(ctx, e, "dedup_global_local answer counts");
        if (!rc && (e = hipStreamSynchronize(st)) != hipSuccess)
            rc = fail(ctx, e, "dedup_global_local answer counts");
        if (!rc)
            an->load(hans, nranks);
        for (int q = 0; q < nranks && !rc; q++)
            for (int p = 0; p < nranks && !rc; p++)
                if (p != q && an->a[q][p]) {
                    if ((e = hipMemcpyAsync(s[p].back + 16 * an->boff(p, q), s[q].ans + 16 * pl->roff(q, p),
                                            16 * an->a[q][p], hipMemcpyDeviceToDevice, st)) != hipSuccess)
                        rc = fail(ctx, e, "dedup_global_local answer copy");
                    ctx->x_ans_bytes += 16 * an->a[q][p];
                }
        // 5. every rank's records over its pre-filled answers
        for (int p = 0; p < nranks && !rc; p++)
            if ((e = dg_apply(s[p], pl->cnt[p][p], an->recv_total(p, nranks), st)) != hipSuccess)
                rc = fail(ctx, e, "dedup_global_local apply");
    }
    // the buffers are freed only once the stream is done with them
    e = hipStreamSynchronize(st);
    if (!rc && e != hipSuccess)
        rc = fail(ctx, e, "dedup_global_local");
    (void)hipFree(amem);
    if (bmem)
        (void)hipFree(bmem);
    delete pl;
    delete an;
    return rc;
}

int fdfs_gpu_dedup_global_stats(fdfs_gpu_ctx *ctx, uint64_t *row_bytes, uint64_t *answer_bytes)
{
    if (!ctx || !row_bytes || !answer_bytes)
        return EINVAL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    *row_bytes = ctx->x_row_bytes;
    *answer_bytes = ctx->x_ans_bytes;
    return 0;
}

// ---- split-file CRC over N GPUs -------------------------------

extern "C++" {

static int cg_check(const fdfs_gpu_batch *pieces, const uint64_t *pfile, const uint64_t *pstart,
                    const uint64_t *fsize, uint64_t nfiles, const uint32_t *crc_out)
{
    if (!pieces)
        return EINVAL;
    if (pieces->n && (!pieces->base || !pieces->offset || !pieces->size || !pfile || !pstart))
        return EINVAL;
    if (nfiles && (!fsize || !crc_out))
        return EINVAL;
    return 0;
}

// The segmented pass over one rank's pieces (their CRC32_ex from XINIT) and
// the pieces' terms in that rank's block of `blk` (zeroed first).
static size_t cg_ws_bytes(uint64_t np) { return align_up(4 * np) + sig_ws_bytes(np); }

static hipError_t cg_pieces(fdfs_gpu_ctx *ctx, const fdfs_gpu_batch *pieces, const uint64_t *pfile,
                            const uint64_t *pstart, const uint64_t *fsize, uint64_t nfiles, const fdfs::CrcParts &blk,
                            uint32_t r, hipStream_t st)
{
    fdfs::CrcParts mine = blk;
    mine.base = blk.base + r * blk.stride;
    hipError_t e = fdfs::launch_zero_u32(mine.base, fdfs::CrcParts::block_bytes(nfiles) / 4, st);
    const uint32_t np = pieces->n;
    if (e != hipSuccess || !np)
        return e;
    Carve cv{static_cast<char *>(ctx->ws)};
    uint32_t *crc = cv.take<uint32_t>(np);
    uint64_t *nseg = cv.take<uint64_t>(2 * (size_t)np);
    uint64_t *first = cv.take<uint64_t>(2 * ((size_t)np + 1));
    uint64_t *bsum = cv.take<uint64_t>(2 * fdfs::scan_workspace_elems(np));
    hipEvent_t a, b;
    timing_pair(ctx, FDFS_KERNEL_CRC_SEG, a, b);
    e = fdfs::launch_crc_seg(ctx->sar, static_cast<const uint8_t *>(pieces->base), pieces->offset, pieces->size, np,
                             nseg, first, bsum, ctx->d_tabs, crc, ctx->ncu, st, a, b);
    if (e == hipSuccess)
        e = fdfs::launch_crc_pieces(crc, pfile, pstart, pieces->size, np, fsize, nfiles, mine, ctx->d_tabs, st);
    return e;
}

// The fold of every rank's block into crc_out, then the error words to the
// host (the call's last synchronisation): 0, or EINVAL with the reason.
static int cg_fold(fdfs_gpu_ctx *ctx, const fdfs::CrcParts &blk, int nranks, const uint64_t *fsize, uint64_t nfiles,
                   uint32_t *crc_out, hipStream_t st, const char *who)
{
    uint64_t *derr = ctx->dann + kAnnMax + 64 * kAnnMax + 4;
    uint64_t *herr = ctx->hann + 64 * kAnnTail + 64 * kAnnMax + 4;
    hipError_t e = fdfs::launch_zero_u32(derr, 4, st);
    if (e == hipSuccess)
        e = fdfs::launch_crc_fold(blk, (uint32_t)nranks, fsize, nfiles, crc_out, derr, ctx->d_tabs, st);
    if (e == hipSuccess)
        e = hipMemcpyAsync(herr, derr, 16, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess)
        e = hipStreamSynchronize(st);
    if (e != hipSuccess)
        return fail(ctx, e, who);
    if (herr[0] || herr[1]) {
        std::snprintf(ctx->err, sizeof(ctx->err),
                      "%s: pieces outside their files on rank mask 0x%llx; %llu files not covered exactly by "
                      "their pieces (crc_out invalid)",
                      who, (unsigned long long)herr[0], (unsigned long long)herr[1]);
        return EINVAL;
    }
    return 0;
}

}  // extern "C++"

int fdfs_gpu_crc_batch_global(fdfs_gpu_ctx *ctx, void *comm, const fdfs_gpu_batch *pieces, const uint64_t *piece_file,
                              const uint64_t *piece_start, const uint64_t *file_size, uint64_t nfiles,
                              uint32_t *crc_out, void *stream)
{
    if (!ctx || !comm)
        return EINVAL;
    ncclComm_t c = static_cast<ncclComm_t>(comm);
    int nranks = 0, me = 0;
    if (ncclCommCount(c, &nranks) != ncclSuccess || ncclCommUserRank(c, &me) != ncclSuccess ||
        nranks < 1 || nranks > 64)
        return EINVAL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    // as in dedup_global: not capturable (EINVAL before any collective), and
    // a local error is announced, not returned, so that no rank waits alone
    // in a collective
    if (capturing(st)) {
        std::snprintf(ctx->err, sizeof(ctx->err), "crc_batch_global synchronises; not capturable");
        return EINVAL;
    }
    int err = cg_check(pieces, piece_file, piece_start, file_size, nfiles, crc_out);
    const uint64_t bb = fdfs::CrcParts::block_bytes(nfiles);
    if (!err)
        err = ensure_buf(ctx, &ctx->xa, &ctx->xa_bytes, bb * nranks, st);
    if (!err)
        err = ensure_ws(ctx, cg_ws_bytes(pieces->n), st);
    WsScope wsc(ctx, st);
    uint64_t *ann = ctx->dann, *all = ctx->dann + kAnnMax;
    uint64_t *htail = ctx->hann, *hall = ctx->hann + 64 * kAnnTail;
    htail[0] = nfiles;
    htail[1] = (uint64_t)err;
    // 1. announcement {nfiles, errno} of every rank: the sizes of the
    //    exchange agree, or every rank returns the first rank's error
    hipError_t e = hipMemcpyAsync(ann, htail, 16, hipMemcpyHostToDevice, st);
    if (e != hipSuccess)
        return fail(ctx, e, "crc_batch_global announce");
    ncclResult_t r = ncclAllGather(ann, all, 2, ncclUint64, c, st);
    if (r != ncclSuccess)
        return nccl_fail(ctx, r, "ncclAllGather announcements");
    if ((e = hipMemcpyAsync(hall, all, 16ull * nranks, hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return fail(ctx, e, "crc_batch_global announcements");
    for (int p = 0; p < nranks; p++) {
        if (hall[2 * p + 1] || hall[2 * p] != nfiles) {
            const int perr = hall[2 * p + 1] ? (int)hall[2 * p + 1] : EINVAL;
            std::snprintf(ctx->err, sizeof(ctx->err), "crc_batch_global: rank %d %s", p,
                          hall[2 * p + 1] ? (perr == ENOMEM ? "is out of memory" : "has invalid arguments")
                                          : "passed a different file count");
            return perr;
        }
    }
    // 2. this rank's pieces into its block of the all-gather buffer,
    // 3. the blocks to every rank (in place), 4. the fold
    const fdfs::CrcParts blk{static_cast<char *>(ctx->xa), nfiles, bb};
    if ((e = cg_pieces(ctx, pieces, piece_file, piece_start, file_size, nfiles, blk, (uint32_t)me, st)) != hipSuccess)
        return fail(ctx, e, "crc_batch_global pieces");
    if ((r = ncclAllGather(blk.base + me * bb, blk.base, bb, ncclUint8, c, st)) != ncclSuccess)
        return nccl_fail(ctx, r, "ncclAllGather crc blocks");
    return cg_fold(ctx, blk, nranks, file_size, nfiles, crc_out, st, "crc_batch_global");
}

int fdfs_gpu_crc_batch_global_local(fdfs_gpu_ctx *ctx, int nranks, const fdfs_gpu_batch *pieces,
                                    const uint64_t *const *piece_file, const uint64_t *const *piece_start,
                                    const uint64_t *file_size, uint64_t nfiles, uint32_t *crc_out, void *stream)
{
    if (!ctx || nranks < 1 || nranks > 64 || !pieces || !piece_file || !piece_start)
        return EINVAL;
    uint32_t maxp = 0;
    for (int p = 0; p < nranks; p++) {
        if (cg_check(&pieces[p], piece_file[p], piece_start[p], file_size, nfiles, crc_out))
            return EINVAL;
        maxp = std::max(maxp, pieces[p].n);
    }
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (capturing(st)) {
        std::snprintf(ctx->err, sizeof(ctx->err), "crc_batch_global_local synchronises; not capturable");
        return EINVAL;
    }
    const uint64_t bb = fdfs::CrcParts::block_bytes(nfiles);
    int rc = ensure_buf(ctx, &ctx->xa, &ctx->xa_bytes, bb * nranks, st);
    if (!rc)
        rc = ensure_ws(ctx, cg_ws_bytes(maxp), st);
    if (rc)
        return rc;
    WsScope wsc(ctx, st);
    // every virtual rank's block where the all-gather would put it (the
    // ranks' segmented passes share the workspace, stream-ordered)
    const fdfs::CrcParts blk{static_cast<char *>(ctx->xa), nfiles, bb};
    for (int p = 0; p < nranks; p++) {
        const hipError_t e =
            cg_pieces(ctx, &pieces[p], piece_file[p], piece_start[p], file_size, nfiles, blk, (uint32_t)p, st);
        if (e != hipSuccess)
            return fail(ctx, e, "crc_batch_global_local pieces");
    }
    return cg_fold(ctx, blk, nranks, file_size, nfiles, crc_out, st, "crc_batch_global_local");
}

// ---- formats that consume the CRC, FastDHT routing, scrub ----

int fdfs_gpu_file_ids(fdfs_gpu_ctx *ctx, uint32_t server_id, const uint32_t *crc32,
                      const int64_t *file_size, const int32_t *timestamp, const uint32_t *rnd,
                      uint32_t n, uint32_t subdir_count, char *name_out, uint8_t *sub_path_out,
                      void *stream)
{
    if (!ctx || subdir_count == 0 || subdir_count > 256)
        return EINVAL;
    if (n == 0)
        return 0;
    if (!crc32 || !file_size || !timestamp || !rnd || !name_out || !sub_path_out)
        return EINVAL;
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipError_t e = fdfs::launch_file_ids(ctx->sar, server_id, crc32, file_size, timestamp, rnd, n,
                                         subdir_count, name_out, sub_path_out,
                                         reinterpret_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : fail(ctx, e, "file_ids launch");
}

int fdfs_gpu_parse_file_ids(fdfs_gpu_ctx *ctx, const char *names, uint32_t n,
                            uint32_t *server_id_out, int32_t *timestamp_out,
                            int64_t *file_size_out, uint32_t *crc32_out, void *stream)
{
    if (!ctx)
        return EINVAL;
    if (n == 0)
        return 0;
    if (!names || !server_id_out || !timestamp_out || !file_size_out || !crc32_out)
        return EINVAL;
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipError_t e = fdfs::launch_parse_file_ids(reinterpret_cast<const uint8_t *>(names), n,
                                               server_id_out, timestamp_out, file_size_out,
                                               crc32_out, reinterpret_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : fail(ctx, e, "parse_file_ids launch");
}

int fdfs_gpu_trunk_pack(fdfs_gpu_ctx *ctx, const uint8_t *file_type, const int32_t *alloc_size,
                        const int32_t *file_size, const uint32_t *crc32, const int32_t *mtime,
                        const char *ext, uint32_t n, uint8_t *hdr_out, void *stream)
{
    if (!ctx)
        return EINVAL;
    if (n == 0)
        return 0;
    if (!file_type || !alloc_size || !file_size || !crc32 || !mtime || !ext || !hdr_out)
        return EINVAL;
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipError_t e = fdfs::launch_trunk_pack(file_type, alloc_size, file_size, crc32, mtime,
                                           reinterpret_cast<const uint8_t *>(ext), n, hdr_out,
                                           reinterpret_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : fail(ctx, e, "trunk_pack launch");
}

int fdfs_gpu_trunk_unpack(fdfs_gpu_ctx *ctx, const uint8_t *hdr, uint32_t n, uint8_t *file_type,
                          int32_t *alloc_size, int32_t *file_size, uint32_t *crc32,
                          int32_t *mtime, char *ext, void *stream)
{
    if (!ctx)
        return EINVAL;
    if (n == 0)
        return 0;
    if (!hdr || !file_type || !alloc_size || !file_size || !crc32 || !mtime || !ext)
        return EINVAL;
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipError_t e = fdfs::launch_trunk_unpack(hdr, n, file_type, alloc_size, file_size, crc32, mtime,
                                             reinterpret_cast<uint8_t *>(ext),
                                             reinterpret_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : fail(ctx, e, "trunk_unpack launch");
}

int fdfs_gpu_fdht_route_keys(fdfs_gpu_ctx *ctx, const uint8_t *keys, uint32_t key_stride,
                             const uint32_t *key_len, uint64_t n, const char *ns, int ns_len,
                             uint32_t group_count, const uint32_t *servers_per_group,
                             int32_t *key_hash_out, uint32_t *group_out, uint32_t *server_out,
                             uint64_t *order_out, uint64_t *group_start_out, void *stream)
{
    // FDHT_MAX_NAMESPACE_LEN / FDHT_MAX_OBJECT_ID_LEN (storage/fdht_client/fdht_types.h:23-24);
    // an empty namespace is rejected like CALC_KEY_HASH_CODE does with an object id
    if (!ctx || !ns || ns_len <= 0 || ns_len > 64 || group_count == 0 || !group_start_out)
        return EINVAL;
    if (key_stride == 0 || key_stride > 128 || (key_stride & 3))
        return EINVAL;
    if (n && (!keys || !key_hash_out || !group_out || !server_out))
        return EINVAL;
    if (reinterpret_cast<uintptr_t>(keys) & 3)  // the kernel reads each key as u32 words
        return EINVAL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int rc = ensure_ws(ctx, align_up(4ull * group_count) + align_up(8ull * group_count), st);
    if (rc)
        return rc;
    WsScope wsc(ctx, st);
    Carve cv{static_cast<char *>(ctx->ws)};
    uint32_t *gcount = cv.take<uint32_t>(group_count);
    uint64_t *cursor = cv.take<uint64_t>(group_count);
    const uint32_t h0 = fdfs::pjw_prefix(ctx->sar, ns, ns_len);
    hipError_t e = fdfs::launch_fdht_route(ctx->sar, keys, key_stride, key_len, n, nullptr, h0,
                                           group_count, servers_per_group, key_hash_out, group_out,
                                           server_out, gcount, group_start_out, cursor, order_out, st);
    return e == hipSuccess ? 0 : fail(ctx, e, "fdht_route launch");
}

int fdfs_gpu_fdht_route(fdfs_gpu_ctx *ctx, const uint8_t *sig, uint64_t n, const char *ns,
                        int ns_len, uint32_t group_count, const uint32_t *servers_per_group,
                        int32_t *key_hash_out, uint32_t *group_out, uint32_t *server_out,
                        uint64_t *order_out, uint64_t *group_start_out, void *stream)
{
    return fdfs_gpu_fdht_route_keys(ctx, sig, 24, nullptr, n, ns, ns_len, group_count,
                                    servers_per_group, key_hash_out, group_out, server_out, order_out,
                                    group_start_out, stream);
}

int fdfs_gpu_recovery_batch(fdfs_gpu_ctx *ctx, const fdfs_gpu_batch *batch, int method,
                            const uint8_t *file_ids, uint32_t id_stride, const uint32_t *id_len,
                            const char *ns, int ns_len, uint32_t group_count,
                            const uint32_t *servers_per_group, fdfs_gpu_recovery_out *out,
                            void *stream)
{
    if (!ctx || !batch || !out || (method != FDFS_SIG_HASH && method != FDFS_SIG_MD5))
        return EINVAL;
    if (!ns || ns_len <= 0 || ns_len > 64 || group_count == 0)
        return EINVAL;
    if (id_stride == 0 || id_stride > 128 || (id_stride & 3) ||
        (reinterpret_cast<uintptr_t>(file_ids) & 3))
        return EINVAL;
    const uint64_t n = batch->n;
    const fdfs_gpu_routed *sets[3] = {&out->fid, &out->ref_rec, &out->sig_rec};
    for (const fdfs_gpu_routed *r : sets)
        if (!r->group_start || (n && (!r->index || !r->key_hash || !r->group || !r->server)))
            return EINVAL;
    if (n && (!file_ids || !out->crc || !out->sig || !out->rep || !out->ref || !out->nsources))
        return EINVAL;
    if ((reinterpret_cast<uintptr_t>(out->sig) | reinterpret_cast<uintptr_t>(out->rep)) & 7)
        return EINVAL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (n == 0) {
        for (const fdfs_gpu_routed *r : sets)
            if (fdfs::launch_zero_u32(r->group_start, 2ull * (group_count + 1), st) != hipSuccess)
                return fail(ctx, hipGetLastError(), "recovery_batch memset");
        return 0;
    }
    // workspace: region A (offset 0) is what the sig / dedup / route calls
    // below carve for themselves; region B after it holds the compacted
    // class sources, which must live across those calls
    const size_t a_bytes = std::max(std::max(sig_ws_bytes(n), dedup_ws_bytes(n)),
                                    align_up(4ull * group_count) + align_up(8ull * group_count));
    const size_t b_bytes = align_up(8 * n) + align_up(8 * (n + 1)) +
                           align_up(8 * fdfs::scan_workspace_elems(n)) + align_up(24 * n) +
                           align_up((size_t)id_stride * n) + align_up(4 * n);
    int rc = ensure_ws(ctx, a_bytes + b_bytes, st);
    if (rc)
        return rc;
    WsScope wsc(ctx, st);
    Carve cv{static_cast<char *>(ctx->ws) + a_bytes};
    uint64_t *flag = cv.take<uint64_t>(n);
    uint64_t *pos = cv.take<uint64_t>(n + 1);
    uint64_t *bsum = cv.take<uint64_t>(fdfs::scan_workspace_elems(n));
    uint8_t *csig = cv.take<uint8_t>(24 * n);
    uint8_t *cids = cv.take<uint8_t>((size_t)id_stride * n);
    uint32_t *clen = cv.take<uint32_t>(n);
    // 1. CRC32 + signature, 2. the dedup decision over the batch in order
    if ((rc = fdfs_gpu_sig_batch(ctx, batch, method, out->crc, out->sig, nullptr, stream)))
        return rc;
    if ((rc = fdfs_gpu_dedup(ctx, out->sig, nullptr, n, out->rep, out->ref, stream)))
        return rc;
    // 3. class sources (rep[i] == i), compacted; sig_rec.index = 0..n-1
    hipError_t e = fdfs::launch_sources(out->rep, n, out->sig, file_ids, id_stride, id_len, flag, pos,
                                        bsum, out->sig_rec.index, out->fid.index, csig, cids, clen,
                                        out->nsources, st);
    if (e != hipSuccess)
        return fail(ctx, e, "recovery_batch sources");
    if (hipMemcpyAsync(out->ref_rec.index, out->fid.index, 8 * n, hipMemcpyDeviceToDevice, st) !=
        hipSuccess)
        return fail(ctx, hipGetLastError(), "recovery_batch copy");
    // 4. the three record sets, routed per FastDHT group
    Carve ca{static_cast<char *>(ctx->ws)};
    uint32_t *gcount = ca.take<uint32_t>(group_count);
    uint64_t *cursor = ca.take<uint64_t>(group_count);
    const uint32_t h0 = fdfs::pjw_prefix(ctx->sar, ns, ns_len);
    struct Job {
        const fdfs_gpu_routed *r;
        const uint8_t *keys;
        uint32_t stride;
        const uint32_t *lens;
        const uint64_t *dcount;
    } jobs[3] = {{&out->fid, csig, 24, nullptr, out->nsources},
                 {&out->ref_rec, cids, id_stride, clen, out->nsources},
                 {&out->sig_rec, file_ids, id_stride, id_len, nullptr}};
    for (const Job &j : jobs) {
        e = fdfs::launch_fdht_route(ctx->sar, j.keys, j.stride, j.lens, n, j.dcount, h0, group_count,
                                    servers_per_group, j.r->key_hash, j.r->group, j.r->server, gcount,
                                    j.r->group_start, cursor, j.r->order, st);
        if (e != hipSuccess)
            return fail(ctx, e, "recovery_batch route");
    }
    return 0;
}

int fdfs_gpu_scrub(fdfs_gpu_ctx *ctx, const fdfs_gpu_batch *batch, const uint32_t *expected_crc,
                   uint32_t *crc_out, uint8_t *bad_out, uint32_t *nbad_out, void *stream)
{
    if (!ctx || !batch || !expected_crc || !crc_out || !bad_out || !nbad_out)
        return EINVAL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    int rc = fdfs_gpu_sig_batch(ctx, batch, FDFS_SIG_CRC_ONLY, crc_out, nullptr, nullptr, stream);
    if (rc || batch->n == 0)
        return rc;
    DeviceGuard g(ctx->device);
    if (!g.ok)
        return ENODEV;
    hipError_t e = fdfs::launch_scrub(crc_out, expected_crc, batch->n, bad_out, nbad_out,
                                      reinterpret_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : fail(ctx, e, "scrub launch");
}

}  // extern "C"
