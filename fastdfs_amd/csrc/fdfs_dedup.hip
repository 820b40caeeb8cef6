// libfdfs_gpu bulk duplicate grouping (gfx950).
//
// Replaces the per-file FastDHT round trips of the upload-done handler
// (storage/storage_service.c:2652 get "fid", :2714 set "fid", :2734 set "ref",
// :2984 inc "ref") for bulk / recovery ingest.  Output per record, in input
// order: rep = smallest ingest index with the same 24-byte signature (the
// file that became the "fid" source), ref = number of records sharing it
// (the "ref" count after every link).
//
//  * dedup_bucket: owner rank = hash(sig) mod nranks; rows {sig[24], gidx}
//    packed per owner for one all-to-all over RCCL (the FastDHT key
//    partition, storage/fdht_client/fdht_client.c:301-305, re-expressed as a
//    GPU bucket).
//  * dedup_group: partition, then group each partition in LDS.
//      K1 dp_keys      key32 = low half of a 64-bit mix of the signature;
//                      per-tile LDS histogram of its top D1 bits
//      K2 scan         exclusive scan of the [digit][tile] counts
//      K3 dp_scatter   (key32, record) pairs to their D1 bucket (LDS ranks)
//      K4 dp_split     one workgroup per D1 bucket splits it by the next D2
//                      bits (LDS histogram + scan + LDS cursors)
//      K5 dp_group     one workgroup per partition (~1K records): an
//                      open-addressing table in LDS keyed by key32, a slot
//                      is claimed by 64-bit CAS of {key32, claimer} and never
//                      changes, equal keys are confirmed on the full 24 bytes
//                      against the claimer's row, class min(gidx) and size
//                      by LDS atomics, then rep/ref written per record.
//    Every random-access atomic stays in LDS: device-scope atomics to
//    random addresses run at a few percent of the HBM rate on MI355X
//    (MI355X_MICROARCH.md, global atomics), which is what bounded the
//    single global hash table this replaces (20 ms for 100M records).
//    A partition with more records than the LDS table holds (heavy
//    duplication of one signature, or adversarial keys) is grouped by the
//    same code on a table in HBM, in a region of the workspace that belongs
//    to that partition alone; results do not depend on arrival order.
#include "fdfs_device.hpp"
#include "fdfs_kernels.hpp"

#include <cstdlib>

namespace fdfs {

__device__ __forceinline__ uint64_t fmix64(uint64_t k)
{
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

__device__ __forceinline__ void load_sig(const uint8_t *row, uint64_t &a, uint64_t &b, uint64_t &c)
{
    const uint64_t *p = reinterpret_cast<const uint64_t *>(row);
    a = p[0];
    b = p[1];
    c = p[2];
}

__device__ __forceinline__ uint64_t sig_hash(uint64_t a, uint64_t b, uint64_t c)
{
    return fmix64(a ^ fmix64(b ^ fmix64(c + 0x9E3779B97F4A7C15ull)));
}

__device__ __forceinline__ bool sig_equal(const uint8_t *sig, uint32_t stride, uint32_t x, uint32_t y)
{
    uint64_t a, b, c, a2, b2, c2;
    load_sig(sig + (uint64_t)x * stride, a, b, c);
    load_sig(sig + (uint64_t)y * stride, a2, b2, c2);
    return a == a2 && b == b2 && c == c2;
}

constexpr int kDpTileThreads = 256;
constexpr int kDpTileItems = 16;
constexpr int kDpTile = kDpTileThreads * kDpTileItems;  // records per K1/K3 tile
constexpr int kDpMaxD1 = 8;
constexpr int kDpMaxD2 = 12;
constexpr int kDpSlotsLog = 11;  // LDS table: 2048 slots
constexpr int kDpSlots = 1 << kDpSlotsLog;
constexpr uint32_t kDpCap = kDpSlots * 3 / 4;  // records per partition grouped in LDS
constexpr uint64_t kDpEmpty = ~0ull;
constexpr int kDpGroupThreads = 512;

struct DpPlan {
    int d1, d2;          // partition bits: top d1 of key32 (K3), next d2 (K4)
    uint64_t tiles;      // K1/K3 tiles
    uint64_t nparts() const { return 1ull << (d1 + d2); }
};

DpPlan dp_plan(uint64_t n)
{
    int p = 1;  // partitions of ~1K records: mean n / 2^p <= 1024
    while (p < kDpMaxD1 + kDpMaxD2 && (n >> p) > 1024)
        p++;
    DpPlan pl;
    pl.d1 = p < kDpMaxD1 ? p : kDpMaxD1;
    pl.d2 = p - pl.d1;
    pl.tiles = (n + kDpTile - 1) / kDpTile;
    return pl;
}

// K1: key32 per record + the tile's histogram of the top d1 bits; the
// singleton answer (rep = own gidx, ref = 1) for every record
__global__ __launch_bounds__(kDpTileThreads) void dp_keys_kernel(
    const uint8_t *__restrict__ sig, uint32_t stride, const uint64_t *__restrict__ gidx,
    uint32_t gstride, uint64_t n, int d1, uint64_t tiles, uint32_t *__restrict__ keys,
    uint64_t *__restrict__ rep_out, uint32_t *__restrict__ ref_out, uint64_t *__restrict__ counts)
{
    __shared__ uint32_t h[1 << kDpMaxD1];
    for (int k = threadIdx.x; k < (1 << d1); k += blockDim.x)
        h[k] = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * kDpTile;
    for (int it = 0; it < kDpTileItems; it++) {
        const uint64_t r = t0 + (uint64_t)it * kDpTileThreads + threadIdx.x;
        if (r < n) {
            uint64_t a, b, c;
            load_sig(sig + r * stride, a, b, c);
            const uint32_t key = (uint32_t)sig_hash(a, b, c);
            keys[r] = key;
            // every record starts as its own class; dp_group overwrites the
            // records of classes with more than one member
            rep_out[r] = gstride ? gidx[r * gstride] : r;
            ref_out[r] = 1;
            atomicAdd(&h[key >> (32 - d1)], 1u);
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < (1 << d1); k += blockDim.x)
        counts[(uint64_t)k * tiles + blockIdx.x] = h[k];
}

// Exclusive scan of cnt[0, nb) into out[] by the whole block (each thread
// owns PER consecutive bins; nb <= PER * blockDim.x).
template <int PER, int NT>
__device__ __forceinline__ void block_scan_bins(const uint32_t *cnt, uint32_t *out, uint32_t nb,
                                                uint32_t *wsum)
{
    uint32_t v[PER], sum = 0;
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const uint32_t k = threadIdx.x * PER + q;
        v[q] = k < nb ? cnt[k] : 0u;
        sum += v[q];
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o)
            x += y;
    }
    if (lane == 63)
        wsum[wid] = x;
    __syncthreads();
    uint32_t run = x - sum;
    for (int k = 0; k < wid; k++)
        run += wsum[k];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const uint32_t k = threadIdx.x * PER + q;
        if (k < nb)
            out[k] = run;
        run += v[q];
    }
    __syncthreads();
}

// K3: the 8-byte entry {key32 << 32 | record} to its d1 bucket.  The tile is
// ranked by LDS counters (unstable: order inside a partition does not
// matter), sorted by digit in LDS and written out as contiguous runs (one run
// per digit).  The ingest index is not carried: dp_group reads it only for
// records of multi-member classes.
__global__ __launch_bounds__(kDpTileThreads) void dp_scatter_kernel(
    const uint32_t *__restrict__ keys, uint64_t n, int d1, uint64_t tiles,
    const uint64_t *__restrict__ off, uint64_t *__restrict__ ent)
{
    __shared__ uint32_t cnt[1 << kDpMaxD1];
    __shared__ uint32_t lst[1 << kDpMaxD1];
    __shared__ uint64_t bas[1 << kDpMaxD1];
    __shared__ uint32_t wsum[kDpTileThreads / 64];
    __shared__ uint64_t stage[kDpTile];
    const uint32_t nb = 1u << d1;
    for (uint32_t k = threadIdx.x; k < nb; k += blockDim.x) {
        cnt[k] = 0;
        bas[k] = off[(uint64_t)k * tiles + blockIdx.x];
    }
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * kDpTile;
    const uint32_t m = (uint32_t)((n - t0) < (uint64_t)kDpTile ? (n - t0) : (uint64_t)kDpTile);
    uint32_t key[kDpTileItems], rank[kDpTileItems];
#pragma unroll
    for (int it = 0; it < kDpTileItems; it++) {
        const uint32_t l = it * kDpTileThreads + threadIdx.x;
        if (l < m) {
            key[it] = keys[t0 + l];
            rank[it] = atomicAdd(&cnt[key[it] >> (32 - d1)], 1u);
        }
    }
    __syncthreads();
    block_scan_bins<1, kDpTileThreads>(cnt, lst, nb, wsum);
#pragma unroll
    for (int it = 0; it < kDpTileItems; it++) {
        const uint32_t l = it * kDpTileThreads + threadIdx.x;
        if (l < m)
            stage[lst[key[it] >> (32 - d1)] + rank[it]] = ((uint64_t)key[it] << 32) | (uint32_t)(t0 + l);
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < m; j += blockDim.x) {
        const uint64_t en = stage[j];
        const uint32_t d = (uint32_t)(en >> (64 - d1));
        ent[bas[d] + (j - lst[d])] = en;
    }
}

// K4: one workgroup per d1 bucket: split by the next d2 bits into ent2 and
// write the partition starts (pstart[nparts] = n).  A first pass counts the
// whole bucket; the second goes chunk by chunk (rank, LDS sort by digit,
// contiguous runs out, per-digit cursors advanced by the chunk's counts).
constexpr int kDpSplitThreads = 1024;
constexpr int kDpSplitPer = 8;  // entries per thread per chunk (FDFS_GPU_DEDUP_SPLIT=4: A/B)

template <int PER_T>
__global__ __launch_bounds__(kDpSplitThreads) void dp_split_kernel(
    const uint64_t *__restrict__ ent, uint64_t n, int d1, int d2, uint64_t tiles,
    const uint64_t *__restrict__ off, uint64_t *__restrict__ ent2, uint32_t *__restrict__ pstart)
{
    constexpr int NB = 1 << kDpMaxD2;
    constexpr int PER = NB / kDpSplitThreads;
    __shared__ uint32_t h[NB];    // bucket counts, then the running cursor (relative to s)
    __shared__ uint32_t cc[NB];   // chunk counts
    __shared__ uint32_t cl[NB];   // chunk-local starts
    __shared__ uint32_t wsum[kDpSplitThreads / 64];
    constexpr int kDpChunk = kDpSplitThreads * PER_T;
    __shared__ uint64_t stage[kDpChunk];
    const uint32_t nd2 = 1u << d2;
    const uint64_t s = off[(uint64_t)blockIdx.x * tiles];
    const uint64_t e = (blockIdx.x + 1 == (1u << d1)) ? n : off[(uint64_t)(blockIdx.x + 1) * tiles];
    const int sh = 64 - d1 - d2;  // d2 digit = (entry.x >> sh) & (nd2 - 1)
    for (uint32_t k = threadIdx.x; k < nd2; k += blockDim.x)
        h[k] = 0;
    __syncthreads();
    for (uint64_t i = s + threadIdx.x; i < e; i += blockDim.x)
        atomicAdd(&h[(uint32_t)(ent[i] >> sh) & (nd2 - 1)], 1u);
    __syncthreads();
    block_scan_bins<PER, kDpSplitThreads>(h, h, nd2, wsum);
    for (uint32_t k = threadIdx.x; k < nd2; k += blockDim.x)
        pstart[((uint64_t)blockIdx.x << d2) + k] = (uint32_t)(s + h[k]);
    if (blockIdx.x + 1 == (1u << d1) && threadIdx.x == 0)
        pstart[(uint64_t)1 << (d1 + d2)] = (uint32_t)n;
    for (uint64_t c0 = s; c0 < e; c0 += kDpChunk) {
        const uint32_t m = (uint32_t)((e - c0) < (uint64_t)kDpChunk ? (e - c0) : (uint64_t)kDpChunk);
        for (uint32_t k = threadIdx.x; k < nd2; k += blockDim.x)
            cc[k] = 0;
        __syncthreads();
        uint64_t en[PER_T];
        uint32_t rk[PER_T];
#pragma unroll
        for (int q = 0; q < PER_T; q++) {
            const uint32_t l = q * kDpSplitThreads + threadIdx.x;
            if (l < m) {
                en[q] = ent[c0 + l];
                rk[q] = atomicAdd(&cc[(uint32_t)(en[q] >> sh) & (nd2 - 1)], 1u);
            }
        }
        __syncthreads();
        block_scan_bins<PER, kDpSplitThreads>(cc, cl, nd2, wsum);
#pragma unroll
        for (int q = 0; q < PER_T; q++) {
            const uint32_t l = q * kDpSplitThreads + threadIdx.x;
            if (l < m)
                stage[cl[(uint32_t)(en[q] >> sh) & (nd2 - 1)] + rk[q]] = en[q];
        }
        __syncthreads();
        for (uint32_t j = threadIdx.x; j < m; j += blockDim.x) {
            const uint64_t v = stage[j];
            const uint32_t d = (uint32_t)(v >> sh) & (nd2 - 1);
            ent2[s + h[d] + (j - cl[d])] = v;
        }
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < nd2; k += blockDim.x)
            h[k] += cc[k];
        __syncthreads();
    }
}

// d2 == 0: the d1 buckets are the partitions
__global__ void dp_starts_kernel(const uint64_t *__restrict__ off, uint64_t n, int d1,
                                 uint64_t tiles, uint32_t *__restrict__ pstart)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < (1u << d1))
        pstart[k] = (uint32_t)off[(uint64_t)k * tiles];
    if (k == 0)
        pstart[1u << d1] = (uint32_t)n;
}

// Open-addressing tables (LDS or a partition's HBM region) hold one 64-bit
// word per slot: {key32, claimer record}, set once by CAS and never changed.
__device__ __forceinline__ uint32_t dp_home(uint32_t key, uint32_t size, bool masked)
{
    return masked ? ((key * 0x9E3779B1u) >> (32 - kDpSlotsLog))
                  : (uint32_t)(((uint64_t)(key * 0x9E3779B1u) * size) >> 32);
}

__device__ __forceinline__ uint32_t dp_next(uint32_t slot, uint32_t size, bool masked)
{
    return masked ? ((slot + 1) & (kDpSlots - 1)) : (slot + 1 == size ? 0 : slot + 1);
}

// Key-only probe from `slot`: claim the first empty slot, or stop at the
// first slot whose key equals ours.  Returns the slot; `owner` = its claimer
// (r itself when this record claimed it).  Equal keys still need the
// full-signature check (dp_insert continues past a mismatch).
template <bool MASKED>
__device__ __forceinline__ uint32_t dp_probe(uint64_t *word, uint32_t size, uint32_t key, uint32_t r,
                                             uint32_t slot, uint32_t &owner)
{
    const uint64_t mine = ((uint64_t)key << 32) | r;
    for (;;) {
        uint64_t cur = word[slot];
        if (cur == kDpEmpty) {
            cur = atomicCAS(reinterpret_cast<unsigned long long *>(&word[slot]), kDpEmpty, mine);
            if (cur == kDpEmpty) {
                owner = r;
                return slot;  // claimed
            }
        }
        if ((uint32_t)(cur >> 32) == key) {
            owner = (uint32_t)cur;
            return slot;
        }
        slot = dp_next(slot, size, MASKED);
    }
}

// Full insert from `slot`: probe, confirm an equal key on the 24 bytes, walk
// on past a key collision with a different signature.
template <bool MASKED>
__device__ __forceinline__ uint32_t dp_insert(uint64_t *word, uint32_t size, uint32_t key, uint32_t r,
                                              uint32_t slot, const uint8_t *sig, uint32_t stride,
                                              uint32_t &owner)
{
    for (;;) {
        slot = dp_probe<MASKED>(word, size, key, r, slot, owner);
        if (owner == r || sig_equal(sig, stride, r, owner))
            return slot;
        slot = dp_next(slot, size, MASKED);
    }
}

// A record's ingest index for the class minimum (only multi-member classes
// read it).  GM_ROW: the 32-byte exchange rows carry it at byte 24, on the
// line the confirmation just read.  GM_REP: from the record's own rep_out
// slot (dp_keys wrote gidx[r] there): the line its final store lands on,
// instead of a third array.  GM_INDEX: no gidx, the record index itself.
enum { GM_INDEX = 0, GM_REP = 1, GM_ROW = 2 };

__device__ __forceinline__ uint64_t gidx_of(const uint64_t *rep, const uint8_t *sig, uint32_t stride,
                                            int gmode, uint32_t r)
{
    if (gmode == GM_ROW)
        return *reinterpret_cast<const uint64_t *>(sig + (uint64_t)r * stride + 24);
    return gmode == GM_REP ? rep[r] : (uint64_t)r;
}
// Only records of classes with more than one member are written (random
// stores); K1 already wrote every record's singleton answer.  The class
// minimum needs ingest indices only there: every member that joined a
// claimed slot folds min(own, claimer's) into the slot, so a class of k > 1
// members gets all k indices and a singleton reads none.
constexpr int kDpEpt = (kDpCap + kDpGroupThreads - 1) / kDpGroupThreads;  // entries per thread

__global__ __launch_bounds__(kDpGroupThreads) __attribute__((amdgpu_waves_per_eu(8))) void dp_group_kernel(
    const uint64_t *__restrict__ ent, const uint32_t *__restrict__ pstart,
    const uint8_t *__restrict__ sig, uint32_t stride, int gmode, uint64_t *__restrict__ gword, uint64_t *__restrict__ gmin,
    uint32_t *__restrict__ gcnt, uint32_t *__restrict__ gslot, uint64_t *__restrict__ rep_out,
    uint32_t *__restrict__ ref_out)
{
    __shared__ uint64_t word[kDpSlots];
    __shared__ uint64_t mn[kDpSlots];
    __shared__ uint32_t cn[kDpSlots];
    const uint32_t s = pstart[blockIdx.x], e = pstart[blockIdx.x + 1];
    const uint32_t cnt = e - s;
    if (cnt == 0)
        return;
    if (cnt <= kDpCap) {
        // all of this thread's entries in flight at once
        uint64_t en[kDpEpt];
#pragma unroll
        for (int k = 0; k < kDpEpt; k++) {
            const uint32_t l = threadIdx.x + k * kDpGroupThreads;
            en[k] = l < cnt ? ent[s + l] : 0ull;
        }
        for (int k = threadIdx.x; k < kDpSlots; k += blockDim.x) {
            word[k] = kDpEmpty;
            mn[k] = kDpEmpty;
            cn[k] = 0;
        }
        __syncthreads();
        // (1) key-only probes: LDS only
        uint32_t slot[kDpEpt], own[kDpEpt];
#pragma unroll
        for (int k = 0; k < kDpEpt; k++) {
            const uint32_t l = threadIdx.x + k * kDpGroupThreads;
            own[k] = (uint32_t)en[k];
            if (l < cnt) {
                const uint32_t key = (uint32_t)(en[k] >> 32);
                slot[k] = dp_probe<true>(word, kDpSlots, key, (uint32_t)en[k], dp_home(key, kDpSlots, true),
                                         own[k]);
            }
        }
        // (2) confirmations of every joined entry issued together: both
        // signature rows and both ingest indices per entry
        uint64_t ra[kDpEpt], rb[kDpEpt], rc[kDpEpt], oa[kDpEpt], ob[kDpEpt], oc[kDpEpt];
        uint64_t gr[kDpEpt], go[kDpEpt];
#pragma unroll
        for (int k = 0; k < kDpEpt; k++) {
            const uint32_t r = (uint32_t)en[k];
            if (own[k] != r) {
                load_sig(sig + (uint64_t)r * stride, ra[k], rb[k], rc[k]);
                load_sig(sig + (uint64_t)own[k] * stride, oa[k], ob[k], oc[k]);
                gr[k] = gidx_of(rep_out, sig, stride, gmode, r);
                go[k] = gidx_of(rep_out, sig, stride, gmode, own[k]);
            }
        }
#pragma unroll
        for (int k = 0; k < kDpEpt; k++) {
            const uint32_t l = threadIdx.x + k * kDpGroupThreads;
            if (l < cnt) {
                const uint32_t r = (uint32_t)en[k];
                if (own[k] != r && !(ra[k] == oa[k] && rb[k] == ob[k] && rc[k] == oc[k])) {
                    // 32-bit key collision with a different signature: walk on
                    slot[k] = dp_insert<true>(word, kDpSlots, (uint32_t)(en[k] >> 32), r,
                                              dp_next(slot[k], kDpSlots, true), sig, stride, own[k]);
                    if (own[k] != r)
                        go[k] = gidx_of(rep_out, sig, stride, gmode, own[k]);
                }
                atomicAdd(&cn[slot[k]], 1u);
                if (own[k] != r)
                    atomicMin(reinterpret_cast<unsigned long long *>(&mn[slot[k]]),
                              (unsigned long long)(gr[k] < go[k] ? gr[k] : go[k]));
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kDpEpt; k++) {
            const uint32_t l = threadIdx.x + k * kDpGroupThreads;
            if (l < cnt) {
                const uint32_t c = cn[slot[k]];
                if (c > 1) {
                    const uint32_t r = (uint32_t)en[k];
                    rep_out[r] = mn[slot[k]];
                    ref_out[r] = c;
                }
            }
        }
        return;
    }
    // oversized partition: the same grouping on this partition's own HBM
    // region (2 * cnt slots at 2 * s)
    const uint32_t size = 2 * cnt;
    uint64_t *w = gword + 2ull * s;
    uint64_t *m = gmin + 2ull * s;
    uint32_t *c = gcnt + 2ull * s;
    for (uint32_t k = threadIdx.x; k < size; k += blockDim.x) {
        w[k] = kDpEmpty;
        m[k] = kDpEmpty;
        c[k] = 0;
    }
    __syncthreads();
    for (uint32_t l = threadIdx.x; l < cnt; l += blockDim.x) {
        const uint64_t en = ent[s + l];
        const uint32_t r = (uint32_t)en, key = (uint32_t)(en >> 32);
        uint32_t o;
        const uint32_t slot = dp_insert<false>(w, size, key, r, dp_home(key, size, false), sig, stride, o);
        atomicAdd(&c[slot], 1u);
        if (o != r) {
            const uint64_t a = gidx_of(rep_out, sig, stride, gmode, r), b = gidx_of(rep_out, sig, stride, gmode, o);
            atomicMin(reinterpret_cast<unsigned long long *>(&m[slot]), (unsigned long long)(a < b ? a : b));
        }
        gslot[s + l] = slot;
    }
    __syncthreads();
    for (uint32_t l = threadIdx.x; l < cnt; l += blockDim.x) {
        const uint32_t slot = gslot[s + l];
        if (c[slot] > 1) {
            const uint32_t r = (uint32_t)ent[s + l];
            rep_out[r] = m[slot];
            ref_out[r] = c[slot];
        }
    }
}

// Workspace layout of launch_dedup_group (bytes, 256-aligned pieces).
static inline uint64_t al(uint64_t x) { return (x + 255) & ~255ull; }

uint64_t dedup_ws_bytes(uint64_t n)
{
    const DpPlan pl = dp_plan(n);
    const uint64_t ncnt = (1ull << pl.d1) * pl.tiles;
    return al(4 * n) + al(8 * n) + al(8 * (ncnt + 1)) + al(8 * (ncnt + 1)) +
           al(8 * scan_workspace_elems(ncnt)) + al(8 * n) + al(8 * n) + al(4 * (pl.nparts() + 1)) +
           al(16 * n) + al(16 * n);
}

static unsigned grid_for(uint64_t n, unsigned block)
{
    uint64_t g = (n + block - 1) / block;
    if (g > 16384)
        g = 16384;
    return g ? (unsigned)g : 1u;
}

hipError_t launch_dedup_group(const uint8_t *sig, uint32_t sig_stride, const uint64_t *gidx,
                              uint32_t gidx_stride, uint64_t n, void *ws, uint64_t *rep_out,
                              uint32_t *ref_out, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1)
{
    if (n == 0)
        return hipSuccess;
    const DpPlan pl = dp_plan(n);
    const uint64_t ncnt = (1ull << pl.d1) * pl.tiles;
    char *p = static_cast<char *>(ws);
    auto take = [&](uint64_t bytes) {
        char *q = p;
        p += al(bytes);
        return q;
    };
    uint32_t *keys = reinterpret_cast<uint32_t *>(take(4 * n));
    uint64_t *counts = reinterpret_cast<uint64_t *>(take(8 * (ncnt + 1)));
    uint64_t *off = reinterpret_cast<uint64_t *>(take(8 * (ncnt + 1)));
    uint64_t *bsum = reinterpret_cast<uint64_t *>(take(8 * scan_workspace_elems(ncnt)));
    uint64_t *ent = reinterpret_cast<uint64_t *>(take(8 * n));
    uint64_t *ent2 = reinterpret_cast<uint64_t *>(take(8 * n));
    uint32_t *pstart = reinterpret_cast<uint32_t *>(take(4 * (pl.nparts() + 1)));
    uint64_t *gword = reinterpret_cast<uint64_t *>(take(16 * n));  // oversized-partition tables
    uint64_t *gmin = reinterpret_cast<uint64_t *>(take(16 * n));
    uint32_t *gcnt = reinterpret_cast<uint32_t *>(take(8 * n));
    uint32_t *gslot = keys;  // keys are dead after K3
    hipError_t e;
    if (ev0)
        (void)hipEventRecord(ev0, st);
    dp_keys_kernel<<<(unsigned)pl.tiles, kDpTileThreads, 0, st>>>(sig, sig_stride, gidx, gidx_stride, n,
                                                                  pl.d1, pl.tiles, keys, rep_out, ref_out,
                                                                  counts);
    if ((e = launch_exclusive_scan(counts, ncnt, off, bsum, st)) != hipSuccess)
        return e;
    dp_scatter_kernel<<<(unsigned)pl.tiles, kDpTileThreads, 0, st>>>(keys, n, pl.d1, pl.tiles, off, ent);
    const uint64_t *parts = ent;
    if (pl.d2) {
#ifdef FDFS_PROBES
        static int per = -1;
        if (per < 0) {  // A/B (make probes): FDFS_GPU_DEDUP_SPLIT=4 -> 4096-entry chunks
            const char *ev = getenv("FDFS_GPU_DEDUP_SPLIT");
            per = (ev && atoi(ev) == 4) ? 4 : kDpSplitPer;
        }
#else
        constexpr int per = kDpSplitPer;
#endif
        if (per == 4)
            dp_split_kernel<4><<<1u << pl.d1, kDpSplitThreads, 0, st>>>(ent, n, pl.d1, pl.d2, pl.tiles, off,
                                                                     ent2, pstart);
        else
            dp_split_kernel<kDpSplitPer><<<1u << pl.d1, kDpSplitThreads, 0, st>>>(ent, n, pl.d1, pl.d2, pl.tiles,
                                                                               off, ent2, pstart);
        parts = ent2;
    } else {
        dp_starts_kernel<<<((1u << pl.d1) + 255) / 256, 256, 0, st>>>(off, n, pl.d1, pl.tiles, pstart);
    }
    const int gmode = !gidx_stride ? GM_INDEX
                      : (gidx == reinterpret_cast<const uint64_t *>(sig + 24) && 8 * gidx_stride == sig_stride)
                          ? GM_ROW
                          : GM_REP;
    dp_group_kernel<<<(unsigned)pl.nparts(), kDpGroupThreads, 0, st>>>(
        parts, pstart, sig, sig_stride, gmode, gword, gmin, gcnt, gslot, rep_out, ref_out);
    if (ev1)
        (void)hipEventRecord(ev1, st);
    return hipGetLastError();
}

// ------------------------------------------------------------------ bucket

__device__ __forceinline__ uint32_t owner_of(const uint8_t *row, uint32_t nranks)
{
    uint64_t a, b, c;
    load_sig(row, a, b, c);
    return (uint32_t)((sig_hash(a, b, c) >> 32) % nranks);
}

__global__ void bucket_count_kernel(const uint8_t *__restrict__ sig, uint64_t n, uint32_t nranks,
                                    uint64_t *__restrict__ counts)
{
    __shared__ uint32_t h[64];
    for (int k = threadIdx.x; k < 64; k += blockDim.x)
        h[k] = 0;
    __syncthreads();
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
         r += (uint64_t)gridDim.x * blockDim.x)
        atomicAdd(&h[owner_of(sig + 24 * r, nranks)], 1u);
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < nranks; k += blockDim.x)
        if (h[k])
            atomicAdd(reinterpret_cast<unsigned long long *>(&counts[k]), (unsigned long long)h[k]);
}

__global__ void bucket_scatter_kernel(const uint8_t *__restrict__ sig, const uint64_t *__restrict__ gidx,
                                      uint64_t n, uint32_t nranks, const uint64_t *__restrict__ counts,
                                      uint64_t *__restrict__ cursor, uint8_t *__restrict__ rows,
                                      uint64_t *__restrict__ row_of)
{
    __shared__ uint32_t cnt[64];
    __shared__ uint64_t bas[64];
    __shared__ uint64_t start[64];
    if (threadIdx.x == 0) {
        uint64_t run = 0;
        for (uint32_t k = 0; k < nranks; k++) {
            start[k] = run;
            run += counts[k];
        }
    }
    for (uint64_t r0 = (uint64_t)blockIdx.x * blockDim.x; r0 < n; r0 += (uint64_t)gridDim.x * blockDim.x) {
        for (int k = threadIdx.x; k < 64; k += blockDim.x)
            cnt[k] = 0;
        __syncthreads();
        const uint64_t r = r0 + threadIdx.x;
        uint32_t own = 0, rank = 0;
        if (r < n) {
            own = owner_of(sig + 24 * r, nranks);
            rank = atomicAdd(&cnt[own], 1u);
        }
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < nranks; k += blockDim.x)
            if (cnt[k])
                bas[k] = start[k] + atomicAdd(reinterpret_cast<unsigned long long *>(&cursor[k]),
                                              (unsigned long long)cnt[k]);
        __syncthreads();
        if (r < n) {
            const uint64_t pos = bas[own] + rank;
            const uint64_t *s = reinterpret_cast<const uint64_t *>(sig + 24 * r);
            uint64_t *d = reinterpret_cast<uint64_t *>(rows + 32 * pos);
            d[0] = s[0];
            d[1] = s[1];
            d[2] = s[2];
            d[3] = gidx ? gidx[r] : r;
            if (row_of)
                row_of[r] = pos;
        }
        __syncthreads();
    }
}

// Multi-GPU dedup (fdfs_gpu_dedup_global): the owner's per-row answers
// packed as {rep, ref} pairs for the return exchange, and the exchanged
// answers mapped back to the rank's records through row_of.
__global__ void answer_pack_kernel(const uint64_t *__restrict__ rep, const uint32_t *__restrict__ ref,
                                   uint64_t m, uint64_t *__restrict__ ans)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
         i += (uint64_t)gridDim.x * blockDim.x)
        reinterpret_cast<ulonglong2 *>(ans)[i] = make_ulonglong2(rep[i], ref[i]);
}

__global__ void answer_gather_kernel(const uint64_t *__restrict__ back, const uint64_t *__restrict__ row_of,
                                     uint64_t n, uint64_t *__restrict__ rep_out, uint32_t *__restrict__ ref_out)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const ulonglong2 a = reinterpret_cast<const ulonglong2 *>(back)[row_of[i]];
        rep_out[i] = a.x;
        ref_out[i] = (uint32_t)a.y;
    }
}

hipError_t launch_answer_pack(const uint64_t *rep, const uint32_t *ref, uint64_t m, uint64_t *ans,
                              hipStream_t st)
{
    if (m)
        answer_pack_kernel<<<grid_for(m, 256), 256, 0, st>>>(rep, ref, m, ans);
    return hipGetLastError();
}

hipError_t launch_answer_gather(const uint64_t *back, const uint64_t *row_of, uint64_t n, uint64_t *rep_out,
                                uint32_t *ref_out, hipStream_t st)
{
    if (n)
        answer_gather_kernel<<<grid_for(n, 256), 256, 0, st>>>(back, row_of, n, rep_out, ref_out);
    return hipGetLastError();
}

hipError_t launch_dedup_bucket(const uint8_t *sig, const uint64_t *gidx, uint64_t n,
                               uint32_t nranks, uint8_t *records_out, uint64_t *counts_out,
                               uint64_t *cursor, uint64_t *row_of_out, hipStream_t st,
                               hipEvent_t ev0, hipEvent_t ev1)
{
    hipError_t e;
    if ((e = hipMemsetAsync(counts_out, 0, nranks * sizeof(uint64_t), st)) != hipSuccess)
        return e;
    if ((e = hipMemsetAsync(cursor, 0, nranks * sizeof(uint64_t), st)) != hipSuccess)
        return e;
    if (n == 0)
        return hipSuccess;
    if (ev0)
        (void)hipEventRecord(ev0, st);
    bucket_count_kernel<<<grid_for(n, 256), 256, 0, st>>>(sig, n, nranks, counts_out);
    bucket_scatter_kernel<<<grid_for(n, 256), 256, 0, st>>>(sig, gidx, n, nranks, counts_out, cursor,
                                                            records_out, row_of_out);
    if (ev1)
        (void)hipEventRecord(ev1, st);
    return hipGetLastError();
}

}  // namespace fdfs
