// Incremental dedup index: a device-resident signature -> {source, ref}
// table kept across ingest batches.
//
// The FastDHT state the upload path builds one RPC at a time
// (storage/storage_service.c:2652 get "fid": hit -> link to the source;
// :2714 miss -> this file becomes the source; :2734 set "ref" = 0 and
// storage_set_link_file_meta :2984 inc "ref" per link) is, for a stream of
// ingest batches, this table: a batch is first grouped on its own
// (dp_* kernels, fdfs_dedup.hip, record positions as ingest order), then
// one thread per class of the batch looks its signature up in the table:
// a hit keeps the source of an earlier batch and adds the batch's members
// to its ref, a miss inserts the class with its first member as source.
// Every record then reads its class's answer.  After k batches the answers
// equal the one-shot dedup of the concatenated stream (source = first file
// ever with the signature, ref = class size so far).
//
// One thread per class and batch inserts a given signature, so a slot that
// is being written (state BUSY) always holds some other key and is skipped;
// a slot is published with a release store of FULL after its key and
// values, and read after an acquire load of its state.  Random device-scope
// atomics are a few per class (MI355X_MICROARCH.md: global atomics), one
// CAS to claim and one add per hit.
#include "fdfs_device.hpp"
#include "fdfs_kernels.hpp"

namespace fdfs {

constexpr uint32_t kIxEmpty = 0, kIxBusy = 1, kIxFull = 2;

__device__ __forceinline__ uint64_t ix_mix(uint64_t k)
{
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

__device__ __forceinline__ uint64_t ix_hash(uint64_t a, uint64_t b, uint64_t c)
{
    // independent of the dedup partition key (which uses a different seed)
    return ix_mix(c ^ ix_mix(b ^ ix_mix(a + 0x632BE59BD9B4E019ull)));
}

__global__ void index_clear_kernel(uint32_t *__restrict__ state, uint64_t slots)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < slots;
         i += (uint64_t)gridDim.x * blockDim.x)
        state[i] = kIxEmpty;
}

// One thread per class of the batch (its first member, rep_pos[i] == i).
__global__ void index_upsert_kernel(const uint8_t *__restrict__ sig, const uint64_t *__restrict__ gidx,
                                    uint64_t gbase, uint64_t n, const uint64_t *__restrict__ rep_pos,
                                    const uint32_t *__restrict__ ref_b, uint64_t slots,
                                    uint8_t *__restrict__ keys, uint64_t *__restrict__ vrep,
                                    uint32_t *__restrict__ vref, uint32_t *__restrict__ state,
                                    uint64_t *__restrict__ res_rep, uint32_t *__restrict__ res_ref,
                                    unsigned long long *__restrict__ counters)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool inserted = false;
    if (i < n && rep_pos[i] == i) {
        const uint64_t *s = reinterpret_cast<const uint64_t *>(sig + 24 * i);
        const uint64_t a = s[0], b = s[1], c = s[2];
        const uint64_t g = gidx ? gidx[i] : gbase + i;
        const uint32_t cnt = ref_b[i];
        uint64_t slot = ix_hash(a, b, c) & (slots - 1);
        uint64_t rep = g;
        uint32_t ref = cnt;
        bool done = false;
        for (uint64_t probe = 0; probe < slots && !done; probe++, slot = (slot + 1) & (slots - 1)) {
            uint32_t st = __hip_atomic_load(&state[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            if (st == kIxEmpty) {
                uint32_t expect = kIxEmpty;
                if (__hip_atomic_compare_exchange_strong(&state[slot], &expect, kIxBusy, __ATOMIC_ACQ_REL,
                                                         __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) {
                    uint64_t *k = reinterpret_cast<uint64_t *>(keys + 24 * slot);
                    k[0] = a;
                    k[1] = b;
                    k[2] = c;
                    vrep[slot] = g;
                    vref[slot] = cnt;
                    __hip_atomic_store(&state[slot], kIxFull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                    inserted = done = true;
                    continue;
                }
                st = expect;  // claimed by another class meanwhile
            }
            if (st != kIxFull)
                continue;  // BUSY: another class of this batch is writing it
            const uint64_t *k = reinterpret_cast<const uint64_t *>(keys + 24 * slot);
            if (k[0] == a && k[1] == b && k[2] == c) {
                rep = vrep[slot];
                ref = atomicAdd(&vref[slot], cnt) + cnt;
                done = true;
            }
        }
        if (!done)  // table full: answered within the batch, flagged
            atomicAdd(&counters[2], 1ull);
        res_rep[i] = rep;
        res_ref[i] = ref;
    }
    // classes inserted, one atomic per wave
    const uint64_t m = __ballot(inserted);
    if ((threadIdx.x & 63) == 0 && m)
        atomicAdd(&counters[0], (unsigned long long)__popcll(m));
}

__global__ void index_answer_kernel(const uint64_t *__restrict__ rep_pos, uint64_t n,
                                    const uint64_t *__restrict__ res_rep, const uint32_t *__restrict__ res_ref,
                                    uint64_t *__restrict__ rep_out, uint32_t *__restrict__ ref_out)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = rep_pos[i];
        rep_out[i] = res_rep[r];
        ref_out[i] = res_ref[r];
    }
}

// Growth: every full slot of the old table into the new one (distinct keys,
// no concurrent reader: a claim is one CAS, then the fields).
__global__ void index_rehash_kernel(const uint8_t *__restrict__ okeys, const uint64_t *__restrict__ orep,
                                    const uint32_t *__restrict__ oref, const uint32_t *__restrict__ ostate,
                                    uint64_t oslots, uint8_t *__restrict__ keys, uint64_t *__restrict__ vrep,
                                    uint32_t *__restrict__ vref, uint32_t *__restrict__ state, uint64_t slots)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < oslots;
         i += (uint64_t)gridDim.x * blockDim.x) {
        if (ostate[i] != kIxFull)
            continue;
        const uint64_t *k = reinterpret_cast<const uint64_t *>(okeys + 24 * i);
        const uint64_t a = k[0], b = k[1], c = k[2];
        uint64_t slot = ix_hash(a, b, c) & (slots - 1);
        for (;;) {
            if (atomicCAS(&state[slot], kIxEmpty, kIxFull) == kIxEmpty)
                break;
            slot = (slot + 1) & (slots - 1);
        }
        uint64_t *d = reinterpret_cast<uint64_t *>(keys + 24 * slot);
        d[0] = a;
        d[1] = b;
        d[2] = c;
        vrep[slot] = orep[i];
        vref[slot] = oref[i];
    }
}

hipError_t launch_index_rehash(const IndexTable &from, const IndexTable &to, hipStream_t st)
{
    const uint64_t g = (from.slots + 255) / 256;
    index_rehash_kernel<<<(unsigned)(g < 16384 ? g : 16384), 256, 0, st>>>(
        from.keys, from.rep, from.ref, from.state, from.slots, to.keys, to.rep, to.ref, to.state, to.slots);
    return hipGetLastError();
}

hipError_t launch_index_clear(uint32_t *state, uint64_t slots, hipStream_t st)
{
    index_clear_kernel<<<4096, 256, 0, st>>>(state, slots);
    return hipGetLastError();
}

hipError_t launch_index_ingest(const uint8_t *sig, const uint64_t *gidx, uint64_t gbase, uint64_t n,
                               const uint64_t *rep_pos, const uint32_t *ref_b, const IndexTable &t,
                               uint64_t *res_rep, uint32_t *res_ref, uint64_t *rep_out, uint32_t *ref_out,
                               hipStream_t st)
{
    if (n == 0)
        return hipSuccess;
    index_upsert_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(
        sig, gidx, gbase, n, rep_pos, ref_b, t.slots, t.keys, t.rep, t.ref, t.state, res_rep, res_ref,
        reinterpret_cast<unsigned long long *>(t.counters));
    const uint64_t g = (n + 255) / 256;
    index_answer_kernel<<<(unsigned)(g < 16384 ? g : 16384), 256, 0, st>>>(rep_pos, n, res_rep, res_ref, rep_out,
                                                                          ref_out);
    return hipGetLastError();
}

}  // namespace fdfs
