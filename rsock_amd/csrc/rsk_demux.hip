// rsk_demux.hip — receive demux for MI355X (gfx950): stable group-by of a decoded batch's VALID
// packets on selected EncHead / TcpInfo fields (semantics: include/rsk_codec.h).
//
// The reference routes each VALID packet with its own map lookup — INetGroup::Input by connKey
// (conn/INetGroup.cpp:57-83), IAppGroup::Input by cmd (conn/IAppGroup.cpp:76-96), ServerGroup::
// OnRecv by IdBuf (server/ServerGroup.cpp:44-60), SubGroup::OnRecv by (dst, conv)
// (server/SubGroup.cpp:31-50), ClientGroup::OnRecv by conv (client/ClientGroup.cpp:66-80).  Here a
// batch becomes segments (one per key and epoch, ordered by first packet, arrival order inside), so
// the host does one lookup per segment.
//
// Pipeline (all stream-ordered, no host sync; n_valid and the segment count stay on the device),
// 5 + passes launches after one fill (round 2: the block scans are decoupled look-backs inside the
// kernels that produce the counts, and the radix sort is onesweep, one launch per pass):
//   k_dm_fill       look-back state words to all-ones, and the key table unless the previous call on
//                   this scratch left it clean (round 6: k_dm_final clears the slots of batches with
//                   few segments)
//   k_dm_flags_prep per-wave ballots of VALID and VALID-control packets, block offsets by look-back;
//                   cidx[j] = packet of compacted slot j; with CMD_BARRIER pep[packet] = its epoch
//                   (CTRL for singletons; without, every epoch is 0 and nothing is stored)
//   k_dm_insert     open-addressing table: a slot holds a key fingerprint and the packet index of
//                   its key's first packet (lowered by CAS), so key confirmation reads the immutable
//                   input arrays at that index (no lane ever waits on another lane's write); keys
//                   whose epoch lies inside one tile are grouped in LDS only
//   k_dm_leader_rank leader of j = the packet its slot names (or j's own packet for a control
//                   packet); leader ranks = dense segment ids in first-occurrence order by look-back;
//                   rank_at[packet], seg_first, n_seg; the followers (non-leaders) compacted with
//                   their leader
//   k_dm_segof_hist radix keys = segment id of each follower, global digit histograms of every pass
//                   (<= 1024 followers: sorted here by one block)
//   k_dm_onesweep   stable LSD pass of the FOLLOWERS by segment id (8-bit or narrower digits, as many
//                   passes as the segment count needs; passes beyond that, and tiles past the
//                   follower count, return at once), per-digit look-back; ranking wave-local (round 4)
//   k_dm_final      leaders merged with the sorted followers: perm, seg_off, n_seg / n_valid
// (round 2, second half: only followers are sorted — leaders already stand in segment order — so a
// batch of mostly single-packet segments skips the sort's work)
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include "../../include/rsk_codec.h"
#include "rsk_ctx.h"

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr uint32_t kItems = 16;  // items per thread per radix / look-back tile (8: C3 +4 % r03, +13 % r05)
constexpr uint32_t kTile = kBlock * kItems;     // 4096 packets per radix tile
constexpr uint32_t kNone = 0xffffffffu;
constexpr uint32_t kCtrl = 0xffffffffu;         // pep[] marker: control packet (singleton segment)
constexpr uint32_t kScanChunk = 4096;           // elements per block in the multi-block scan

__device__ __forceinline__ uint64_t lanemask_lt(uint32_t lane) { return (1ull << lane) - 1ull; }

// ---- scans ----------------------------------------------------------------------------------
// exclusive scan of 4096 u32 per pass by one 1024-thread block; carry across passes
__device__ __forceinline__ void block_scan_4096(const uint32_t *in, uint32_t *out, uint32_t base, uint32_t cnt,
                                                uint32_t &carry, uint32_t *wsum) {
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const uint32_t idx = base + 4u * t;
    uint32_t c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = idx + k < cnt ? in[idx + k] : 0u;
    const uint32_t tsum = c[0] + c[1] + c[2] + c[3];
    uint32_t inc = tsum;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(inc, off);
        if (lane >= (uint32_t)off) inc += v;
    }
    if (lane == 63u) wsum[wv] = inc;
    __syncthreads();
    uint32_t wpre = 0, total = 0;
#pragma unroll
    for (uint32_t q = 0; q < 16; ++q) {
        const uint32_t v = wsum[q];
        wpre += q < wv ? v : 0u;
        total += v;
    }
    uint32_t run = carry + wpre + inc - tsum;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (idx + k < cnt) out[idx + k] = run;
        run += c[k];
    }
    carry += total;
    __syncthreads();
}

// one block: exclusive scan of cnt elements (any cnt), total to *total if non-null
__global__ __launch_bounds__(1024) void k_dm_scan1(const uint32_t *in, uint32_t *out, uint32_t cnt, uint32_t *total) {
    __shared__ uint32_t wsum[16];
    uint32_t carry = 0;
    for (uint32_t base = 0; base < cnt; base += 4096u) block_scan_4096(in, out, base, cnt, carry, wsum);
    if (threadIdx.x == 0 && total) *total = carry;
}
// multi-block: chunk sums, then (k_dm_scan1 over the sums), then per-chunk scan with its offset
__global__ __launch_bounds__(1024) void k_dm_chunk_sum(const uint32_t *in, uint32_t cnt, uint32_t *sums) {
    __shared__ uint32_t wsum[16];
    const uint32_t base = blockIdx.x * kScanChunk, t = threadIdx.x, lane = t & 63u;
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) s += base + 4u * t + k < cnt ? in[base + 4u * t + k] : 0u;
#pragma unroll
    for (int off = 32; off; off >>= 1) s += __shfl_xor(s, off);
    if (lane == 0) wsum[t >> 6] = s;
    __syncthreads();
    if (t == 0) {
        uint32_t a = 0;
        for (int q = 0; q < 16; ++q) a += wsum[q];
        sums[blockIdx.x] = a;
    }
}
__global__ __launch_bounds__(1024) void k_dm_chunk_apply(const uint32_t *in, uint32_t *out, uint32_t cnt,
                                                         const uint32_t *sum_off) {
    __shared__ uint32_t wsum[16];
    uint32_t carry = sum_off[blockIdx.x];
    block_scan_4096(in, out, blockIdx.x * kScanChunk, cnt, carry, wsum);
}

struct ScanWs {
    uint32_t *sums, *sum_off;  // >= ceil(max cnt / kScanChunk) each
};

int scan_u32(const uint32_t *in, uint32_t *out, uint32_t cnt, uint32_t *total, const ScanWs &w, hipStream_t s) {
    if (cnt <= 4u * kScanChunk) {
        hipLaunchKernelGGL(k_dm_scan1, dim3(1), dim3(1024), 0, s, in, out, cnt, total);
        return rsk::launch_check("k_dm_scan1");
    }
    const uint32_t nc = (cnt + kScanChunk - 1) / kScanChunk;
    hipLaunchKernelGGL(k_dm_chunk_sum, dim3(nc), dim3(1024), 0, s, in, cnt, w.sums);
    hipLaunchKernelGGL(k_dm_scan1, dim3(1), dim3(1024), 0, s, w.sums, w.sum_off, nc, total);
    hipLaunchKernelGGL(k_dm_chunk_apply, dim3(nc), dim3(1024), 0, s, in, out, cnt, w.sum_off);
    return rsk::launch_check("scan_u32");
}

// ---- demux kernels --------------------------------------------------------------------------
struct DmIn {
    const int8_t *status;
    const uint8_t *cmd;
    const uint64_t *id;  // IdBuf as one u64 (8-B aligned)
    const uint32_t *conv;
    const uint64_t *key;
    const uint32_t *dst;
    uint32_t *pep;   // with CMD_BARRIER: epoch of each VALID data packet, by packet index (else null: 0)
    uint32_t *cpos;  // with CMD_BARRIER: packet index of the c-th VALID control packet; cpos[n_ctrl] = n
    const uint32_t *xep;  // second pass of GROUP_BARRIER: a key word per packet (else null: 0)
    uint32_t n, fields;
};

// ---- decoupled look-back: one-pass exclusive scan of per-block counts across a grid -----------
// Block b publishes its aggregate, then reads its predecessors' words (a wave 64 at a time) until it
// meets an inclusive prefix, and publishes its own inclusive prefix.  Blocks are dispatched in
// index order, so a block only ever waits for blocks that are already resident or done.  State
// words start as all-ones (the demux memset); a ready word is the value in bits 0..31 with bit 63
// set for an inclusive prefix.  Device-scope RELAXED atomics (sc1 loads / stores, coherent across
// the XCDs' L2s): the published words are the only data one block reads from another, so no
// ordering is needed, and acquire / release at device scope would add an L2 invalidate / write-back
// per access (first build: 0.56 ms for C4's flags pass instead of ~0.02).  A spin that outlives
// kDlbSpinMax reads gives up (the GPU is not hung): the batch result is then wrong, and the spin sets
// RSK_DEVERR_LOOKBACK in the context's sticky error word (rsk_check_device_errors).
constexpr unsigned long long kDlbEmpty = ~0ull;
constexpr unsigned long long kDlbIncl = 1ull << 63;
constexpr uint32_t kDlbSpinMax = 1u << 22;

__device__ __forceinline__ void dlb_publish(unsigned long long *s, unsigned long long v) {
    __hip_atomic_store(s, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long dlb_wait(unsigned long long *s, uint32_t *err) {
    unsigned long long v;
    uint32_t spins = 0;
    do {
        v = __hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } while (v == kDlbEmpty && ++spins < kDlbSpinMax);
    if (v != kDlbEmpty) return v;
    __hip_atomic_fetch_or(err, RSK_DEVERR_LOOKBACK, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return kDlbIncl;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int off = 32; off; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// Called by all 64 lanes of one wave of block b; agg uniform; returns b's exclusive prefix (uniform).
__device__ uint32_t dlb_wave(unsigned long long *st, uint32_t b, uint32_t agg, uint32_t lane, uint32_t *err) {
    if (b == 0u) {
        if (lane == 0u) dlb_publish(st, kDlbIncl | agg);
        return 0u;
    }
    if (lane == 0u) dlb_publish(st + b, (unsigned long long)agg);
    uint32_t excl = 0;
    for (int64_t top = (int64_t)b - 1;; top -= 64) {
        const int64_t j = top - (int64_t)lane;
        const unsigned long long v = j >= 0 ? dlb_wait(st + j, err) : kDlbIncl;  // before block 0: inclusive 0
        const uint64_t im = __ballot((v & kDlbIncl) != 0ull);
        uint32_t val = (uint32_t)v;
        if (im) {  // the nearest inclusive predecessor ends the walk
            if (lane > (uint32_t)__builtin_ctzll(im)) val = 0u;
            excl += wave_sum(val);
            break;
        }
        excl += wave_sum(val);
    }
    if (lane == 0u) dlb_publish(st + b, kDlbIncl | (unsigned long long)(excl + agg));
    return excl;
}

// Per-digit look-back for the onesweep radix scatter: thread d of tile t publishes its digit count,
// walks back over tiles until an inclusive word, publishes the inclusive count; returns the count
// of digit d in tiles before t.
__device__ uint32_t dlb_digit(unsigned long long *st, uint32_t t, uint32_t d, uint32_t cnt, uint32_t *err) {
    if (t == 0u) {
        dlb_publish(st + d, kDlbIncl | cnt);
        return 0u;
    }
    dlb_publish(st + (uint64_t)t * 256u + d, (unsigned long long)cnt);
    // walk back kLb tiles per step: their words are requested together (one round trip per step,
    // not per tile); a tile before tile 0 reads as an inclusive 0
    constexpr int kLb = 4;
    uint32_t excl = 0;
    for (int64_t j = (int64_t)t - 1; j >= 0; j -= kLb) {
        unsigned long long v[kLb];
#pragma unroll
        for (int q = 0; q < kLb; ++q)
            v[q] = j - q >= 0 ? __hip_atomic_load(st + (uint64_t)(j - q) * 256u + d, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT)
                              : kDlbIncl;
        bool done = false;
#pragma unroll
        for (int q = 0; q < kLb; ++q) {
            if (done) break;
            if (v[q] == kDlbEmpty) v[q] = dlb_wait(st + (uint64_t)(j - q) * 256u + d, err);
            excl += (uint32_t)v[q];
            done = (v[q] & kDlbIncl) != 0ull;
        }
        if (done) break;
    }
    dlb_publish(st + (uint64_t)t * 256u + d, kDlbIncl | (unsigned long long)(excl + cnt));
    return excl;
}

struct Key {
    uint32_t ep, conv, dst, xf;
    uint64_t id, ck;
};

__device__ __forceinline__ Key load_key(const DmIn &a, uint32_t i, uint32_t ep) {
    Key k;
    k.ep = ep;
    k.id = (a.fields & RSK_DEMUX_ID) ? a.id[i] : 0ull;
    k.ck = (a.fields & RSK_DEMUX_CONN_KEY) ? a.key[i] : 0ull;
    k.conv = (a.fields & RSK_DEMUX_CONV) ? a.conv[i] : 0u;
    k.dst = (a.fields & RSK_DEMUX_DST) ? a.dst[i] : 0u;
    k.xf = a.xep ? a.xep[i] : 0u;
    return k;
}
__device__ __forceinline__ bool key_eq(const Key &x, const Key &y) {
    return x.ep == y.ep && x.xf == y.xf && x.id == y.id && x.ck == y.ck && x.conv == y.conv && x.dst == y.dst;
}
__device__ __forceinline__ uint64_t key_hash(const Key &k) {
    uint64_t h = ((uint64_t)k.ep | (uint64_t)k.xf << 32) * 0x9E3779B97F4A7C15ull ^ k.id * 0xC2B2AE3D27D4EB4Full ^
                 k.ck * 0x165667B19E3779F9ull ^ ((uint64_t)k.conv | (uint64_t)k.dst << 32) * 0xD6E8FEB86659FD93ull;
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    return h;
}

// Global table probe: a slot is one u64, fingerprint (hash bits 32..63) << 32 | the compacted index
// of the key's first packet so far.  A slot with another fingerprint is skipped without touching that
// packet's fields, a matching fingerprint is confirmed on the full key, and the index is lowered by
// compare-and-swap (the fingerprint half never changes once claimed).  A relaxed load comes first:
// a hot key's slot is read, not written, by every later tile (no RMW unless the index drops); a new
// key costs the load and one CAS (round 2, first half: a load, a CAS and a separate atomicMin word).
// [es, ee): the packets of the key's epoch (with CMD_BARRIER; cpos) -- an owner outside it has another
// epoch, so its epoch is checked by its index instead of a third gather (round 5)
__device__ __forceinline__ uint32_t global_probe(const DmIn &a,
                                                 unsigned long long *slots, uint32_t mask, const Key &k,
                                                 uint64_t hv, uint32_t j, uint32_t es, uint32_t ee, uint32_t *err) {
    // j is the packet index (monotone with the compacted index, so the minimum is the same packet):
    // a slot's owner is confirmed on the inputs at that index directly (round 5: one dependent
    // gather less than through the compacted index, C3 0.400 -> 0.372 ms with the 512-packet tiles)
    const uint32_t fp = (uint32_t)(hv >> 32);
    const unsigned long long mine = ((unsigned long long)fp << 32) | j;
    uint32_t h = (uint32_t)hv & mask;
    for (uint32_t walked = 0;; ++walked) {
        if (walked > mask) {  // the whole table: it was not clean (RSK_DEVERR_TABLE), give up, no hang
            __hip_atomic_fetch_or(err, RSK_DEVERR_TABLE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return h;
        }
        unsigned long long e = __hip_atomic_load(slots + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (e == ~0ull) {
            e = atomicCAS(slots + h, ~0ull, mine);
            if (e == ~0ull) return h;  // claimed
        }
        if ((uint32_t)(e >> 32) == fp) {
            const uint32_t o = (uint32_t)e;
            if (o >= es && o < ee && key_eq(load_key(a, o, k.ep), k)) {
                while ((uint32_t)e > j) {  // lower the key's first index to j
                    const unsigned long long f = atomicCAS(slots + h, e, mine);
                    if (f == e) break;
                    e = f;
                }
                return h;
            }
        }
        h = (h + 1u) & mask;
    }
}

// One block = kInsTile consecutive compacted packets.  Phase 1 groups them by key in an LDS table
// (same fingerprint scheme, confirmed on the full key) and takes each key's block-minimum index
// with LDS atomics; phase 2: that minimum packet alone probes the global table and lowers its index,
// so a hot key costs one global atomic per block, not one per packet (a single hot word takes
// ~88 atomics/us: MI355X_MICROARCH.md, dequeue row); phase 3 hands every packet its key's slot.
// Epoch-local keys (round 2, second half): with CMD_BARRIER the epoch is part of the key and epochs only grow
// with the packet index, so a key whose epoch lies strictly between the epochs of the tile's first
// and last data packets cannot occur outside the tile: its block minimum IS its first packet and it
// never touches the global table (hslot = kLeadTag | leader).  Only the tile's first and last epochs
// go to the table: C4 (5 % control packets) sends ~2 % of its keys there instead of all of them.
constexpr uint32_t kInsItems = 2;  // round 5: 2 (512-packet tiles; 4: C3 +4 %, 1: 64 connections +7 %)
constexpr uint32_t kLeadTag = 0x80000000u;  // hslot: leader index (table slots are < 2^31)
constexpr uint32_t kInsTile = kBlock * kInsItems;  // 512 packets (12 KB LDS)
constexpr uint32_t kLtab = 2 * kInsTile;           // LDS table slots (power of 2)

__global__ __launch_bounds__(kBlock) void k_dm_insert(DmIn a, const uint32_t *nvp, const uint32_t *cidx,
                                                      unsigned long long *slots,
                                                      uint32_t mask, uint32_t *hslot, uint32_t *err) {
    __shared__ unsigned long long ltab[kLtab];
    __shared__ uint32_t lmin[kLtab];  // block-minimum index per key, then (phase 2b) the key's global slot
    __shared__ uint32_t elo, ehi;     // epochs of the tile's first and last data packets
    __shared__ uint32_t erng[4];      // their packet ranges [start, end) (CMD_BARRIER)
    const uint32_t nv = *nvp;
    const uint32_t base = blockIdx.x * kInsTile, t = threadIdx.x;
    if (base >= nv) return;  // block-uniform
    for (uint32_t q = t; q < kLtab; q += kBlock) {
        ltab[q] = ~0ull;
        lmin[q] = kNone;
    }
    if (t == 0) {
        elo = kNone;
        ehi = 0u;
    }
    __syncthreads();
    // (keys stay in registers; confirming another packet's key reads the immutable inputs: keeping
    // the tile's keys in LDS too cost more occupancy than it saved, 157 -> 179 us on C3)
    Key kr[kInsItems];
    uint32_t lpos[kInsItems], pkr[kInsItems];
#pragma unroll
    for (uint32_t it = 0; it < kInsItems; ++it) {  // every item's loads in flight before the LDS work
        const uint32_t j = base + it * kBlock + t;
        pkr[it] = j < nv ? cidx[j] : kNone;
    }
#pragma unroll
    for (uint32_t it = 0; it < kInsItems; ++it)
        kr[it] = pkr[it] == kNone ? Key{kCtrl, 0, 0, 0, 0, 0} : load_key(a, pkr[it], a.pep ? a.pep[pkr[it]] : 0u);
#pragma unroll
    for (uint32_t it = 0; it < kInsItems; ++it) {
        const uint32_t li = it * kBlock + t, j = base + li;
        lpos[it] = kNone;
        if (kr[it].ep == kCtrl) continue;  // past the batch, or a control packet
        const Key &k = kr[it];
        const uint64_t hv = key_hash(k);
        const uint32_t fp = (uint32_t)(hv >> 32);
        const unsigned long long mine = ((unsigned long long)fp << 32) | li;
        uint32_t h = (uint32_t)(hv ^ (hv >> 40)) & (kLtab - 1u);
        for (;;) {
            unsigned long long e = ltab[h];
            if (e == ~0ull) {
                e = atomicCAS(&ltab[h], ~0ull, mine);
                if (e == ~0ull) break;
            }
            if ((uint32_t)(e >> 32) == fp) {
                const uint32_t jo = base + (uint32_t)e;
                const uint32_t po = cidx[jo];
                if (key_eq(load_key(a, po, a.pep ? a.pep[po] : 0u), k)) break;
            }
            h = (h + 1u) & (kLtab - 1u);
        }
        lpos[it] = h;
        atomicMin(&lmin[h], j);
    }
    {  // the tile's epoch range (data packets only; control packets carry kCtrl)
        uint32_t lo = kNone, hi = 0u;
#pragma unroll
        for (uint32_t it = 0; it < kInsItems; ++it)
            if (lpos[it] != kNone) {
                lo = min(lo, kr[it].ep);
                hi = max(hi, kr[it].ep);
            }
#pragma unroll
        for (int off = 32; off; off >>= 1) {
            lo = min(lo, (uint32_t)__shfl_xor((int)lo, off));
            hi = max(hi, (uint32_t)__shfl_xor((int)hi, off));
        }
        if ((t & 63u) == 0u && lo != kNone) {
            atomicMin(&elo, lo);
            atomicMax(&ehi, hi);
        }
    }
    __syncthreads();
    if (t == 0u) {  // the packets of epochs elo and ehi: between consecutive control packets
        uint32_t r[4] = {0u, ~0u, 0u, ~0u};
        if (a.cpos && elo != kNone) {
            r[0] = elo == 0u ? 0u : a.cpos[elo - 1u] + 1u;
            r[1] = a.cpos[elo];
            r[2] = ehi == 0u ? 0u : a.cpos[ehi - 1u] + 1u;
            r[3] = a.cpos[ehi];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) erng[q] = r[q];
    }
    uint32_t rep = 0;  // bit it: this thread's item `it` is its key's first packet in the block
#pragma unroll
    for (uint32_t it = 0; it < kInsItems; ++it)
        if (lpos[it] != kNone && lmin[lpos[it]] == base + it * kBlock + t) rep |= 1u << it;
    __syncthreads();
#pragma unroll
    for (uint32_t it = 0; it < kInsItems; ++it) {
        if (!((rep >> it) & 1u)) continue;
        const uint32_t j = pkr[it];  // leaders are named by packet index
        const Key &k = kr[it];
        const bool lo = k.ep == elo;
        lmin[lpos[it]] = (lo || k.ep == ehi)
                             ? global_probe(a, slots, mask, k, key_hash(k), j, erng[lo ? 0 : 2], erng[lo ? 1 : 3], err)
                             : kLeadTag | j;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t it = 0; it < kInsItems; ++it) {
        const uint32_t j = base + it * kBlock + t;
        if (j < nv) hslot[j] = lpos[it] == kNone ? kNone : lmin[lpos[it]];
    }
}

// ---- stable LSD radix sort by segment id ------------------------------------------------------
__device__ __forceinline__ uint32_t bits_for(uint32_t nseg) {  // bits of the largest key (< nseg)
    return nseg <= 1u ? 1u : 32u - (uint32_t)__builtin_clz(nseg - 1u);
}
// passes = ceil(bits / 8); the digit width spreads the bits evenly over them (18 bits: 3 x 6, not
// 8 + 8 + 2), so each pass has as few buckets as it can -> longer contiguous runs per tile
__device__ __forceinline__ uint32_t n_passes(uint32_t nseg) { return (bits_for(nseg) + 7u) / 8u; }
__device__ __forceinline__ uint32_t digit_width(uint32_t nseg) {
    const uint32_t b = bits_for(nseg), p = (b + 7u) / 8u;
    return (b + p - 1u) / p;
}

// lanes of this wave holding the same digit (valid lanes only)
__device__ __forceinline__ uint64_t digit_peers(bool v, uint32_t d, uint32_t width) {
    uint64_t peers = __ballot(v);
    for (uint32_t b = 0; b < width; ++b) {  // width is uniform
        const uint64_t m = __ballot(v && ((d >> b) & 1u));
        peers &= ((d >> b) & 1u) ? m : ~m;
    }
    return peers;
}

// Look-back scans run over tiles of kTile items (16 rows of 256) so a 4M-item batch has 1024
// look-back steps in its chain instead of 16384.
constexpr uint32_t kRows = kTile / kBlock;

// flags + both block scans + prep in one pass: per-row ballots of VALID and VALID-control packets,
// the tile's exclusive offsets by decoupled look-back (wave 0: compacted index, wave 1: epoch), then
// cidx[j] = packet of compacted slot j, pep[packet] = its epoch (CTRL for singletons; CMD_BARRIER
// only); the last tile
// writes n_valid.
__global__ __launch_bounds__(kBlock) void k_dm_flags_prep(DmIn a, unsigned long long *st_v,
                                                          unsigned long long *st_c, uint32_t *cidx,
                                                          uint32_t *nvp, uint32_t *err) {
    __shared__ uint64_t mv[kRows][kWaves], mc[kRows][kWaves];
    __shared__ uint32_t pre[2];
    const uint32_t b = blockIdx.x, t = threadIdx.x, w = t >> 6, lane = t & 63u;
    uint32_t flags = 0;  // bit r: row r's item valid; bit 16 + r: control
    int8_t stv[kRows];  // every row's loads in flight before the first ballot
    uint8_t cmv[kRows];
    const bool barrier = (a.fields & RSK_DEMUX_CMD_BARRIER) != 0u;
#pragma unroll
    for (uint32_t r = 0; r < kRows; ++r) {
        const uint64_t i = (uint64_t)b * kTile + r * kBlock + t;
        stv[r] = i < a.n ? a.status[i] : (int8_t)RSK_RECV_DROP;
        cmv[r] = i < a.n && barrier ? a.cmd[i] : (uint8_t)RSK_CMD_DATA;
    }
#pragma unroll
    for (uint32_t r = 0; r < kRows; ++r) {
        const bool valid = stv[r] == RSK_RECV_VALID;
        const bool ctrl = valid && cmv[r] != RSK_CMD_DATA;
        const uint64_t bv = __ballot(valid), bc = __ballot(ctrl);
        if (lane == 0u) {
            mv[r][w] = bv;
            mc[r][w] = bc;
        }
        flags |= (valid ? 1u << r : 0u) | (ctrl ? 1u << (16 + r) : 0u);
    }
    __syncthreads();
    uint32_t av = 0, ac = 0;  // the tile's totals; row offsets are recomputed from LDS below (round 4:
                              // holding 2 x 16 of them cost VGPRs, 181 in all -> 2 waves per SIMD)
#pragma unroll
    for (uint32_t r = 0; r < kRows; ++r)
#pragma unroll
        for (uint32_t q = 0; q < (uint32_t)kWaves; ++q) {
            av += (uint32_t)__popcll(mv[r][q]);
            ac += (uint32_t)__popcll(mc[r][q]);
        }
    if (w == 0u) {
        const uint32_t e = dlb_wave(st_v, b, av, lane, err);
        if (lane == 0u) {
            pre[0] = e;
            if (b == gridDim.x - 1u) *nvp = e + av;
        }
    } else if (w == 1u) {
        const uint32_t e = dlb_wave(st_c, b, ac, lane, err);
        if (lane == 0u) {
            pre[1] = e;
            if (b == gridDim.x - 1u && a.cpos) a.cpos[e + ac] = a.n;  // sentinel: the last epoch ends at n
        }
    }
    __syncthreads();
    const uint64_t lt = lanemask_lt(lane);
    uint32_t accv = pre[0], accc = pre[1];  // + items of the rows before r
#pragma unroll
    for (uint32_t r = 0; r < kRows; ++r) {
        uint32_t bv = 0, bc = 0, tv = 0, tc = 0;  // waves before w in row r; the whole row
#pragma unroll
        for (uint32_t q = 0; q < (uint32_t)kWaves; ++q) {
            const uint32_t cv = (uint32_t)__popcll(mv[r][q]), cc = (uint32_t)__popcll(mc[r][q]);
            if (q < w) {
                bv += cv;
                bc += cc;
            }
            tv += cv;
            tc += cc;
        }
        if ((flags >> r) & 1u) {
            const uint32_t i = b * kTile + r * kBlock + t;
            const uint32_t j = accv + bv + (uint32_t)__popcll(mv[r][w] & lt);
            cidx[j] = i;
            if (a.pep) {
                const bool ctl = ((flags >> (16 + r)) & 1u) != 0u;
                const uint32_t ec = accc + bc + (uint32_t)__popcll(mc[r][w] & lt);  // control packets before i
                a.pep[i] = ctl ? kCtrl : ec;
                if (ctl) a.cpos[ec] = i;
            }
        }
        accv += tv;
        accc += tc;
    }
}

// leader + scan + rank in one pass: the leader of compacted packet j is the first packet of its key
// (the index half of its table slot, or j for a control packet); the leaders' dense ranks (segment
// ids in first-occurrence order) by decoupled look-back; rank_at[leader], seg_first[rank]; the last
// tile writes the segment count.  Followers (every other packet) are compacted by the same count:
// follower f = j - (leaders before j) gets fkey[f] = its leader, fval[f] = its packet index.  Block 0
// also clears the radix digit histograms the next launch accumulates.
__global__ __launch_bounds__(kBlock) void k_dm_leader_rank(const uint32_t *nvp, const uint32_t *hslot,
                                                           const unsigned long long *slots, const uint32_t *cidx,
                                                           unsigned long long *st_l, uint32_t *fkey, uint32_t *fval,
                                                           uint32_t *rank_at, uint32_t *seg_first, uint32_t *seg_slot,
                                                           uint32_t tsize, uint32_t *nsegp, uint32_t *ghist,
                                                           uint32_t *err) {
    __shared__ uint64_t ml[kRows][kWaves];
    __shared__ uint32_t pre;
    const uint32_t nv = *nvp;
    const uint32_t b = blockIdx.x, t = threadIdx.x, w = t >> 6, lane = t & 63u;
    if (b == 0u)
        for (uint32_t q = t; q < 4u * 256u; q += kBlock) ghist[q] = 0u;
    uint32_t isl = 0;  // bit r: row r's item is its key's leader
    uint32_t hs[kRows], lead[kRows];
    uint32_t pks[kRows];  // packet indices, loaded with the slots (before the look-back)
#pragma unroll
    for (uint32_t r = 0; r < kRows; ++r) {
        const uint32_t j = b * kTile + r * kBlock + t;
        hs[r] = j < nv ? hslot[j] : kNone;
        pks[r] = j < nv ? cidx[j] : kNone;
    }
    // leaders by packet index (the table and the epoch-local tag hold packet indices)
#pragma unroll
    for (uint32_t r = 0; r < kRows; ++r)
        lead[r] = hs[r] == kNone ? pks[r] : (hs[r] & kLeadTag) ? hs[r] & ~kLeadTag : (uint32_t)slots[hs[r]];
#pragma unroll
    for (uint32_t r = 0; r < kRows; ++r) {
        const uint32_t j = b * kTile + r * kBlock + t;
        const bool l = j < nv && lead[r] == pks[r];
        const uint64_t bl = __ballot(l);
        if (lane == 0u) ml[r][w] = bl;
        isl |= l ? 1u << r : 0u;
    }
    __syncthreads();
    uint32_t al = 0;  // the tile's leaders; row offsets recomputed from LDS below (as k_dm_flags_prep)
#pragma unroll
    for (uint32_t r = 0; r < kRows; ++r)
#pragma unroll
        for (uint32_t q = 0; q < (uint32_t)kWaves; ++q) al += (uint32_t)__popcll(ml[r][q]);
    if (w == 0u) {
        const uint32_t e = dlb_wave(st_l, b, al, lane, err);
        if (lane == 0u) {
            pre = e;
            if (b == gridDim.x - 1u) *nsegp = e + al;
        }
    }
    __syncthreads();
    const uint64_t lt = lanemask_lt(lane);
    uint32_t acc = pre;  // + leaders of the rows before r
#pragma unroll
    for (uint32_t r = 0; r < kRows; ++r) {
        const uint32_t j = b * kTile + r * kBlock + t;
        uint32_t bw = 0, tw = 0;
#pragma unroll
        for (uint32_t q = 0; q < (uint32_t)kWaves; ++q) {
            const uint32_t c = (uint32_t)__popcll(ml[r][q]);
            if (q < w) bw += c;
            tw += c;
        }
        const uint32_t before = acc + bw + (uint32_t)__popcll(ml[r][w] & lt);  // leaders before j
        acc += tw;
        if (j >= nv) continue;
        const uint32_t pk = pks[r];
        if ((isl >> r) & 1u) {
            rank_at[pk] = before;  // by packet index: followers name their leader by it
            seg_first[before] = pk;
            // the table slot its key claimed (k_dm_final clears it), if the key went to the table; past
            // the clearing limit (k_dm_final: n_seg <= tsize / 16) the next call fills the table instead
            if (before <= (tsize >> 4)) seg_slot[before] = hs[r] == kNone || (hs[r] & kLeadTag) ? kNone : hs[r];
        } else {
            fkey[j - before] = lead[r];
            fval[j - before] = pk;
        }
    }
}

// The followers' radix keys + the global digit histograms of every radix pass: fkey[f] (its leader,
// written by k_dm_leader_rank) becomes the leader's segment id in place; one tile of kTile followers
// per block, LDS histograms per pass, one global atomic per non-empty bin.  Leaders are not sorted:
// they already stand in segment order (k_dm_final).
// At most kSmallF followers (a batch of mostly single-packet segments): block 0 sorts them alone, in
// place, by counting for each follower the followers that precede it in (segment id, arrival) order,
// and the radix passes return at once.
constexpr uint32_t kSmallF = 1024;
__global__ __launch_bounds__(kBlock) void k_dm_segof_hist(const uint32_t *nvp, const uint32_t *nsegp,
                                                          const uint32_t *rank_at, uint32_t *keys, uint32_t *vals,
                                                          uint32_t *ghist) {
    __shared__ uint32_t lh[4][256];
    __shared__ uint32_t sk[kSmallF], sv[kSmallF];
    const uint32_t ns = *nsegp, nf = *nvp - ns, t = threadIdx.x, lane = t & 63u;
    const uint32_t base = blockIdx.x * kTile;
    if (base >= nf) return;  // block-uniform
    if (nf <= kSmallF) {  // block 0 only (base = 0)
        constexpr uint32_t kPer = kSmallF / kBlock;
        uint32_t ld[kPer], kk[kPer], vv[kPer];
#pragma unroll
        for (uint32_t r = 0; r < kPer; ++r) {
            const uint32_t f = r * kBlock + t;
            ld[r] = f < nf ? keys[f] : 0u;
            vv[r] = f < nf ? vals[f] : 0u;
        }
#pragma unroll
        for (uint32_t r = 0; r < kPer; ++r) {
            const uint32_t f = r * kBlock + t;
            kk[r] = f < nf ? rank_at[ld[r]] : 0u;
            if (f < nf) {  // every global read is consumed before the barrier: the writes below are in place
                sk[f] = kk[r];
                sv[f] = vv[r];
            }
        }
        __syncthreads();
        uint32_t pos[kPer] = {};
        for (uint32_t g = 0; g < nf; ++g) {  // sk[g] is an LDS broadcast
            const uint32_t kg = sk[g];
#pragma unroll
            for (uint32_t r = 0; r < kPer; ++r) pos[r] += kg < kk[r] || (kg == kk[r] && g < r * kBlock + t);
        }
        __syncthreads();
#pragma unroll
        for (uint32_t r = 0; r < kPer; ++r) {
            if (r * kBlock + t >= nf) continue;
            keys[pos[r]] = kk[r];
            vals[pos[r]] = sv[r * kBlock + t];
        }
        return;
    }
    const uint32_t np = n_passes(ns), width = digit_width(ns), dm = (1u << width) - 1u;
#pragma unroll
    for (int p = 0; p < 4; ++p) lh[p][t] = 0u;
    __syncthreads();
    uint32_t kk[kItems], ld[kItems];  // all leader loads, then all rank_at gathers, in flight at once
#pragma unroll
    for (uint32_t r = 0; r < kItems; ++r) {
        const uint32_t f = base + r * kBlock + t;
        ld[r] = f < nf ? keys[f] : 0u;
    }
#pragma unroll
    for (uint32_t r = 0; r < kItems; ++r) {
        const uint32_t f = base + r * kBlock + t;
        kk[r] = f < nf ? rank_at[ld[r]] : 0u;
    }
#pragma unroll
    for (uint32_t r = 0; r < kItems; ++r) {
        const uint32_t f = base + r * kBlock + t;
        if (f < nf) keys[f] = kk[r];
    }
    for (uint32_t p = 0; p < np; ++p) {  // np is block-uniform
#pragma unroll
        for (uint32_t r = 0; r < kItems; ++r) {
            // one LDS atomic per lane; a row whose valid lanes all hold one digit (a hot segment)
            // adds its count once (round 5: the per-bit ballot match of every row cost C3 ~20 us)
            const bool v = base + r * kBlock + t < nf;
            const uint32_t d = (kk[r] >> (width * p)) & dm;
            const uint64_t bv = __ballot(v);
            if (bv == 0ull) continue;  // wave-uniform
            const uint32_t first = (uint32_t)__builtin_ctzll(bv);
            const uint32_t df = (uint32_t)__shfl((int)d, (int)first);
            if (__ballot(v && d == df) == bv) {
                if (lane == first) atomicAdd(&lh[p][df], (uint32_t)__popcll(bv));
            } else if (v) {
                atomicAdd(&lh[p][d], 1u);
            }
        }
    }
    __syncthreads();
    for (uint32_t p = 0; p < np; ++p)
        if (lh[p][t]) atomicAdd(ghist + 256u * p + t, lh[p][t]);
}

// One radix pass, onesweep: tile t (= block t, dispatch order) ranks its items stably, gets the count
// of each digit in tiles before it by per-digit decoupled look-back, adds the digit's global start
// (exclusive scan of the pass's global histogram) and writes the tile out digit run by digit run
// (consecutive threads, consecutive addresses).  Round 4: wave w owns items [w * 1024, w * 1024 + 1024)
// of the tile and ranks them row by row (64 items) against its own running digit counts in LDS, so
// the ranking needs no block barrier per row (rounds 2-3: rows across the 4 waves, three block
// barriers per row, 48 per tile); one barrier then turns the per-wave counts into per-wave offsets.
__global__ __launch_bounds__(kBlock) void k_dm_onesweep(uint32_t pass, const uint32_t *nvp, const uint32_t *nsegp,
                                                        const uint32_t *kin, const uint32_t *vin, const uint32_t *ghist,
                                                        unsigned long long *st, uint32_t *kout, uint32_t *vout,
                                                        uint32_t *err) {
    constexpr uint32_t kPerWave = kTile / kWaves;  // 1024 items, kItems rows of 64
    __shared__ uint32_t wcnt[kWaves][256];  // wave's running digit counts, then its exclusive offsets
    __shared__ uint32_t lbase[256], dbase[256];
    __shared__ uint32_t sk[kTile], sv[kTile];
    const uint32_t ns = *nsegp, nv = *nvp - ns, tile = blockIdx.x;  // nv: the followers being sorted
    if (pass >= n_passes(ns) || tile * kTile >= nv || nv <= kSmallF) return;  // block-uniform; no later tile waits
    const uint32_t width = digit_width(ns), sh = width * pass, dm = (1u << width) - 1u;
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint32_t base = tile * kTile, wbase = base + w * kPerWave;
    const uint32_t cnt = nv - base < kTile ? nv - base : kTile;
#pragma unroll
    for (int q = 0; q < kWaves; ++q) wcnt[q][t] = 0;
    uint32_t kk[kItems], vv[kItems], rk[kItems];
#pragma unroll
    for (uint32_t r = 0; r < kItems; ++r) {
        const uint32_t k = wbase + r * 64u + lane;
        kk[r] = k < nv ? kin[k] : 0u;
        vv[r] = k < nv ? vin[k] : 0u;
    }
    __syncthreads();
    const uint64_t lt = lanemask_lt(lane);
#pragma unroll
    for (uint32_t r = 0; r < kItems; ++r) {  // wave-local: the wave's rows in item order
        const bool v = wbase + r * 64u + lane < nv;
        const uint32_t d = (kk[r] >> sh) & dm;
        const uint64_t peers = digit_peers(v, d, width);
        const uint32_t below = (uint32_t)__popcll(peers & lt);
        const uint32_t c = v ? wcnt[w][d] : 0u;
        rk[r] = c + below;
        if (v && below == 0u) wcnt[w][d] = c + (uint32_t)__popcll(peers);  // after every lane's read (in order)
    }
    __syncthreads();
    uint32_t tot = 0;  // digit t: the tile's count, and each wave's exclusive offset
#pragma unroll
    for (int q = 0; q < kWaves; ++q) {
        const uint32_t c = wcnt[q][t];
        wcnt[q][t] = tot;
        tot += c;
    }
    lbase[t] = tot;
    // global position of this tile's first digit-t item: digits before t overall + digit t before this tile
    const uint32_t before = dlb_digit(st + (uint64_t)pass * 256u * gridDim.x, tile, t, tot, err);
    __syncthreads();
    if (w == 0) {  // exclusive scans of the global histogram and of the tile's bins (4 per lane)
        uint32_t g[4], c[4], gs = 0, cs = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            g[q] = ghist[256u * pass + 4u * lane + q];
            c[q] = lbase[4 * lane + q];
            gs += g[q];
            cs += c[q];
        }
        uint32_t gi = gs, ci = cs;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t x = __shfl_up(gi, off), y = __shfl_up(ci, off);
            if (lane >= (uint32_t)off) {
                gi += x;
                ci += y;
            }
        }
        uint32_t ga = gi - gs, ca = ci - cs;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            dbase[4 * lane + q] = ga;
            lbase[4 * lane + q] = ca;
            ga += g[q];
            ca += c[q];
        }
    }
    __syncthreads();
    dbase[t] += before;
#pragma unroll
    for (uint32_t r = 0; r < kItems; ++r) {
        if (wbase + r * 64u + lane >= nv) continue;
        const uint32_t d = (kk[r] >> sh) & dm;
        const uint32_t pos = lbase[d] + wcnt[w][d] + rk[r];
        sk[pos] = kk[r];
        sv[pos] = vv[r];
    }
    __syncthreads();
    for (uint32_t p = t; p < cnt; p += kBlock) {
        const uint32_t key = sk[p], d = (key >> sh) & dm;
        const uint32_t g = dbase[d] + (p - lbase[d]);
        kout[g] = key;
        vout[g] = sv[p];
    }
}

// Merge of the leaders (segment order already) with the sorted followers (segment id, arrival order):
// segment s starts at s + (followers of segments before s), a lower bound in the sorted keys, and its
// leader goes there; the follower at sorted position p with segment id r lands at r + 1 + p (r
// leaders up to and including its own, p followers before it).
__global__ __launch_bounds__(kBlock) void k_dm_final(const uint32_t *nvp, const uint32_t *nsegp, const uint32_t *kA,
                                                     const uint32_t *vA, const uint32_t *kB, const uint32_t *vB,
                                                     const uint32_t *seg_first, uint32_t *perm, uint32_t *seg_off,
                                                     uint32_t *n_seg, uint32_t *n_valid, const uint32_t *seg_slot,
                                                     unsigned long long *slots, uint32_t tsize, uint32_t clear_max,
                                                     uint32_t *tflag, uint32_t *hint) {
    const uint32_t nv = *nvp, ns = *nsegp, nf = nv - ns;
    const uint32_t passes = n_passes(ns);  // effective passes; pass p writes B when p is even
    const bool inB = nf > kSmallF && ((passes - 1u) & 1u) == 0u;  // small: sorted in place in A
    const uint32_t *keys = inB ? kB : kA;
    const uint32_t *vals = inB ? vB : vA;
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    // few segments: clear the slots their keys claimed and mark the table clean for the next call of
    // this size; many (up to one per packet): leave it to the next call's fill (scattered 8-B clears
    // of 3.4 M slots cost more than the 64-MB fill: server shape 0.474 -> 0.500 ms)
    const bool clear = ns <= clear_max;
    if (k == 0) {
        *n_seg = ns;
        *n_valid = nv;
        seg_off[ns] = nv;
        *tflag = clear ? tsize : 0u;
        if (hint) __hip_atomic_store(hint, clear ? tsize : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (k < ns) {
        uint32_t lo = 0, hi = nf;  // followers with segment id < k
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (keys[mid] < k) lo = mid + 1u;
            else hi = mid;
        }
        seg_off[k] = k + lo;
        perm[k + lo] = seg_first[k];
        // every slot the call claimed belongs to one key, hence one leader: all-ones again for the
        // next call (round 6: instead of a fill of the whole table, 12.5 us for C3's 64 MB)
        if (clear) {
            const uint32_t ss = seg_slot[k];
            if (ss != kNone) slots[ss] = ~0ull;
        }
    }
    if (k < nf) perm[keys[k] + 1u + k] = vals[k];
}

// The per-call fill: the look-back state words always, the key table unless the last call on this
// scratch left it clean for this table size (*tflag == tsize, k_dm_final).  16-B stores, grid-stride.
__global__ __launch_bounds__(kBlock) void k_dm_fill(const uint32_t *tflag, uint32_t tsize, uint4 *slots,
                                                    uint64_t slot16, uint4 *states, uint64_t state16) {
    const bool table = *tflag != tsize;  // uniform
    const uint4 ones = make_uint4(~0u, ~0u, ~0u, ~0u);
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < state16; i += stride) states[i] = ones;
    if (table)
        for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < slot16; i += stride) slots[i] = ones;
}

// ---- workspace ------------------------------------------------------------------------------
struct DmWs {
    uint32_t *cidx, *hslot, *rank_at, *pep, *cpos, *seg_slot;
    uint32_t *kA, *vA, *kB, *vB;
    uint32_t *ghist;
    unsigned long long *slots;  // the key table, then the look-back states (k_dm_fill)
    unsigned long long *st_v, *st_c, *st_l, *st_r;
    size_t state_bytes;
    uint32_t *tflag;  // == tsize: the table is all-ones for this size (k_dm_final), else the fill writes it
    uint32_t *nv, *nseg;
    uint32_t nb, nt, tsize;
};

uint32_t table_size(uint32_t n) {  // power of two >= 2 n (n <= 2^30, checked by the entry point)
    uint64_t t = 64;
    while (t < 2ull * n) t <<= 1;
    return (uint32_t)t;
}

size_t dm_layout(uint32_t n, uint8_t *base, DmWs *w) {
    const uint32_t nb = (n + kBlock - 1) / kBlock, nt = (n + kTile - 1) / kTile, T = table_size(n);
    size_t off = 0;
    auto take = [&](size_t bytes) -> uint8_t * {
        uint8_t *p = base ? base + off : nullptr;
        off += (bytes + 255) & ~size_t(255);
        return p;
    };
    DmWs d;
    d.tflag = (uint32_t *)take(8);  // first, at a fixed place for every batch size
    d.cidx = (uint32_t *)take(4ull * n);
    d.hslot = (uint32_t *)take(4ull * n);
    d.rank_at = (uint32_t *)take(4ull * n);
    d.pep = (uint32_t *)take(4ull * n);
    d.cpos = (uint32_t *)take(4ull * n + 4ull);
    d.seg_slot = (uint32_t *)take(4ull * n);
    d.kA = (uint32_t *)take(4ull * n);
    d.vA = (uint32_t *)take(4ull * n);
    d.kB = (uint32_t *)take(4ull * n);
    d.vB = (uint32_t *)take(4ull * n);
    d.ghist = (uint32_t *)take(4ull * 4 * 256);
    d.nv = (uint32_t *)take(8);
    d.nseg = (uint32_t *)take(8);
    d.slots = (unsigned long long *)take(8ull * T);
    const size_t st0 = off;
    d.st_v = (unsigned long long *)take(8ull * nt);
    d.st_c = (unsigned long long *)take(8ull * nt);
    d.st_l = (unsigned long long *)take(8ull * nt);
    d.st_r = (unsigned long long *)take(8ull * 4 * 256 * nt);
    d.state_bytes = off - st0;
    d.nb = nb;
    d.nt = nt;
    d.tsize = T;
    if (w) *w = d;
    return off;
}

// ---- GROUP_BARRIER: each DATA packet's epoch inside its IdBuf -------------------------------
// The first pass groups only the VALID CONTROL packets by IdBuf (k_dm_gstatus hides every other
// packet), so its table maps an IdBuf to the first control packet of that IdBuf and its segments list
// each IdBuf's control packets in arrival order.  k_dm_gep then gives every VALID DATA packet i the
// number of its IdBuf's control packets before it -- a probe of that table by IdBuf, the segment of
// the owner, a binary search of i among the segment's packet indices -- as its key word for the
// second pass; a control packet gets kLeadTag | its own index, a key no other packet has (a
// singleton segment).  (First build: a group-by of every packet by IdBuf and a scan, 0.82 ms on the
// server shape.)
__global__ __launch_bounds__(kBlock) void k_dm_gstatus(const int8_t *status, const uint8_t *cmd, uint32_t n,
                                                       int8_t *st2) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) st2[i] = status[i] == RSK_RECV_VALID && cmd[i] != RSK_CMD_DATA ? (int8_t)RSK_RECV_VALID
                                                                            : (int8_t)RSK_RECV_DROP;
}
__global__ __launch_bounds__(kBlock) void k_dm_gep(DmIn a, const unsigned long long *slots, uint32_t mask,
                                                   const uint32_t *rank_at, const uint32_t *perm,
                                                   const uint32_t *seg_off, uint32_t *xep, uint32_t *err) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= a.n || a.status[i] != RSK_RECV_VALID) return;
    if (a.cmd[i] != RSK_CMD_DATA) {
        xep[i] = kLeadTag | i;
        return;
    }
    const Key k = load_key(a, i, 0u);  // the IdBuf alone (a.fields = RSK_DEMUX_ID, no epoch, no word)
    const uint64_t hv = key_hash(k);
    const uint32_t fp = (uint32_t)(hv >> 32);
    uint32_t h = (uint32_t)hv & mask, cnt = 0;
    for (uint32_t walked = 0; walked <= mask; ++walked) {  // read-only probe: the table is complete
        const unsigned long long e = slots[h];
        if (e == ~0ull) break;  // no control packet of this IdBuf
        if ((uint32_t)(e >> 32) == fp && a.id[(uint32_t)e] == k.id) {
            const uint32_t sg = rank_at[(uint32_t)e];
            uint32_t lo = seg_off[sg], hi = seg_off[sg + 1u];  // the IdBuf's control packets, in order
            while (lo < hi) {  // how many of them precede i
                const uint32_t mid = (lo + hi) >> 1;
                if (perm[mid] < i) lo = mid + 1u;
                else hi = mid;
            }
            cnt = lo - seg_off[sg];
            break;
        }
        h = (h + 1u) & mask;
        if (walked == mask) __hip_atomic_fetch_or(err, RSK_DEVERR_TABLE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    xep[i] = cnt;
}

// One group-by pass over the batch (the whole rsk_demux_batch without GROUP_BARRIER); keep_table:
// k_dm_final leaves the key table as it is (GROUP_BARRIER's first pass: k_dm_gep reads it).
int demux_pass(rsk_ctx *c, const DmIn &a, const DmWs &w, const rsk_demux_out *out, hipStream_t s,
               bool keep_table = false) {
    const uint32_t n = a.n;
    int r;
    // the look-back state words start as all-ones, and so does the key table, unless the last call
    // left it clean for this size (k_dm_final clears the slots of batches with few segments); fresh
    // scratch (or scratch after a device error) gets its flag word reset first
    if (!rsk::ws_clean(c, s, rsk::WS_DEMUX)) {
        hipError_t e = hipMemsetAsync(w.tflag, 0, 4, s);
        if (e != hipSuccess) { rsk::set_error("hipMemsetAsync(table flag)", e); return RSK_EDEVICE; }
        rsk::set_ws_clean(c, s, rsk::WS_DEMUX, true);
    }
    // the host-mapped hint (k_dm_final's last verdict, read without synchronisation) picks the form:
    // likely dirty -> one memset of table and states (a blit, faster than the kernel: C4 0.080 vs
    // 0.085 ms); likely clean -> k_dm_fill, which checks the device flag itself (a stale hint is only
    // slower, never wrong)
    uint32_t *hint = c->enc_stat_dev ? c->enc_stat_dev + 1 : nullptr;
    const bool likely_clean = c->enc_stat_host && __atomic_load_n(c->enc_stat_host + 1, __ATOMIC_RELAXED) == w.tsize;
    if (!likely_clean) {
        hipError_t e = hipMemsetAsync(w.slots, 0xff, (size_t)w.tsize * 8u + w.state_bytes, s);
        if (e != hipSuccess) { rsk::set_error("hipMemsetAsync(table)", e); return RSK_EDEVICE; }
    } else {
        const uint64_t slot16 = ((uint64_t)w.tsize * 8u) / 16u, state16 = w.state_bytes / 16u;
        const unsigned fg = (unsigned)std::min<uint64_t>(4096u, (slot16 + kBlock - 1) / kBlock);
        hipLaunchKernelGGL(k_dm_fill, dim3(fg), dim3(kBlock), 0, s, w.tflag, w.tsize, reinterpret_cast<uint4 *>(w.slots),
                           slot16, reinterpret_cast<uint4 *>(w.st_v), state16);
    }
    hipLaunchKernelGGL(k_dm_flags_prep, dim3(w.nt), dim3(kBlock), 0, s, a, w.st_v, w.st_c, w.cidx, w.nv,
                       c->err_dev);
    hipLaunchKernelGGL(k_dm_insert, dim3((n + kInsTile - 1) / kInsTile), dim3(kBlock), 0, s, a, w.nv, w.cidx,
                       w.slots, w.tsize - 1u, w.hslot, c->err_dev);
    hipLaunchKernelGGL(k_dm_leader_rank, dim3(w.nt), dim3(kBlock), 0, s, w.nv, w.hslot, w.slots, w.cidx, w.st_l,
                       w.kA, w.vA, w.rank_at, out->seg_first, w.seg_slot, w.tsize, w.nseg, w.ghist, c->err_dev);
    hipLaunchKernelGGL(k_dm_segof_hist, dim3(w.nt), dim3(kBlock), 0, s, w.nv, w.nseg, w.rank_at, w.kA, w.vA,
                       w.ghist);
    if ((r = rsk::launch_check("k_dm_segof_hist"))) return r;
    // passes for the largest possible segment count (n); surplus passes return at once
    uint32_t maxbits = 1;
    while (maxbits < 32 && (1ull << maxbits) < n) ++maxbits;
    const uint32_t passes = (maxbits + 7) / 8;
    for (uint32_t p = 0; p < passes; ++p) {
        const uint32_t *kin = (p & 1u) ? w.kB : w.kA, *vin = (p & 1u) ? w.vB : w.vA;
        uint32_t *kout = (p & 1u) ? w.kA : w.kB, *vout = (p & 1u) ? w.vA : w.vB;
        hipLaunchKernelGGL(k_dm_onesweep, dim3(w.nt), dim3(kBlock), 0, s, p, w.nv, w.nseg, kin, vin, w.ghist, w.st_r,
                           kout, vout, c->err_dev);
        if ((r = rsk::launch_check("k_dm_onesweep"))) return r;
    }
    hipLaunchKernelGGL(k_dm_final, dim3(w.nb), dim3(kBlock), 0, s, w.nv, w.nseg, w.kA, w.vA, w.kB, w.vB,
                       out->seg_first, out->perm, out->seg_off, out->n_seg, out->n_valid, w.seg_slot, w.slots,
                       w.tsize, keep_table ? 0u : w.tsize >> 4, w.tflag, hint);
    return rsk::launch_check("k_dm_final");
}

}  // namespace

extern "C" int rsk_demux_batch(rsk_ctx *c, uint32_t n, const rsk_demux_in *in, uint32_t fields,
                               const rsk_demux_out *out, void *stream) {
    if (!c || !in || !out || !out->perm || !out->seg_off || !out->seg_first || !out->n_seg || !out->n_valid)
        return RSK_EINVAL;
    if (fields & ~0x3fu) return RSK_EINVAL;
    const bool group = (fields & RSK_DEMUX_GROUP_BARRIER) != 0u;
    if (group && ((fields & RSK_DEMUX_CMD_BARRIER) || !(fields & RSK_DEMUX_ID))) return RSK_EINVAL;
    if (n && (!in->status || !in->cmd)) return RSK_EINVAL;
    if (n && (fields & RSK_DEMUX_ID) && (!in->id || (reinterpret_cast<uintptr_t>(in->id) & 7u))) return RSK_EINVAL;
    if (n && (fields & RSK_DEMUX_CONN_KEY) && !in->conn_key) return RSK_EINVAL;
    if (n && (fields & RSK_DEMUX_CONV) && !in->conv) return RSK_EINVAL;
    if (n && (fields & RSK_DEMUX_DST) && !in->dst) return RSK_EINVAL;
    if (n > (1u << 30)) return RSK_EINVAL;  // table of 2^31 slots max (uint32 slot indices)
    rsk::DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        hipError_t e = hipMemsetAsync(out->n_seg, 0, 4, s);
        if (e == hipSuccess) e = hipMemsetAsync(out->n_valid, 0, 4, s);
        if (e == hipSuccess) e = hipMemsetAsync(out->seg_off, 0, 4, s);
        if (e != hipSuccess) { rsk::set_error("hipMemsetAsync", e); return RSK_EDEVICE; }
        return RSK_OK;
    }
    void *wsp = nullptr;
    int r = rsk::stream_ws(c, s, rsk::WS_DEMUX, dm_layout(n, nullptr, nullptr), &wsp);
    if (r) return r;
    DmWs w;
    dm_layout(n, static_cast<uint8_t *>(wsp), &w);
    DmIn a;
    a.status = in->status;
    a.cmd = in->cmd;
    a.id = reinterpret_cast<const uint64_t *>(in->id);
    a.conv = in->conv;
    a.key = in->conn_key;
    a.dst = in->dst;
    a.n = n;
    a.fields = fields & ~RSK_DEMUX_GROUP_BARRIER;
    a.pep = (fields & RSK_DEMUX_CMD_BARRIER) ? w.pep : nullptr;
    a.cpos = (fields & RSK_DEMUX_CMD_BARRIER) ? w.cpos : nullptr;
    a.xep = nullptr;
    if (!group) return demux_pass(c, a, w, out, s);
    // GROUP_BARRIER: the control packets alone by IdBuf (into out; their VALID mask in pep, which
    // neither pass uses otherwise), each DATA packet's epoch inside its IdBuf into pep (k_dm_gep, over
    // the first pass's table and segments), then the key with that epoch (over out again)
    int8_t *st2 = reinterpret_cast<int8_t *>(w.pep);
    hipLaunchKernelGGL(k_dm_gstatus, dim3(w.nb), dim3(kBlock), 0, s, a.status, a.cmd, n, st2);
    DmIn ga = a;
    ga.status = st2;
    ga.fields = RSK_DEMUX_ID;
    if ((r = demux_pass(c, ga, w, out, s, true))) return r;
    DmIn gk = a;  // the batch's own VALID mask (st2 is overwritten by the epochs), the IdBuf as the key
    gk.fields = RSK_DEMUX_ID;
    hipLaunchKernelGGL(k_dm_gep, dim3(w.nb), dim3(kBlock), 0, s, gk, w.slots, w.tsize - 1u, w.rank_at, out->perm,
                       out->seg_off, w.pep, c->err_dev);
    if ((r = rsk::launch_check("k_dm_gep"))) return r;
    a.xep = w.pep;
    return demux_pass(c, a, w, out, s);
}

// =============================================================================================
// Connection state of the fake-TCP path around the codec: FakeTcp::Output's seq advance and
// RawTcp::Output's IP id counter (send), FakeTcp::OnRecv's ack (receive).  include/rsk_codec.h.
// =============================================================================================
namespace {

// framed packets of known connections take part in the group-by (status VALID), the rest do not
__global__ __launch_bounds__(kBlock) void k_sq_flags(const uint32_t *conn, const int32_t *status, uint32_t n,
                                                     uint32_t n_conn, int8_t *part, uint8_t *cmd0, uint32_t *framed) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const bool fr = status[i] > 0;                                  // RConn::Output framed it
    part[i] = (int8_t)(fr && conn[i] < n_conn ? RSK_RECV_VALID : RSK_RECV_DROP);
    cmd0[i] = 0;
    framed[i] = fr ? 1u : 0u;
}

// frame lengths in segment (= connection) order, 0 past n_valid (the scan runs over n + 1 slots)
__global__ __launch_bounds__(kBlock) void k_sq_lens(const uint32_t *perm, const uint32_t *nvp, const int32_t *status,
                                                    uint32_t n, uint32_t *v) {
    const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    if (j > n) return;
    v[j] = j < *nvp ? (uint32_t)status[perm[j]] : 0u;
}

// one thread per segment: the connection's seq before the batch, relative to the scan, and its
// advance over the batch (every connection is exactly one segment, so no two threads share it)
__global__ __launch_bounds__(kBlock) void k_sq_conn(const uint32_t *nsegp, const uint32_t *seg_off,
                                                    const uint32_t *seg_first, const uint32_t *conn,
                                                    const uint32_t *pre, uint32_t *conn_seq, uint32_t *base) {
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= *nsegp) return;
    const uint32_t c = conn[seg_first[s]];
    const uint32_t p0 = pre[seg_off[s]], p1 = pre[seg_off[s + 1]];
    const uint32_t before = conn_seq[c];
    base[c] = before - p0;          // mod 2^32, as TcpInfo::seq wraps
    conn_seq[c] = before + (p1 - p0);
}

__global__ __launch_bounds__(kBlock) void k_sq_seq(const uint32_t *perm, const uint32_t *nvp, const uint32_t *conn,
                                                   const uint32_t *base, const uint32_t *pre, uint32_t *seq) {
    const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    if (j >= *nvp) return;
    const uint32_t i = perm[j];
    seq[i] = base[conn[i]] + pre[j];
}

__global__ __launch_bounds__(kBlock) void k_sq_ipid(const uint32_t *framed, const uint32_t *rank, uint32_t n,
                                                    const uint16_t *ip_next, uint16_t *ip_id) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    ip_id[i] = framed[i] ? (uint16_t)(*ip_next + rank[i]) : (uint16_t)0;  // mIpId++ wraps at 2^16
}

__global__ void k_sq_ipid_advance(uint16_t *ip_next, const uint32_t *nfr) { *ip_next = (uint16_t)(*ip_next + *nfr); }

__global__ __launch_bounds__(kBlock) void k_ack(const uint32_t *conn, const uint8_t *delivered, const uint32_t *seq,
                                                uint32_t n, uint32_t n_conn, uint32_t *conn_ack) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n || !delivered[i] || conn[i] >= n_conn) return;
    atomicMax(conn_ack + conn[i], seq[i]);  // FakeTcp.cpp:60-64: ack = seq when mInfo.ack < seq
}

// n_conn <= kAckLds: each workgroup folds a 4096-packet tile into an LDS table first, then issues one
// global atomicMax per connection it saw (a few hot connections would otherwise serialise every
// packet's atomic on a handful of words: 1.23 ms for 4M packets over 64 connections).
constexpr uint32_t kAckLds = 8192;
constexpr uint32_t kAckTile = 4096;
__global__ __launch_bounds__(kBlock) void k_ack_lds(const uint32_t *conn, const uint8_t *delivered, const uint32_t *seq,
                                                    uint32_t n, uint32_t n_conn, uint32_t *conn_ack) {
    __shared__ uint32_t tab[kAckLds];
    for (uint32_t c = threadIdx.x; c < n_conn; c += kBlock) tab[c] = 0u;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * kAckTile;
    for (uint32_t k = threadIdx.x; k < kAckTile; k += kBlock) {
        const uint64_t i = t0 + k;
        if (i < n && delivered[i] && conn[i] < n_conn) atomicMax(tab + conn[i], seq[i]);
    }
    __syncthreads();
    for (uint32_t c = threadIdx.x; c < n_conn; c += kBlock)
        if (tab[c]) atomicMax(conn_ack + c, tab[c]);  // max with 0 changes nothing
}

// ---- send seq / IP id, table path (n_conn + 1 <= kSqCols) --------------------------------------
// Without the group-by: the batch is cut into wave tiles of W packets (W >= n_conn + 1, so the table
// below is at most 4 B per packet).  Column c < n_conn of a tile's row is connection c's framed
// bytes in the tile, column n_conn its framed-packet count (the IP id column).
//   k_sqt_sum    per wave tile, a wave-private LDS row (ds_add), written to tab[tile][col]
//   k_sqt_csum / k_sqt_cscan   per column, exclusive scan down the tiles, rebased on conn_seq[c] /
//                *ip_id_next, in place; the column's total advances the state (k_sqt_scan: the
//                one-kernel form, A/B)
//   k_sqt_apply  per wave tile in batch order: the row back into LDS, then per 64-packet round the
//                in-wave per-connection exclusive prefix by a readlane walk of the 64 lanes; the last
//                lane of each connection carries the row forward
// Every packet is read twice (conn + status, 8 B) and written once (seq + ip_id, 6 B).
constexpr uint32_t kSqCols = 2048;
constexpr uint32_t kSqScanThreads = 1024;

__device__ __forceinline__ void sqt_load4(const uint32_t *conn, const int32_t *status, uint64_t r, uint64_t end,
                                          uint32_t lane, int32_t (&st)[4], uint32_t (&cn)[4]) {
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint64_t i = r + 64u * k + lane;
        const bool in = i < end;
        st[k] = in ? status[i] : 0;
        cn[k] = in ? conn[i] : 0u;
    }
}

__global__ __launch_bounds__(kBlock) void k_sqt_sum(const uint32_t *conn, const int32_t *status, uint32_t n,
                                                    uint32_t n_conn, uint32_t W, uint32_t nwt, uint32_t *tab) {
    extern __shared__ uint32_t sq_lds[];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, ncol = n_conn + 1u;
    const uint32_t wt = blockIdx.x * kWaves + wv;
    uint32_t *t = sq_lds + wv * ncol;
    for (uint32_t c = lane; c < n_conn; c += 64u) t[c] = 0u;
    __syncthreads();
    uint32_t nfr = 0;
    if (wt < nwt) {
        const uint64_t base = (uint64_t)wt * W, end = base + W < n ? base + W : n;
        for (uint64_t r = base; r < end; r += 256u) {
            int32_t st[4];
            uint32_t cn[4];
            sqt_load4(conn, status, r, end, lane, st, cn);
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
                const bool fr = st[k] > 0;
                nfr += (uint32_t)__popcll(__ballot(fr));
                if (fr && cn[k] < n_conn) atomicAdd(t + cn[k], (uint32_t)st[k]);
            }
        }
    }
    __syncthreads();
    if (wt < nwt) {
        uint32_t *row = tab + (uint64_t)wt * ncol;
        for (uint32_t c = lane; c < n_conn; c += 64u) row[c] = t[c];
        if (lane == 0) row[n_conn] = nfr;
    }
}

// cb columns per block (a power of two), 1024 / cb row groups; group g scans rows [g R, (g + 1) R)
__global__ __launch_bounds__(kSqScanThreads) void k_sqt_scan(uint32_t *tab, uint32_t nwt, uint32_t n_conn, uint32_t cb,
                                                             uint32_t *conn_seq, uint16_t *ip_next) {
    __shared__ uint32_t part[kSqScanThreads];
    const uint32_t ncol = n_conn + 1u, cl = threadIdx.x % cb, g = threadIdx.x / cb, ng = kSqScanThreads / cb;
    const uint32_t c = blockIdx.x * cb + cl;
    const bool ok = c < ncol;
    const uint32_t R = (nwt + ng - 1u) / ng, r0 = g * R < nwt ? g * R : nwt, r1 = r0 + R < nwt ? r0 + R : nwt;
    const uint32_t state = ok ? (c < n_conn ? conn_seq[c] : (uint32_t)*ip_next) : 0u;  // read before any write
    uint32_t s = 0;
    if (ok) {
        uint32_t r = r0;
        for (; r + 8u <= r1; r += 8u) {
            uint32_t v[8];
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) v[k] = tab[(uint64_t)(r + k) * ncol + c];
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) s += v[k];
        }
        for (; r < r1; ++r) s += tab[(uint64_t)r * ncol + c];
    }
    // inclusive scan of the group sums down each column (Hillis-Steele over the ng groups)
    part[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t off = 1; off < ng; off <<= 1) {
        const uint32_t v = part[threadIdx.x] + (g >= off ? part[threadIdx.x - off * cb] : 0u);
        __syncthreads();
        part[threadIdx.x] = v;
        __syncthreads();
    }
    if (!ok) return;
    uint32_t run = state + part[threadIdx.x] - s;  // mod 2^32 (TcpInfo::seq) / mod 2^16 once stored (mIpId)
    uint32_t r = r0;
    for (; r + 8u <= r1; r += 8u) {
        uint32_t v[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) v[k] = tab[(uint64_t)(r + k) * ncol + c];
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) {
            tab[(uint64_t)(r + k) * ncol + c] = run;
            run += v[k];
        }
    }
    for (; r < r1; ++r) {
        const uint32_t v = tab[(uint64_t)r * ncol + c];
        tab[(uint64_t)r * ncol + c] = run;
        run += v;
    }
    if (g == ng - 1u) {  // the last group ends on the column's total
        if (c < n_conn) conn_seq[c] = run;
        else *ip_next = (uint16_t)run;
    }
}

// Coalesced two-kernel form of the column scan: a wave reads 64 adjacent columns of one row per
// load.  Rows are cut into nch chunks of RC rows (RC a multiple of 16, nch <= 64); grid (column
// blocks of 64, chunks), 16 waves per block, wave w owns RC / 16 consecutive rows of the chunk.
//   k_sqt_csum   chunk sums per column -> csum[chunk][col]; chunk 0 snapshots the state into st0
//   k_sqt_cscan  chunk offset = st0 + earlier chunks' sums, wave offsets by LDS, rows rewritten as
//                exclusive prefixes; the last chunk's last wave advances the state
constexpr uint32_t kSqcWaves = 16;
__global__ __launch_bounds__(kSqcWaves * 64) void k_sqt_csum(const uint32_t *tab, uint32_t nwt, uint32_t n_conn,
                                                             uint32_t RC, uint32_t *csum, uint32_t *st0,
                                                             const uint32_t *conn_seq, const uint16_t *ip_next) {
    __shared__ uint32_t part[kSqcWaves][64];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, ncol = n_conn + 1u;
    const uint32_t c = blockIdx.x * 64u + lane, ch = blockIdx.y, RW = RC / kSqcWaves;
    const bool ok = c < ncol;
    const uint32_t r0 = ch * RC + wv * RW;
    uint32_t sm = 0;
    if (ok) {
#pragma unroll 16
        for (uint32_t k = 0; k < RW; ++k)
            if (r0 + k < nwt) sm += tab[(uint64_t)(r0 + k) * ncol + c];
    }
    part[wv][lane] = sm;
    __syncthreads();
    if (wv == 0 && ok) {
        uint32_t tot = 0;
#pragma unroll
        for (uint32_t q = 0; q < kSqcWaves; ++q) tot += part[q][lane];
        csum[(uint64_t)ch * ncol + c] = tot;
        if (ch == 0) st0[c] = c < n_conn ? conn_seq[c] : (uint32_t)*ip_next;
    }
}

__global__ __launch_bounds__(kSqcWaves * 64) void k_sqt_cscan(uint32_t *tab, uint32_t nwt, uint32_t n_conn,
                                                              uint32_t RC, uint32_t nch, const uint32_t *csum,
                                                              const uint32_t *st0, uint32_t *conn_seq,
                                                              uint16_t *ip_next) {
    __shared__ uint32_t part[kSqcWaves][64];
    __shared__ uint32_t cbase[64];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, ncol = n_conn + 1u;
    const uint32_t c = blockIdx.x * 64u + lane, ch = blockIdx.y, RW = RC / kSqcWaves;
    const bool ok = c < ncol;
    const uint32_t r0 = ch * RC + wv * RW;
    uint32_t sm = 0;
    if (ok) {
#pragma unroll 16
        for (uint32_t k = 0; k < RW; ++k)
            if (r0 + k < nwt) sm += tab[(uint64_t)(r0 + k) * ncol + c];
    }
    part[wv][lane] = sm;
    if (wv == 0) {
        uint32_t b = ok ? st0[c] : 0u;
        if (ok)
            for (uint32_t q = 0; q < ch; ++q) b += csum[(uint64_t)q * ncol + c];
        cbase[lane] = b;
    }
    __syncthreads();
    if (!ok) return;
    uint32_t run = cbase[lane];  // mod 2^32 (TcpInfo::seq) / mod 2^16 once stored (mIpId)
    for (uint32_t q = 0; q < wv; ++q) run += part[q][lane];
#pragma unroll 16
    for (uint32_t k = 0; k < RW; ++k) {
        if (r0 + k >= nwt) break;
        uint32_t *e = tab + (uint64_t)(r0 + k) * ncol + c;
        const uint32_t v = *e;
        *e = run;
        run += v;
    }
    if (ch == nch - 1u && wv == kSqcWaves - 1u) {
        if (c < n_conn) conn_seq[c] = run;
        else *ip_next = (uint16_t)run;
    }
}

__global__ __launch_bounds__(kBlock) void k_sqt_apply(const uint32_t *conn, const int32_t *status, uint32_t n,
                                                      uint32_t n_conn, uint32_t W, uint32_t nwt, const uint32_t *tab,
                                                      uint32_t *seq, uint16_t *ip_id) {
    extern __shared__ uint32_t sq_lds[];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, ncol = n_conn + 1u;
    const uint32_t wt = blockIdx.x * kWaves + wv;
    uint32_t *t = sq_lds + wv * ncol;
    uint32_t ip = 0;
    if (wt < nwt) {
        const uint32_t *row = tab + (uint64_t)wt * ncol;
        for (uint32_t c = lane; c < n_conn; c += 64u) t[c] = row[c];
        ip = row[n_conn];
    }
    __syncthreads();
    if (wt >= nwt) return;
    const uint64_t lt = lanemask_lt(lane);
    const uint64_t base = (uint64_t)wt * W, end = base + W < n ? base + W : n;
    for (uint64_t r = base; r < end; r += 256u) {
        int32_t st[4];
        uint32_t cn[4];
        sqt_load4(conn, status, r, end, lane, st, cn);
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const uint64_t i = r + 64u * k + lane;
            const bool fr = st[k] > 0;
            const uint32_t key = fr && cn[k] < n_conn ? cn[k] : kNone;
            const uint32_t len = fr ? (uint32_t)st[k] : 0u;
            const uint64_t m = __ballot(fr);
            const uint32_t my_ip = ip + (uint32_t)__popcll(m & lt);
            ip += (uint32_t)__popcll(m);
            // FakeTcp::Output order inside the round: earlier lanes of the same connection go first.
            // Lane d's peers are one compare into an SGPR mask: the peers above d add lane d's len (the
            // mask drives the select directly, no per-lane index compare) and the peers below d have a
            // later lane of their connection (scalar OR).  6 VALU per d; a scalar loop over the
            // distinct connections of the round instead was slower (branches), DESIGN.md §4.8
            uint32_t ex = 0;
            uint64_t laterm = 0;  // lanes with a later lane of their connection (scalar)
#pragma unroll
            for (int d = 0; d < 64; ++d) {
                const uint32_t sk = (uint32_t)__builtin_amdgcn_readlane((int)key, d);
                const uint32_t sl = (uint32_t)__builtin_amdgcn_readlane((int)len, d);
                const uint64_t eq = __ballot(key == sk);
                const uint64_t above = d == 63 ? 0ull : eq & (~0ull << (d + 1));
                uint32_t ex1 = ex + sl;                  // v_add with the SGPR operand, then a select on
                asm volatile("" : "+v"(ex1));            // the mask (not folded back into add(select))
                ex = __builtin_amdgcn_inverse_ballot_w64(above) ? ex1 : ex;
                laterm |= eq & ((1ull << d) - 1ull);
                asm volatile("" : "+v"(ex), "+s"(laterm));  // no sinking: consume each mask in its own step
            }
            const bool later = __builtin_amdgcn_inverse_ballot_w64(laterm);
            uint32_t sv = 0;
            if (key != kNone) {
                const uint32_t pre = t[key];
                sv = pre + ex;
                if (!later) t[key] = sv + len;  // one lane per connection carries the row
            }
            __builtin_amdgcn_wave_barrier();
            if (i < end) {
                seq[i] = sv;
                ip_id[i] = fr ? (uint16_t)my_ip : (uint16_t)0;
            }
        }
    }
}

uint32_t sqt_wave_tile(uint32_t n_conn) {
    uint32_t w = 512;
    while (w < n_conn + 1u) w <<= 1;
    return w;
}

struct SqWs {
    int8_t *part;
    uint8_t *cmd0;
    uint32_t *framed, *rank, *perm, *seg_off, *seg_first, *v, *pre, *base, *nseg, *nvalid, *nfr;
    ScanWs scan;
};

size_t sq_layout(uint32_t n, uint32_t n_conn, uint8_t *b, SqWs *w) {
    size_t off = 0;
    auto take = [&](size_t bytes) -> uint8_t * {
        uint8_t *p = b ? b + off : nullptr;
        off += (bytes + 255) & ~size_t(255);
        return p;
    };
    SqWs d;
    const size_t nc = (n + 1 + kScanChunk - 1) / kScanChunk + 1;
    d.part = (int8_t *)take(n);
    d.cmd0 = take(n);
    d.framed = (uint32_t *)take(4ull * n);
    d.rank = (uint32_t *)take(4ull * n);
    d.perm = (uint32_t *)take(4ull * n);
    d.seg_off = (uint32_t *)take(4ull * (n + 1));
    d.seg_first = (uint32_t *)take(4ull * n);
    d.v = (uint32_t *)take(4ull * (n + 1));
    d.pre = (uint32_t *)take(4ull * (n + 1));
    d.base = (uint32_t *)take(4ull * n_conn);
    d.nseg = (uint32_t *)take(4);
    d.nvalid = (uint32_t *)take(4);
    d.nfr = (uint32_t *)take(4);
    d.scan.sums = (uint32_t *)take(4ull * nc);
    d.scan.sum_off = (uint32_t *)take(4ull * nc);
    if (w) *w = d;
    return off;
}

}  // namespace

extern "C" int rsk_tcp_send_seq_batch(rsk_ctx *c, uint32_t n, const uint32_t *conn, const int32_t *status,
                                      uint32_t n_conn, uint32_t *conn_seq, uint16_t *ip_id_next, uint32_t *seq,
                                      uint16_t *ip_id, void *stream) {
    if (!c) return RSK_EINVAL;
    if (n == 0) return RSK_OK;
    if (n > RSK_MAX_BATCH) return RSK_EINVAL;  // grids of one lane per packet
    if (!conn || !status || !ip_id_next || !seq || !ip_id || (n_conn && !conn_seq)) return RSK_EINVAL;
    if (n > (1u << 30)) return RSK_EINVAL;
    rsk::DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    hipStream_t s = (hipStream_t)stream;
    const bool table = n_conn + 1ull <= kSqCols && !c->sq_force_groupby;
    const uint32_t W = sqt_wave_tile(n_conn), nwt = (uint32_t)((n + (uint64_t)W - 1) / W);
    const size_t need = table ? 4ull * (nwt + 64ull + 1ull) * (n_conn + 1ull) : sq_layout(n, n_conn, nullptr, nullptr);
    void *sq_ws = nullptr;
    int r = rsk::stream_ws(c, s, rsk::WS_SEQ, need, &sq_ws);
    if (r) return r;
    if (table) {
        uint32_t *tab = static_cast<uint32_t *>(sq_ws);
        const unsigned nbt = (nwt + kWaves - 1) / kWaves;
        const size_t lds = 4ull * kWaves * (n_conn + 1ull);
        hipLaunchKernelGGL(k_sqt_sum, dim3(nbt), dim3(kBlock), lds, s, conn, status, n, n_conn, W, nwt, tab);
        if (c->sq_scan_variant == 1) {
            const uint32_t cb = n_conn + 1u <= 128u ? 1u : n_conn + 1u <= 512u ? 16u : 64u;  // more row groups when narrow
            hipLaunchKernelGGL(k_sqt_scan, dim3((n_conn + cb) / cb), dim3(kSqScanThreads), 0, s, tab, nwt, n_conn, cb,
                               conn_seq, ip_id_next);
        } else {
            uint32_t RC = 256;
            while ((nwt + RC - 1) / RC > 64u) RC <<= 1;
            const uint32_t nch = (nwt + RC - 1) / RC;
            uint32_t *csum = tab + (size_t)nwt * (n_conn + 1u), *st0 = csum + (size_t)nch * (n_conn + 1u);
            const dim3 g((n_conn + 64u) / 64u, nch);
            hipLaunchKernelGGL(k_sqt_csum, g, dim3(kSqcWaves * 64), 0, s, tab, nwt, n_conn, RC, csum, st0, conn_seq,
                               ip_id_next);
            hipLaunchKernelGGL(k_sqt_cscan, g, dim3(kSqcWaves * 64), 0, s, tab, nwt, n_conn, RC, nch, csum, st0,
                               conn_seq, ip_id_next);
        }
        hipLaunchKernelGGL(k_sqt_apply, dim3(nbt), dim3(kBlock), lds, s, conn, status, n, n_conn, W, nwt, tab, seq,
                           ip_id);
        return rsk::launch_check("k_sqt_apply");
    }
    SqWs w;
    sq_layout(n, n_conn, static_cast<uint8_t *>(sq_ws), &w);
    const unsigned nb = (n + kBlock - 1) / kBlock, nb1 = (n + 1 + kBlock - 1) / kBlock;
    hipError_t e = hipMemsetAsync(seq, 0, 4ull * n, s);
    if (e != hipSuccess) { rsk::set_error("hipMemsetAsync(seq)", e); return RSK_EDEVICE; }
    hipLaunchKernelGGL(k_sq_flags, dim3(nb), dim3(kBlock), 0, s, conn, status, n, n_conn, w.part, w.cmd0, w.framed);
    if ((r = rsk::launch_check("k_sq_flags"))) return r;
    // IP ids: RawTcp::Output's mIpId++ over the framed packets in batch order (conn/RawTcp.cpp:119)
    if ((r = scan_u32(w.framed, w.rank, n, w.nfr, w.scan, s))) return r;
    hipLaunchKernelGGL(k_sq_ipid, dim3(nb), dim3(kBlock), 0, s, w.framed, w.rank, n, ip_id_next, ip_id);
    hipLaunchKernelGGL(k_sq_ipid_advance, dim3(1), dim3(1), 0, s, ip_id_next, w.nfr);
    if ((r = rsk::launch_check("k_sq_ipid"))) return r;
    // seq: FakeTcp::Output's UpdateSeq(seq + 31 + nread) per connection, in batch order (FakeTcp.cpp:43-49):
    // group the framed packets by connection (stable), one scan of their frame lengths in that order
    rsk_demux_in din{};
    din.status = w.part;
    din.cmd = w.cmd0;
    din.conv = conn;
    rsk_demux_out dout{w.perm, w.seg_off, w.seg_first, w.nseg, w.nvalid};
    if ((r = rsk_demux_batch(c, n, &din, RSK_DEMUX_CONV, &dout, stream))) return r;
    hipLaunchKernelGGL(k_sq_lens, dim3(nb1), dim3(kBlock), 0, s, w.perm, w.nvalid, status, n, w.v);
    if ((r = rsk::launch_check("k_sq_lens"))) return r;
    if ((r = scan_u32(w.v, w.pre, n + 1, nullptr, w.scan, s))) return r;
    hipLaunchKernelGGL(k_sq_conn, dim3(nb), dim3(kBlock), 0, s, w.nseg, w.seg_off, w.seg_first, conn, w.pre, conn_seq,
                       w.base);
    hipLaunchKernelGGL(k_sq_seq, dim3(nb), dim3(kBlock), 0, s, w.perm, w.nvalid, conn, w.base, w.pre, seq);
    return rsk::launch_check("k_sq_seq");
}

// internal A/B + test knob (not in the public header): 1 sends every n_conn through the group-by path,
// 2 keeps the table path with the one-kernel column scan (k_sqt_scan, A/B)
extern "C" int rsk__set_send_seq_groupby(rsk_ctx *c, int v) {
    if (!c || v < 0 || v > 2) return RSK_EINVAL;
    c->sq_force_groupby = v == 1;
    c->sq_scan_variant = v == 2 ? 1 : 0;
    return RSK_OK;
}

extern "C" int rsk_tcp_recv_ack_batch(rsk_ctx *c, uint32_t n, const uint32_t *conn, const uint8_t *delivered,
                                      const uint32_t *seq, uint32_t n_conn, uint32_t *conn_ack, void *stream) {
    if (!c) return RSK_EINVAL;
    if (n == 0) return RSK_OK;
    if (n > RSK_MAX_BATCH) return RSK_EINVAL;  // grids of one lane per packet
    if (!conn || !delivered || !seq || (n_conn && !conn_ack)) return RSK_EINVAL;
    if (n > (1u << 30)) return RSK_EINVAL;  // as rsk_tcp_send_seq_batch: 32-bit grid arithmetic stays exact
    rsk::DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    if (n_conn <= kAckLds)
        hipLaunchKernelGGL(k_ack_lds, dim3((n + kAckTile - 1) / kAckTile), dim3(kBlock), 0, (hipStream_t)stream, conn,
                           delivered, seq, n, n_conn, conn_ack);
    else
        hipLaunchKernelGGL(k_ack, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, (hipStream_t)stream, conn,
                           delivered, seq, n, n_conn, conn_ack);
    return rsk::launch_check("k_ack");
}
