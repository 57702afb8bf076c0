// rsk_kernels.hip — MI355X (gfx950) HIP implementation of the rsock framing codec + its C ABI.
//
// Kernels (DESIGN.md §4 has the roofline and the algorithmic bytes of each):
//   k_encode        RConn::Output framing (conn/RConn.cpp:87-105): per 64-packet set (8 groups of 8
//                   consecutive packets, interleaved across 1024 waves), one lane per packet computes
//                   status and the 31 header bytes (the tag: one MD5 compression per lane, or in
//                   RSK_TAG_TABLE mode the key's 256-entry table staged in LDS); then, per wave,
//                   the software-pipelined per-packet copy (4-packet batches of 16-B chunks, one
//                   aligned payload load per chunk, funnel partner from the next lane by DPP) or
//                   the flat chunk list for short frames; for batches of long frames the two-pass
//                   form k_encode_heads + k_encode_copy (K = 1, 2 or 4 packets per copy wave).
//   k_encode_wire   RConn::Output + RawTcp::SendRawTcp (conn/RawTcp.cpp:280-341): frames plus the
//                   IPv4/TCP headers and checksums libnet writes, two-launch hybrid.
//   k_encode_hdr /  header-only framing / verification on 32-B slots (host-resident deployments:
//   k_decode_hdr    the payload never crosses PCIe).
//   k_decode        RConn::OnRecv (conn/RConn.cpp:64-85): one lane per frame, 32-B header window,
//                   tag verify (MD5 per lane / LDS table), SoA field stores, per-wave VALID ballot for k_compact.
//   k_parse_decode  RawTcp::RawInput (conn/RawTcp.cpp:138-244) fused with k_decode's body.
//   k_capture_filter the pcap predicate of BuildFilterStr (cap/cap_util.cpp:67-144), SURVEY §8f-4.
//   k_compact       order-stable VALID index list from the decode launches' per-wave ballots, one
//                   pass (decoupled look-back over 4096-packet tiles).
//   k_tcpinfo_encode 21-B TcpInfo hand-off records (bean/TcpInfo.cpp:20-32), staged through LDS.
//   k_shim          the single-call shims (reference signatures) on a batch of one.
//   k_tag_table     the key's 256 tags (MD5(key || b)[8..15], b = 0..255), once per context.
//   k_fill_splitmix synthetic workload generator (bench/tests only).
// The receive demux is in rsk_demux.hip; host batch helpers in rsk_host.cpp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cassert>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rsk_codec.h"
#include "rsk_ctx.h"
#include "rsk_device.h"
#include "rsk_md5.h"

using rsk::KeySched;

namespace {

constexpr int kBlock = 256;  // 4 waves of 64
constexpr int kWavesPerBlock = kBlock / 64;

using rsk::DeviceGuard;
using rsk::g_last_error;
using rsk::launch_check;
using rsk::set_error;

// ---------------------------------------------------------------------------------------------
// Encode
// ---------------------------------------------------------------------------------------------
struct EncArgs {
    const uint8_t *payload;
    const uint64_t *pay_off;
    const uint16_t *pay_len;
    const uint8_t *cmd;
    const uint32_t *conv;
    const uint64_t *conn_key;
    const uint8_t *id;  // n*8, 8-byte aligned, or null
    uint8_t *frame;
    const uint64_t *frame_off;
    int32_t *status;
    uint32_t id_lo, id_hi;
    uint32_t n;
    uint32_t pad;  // log2 of the zero-pad granularity (4: RSK_ENC_ZERO_PAD16, 7: RSK_ENC_ZERO_PAD128), 0 = none
};

__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t j) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)j);
}
__device__ __forceinline__ uint64_t rdl64(uint64_t v, uint32_t j) {
    return (uint64_t)rdl((uint32_t)v, j) | ((uint64_t)rdl((uint32_t)(v >> 32), j) << 32);
}

// ---- the tag (util/rhash.cpp:20-41): MD5(key || payload[0])[8..15].  Two modes, chosen per context
// at run time (rsk_set_tag_mode, uniform per launch through KeySched::tag_mode):
//   RSK_TAG_MD5 (default)  every lane runs the MD5 compression of rsk_md5.h for its packet, as the
//                          reference does per packet (rhash.cpp:20-41): the key's message words are
//                          kernel arguments (SGPRs), only the word holding payload[0] is per lane, the
//                          round constants are instruction immediates;
//   RSK_TAG_TABLE          the tag depends on one payload byte, so a key has 256 tags: k_tag_table
//                          computes them once per context and every kernel that frames or verifies
//                          stages the 2-KB table in LDS (one entry per thread of the 256-thread block,
//                          before any early exit) and looks the tag up with one ds_read_b64.
// Round 3 measured the MD5 round constants staged in LDS per block (the north star's "MD5 round
// constants ... staged in LDS") against instruction immediates and kept immediates
// (profiles/r03_ab_md5_lds.json; that build is in the git history).
__shared__ uint2 s_tags[256];

__device__ __forceinline__ void stage_tags(const KeySched &ks) {
    static_assert(kBlock == 256, "one tag-table entry per thread");
    if (ks.tag_mode == RSK_TAG_TABLE) {  // uniform: the whole block takes the barrier or none does
        s_tags[threadIdx.x] = ks.tab[threadIdx.x];
        __syncthreads();
    }
}

// LANE: the payload-word-specialised schedule (rsk_md5.h md5_tag_lane: 4 VALU per step instead of 5,
// 16 instantiations behind one scalar branch).  Who uses it: the decode kernels (registers to spare,
// ~1 %) and the two-pass header pass.  The framing kernels keep the generic schedule: in k_encode's
// per-packet sets the specialised one raised the register budget past 128 VGPRs (3 waves per SIMD
// instead of 4) and cost C2 / C4 13-16 % (profiles/r04_ab_md5_isa.json); for its flat sets (MODE 12)
// round 4 measured a gain on a build that specialised key word 2 only -- on the full build MODE 11
// (generic) is as fast or 1 % faster (C2 0.0498-0.0501 vs 0.0499-0.0503 ms; 128 / 200-B batches -1 %,
// profiles/r05_md5_mode11_vs_12.json), so the shipped per-set kernel is k_encode<11>.
template <bool LANE = false>
__device__ __forceinline__ void tag_of(const KeySched &ks, uint32_t b, uint32_t &t0, uint32_t &t1) {
    if (ks.tag_mode == RSK_TAG_TABLE) {
        const uint2 t = s_tags[b & 255u];
        t0 = t.x;
        t1 = t.y;
        return;
    }
    if constexpr (LANE) rsk::md5_tag_lane(ks, b & 255u, t0, t1);
    else rsk::md5_tag(ks, b & 255u, t0, t1);
}

// Frame bytes 8..31 as words H[2..7] (bean/EncHead.cpp:9-24 field order; byte 30 reserved = 0,
// byte 31 = payload[0], which belongs to the payload but shares the word).
__device__ __forceinline__ void head_words(uint32_t cmd, uint32_t id0, uint32_t id1, uint32_t conv,
                                           uint64_t key, uint32_t b0, uint32_t (&H)[8]) {
    H[2] = (uint32_t)RSK_ENC_HEAD_SIZE | (cmd << 8) | (id0 << 16);
    H[3] = (id0 >> 16) | (id1 << 16);
    H[4] = (id1 >> 16) | (conv << 16);
    H[5] = (conv >> 16) | ((uint32_t)key << 16);
    H[6] = (uint32_t)(key >> 16);
    H[7] = (uint32_t)(key >> 48) | (b0 << 24);
}

// ---- phase 1: one lane per packet ---------------------------------------------------------------
// status (RConn.cpp:88-98), tag (rhash.cpp:20-41 via md5_tag), frame words 0..7 (tag + EncHead +
// payload[0]); `slow` marks a framed packet whose frame is not 16-B aligned (k_encode_wire: the
// shifted copies).
struct Lane1 {
    int32_t st;
    uint64_t po, fo;
    uint32_t H[8];
    bool slow;
};

// SADD: added to a framed packet's status (the two-pass wire build: the wire length, HL + 31 + P)
template <bool TAG = true, bool LANE = false, int SADD = 0>
__device__ __forceinline__ Lane1 encode_phase1(const EncArgs &a, const KeySched &ks, uint64_t i) {
    Lane1 L;
    L.st = 0;
    L.po = 0;
    L.fo = 0;
    L.slow = false;
#pragma unroll
    for (int q = 0; q < 8; ++q) L.H[q] = 0;
    if (i < a.n) {
        L.po = a.pay_off[i];
        const uint32_t P = a.pay_len[i];
        L.fo = a.frame_off[i];
        L.st = P == 0 ? RSK_SEND_RESET
                      : (P > RSK_MAX_PAYLOAD ? RSK_SEND_OVERSIZE : (int32_t)(RSK_HEAD_SIZE + P));
        if (L.st > 0) {
            const uint32_t b0 = TAG ? a.payload[L.po] : 0u;
            if (TAG) tag_of<LANE>(ks, b0, L.H[0], L.H[1]);
            uint32_t id0 = a.id_lo, id1 = a.id_hi;
            if (a.id) {
                const uint2 v = *reinterpret_cast<const uint2 *>(a.id + 8 * i);
                id0 = v.x;
                id1 = v.y;
            }
            head_words(a.cmd[i], id0, id1, a.conv[i], a.conn_key[i], b0, L.H);
            L.slow = (reinterpret_cast<uintptr_t>(a.frame + L.fo) & 15u) != 0;
        }
        a.status[i] = L.st > 0 ? L.st + SADD : L.st;
    }
    return L;
}

// The tag half of phase 1 for a set that skipped it (encode_phase1<false>): payload[0], MD5, and
// payload[0] into frame byte 31 (H[7]).
__device__ __forceinline__ void encode_tag(const EncArgs &a, const KeySched &ks, Lane1 &L) {
    if (L.st > 0) {
        const uint32_t b0 = a.payload[L.po];
        tag_of(ks, b0, L.H[0], L.H[1]);
        L.H[7] |= b0 << 24;
    }
}

// The batch statistic behind the next calls' choice of encode path (rsk_encode_batch, enc_path): one
// wave reads pay_len at 64 evenly spaced packets and stores their mean payload length (bit 31 set:
// valid) to a host-mapped word of the context.  k_encode_heads does it in its block 0; calls on the
// other paths launch k_enc_sample behind the encode (the per-set kernel itself carries no extra
// argument: one more pointer in its arguments cost C4 12 % through SGPR spills, gpurun_out/r04o).
constexpr uint32_t kStatValid = 0x80000000u;
constexpr uint32_t kStatPacked = 0x40000000u;  // the sampled frames lie back to back (output-stationary copy)
constexpr uint32_t kStatMean = 0xffffu;        // the sampled mean payload
// AUTO's choice (rsk_encode_batch, enc_path / copy_k): batches of at least kTwoPassMinPackets by the mean
// payload of the context's last sampled batch (below that, and in a capture before any sample, the
// per-set kernel).
// Measured on uniform and mixed lengths, 2M packets per case, one process per box
// (tools/path_threshold.py, profiles/r05_path_threshold.json): the per-set kernel is fastest up to a
// mean of ~200 B, except C2's 64 B where the short-frame kernel is (profiles/r05_enc_paths.json); the
// short-frame kernel (every set on the flat chunk list) at 250-350 B, where the per-set kernel's sets
// cross its 256-B flat limit; the two-pass form with 4 packets per copy wave from 450 B (and C4's
// mixed 64-1400 B), 2 packets around 900-1100 B and mixed 700-1400 B, 1 packet from 1200 B (C3).
constexpr uint32_t kTwoPassMinPackets = 16384;
constexpr uint32_t kAutoShortMax = 96;     // mean payload <= this: the short-frame kernel (C2)
constexpr uint32_t kAutoPerSetBelow = 224;  // .. below this: the per-set kernel
constexpr uint32_t kAutoShortBelow = 400;   // .. below this: the short-frame kernel again
constexpr uint32_t kAutoK4Below = 880;      // .. below this: two-pass, 4 packets per copy wave (C4)
constexpr uint32_t kAutoK2Below = 1160;     // .. below this: two-pass, 2 packets per copy wave; above: 1 (C3)
constexpr uint64_t kCopyMaxPackets = 1ull << 25;  // per k_encode_copy launch (2^31 work-items)
// the output-stationary copy's block map: 2 blocks per packet (frames of <= 1531 B + pad, back to back:
// <= 2 KB each)
__host__ __device__ constexpr uint64_t os_bcap(uint64_t n) { return 2ull * n + 2ull; }
// the two-pass encode's workspace: 32-B records, the block map and its two control words
__host__ __device__ constexpr uint64_t enc_ws_bytes(uint64_t n) { return 32ull * n + 4ull * os_bcap(n) + 16ull; }
// With frame_off (round 6) it also checks whether each sampled packet's frame ends where the next
// packet's begins, inside a 16-B chunk (byte-packed frames without a pad share their boundary
// chunks): three in four -> kStatPacked, which lets AUTO take the output-stationary copy
// (k_encode_os).  Frames packed at a 16-B pitch share nothing, and the packet copies are faster
// there (C4 16-B packed: 0.36 vs 0.435 ms).  A hint only: every copy writes the same bytes.
__device__ __forceinline__ void enc_sample(const uint16_t *pay_len, uint32_t n, uint32_t *stat,
                                           const uint64_t *frame_off = nullptr, uint32_t pad = 0u) {
    if (stat == nullptr || blockIdx.x != 0u || threadIdx.x >= 64u) return;  // one wave of block 0
    const uint64_t i = ((uint64_t)threadIdx.x * n) >> 6;
    const uint32_t P = pay_len[i];
    uint32_t v = P;
    bool packed = false;
    if (frame_off && pad == 0u && i + 1u < n && P != 0u && P <= (uint32_t)RSK_MAX_PAYLOAD) {
        const uint64_t e = frame_off[i] + RSK_HEAD_SIZE + P;
        packed = frame_off[i + 1] == e && (e & 15u) != 0u;  // the next frame starts inside e's 16-B chunk
    }
    const uint32_t np = (uint32_t)__popcll(__ballot(packed));
#pragma unroll
    for (int off = 32; off; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off);
    if (threadIdx.x == 0u)
        __hip_atomic_store(stat, kStatValid | (np >= 48u ? kStatPacked : 0u) | (v >> 6), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ __launch_bounds__(64) void k_enc_sample(const uint16_t *pay_len, uint32_t n, uint32_t *stat,
                                                   const uint64_t *frame_off, uint32_t pad) {
    enc_sample(pay_len, n, stat, frame_off, pad);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int NT>
__device__ __forceinline__ uint4 ld16(const uint8_t *p) {
    const RSK_GLOBAL u32x4 *g = reinterpret_cast<const RSK_GLOBAL u32x4 *>(rsk::gptr(p));
    u32x4 v;
    if constexpr (NT & 1) v = __builtin_nontemporal_load(g);
    else v = *g;
    return make_uint4(v.x, v.y, v.z, v.w);
}
template <int NT>
__device__ __forceinline__ void st16(uint8_t *p, const uint4 &v) {
    RSK_GLOBAL u32x4 *g = reinterpret_cast<RSK_GLOBAL u32x4 *>(rsk::gptr(p));
    const u32x4 w = {v.x, v.y, v.z, v.w};
    if constexpr (NT & 2) __builtin_nontemporal_store(w, g);
    else *g = w;
}
// Store chunk data v whose first `lim` bytes belong to the frame: whole chunk when lim >= 16;
// with padding, the tail (or the whole chunk, lim <= 0) is zeroed; without, only [0, lim).
template <int NT>
__device__ __forceinline__ void store_last16(uint8_t *d, const uint4 &v, int lim, bool pad) {
    if (lim >= 16) st16<NT>(d, v);
    else if (pad) st16<NT>(d, lim > 0 ? rsk::keep_bytes16(v, lim) : make_uint4(0u, 0u, 0u, 0u));
    else rsk::store_partial16(d, v, lim);
}

// Bytes written for a frame of flen bytes at d: flen, or up to the next 2^pad boundary.
__device__ __forceinline__ uint32_t padded_len(const uint8_t *d, uint32_t flen, uint32_t pad) {
    if (!pad) return flen;
    const uint32_t m = (1u << pad) - 1u;
    return flen + ((m + 1u - ((uint32_t)(reinterpret_cast<uintptr_t>(d) + flen) & m)) & m);
}

struct alignas(16) CopyRec {
    const uint8_t *src_al;  // 16-B aligned source of chunk 2 (payload + 1 - sh; wire: its own base)
    uint8_t *dst;           // 16-B aligned destination of chunk 0
    uint32_t cstart;        // first flat chunk index of this packet within the set
    uint32_t sh;            // funnel shift (bits 0-3) | frame offset r << 4 (encode)
    int32_t last_rel;       // last payload byte, relative to src_al
    uint32_t flen;          // frame length (31 + P)
};

// 16 bytes at byte offset sh (0..15, per lane) of A||B, branch-free
__device__ __forceinline__ uint4 funnel16_lane(const uint4 &A, const uint4 &B, uint32_t sh) {
    const uint32_t q = sh >> 2, r = sh & 3u;
    const uint32_t W[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
    uint32_t E[5];
#pragma unroll
    for (int d = 0; d < 5; ++d) {
        const uint32_t w0 = W[d], w1 = d + 1 < 8 ? W[d + 1] : 0u, w2 = d + 2 < 8 ? W[d + 2] : 0u,
                       w3 = d + 3 < 8 ? W[d + 3] : 0u;
        E[d] = q == 0 ? w0 : q == 1 ? w1 : q == 2 ? w2 : w3;
    }
    uint4 o;
    o.x = rsk::funnel(E[1], E[0], r);
    o.y = rsk::funnel(E[2], E[1], r);
    o.z = rsk::funnel(E[3], E[2], r);
    o.w = rsk::funnel(E[4], E[3], r);
    return o;
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- frame geometry: any destination alignment ---------------------------------------------------
// A frame whose first byte sits r = dst mod 16 bytes into a 16-B chunk is written as destination
// chunks k = 0 .. nst-1 at d0 = dst - r; chunk k holds frame-image bytes [16k - r, 16k - r + 16),
// the image being the 31 header bytes (tag | EncHead) followed by the payload (image byte 31 =
// payload[0]).  Chunks 0 and 1 and the first max(r, 1) - 1 bytes of chunk 2 are header bytes: the
// packet's own lane stores them from its 8 header words (store_head).  Everything from image byte
// 31 on is payload: chunk k >= 2 is the 16 bytes at offset sh of aligned source chunks k - 2 and
// k - 1 of srcp = src + 1 - r - sh (sh = (src + 1 - r) mod 16), one funnel shift per chunk, stored
// from byte max(r, 1) - 1 for k = 2 (r = 0 puts payload[0] in chunk 1, with the header words).
// Chunk 0 of an unaligned frame is stored from byte r on and the last chunk up to the frame's end
// (or, padded, to the 16-B boundary), so neighbouring frames packed at any byte offset are never
// touched.  r = 0 is the aligned case.
struct FrameGeo {
    uint8_t *d0;           // 16-B aligned destination of chunk 0
    const uint8_t *srcp;   // 16-B aligned source of chunk 2
    uint32_t r, sh;        // dst mod 16, funnel shift
    uint32_t nst;          // destination chunks stored
    int32_t first_rel;     // payload[0]   relative to srcp (-1 .. 29)
    int32_t last_rel;      // payload[P-1] relative to srcp
};

__device__ __forceinline__ FrameGeo frame_geo(const uint8_t *src, uint8_t *dst, uint32_t flen, uint32_t pad) {
    FrameGeo g;
    g.r = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15u);
    g.d0 = dst - g.r;
    g.sh = (uint32_t)((reinterpret_cast<uintptr_t>(src) + 1u - g.r) & 15u);
    g.srcp = src + 1 - (int)g.r - (int)g.sh;
    g.first_rel = (int32_t)(g.r + g.sh) - 1;
    g.last_rel = g.first_rel + (int32_t)flen - RSK_HEAD_SIZE - 1;
    g.nst = (g.r + padded_len(dst, flen, pad) + 15u) >> 4;
    return g;
}

// aligned source chunk m (relative to srcp) holds at least one payload byte
__device__ __forceinline__ bool src_chunk_live(int32_t m, int32_t first_rel, int32_t last_rel) {
    return 16 * m <= last_rel && 16 * m + 16 > first_rel;
}

// first byte of chunk 2 that is payload (the header's last bytes precede it when r >= 2)
__device__ __forceinline__ uint32_t chunk2_lo(uint32_t r) { return r >= 2u ? r - 1u : 0u; }

// Store the bytes [lo, ...) of payload chunk v at p (16-B aligned) that belong to the frame: lim =
// frame bytes from the chunk's start (>= 16: the whole chunk); with pad the tail is zero-filled to
// the chunk's end.
template <int NT>
__device__ __forceinline__ void store_piece(uint8_t *p, uint4 v, uint32_t lo, int lim, bool pad) {
    if (lim < 16 && pad) v = rsk::keep_bytes16(v, lim);
    const uint32_t hi = lim < 16 && !pad ? (uint32_t)lim : 16u;
    if (lo == 0u && hi == 16u) st16<NT>(p, v);
    else rsk::store_range16(p, v, lo, hi);
}

// The header bytes of the lane's own frame (image bytes [0, 31), plus payload[0] at 31 when r = 0):
// H = tag words, EncHead words and payload[0] in H[7]'s top byte.
__device__ __forceinline__ void store_head(const uint32_t (&H)[8], uint8_t *dst) {
    const uint32_t r = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15u);
    uint8_t *d0 = dst - r;
    const uint4 lo = make_uint4(H[0], H[1], H[2], H[3]), hi = make_uint4(H[4], H[5], H[6], H[7]);
    if (r == 0u) {
        st16<0>(d0, lo);
        st16<0>(d0 + 16, hi);
        return;
    }
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    rsk::store_range16(d0, funnel16_lane(z, lo, 16u - r), r, 16u);
    st16<0>(d0 + 16, funnel16_lane(lo, hi, 16u - r));
    if (r >= 2u) rsk::store_range16(d0 + 32, funnel16_lane(hi, z, 16u - r), 0u, r - 1u);
}

// ---- per-packet copy: the wave streams the payload chunks (k >= 2) of the frames of the packets
// in `vm`, PU packets per iteration.  A frame spans at most 95 destination chunks (1500 B + 15 B of
// offset), so chunk slots k = lane and k = lane + 64 cover it; all PU x 2 slots' loads are issued
// before any store.  Lane k loads only aligned source chunk k - 2 and takes the funnel partner
// (chunk k - 1) from lane k + 1 by a DPP wave shift (lane 63 of slot 0 from lane 0 of slot 1), so
// a packet holds 2 uint4 registers per lane.  The shifts run with every lane active (DPP reads
// disabled lanes as 0).  Lane p of an iteration stores the header chunks of the iteration's packet p
// (store_head, header words fetched from the packet's lane by one ds_bpermute each).
// tag (sets of long frames): phase 1 skipped payload[0] and the MD5, because that byte load
// fetches the payload's first line well before the copy reaches the packet and the line is gone
// from L2 by then; here lane p loads payload[0] of the iteration's packet p first, then the chunks,
// and runs the MD5 of the PU packets while the chunk loads are in flight.
__device__ __forceinline__ uint32_t wave_shl1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false);  // wave_shl:1
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src) {
    return (uint64_t)(uint32_t)__shfl((int)(uint32_t)v, (int)src) |
           ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)src) << 32);
}

// Header-bearing destination chunk k < kh (kh = 2, or 3 when r >= 2) of a frame at offset r, for the
// slot lanes 0..2 (TAG form): header image bytes [16k - r, 16k - r + 16) from the packet's header
// words Hj (uniform, SGPRs), for k = 2 only its first r bytes, the rest from the payload funnel V.
__device__ __forceinline__ uint4 head_chunk(const uint32_t (&H)[8], uint32_t k, uint32_t r, const uint4 &V) {
    const uint4 lo = make_uint4(H[0], H[1], H[2], H[3]), hi = make_uint4(H[4], H[5], H[6], H[7]);
    if (r == 0u) return k == 0u ? lo : hi;
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    const uint4 X = k == 0u ? z : k == 1u ? lo : hi, Y = k == 0u ? lo : k == 1u ? hi : z;
    const uint4 hs = rsk::funnel16(X, Y, 16u - r);  // r uniform: one scalar branch
    if (k < 2u) return hs;
    const uint4 m = rsk::keep_bytes16(make_uint4(~0u, ~0u, ~0u, ~0u), (int)r);  // first r bytes
    return make_uint4((hs.x & m.x) | (V.x & ~m.x), (hs.y & m.y) | (V.y & ~m.y), (hs.z & m.z) | (V.z & ~m.z),
                      (hs.w & m.w) | (V.w & ~m.w));
}

// ---- software-pipelined per-packet copy: the chunk loads of the next PU packets are issued before
// the current PU packets are shifted and stored, so each wave keeps a batch of loads in flight
// while it stores (an unpipelined copy waits for its own loads, then stores, then loads again; the
// round-1 form, measured in profiles/r01_ab_store_policy.json and r02_ab_encode_v2.json).  Two register
// buffers of PU packets, the roles swapped by a 2x unrolled loop.  Every load instruction runs with
// all lanes (a dead lane reads the arena's first chunk, which stays cached) so the batch's load
// count is static and the wait for the older batch leaves the newer one in flight.
template <int PU>
__device__ __forceinline__ uint64_t take_batch(uint64_t &vm) {
    uint64_t m = 0;
#pragma unroll
    for (int p = 0; p < PU; ++p) {
        const uint64_t b = vm & (~vm + 1ull);
        m |= b;
        vm ^= b;
    }
    return m;
}

template <int PU>
__device__ __forceinline__ void batch_slots(uint64_t bm, uint32_t lane, uint32_t (&js)[PU], bool (&on)[PU],
                                            uint32_t &myj, bool &mine) {
    myj = 0;
    mine = false;
#pragma unroll
    for (int p = 0; p < PU; ++p) {
        on[p] = bm != 0ull;
        js[p] = on[p] ? (uint32_t)__builtin_ctzll(bm) : 0u;
        if (on[p]) bm &= bm - 1ull;
        if (lane == (uint32_t)p) {
            myj = js[p];
            mine = on[p];
        }
    }
}

template <int PU, int NT, bool TAG, int TG = 0>
__device__ __forceinline__ void pkt_issue(const EncArgs &a, const Lane1 &L, uint32_t lane, uint64_t bm,
                                          uint4 (&A)[PU][2], uint32_t &b0) {
    uint32_t js[PU], myj;
    bool on[PU], mine;
    batch_slots<PU>(bm, lane, js, on, myj, mine);
    if constexpr (TAG && TG == 0) {  // payload[0] of the lane's slot packet, ahead of the chunk loads
        const uint64_t po = shfl64(L.po, myj);
        b0 = rsk::gptr(a.payload)[mine ? po : 0u];
    }
#pragma unroll
    for (int p = 0; p < PU; ++p) {
        const uint32_t flen = on[p] ? rdl((uint32_t)L.st, js[p]) : 0u;
        const uint8_t *src = a.payload + rdl64(L.po, js[p]);
        const FrameGeo g = frame_geo(src, a.frame + rdl64(L.fo, js[p]), flen, a.pad);
        // a dead lane reads the aligned chunk that holds the packet's payload[0] (mapped, cached)
        const uint8_t *dummy = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(src) & ~(uintptr_t)15);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int32_t m = (int32_t)(lane + 64u * q) - 2;
            const bool live = on[p] && m >= 0 && src_chunk_live(m, g.first_rel, g.last_rel);
            const uint4 v = ld16<NT>(live ? g.srcp + 16 * m : dummy);
            // zeroed here, which makes the compiler wait for the batch's loads at issue: round 4 moved
            // the zeroing after the wait (true two-batch overlap, vmcnt(6-7) instead of vmcnt(0)) and
            // measured C3 unchanged, C4 +2 % (profiles/r04_ab_pipeline.json): the memory system, not
            // the per-wave depth, sets the pace
            A[p][q] = live ? v : make_uint4(0u, 0u, 0u, 0u);
        }
    }
}

// A frame's last chunk, held back (wave-uniform, SGPRs) to be stored together with the next frame's
// first chunk: frames packed back to back at byte granularity share that 16-B chunk, and two partial
// stores from two lanes (up to 2 x 5 byte / short / dword stores) become one 16-B store.
struct TailCarry {
    uint4 t;       // the chunk: its first bytes are the previous frame's tail
    uintptr_t at;  // its 16-B aligned address
    bool on;
};

__device__ __forceinline__ uint4 rdl4(const uint4 &v, uint32_t j) {
    return make_uint4(rdl(v.x, j), rdl(v.y, j), rdl(v.z, j), rdl(v.w, j));
}

// bytes [0, r) of t, bytes [r, 16) of v
__device__ __forceinline__ uint4 merge16(const uint4 &t, const uint4 &v, uint32_t r) {
    const uint4 m = rsk::keep_bytes16(make_uint4(~0u, ~0u, ~0u, ~0u), (int)r);
    return make_uint4((t.x & m.x) | (v.x & ~m.x), (t.y & m.y) | (v.y & ~m.y), (t.z & m.z) | (v.z & ~m.z),
                      (t.w & m.w) | (v.w & ~m.w));
}

// nxt_bm: the packets of the batch stored after this one (its lowest set bit is the next frame in
// store order), for the TailCarry hand-over; tc carries a held-back tail chunk between calls.
template <int PU, int NT, bool TAG, int TG = 0, bool MRG = false>
__device__ __forceinline__ void pkt_store(const EncArgs &a, const KeySched &ks, const Lane1 &L, uint32_t lane,
                                          uint64_t bm, const uint4 (&A)[PU][2], uint32_t my_b0, uint64_t nxt_bm,
                                          TailCarry &tc) {
    uint32_t js[PU], myj;
    bool on[PU], mine;
    batch_slots<PU>(bm, lane, js, on, myj, mine);
    uint32_t t0 = 0, t1 = 0;
    if constexpr (TAG && TG == 0) {
        tag_of(ks, my_b0, t0, t1);
    } else if constexpr (TAG) {
        // the tag prepass (copy_pkt_pipe) left each packet's tag and payload[0] in its own lane's H
    } else {  // lane p: the header chunks of its slot packet (store_head)
        uint32_t H[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) H[t] = (uint32_t)__shfl((int)L.H[t], (int)myj);
        const uint64_t my_fo = shfl64(L.fo, myj);
        if (mine) store_head(H, a.frame + my_fo);
    }
#pragma unroll
    for (int p = 0; p < PU; ++p) {
        if (!on[p]) continue;
        const uint32_t fl = rdl((uint32_t)L.st, js[p]);
        const FrameGeo g = frame_geo(a.payload + rdl64(L.po, js[p]), a.frame + rdl64(L.fo, js[p]), fl, a.pad);
        const uint32_t flen = fl + g.r, nst = g.nst;
        const uint4 (&Ap)[2] = A[p];
        uint4 B[2];
        B[0] = make_uint4(wave_shl1(Ap[0].x), wave_shl1(Ap[0].y), wave_shl1(Ap[0].z), wave_shl1(Ap[0].w));
        B[1] = make_uint4(0u, 0u, 0u, 0u);
        if (nst >= 64u) {  // uniform: the frame reaches slot 1
            const uint4 l0 = make_uint4(rdl(Ap[1].x, 0), rdl(Ap[1].y, 0), rdl(Ap[1].z, 0), rdl(Ap[1].w, 0));
            if (lane == 63u) B[0] = l0;
            if (nst > 64u)
                B[1] = make_uint4(wave_shl1(Ap[1].x), wave_shl1(Ap[1].y), wave_shl1(Ap[1].z), wave_shl1(Ap[1].w));
        }
        uint32_t Hj[8];
        bool hmerge = false, tmerge = false;
        uint32_t kt = 0;
        if constexpr (TAG) {
#pragma unroll
            for (int t = 2; t < 8; ++t) Hj[t] = rdl(L.H[t], js[p]);
            if constexpr (TG == 0) {
                Hj[0] = rdl(t0, (uint32_t)p);
                Hj[1] = rdl(t1, (uint32_t)p);
                Hj[7] |= rdl(my_b0, (uint32_t)p) << 24;
            } else {
                Hj[0] = rdl(L.H[0], js[p]);
                Hj[1] = rdl(L.H[1], js[p]);
            }
            if constexpr (MRG) {
                // byte-packed neighbours (no padding): this frame's first chunk completes the held-back
                // tail of the previous frame; its own last chunk is held back when the next frame in
                // store order starts inside it.  All uniform.
                hmerge = tc.on && tc.at == reinterpret_cast<uintptr_t>(g.d0);
                tc.on = false;
                const uint64_t nb = p + 1 < PU && on[p + 1] ? 0ull : nxt_bm;
                const bool has_next = (p + 1 < PU && on[p + 1]) || nb != 0ull;
                const uint32_t jn =
                    p + 1 < PU && on[p + 1] ? js[p + 1] : (uint32_t)__builtin_ctzll(nb | (1ull << 63));
                const uintptr_t end = reinterpret_cast<uintptr_t>(a.frame + rdl64(L.fo, js[p])) + fl;
                tmerge = a.pad == 0u && has_next && (end & 15u) != 0u &&
                         reinterpret_cast<uintptr_t>(a.frame + rdl64(L.fo, jn)) == end;
                kt = nst - 1u;
            }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const uint32_t k = lane + 64u * q;
            if (q == 1 && nst <= 64u) continue;  // uniform
            if constexpr (TAG) {
                const uint4 V = rsk::funnel16(Ap[q], B[q], g.sh);
                uint4 v = k < (g.r >= 2u ? 3u : 2u) ? head_chunk(Hj, k, g.r, V) : V;
                uint32_t lo = k == 0u ? g.r : 0u;
                if constexpr (MRG) {
                    if (hmerge && k == 0u) {
                        v = merge16(tc.t, v, g.r);
                        lo = 0u;
                    }
                    if (tmerge && (kt >> 6) == (uint32_t)q) {  // uniform: hold the last chunk back
                        tc.t = rdl4(v, kt & 63u);
                        tc.at = reinterpret_cast<uintptr_t>(g.d0) + 16u * kt;
                        tc.on = true;
                    }
                }
                if (k >= nst || (MRG && tmerge && k == kt)) continue;
                store_piece<NT>(g.d0 + 16u * k, v, lo, (int)flen - 16 * (int)k, a.pad != 0u);
            } else {
                if (k >= nst || k < 2u) continue;
                const uint4 V = rsk::funnel16(Ap[q], B[q], g.sh);
                store_piece<NT>(g.d0 + 16u * k, V, k == 2u ? chunk2_lo(g.r) : 0u, (int)flen - 16 * (int)k,
                                a.pad != 0u);
            }
        }
    }
}

// Tag prepass (TAG form, TG > 0): before the batch that needs them, the lanes of the next TG packets
// (in copy order) load their payload[0] and run their MD5 together, one compression pass per TG
// packets instead of one per batch of PU packets (a pass costs the same VALU issue however few lanes
// are active); the byte loads fetch each payload's first line at most TG / PU batches before its
// chunk loads.  TG == 0: payload[0] loaded beside the batch's chunk loads, MD5 per batch (round 2).
template <int TG>
__device__ __forceinline__ void tag_prepass(const EncArgs &a, const KeySched &ks, Lane1 &L, uint32_t lane,
                                            uint64_t bm, uint64_t &untagged) {
    if constexpr (TG > 0) {
        if (!(bm & untagged)) return;  // uniform
        uint64_t m = 0;
#pragma unroll
        for (int k = 0; k < TG; ++k) {
            const uint64_t b = untagged & (~untagged + 1ull);
            m |= b;
            untagged ^= b;
        }
        if ((m >> lane) & 1ull) encode_tag(a, ks, L);
    }
}

// MRG: the TailCarry hand-over between byte-packed neighbours (sets with an unaligned frame end and
// no padding only: the carried chunk costs SGPRs the other sets spend on the pipelined copy).
template <int PU, int NT, bool TAG, int TG = 0, bool MRG = false>
__device__ __forceinline__ void copy_pkt_pipe(const EncArgs &a, const KeySched &ks, Lane1 &L, uint32_t lane,
                                              uint64_t vm) {
    uint4 A0[PU][2], A1[PU][2];
    uint32_t b0a = 0, b0b = 0;
    TailCarry tc;
    tc.t = make_uint4(0u, 0u, 0u, 0u);
    tc.at = 0;
    tc.on = false;
    uint64_t untagged = TAG ? vm : 0ull;
    uint64_t cur = take_batch<PU>(vm);
    if (!cur) return;
    pkt_issue<PU, NT, TAG, TG>(a, L, lane, cur, A0, b0a);
    while (true) {
        const uint64_t nxt = take_batch<PU>(vm);
        if (nxt) pkt_issue<PU, NT, TAG, TG>(a, L, lane, nxt, A1, b0b);
        if constexpr (TAG) tag_prepass<TG>(a, ks, L, lane, cur, untagged);
        pkt_store<PU, NT, TAG, TG, MRG>(a, ks, L, lane, cur, A0, b0a, nxt, tc);
        if (!nxt) break;
        cur = take_batch<PU>(vm);
        if (cur) pkt_issue<PU, NT, TAG, TG>(a, L, lane, cur, A0, b0a);
        if constexpr (TAG) tag_prepass<TG>(a, ks, L, lane, nxt, untagged);
        pkt_store<PU, NT, TAG, TG, MRG>(a, ks, L, lane, nxt, A1, b0b, cur, tc);
        if (!cur) break;
    }
}

// ---- flat copy: the payload chunks (k >= 2) of every packet in `vm` as one list of 16-B chunks;
// lane l of iteration t takes chunk g = 64(U t + u) + l and finds its packet by a 6-step binary
// search over the set's prefix sums in this wave's LDS slice.  Wave-local: no block barrier, so
// waves of one block may take different copy paths.
// TAGQ: phase 1 left the tag; `payload[0]` is loaded right after the first iteration's chunk loads
// (both depend only on the descriptors) and the packet's lane then stores its header chunks, so
// the set pays one dependent global round trip less than with the tag before the copy.
template <int U, bool TAGQ = false, bool LANE = false>
__device__ __forceinline__ void flat_head(const EncArgs &a, const KeySched &ks, const Lane1 &L, bool mine) {
    if constexpr (TAGQ) {
        if (mine) {
            const uint32_t b0 = rsk::gptr(a.payload)[L.po];
            uint32_t H[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) H[q] = L.H[q];
            tag_of<LANE>(ks, b0, H[0], H[1]);
            H[7] |= b0 << 24;
            store_head(H, a.frame + L.fo);
        }
    }
}

template <int U, bool TAGQ = false, bool LANE = false>
__device__ __forceinline__ void copy_flat(const EncArgs &a, const KeySched &ks, const Lane1 &L, uint32_t lane,
                                          bool mine, CopyRec *recs, uint32_t *cend) {
    uint32_t cc = 0;
    CopyRec r;
    r.src_al = nullptr; r.dst = nullptr; r.cstart = 0; r.sh = 0; r.last_rel = 0; r.flen = 0;
    if (mine) {
        const uint32_t flen = (uint32_t)L.st;
        const FrameGeo g = frame_geo(a.payload + L.po, a.frame + L.fo, flen, a.pad);
        cc = g.nst - 2u;
        r.src_al = g.srcp;
        r.dst = g.d0;
        r.sh = g.sh | (g.r << 4);
        r.last_rel = g.last_rel;
        r.flen = flen + g.r;  // frame bytes counted from d0
    }
    uint32_t inc = cc;  // wave-inclusive scan -> set chunk table
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(inc, off);
        if (lane >= (uint32_t)off) inc += v;
    }
    r.cstart = inc - cc;
    recs[lane] = r;
    cend[lane] = inc;
    const uint32_t C = (uint32_t)__shfl((int)inc, 63);
    wave_lds_sync();
    for (uint32_t g0 = 0; g0 < C; g0 += 64u * U) {
        uint4 A[U], B[U];
        uint8_t *dsts[U];
        uint32_t shs[U], los[U];
        int32_t lims[U];
        bool act[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t g = g0 + 64u * u + lane;
            act[u] = g < C;
            A[u] = make_uint4(0u, 0u, 0u, 0u);
            B[u] = make_uint4(0u, 0u, 0u, 0u);
            shs[u] = 0;
            los[u] = 0;
            lims[u] = 0;
            dsts[u] = nullptr;
            if (act[u]) {
                uint32_t lo = 0;
#pragma unroll
                for (uint32_t st = 32; st; st >>= 1)
                    if (cend[lo + st - 1] <= g) lo += st;
                const CopyRec rr = recs[lo];
                const uint32_t rf = rr.sh >> 4, sh = rr.sh & 15u;
                const int32_t m = (int32_t)(g - rr.cstart);  // source chunk of destination chunk m + 2
                const int32_t first_rel = (int32_t)(rf + sh) - 1;
                if (src_chunk_live(m, first_rel, rr.last_rel)) A[u] = ld16<0>(rr.src_al + 16 * m);
                if (src_chunk_live(m + 1, first_rel, rr.last_rel)) B[u] = ld16<0>(rr.src_al + 16 * m + 16);
                shs[u] = sh;
                los[u] = m == 0 ? chunk2_lo(rf) : 0u;
                dsts[u] = rr.dst + 32u + 16u * (uint32_t)m;
                lims[u] = (int32_t)rr.flen - 32 - 16 * m;
            }
        }
        if (TAGQ && g0 == 0u) flat_head<U, TAGQ, LANE>(a, ks, L, mine);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (act[u]) store_piece<0>(dsts[u], funnel16_lane(A[u], B[u], shs[u]), los[u], lims[u], a.pad != 0u);
    }
    if (TAGQ && C == 0u) flat_head<U, TAGQ, LANE>(a, ks, L, mine);
    wave_lds_sync();  // LDS slice reusable by the caller afterwards
}

// Copy-path choice for the hybrid kernel: the per-packet loop wastes lanes on short frames (a
// 95-B frame uses 6 of 64 lanes), the flat list costs a binary search + LDS table per chunk.
// Measured crossover: flat wins below a set-mean frame of ~256 B.
constexpr uint32_t kFlatBelowMeanBytes = 256;
// The tag moves into the copy loop for sets of long frames only; with short frames an iteration
// carries fewer bytes per MD5 (C4: +10 % with the tag deferred).
constexpr uint32_t kDeferTagMeanBytes = 1024;

// One 64-packet set per wave: phase 1, then the chosen copy path.  MODE 11 (the per-set kernel):
// per-wave choice of path -- the flat chunk list for sets of short frames (tag and header stores
// behind the first chunk loads), the software-pipelined per-packet copy otherwise, with the tag
// deferred into the copy loop for sets of long frames; MODE 19 (the short path): every set on the
// flat list, for batches of short frames only (the per-packet copy's registers out of the kernel).
// The store policy is chosen per set (below).
template <int MODE, int PU, int U, int GRP = 64, int TG = 0>
__device__ __forceinline__ void encode_set(const EncArgs &a, const KeySched &ks, uint64_t i, uint32_t lane,
                                           CopyRec *recs, uint32_t *cend) {
    static_assert(MODE == 11 || MODE == 19, "the per-set kernel and its flat-only build");
    Lane1 L = encode_phase1<false>(a, ks, i);
    const bool vec = L.st > 0;  // every framed packet takes a vector path, at any alignment
    const uint64_t vm = __ballot(vec);
    // set mean frame length over framed packets (wave reduction)
    uint32_t fl = vec ? (uint32_t)L.st : 0u;
#pragma unroll
    for (int off = 32; off; off >>= 1) fl += __shfl_xor(fl, off);
    const uint32_t cnt = (uint32_t)__popcll(vm);
    const bool flat = MODE == 19 ? true : fl < kFlatBelowMeanBytes * cnt;
    const bool defer = !flat && fl >= kDeferTagMeanBytes * cnt;
    if (!defer && !flat) encode_tag(a, ks, L);  // the flat list and the deferred copy take it themselves
    if (flat) {
        copy_flat<U, true, false>(a, ks, L, lane, vec, recs, cend);
        return;
    }
    if constexpr (MODE == 11) {
        // Store policy per set: frames packed back to back (each frame's padded end is the next
        // frame's start, so every line of the span is written in full) keep normal stores; any gap
        // leaves partially written lines, which nontemporal stores write without the memory-side
        // read-modify-write (C4's 1440-B slots: -13 %; C3's packed frames: +4 % if streamed).
        const uint32_t fend = vec ? padded_len(a.frame + L.fo, (uint32_t)L.st, a.pad) : 0u;
        const uint64_t end = L.fo + fend;
        const uint64_t nfo = (uint64_t)(uint32_t)__shfl_down((int)(uint32_t)L.fo, 1) |
                             ((uint64_t)(uint32_t)__shfl_down((int)(uint32_t)(L.fo >> 32), 1) << 32);
        const bool nvec = __shfl_down((int)vec, 1) != 0;
        // (lanes of the last packet of a group: the next lane's packet is not the next frame)
        const bool nt = __ballot(vec && nvec && lane % GRP != GRP - 1u && end != nfo) != 0ull;
        // Header chunks: sets with the tag in the copy loop (long frames) store them in the packet's
        // first slot store (lanes 0..2, words by readlane); the others by the slot lane (store_head).
        // Measured (profiles/r02_ab_head.json): C3 2.34 vs 2.55 ms with the first; C4 0.389 vs
        // 0.420 ms with the second.
        // Byte-packed long frames (no pad; a frame ends mid-chunk and the next packet's frame
        // starts there): the TAG-form copy with the boundary-chunk merge (TailCarry), which writes
        // each shared chunk as one 16-B store.  Only sets that really have such a pair take it: the
        // carry costs ~8 % where nothing merges (C3 frames at odd offsets 0.769 -> 0.704 ms, C3
        // slots without padding 0.682 -> 0.630 ms, gpurun_out/r03lay).  Short-frame sets keep
        // their copy: the TAG form with the tag from phase 1 (TG = -1) was slower on C4's
        // byte-packed frames (0.486 vs 0.466 ms).
        bool mrg = false;
        if (a.pad == 0u && defer) {
            const uint64_t fe = reinterpret_cast<uintptr_t>(a.frame + L.fo) + (uint32_t)L.st;
            mrg = __ballot(vec && nvec && lane % GRP != GRP - 1u && (fe & 15u) != 0u &&
                           reinterpret_cast<uintptr_t>(a.frame + nfo) == fe) != 0ull;
        }
        if (defer) {
            if (mrg) copy_pkt_pipe<PU, 0, true, TG, true>(a, ks, L, lane, vm);
            else if (nt) copy_pkt_pipe<PU, 2, true, TG>(a, ks, L, lane, vm);
            else copy_pkt_pipe<PU, 0, true, TG>(a, ks, L, lane, vm);
        } else {
            if (nt) copy_pkt_pipe<PU, 2, false>(a, ks, L, lane, vm);
            else copy_pkt_pipe<PU, 0, false>(a, ks, L, lane, vm);
        }
    }
}

// ---- the two-pass form for batches of long frames (round 4) ---------------------------------------
// Pass 1, k_encode_heads: phase 1 one lane per packet (status, the MD5 tag, EncHead, payload[0]; the
// same code as k_encode's phase 1) into a 32-B record per packet in the stream's workspace.  Pass 2,
// k_encode_copy: ONE WAVE PER PACKET -- descriptors and the record by scalar loads, the packet's chunk
// loads, the DPP funnel, the header chunks from the record, nontemporal loads and stores -- so waves are short-lived
// and independent.  That is the access shape of the fastest plain copy measured on this chip for C3's
// arenas (one wave per packet: 6.0 TB/s, against 5.2 TB/s for k_encode's 64-packet sets; DESIGN.md §4.1,
// profiles/r04_c3_ceiling.json), which k_encode cannot take: a one-packet wave would run a whole MD5
// compression for one packet (~300 VALU whatever its active lanes; 4.5 ms for C3).  Pass 1 runs the
// compressions 64 to a wave instead.  rsk_encode_batch takes this form for batches of long frames
// (enc_path); for short frames one packet per wave idles most lanes and the per-set kernel stays.
// base: the first packet of this launch (a chunked call runs heads / copy per chunk of packets)
// Records chunk-major (round 6): chunk 0 of packet i at heads[i], chunk 1 at heads[nr + i] (nr = the
// records' capacity in packets), so each store instruction of a wave writes 1 KB contiguous instead of
// 16-B pieces at a 32-B stride.
template <int SADD = 0>
__global__ __launch_bounds__(kBlock) void k_encode_heads(EncArgs a, KeySched ks, uint4 *heads, uint32_t *stat,
                                                         uint64_t base, uint64_t nr) {
    stage_tags(ks);
    enc_sample(a.pay_len, a.n, stat, a.frame_off, a.pad);
    const uint64_t i = base + (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const Lane1 L = encode_phase1<true, true, SADD>(a, ks, i < a.n ? i : a.n);
    if (i < a.n && L.st > 0) {
        heads[i] = make_uint4(L.H[0], L.H[1], L.H[2], L.H[3]);
        heads[nr + i] = make_uint4(L.H[4], L.H[5], L.H[6], L.H[7]);
    }
}

// ---- K packets per wave, one wave-instruction stream: the two-pass form's copy ------------------------
// Issue: lanes 0..K-1 load the K packets' pay_len / pay_off / frame_off together (ONE dependent round
// trip for all descriptors; pay_len has no scalar 16-bit load, and a vector load per packet made the
// compiler wait for every earlier packet's chunk loads before the next packet's descriptors -- K
// packets ran one after another), then every chunk load of the K packets with all lanes (no exec
// mask: dead lanes re-read a chunk a live lane of the instruction reads), so the stores of packet p
// wait for packet p's loads, not for the later packets'.  Dead lanes' data only ever reaches bytes no
// store writes (past the frame's end, masked by store_piece; before payload[0], header bytes).
template <int K>
struct CopyK {
    uint4 A[K][2];
    FrameGeo g[K];
    uint32_t flen[K];  // frame bytes counted from g.d0 (31 + P + r); 0: packet not framed
};

template <int K, int NT>
__device__ __forceinline__ void copyk_issue(const EncArgs &a, uint64_t i0, uint32_t lane, CopyK<K> &c) {
    uint32_t dP = 0;
    uint64_t dpo = 0, dfo = 0;
    if constexpr (K > 1) {
        const uint64_t il = i0 + lane;
        if (lane < (uint32_t)K && il < a.n) {
            dP = a.pay_len[il];
            dpo = a.pay_off[il];
            dfo = a.frame_off[il];
        }
    }
#pragma unroll
    for (int p = 0; p < K; ++p) {
        uint32_t P;
        const uint8_t *src;
        uint8_t *dst;
        if constexpr (K > 1) {
            P = rdl(dP, (uint32_t)p);
            src = a.payload + rdl64(dpo, (uint32_t)p);
            dst = a.frame + rdl64(dfo, (uint32_t)p);
        } else {
            // one packet: pay_len, then the offsets of a framed packet only (uniform addresses).  Loading
            // all three at once shortens each wave by a round trip yet made C3's copy 6 % SLOWER
            // (gpurun_out/r05k: 2.22 vs 2.08 ms) -- the copy is bound by the memory side, and waves
            // that start their payload loads together contend for it
            P = i0 < a.n ? a.pay_len[i0] : 0u;
            const bool ok = P != 0u && P <= (uint32_t)RSK_MAX_PAYLOAD;
            src = a.payload + (ok ? a.pay_off[i0] : 0u);
            dst = a.frame + (ok ? a.frame_off[i0] : 0u);
        }
        const bool on = P != 0u && P <= (uint32_t)RSK_MAX_PAYLOAD;  // uniform; status written elsewhere
        c.g[p] = frame_geo(src, dst, RSK_HEAD_SIZE + P, a.pad);
        c.flen[p] = on ? RSK_HEAD_SIZE + P + c.g[p].r : 0u;
        if (!on) c.g[p].nst = 0u;
        // source chunks holding payload bytes: m_lo .. m_hi (relative to srcp; none when P = 1 and
        // payload[0] sits in destination chunk 1: no load at all)
        const int32_t m_lo = c.g[p].first_rel >= 16 ? 1 : 0, m_hi = c.g[p].last_rel >> 4;
        // lane k loads aligned source chunk k - 2 of slot q (destination chunk k + 64 q); the funnel
        // partner (chunk k - 1) comes from lane k + 1 by a DPP shift, lane 63 of slot 0 from lane 0 of slot 1.
        // A lane outside m_lo .. m_hi loads the nearest chunk of that range, which a live lane of the same
        // instruction requests too: the instruction costs no extra memory request.  Instructions with no
        // live lane (packet not framed; slot 1 of a frame under 64 chunks) are skipped by a uniform branch.
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            c.A[p][q] = make_uint4(0u, 0u, 0u, 0u);
            if (!on || m_hi < m_lo || (q == 1 && c.g[p].nst < 64u)) continue;  // uniform
            const int32_t m = (int32_t)(lane + 64u * q) - 2;
            const int32_t mc = m < m_lo ? m_lo : m > m_hi ? m_hi : m;
            c.A[p][q] = ld16<NT>(c.g[p].srcp + 16 * mc);  // uniform base + lane offset
        }
    }
}

// Store packet p's chunks, the header chunks from the packet's 8 header words Hj (its pass-1 record).
template <int K, int NT>
__device__ __forceinline__ void copyk_store(const EncArgs &a, const CopyK<K> &c, int p, uint32_t lane,
                                            const uint32_t (&Hj)[8]) {
    const FrameGeo &g = c.g[p];
    const uint32_t nst = g.nst, fl = c.flen[p];
    uint4 B[2];
    B[0] = make_uint4(wave_shl1(c.A[p][0].x), wave_shl1(c.A[p][0].y), wave_shl1(c.A[p][0].z), wave_shl1(c.A[p][0].w));
    B[1] = make_uint4(0u, 0u, 0u, 0u);
    if (nst >= 64u) {
        const uint4 l0 = rdl4(c.A[p][1], 0);
        if (lane == 63u) B[0] = l0;
        if (nst > 64u)
            B[1] = make_uint4(wave_shl1(c.A[p][1].x), wave_shl1(c.A[p][1].y), wave_shl1(c.A[p][1].z),
                              wave_shl1(c.A[p][1].w));
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const uint32_t k = lane + 64u * q;
        if (q == 1 && nst <= 64u) continue;  // uniform
        const uint4 V = rsk::funnel16(c.A[p][q], B[q], g.sh);
        const uint4 v = k < (g.r >= 2u ? 3u : 2u) ? head_chunk(Hj, k, g.r, V) : V;
        if (k >= nst) continue;
        store_piece<NT>(g.d0 + 16u * k, v, k == 0u ? g.r : 0u, (int)fl - 16 * (int)k, a.pad != 0u);
    }
}

// NT: bit 0 nontemporal loads, bit 1 nontemporal stores (shipped: 3; C3 -1.4 % against 2, and 256-thread
// blocks against 64 / 512 / 1024: profiles/r04r_two_pass_ab.json).  K: packets per wave (round 5):
// every chunk load of the K packets is issued before any store, so a wave carries K frames' bytes in
// flight -- the chip retires a bounded number of waves per second (the one-packet waves of C3 run at
// ~2 G waves/s), so short frames need several per wave to keep the memory system busy.
// base: the launch's first packet (a grid is limited to 2^32 - 1 work-items, i.e. 2^26 packets at 64
// per packet: larger batches take several launches, kCopyMaxPackets each).
template <int NT, int K = 1>
__global__ __launch_bounds__(kBlock) void k_encode_copy(EncArgs a, const uint32_t *heads, uint64_t base, uint64_t nr) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint64_t i0 = base + ((uint64_t)blockIdx.x * kWavesPerBlock + w) * K;
    if (i0 >= a.n) return;
    CopyK<K> c;
    copyk_issue<K, NT>(a, i0, lane, c);
#pragma unroll
    for (int p = 0; p < K; ++p) {
        if (!c.flen[p]) continue;  // uniform
        uint32_t Hj[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) Hj[t] = heads[4 * ((t < 4 ? 0 : nr) + i0 + p) + (t & 3)];  // uniform: scalar loads
        copyk_store<K, NT>(a, c, p, lane, Hj);
    }
}

// ---- the output-stationary copy for frames laid back to back (round 6) -------
// When frames are byte-packed, the 16-B chunk where one frame ends and the next begins is written by
// two packet-stationary waves, each with byte stores for its part (store_range16: up to five
// stores), and the write pattern costs what the copy saves: tools/bench_layouts.py --probe writes
// C4's frames in the encode's access shape at 0.348 ms with whole-chunk stores and 0.572 ms with the
// byte-exact edges (profiles/r06_layout_probe.json).  Here waves own OUTPUT: block b = kOsBlock bytes
// of the arena from r0 = (frame + frame_off[0]) rounded down, each lane one 16-B chunk, assembled from
// at most two frames (frames are >= 32 B: a chunk holds the tail of frame F1 -- header words from its
// pass-1 record, payload through a per-lane funnel, pad zeros -- and the first header bytes of F2), so
// every chunk a frame touches is written once, whole, unless it also holds bytes outside every frame.
// The header pass (k_encode_heads_os) maps each block to the first packet that can reach it and
// checks that the frames are laid out in packet order without overlap; otherwise (or when the gaps
// are wide) k_encode_os copies packet by packet as k_encode_copy<NT, 1> does.
constexpr uint32_t kOsBlock = 2048;  // bytes per wave-iteration: 2 chunks per lane (1 KB: 0.487 ms on C4 byte-packed; 4 KB: 141 VGPRs)
constexpr uint32_t kOsMaxGapBlocks = 16;  // blocks one packet may map (wider gaps: the fallback)
struct OsMap {
    uint32_t *bfirst;  // [bcap] first packet of block b
    uint32_t *ctl;     // [0] = epoch: the layout failed a check in this call; [1] = block count
    uint32_t bcap, epoch;
};
__device__ __forceinline__ uint32_t os_ext(const EncArgs &a, uint64_t fo, uint32_t P) {
    return P != 0u && P <= (uint32_t)RSK_MAX_PAYLOAD ? padded_len(a.frame + fo, RSK_HEAD_SIZE + P, a.pad) : 0u;
}

template <int SADD = 0>
__global__ __launch_bounds__(kBlock) void k_encode_heads_os(EncArgs a, KeySched ks, uint4 *heads, uint32_t *stat,
                                                            uint64_t nr, OsMap m) {
    stage_tags(ks);
    enc_sample(a.pay_len, a.n, stat, a.frame_off, a.pad);
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const Lane1 L = encode_phase1<true, true, SADD>(a, ks, i < a.n ? i : a.n);
    bool bad = false;
    if (i < a.n) {
        if (L.st > 0) {
            heads[i] = make_uint4(L.H[0], L.H[1], L.H[2], L.H[3]);
            heads[nr + i] = make_uint4(L.H[4], L.H[5], L.H[6], L.H[7]);
        }
        const uint64_t base = reinterpret_cast<uintptr_t>(a.frame);
        const uint64_t r0 = (base + a.frame_off[0]) & ~(uint64_t)(kOsBlock - 1u);
        const uint64_t s = base + L.fo, e = s + (L.st > 0 ? padded_len(a.frame + L.fo, (uint32_t)L.st, a.pad) : 0u);
        uint64_t ep = r0;  // the previous packet's end
        if (i > 0) {
            const uint64_t fp = a.frame_off[i - 1];
            ep = base + fp + os_ext(a, fp, a.pay_len[i - 1]);
        }
        bad = s < ep;
        if (!bad) {  // blocks starting in [ep, e): this packet is the first that can reach them
            uint64_t b = (ep - r0 + kOsBlock - 1u) / kOsBlock;
            const uint64_t bend = e > r0 ? (e - r0 + kOsBlock - 1u) / kOsBlock : 0u;
            if (bend > b + kOsMaxGapBlocks || bend > m.bcap) bad = true;
            else
                for (; b < bend; ++b) m.bfirst[b] = (uint32_t)i;
        }
        if (i == a.n - 1u) m.ctl[1] = e > r0 ? (uint32_t)((e - r0 + kOsBlock - 1u) / kOsBlock) : 0u;
    }
    if (__ballot(bad) != 0ull && (threadIdx.x & 63u) == 0u)
        __hip_atomic_store(m.ctl, m.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The frame a lane's chunk takes bytes from: payload offset and length, packet index (its record).
struct OsFrame {
    uint64_t po;
    uint32_t P, p;
};

// The 16 bytes of frame F's image at image offset t (t >= 0): header words from its record for
// t < 32, the payload through the per-lane funnel from t + 16 > 32 on (payload byte x at image
// 31 + x), zero past 31 + P (the pad).  Split in two so that a block issues every load of all its
// chunks before the first use (a load inside a divergent branch waits for the branch: the first
// build, with the loads in branches, ran C4's byte-packed frames at 0.66 ms): os_load always loads
// (addresses clamped into the payload and the records), os_compose only selects.
struct OsLd {
    uint4 A, B, H0, H1;
    uint32_t sh;
};
template <int NT>
__device__ __forceinline__ OsLd os_load(const EncArgs &a, const uint4 *heads, uint64_t nr, const OsFrame &F,
                                        uint32_t t) {
    OsLd L;
    const uint64_t lo = F.po & ~15ull, hi = (F.po + (F.P ? F.P : 1u) - 1u) & ~15ull;
    const int64_t src = (int64_t)F.po + (int64_t)t - RSK_HEAD_SIZE;  // payload address of chunk byte 0
    const uint64_t c0 = (uint64_t)(src & ~(int64_t)15);
    L.sh = (uint32_t)(src & 15);
    const int64_t c1 = (int64_t)c0 + 16;  // chunks outside the payload: any payload chunk (masked)
    const uint64_t a0 = (int64_t)c0 < (int64_t)lo ? lo : c0 > hi ? hi : c0;
    const uint64_t a1 = c1 < (int64_t)lo ? lo : (uint64_t)c1 > hi ? hi : (uint64_t)c1;
    L.A = ld16<NT & 1>(a.payload + a0);
    L.B = ld16<NT & 1>(a.payload + a1);
    L.H0 = heads[F.p];
    L.H1 = heads[nr + F.p];
    return L;
}
__device__ __forceinline__ uint4 os_compose(const OsFrame &F, const OsLd &L, uint32_t t) {
    const uint32_t flen = RSK_HEAD_SIZE + F.P;
    uint4 v = funnel16_lane(L.A, L.B, L.sh);
    const int lim = (int)flen - (int)t;  // payload bytes end at image flen
    if (lim < 16) v = lim > 0 ? rsk::keep_bytes16(v, lim) : make_uint4(0u, 0u, 0u, 0u);
    if (t < 32u) {  // header words (bytes [0, 32) of the record, byte 31 = payload[0])
        const uint4 z = make_uint4(0u, 0u, 0u, 0u);
        const uint4 hv = t < 16u ? funnel16_lane(L.H0, L.H1, t) : funnel16_lane(L.H1, z, t - 16u);
        const int nh = 32 - (int)t;  // chunk bytes [0, nh) are header bytes
        const uint4 mk = nh >= 16 ? make_uint4(~0u, ~0u, ~0u, ~0u) : rsk::keep_bytes16(make_uint4(~0u, ~0u, ~0u, ~0u), nh);
        v = make_uint4((hv.x & mk.x) | (v.x & ~mk.x), (hv.y & mk.y) | (v.y & ~mk.y), (hv.z & mk.z) | (v.z & ~mk.z),
                       (hv.w & mk.w) | (v.w & ~mk.w));
    }
    return v;
}

// A wave's window: descriptors of 64 consecutive packets from p0, one per lane.
struct OsWin {
    uint32_t p0;
    uint64_t s, e, po;  // lane j: packet p0 + j's frame [s, e) (absolute; e = s when not framed), payload offset
    uint32_t P;
};
__device__ __forceinline__ OsWin os_window(const EncArgs &a, uint32_t p0, uint32_t lane) {
    OsWin W;
    W.p0 = p0;
    const uint64_t pj = (uint64_t)p0 + lane;
    uint64_t fo = 0, po = 0;
    uint32_t P = 0;
    if (pj < a.n) {
        P = a.pay_len[pj];
        fo = a.frame_off[pj];
        po = a.pay_off[pj];
    }
    W.s = pj < a.n ? reinterpret_cast<uintptr_t>(a.frame) + fo : ~0ull;  // past the batch: starts nowhere
    W.e = pj < a.n ? W.s + os_ext(a, fo, P) : ~0ull;
    W.po = po;
    W.P = P;
    return W;
}

// Block [B0, B0 + kOsBlock): every packet overlapping it lies in the window lanes [jlo, jhi] (the
// caller slides the window).  Chunk u of lane l (q = B0 + 1024 u + 16 l) takes F1 = the last packet
// starting at or before q (a dropped one has no bytes: with frames in order nothing earlier reaches q
// then) and F2 = the first framed packet starting inside the chunk; the loop over the block's packets
// only counts (32-bit starts relative to B0), the frames' fields come from their window lanes by one
// ds_bpermute each (round 6: selecting whole frame records in the loop cost ~200 VALU per block).
template <int NT>
__device__ __forceinline__ void os_block(const EncArgs &a, const uint4 *heads, uint64_t nr, const OsWin &W,
                                         uint32_t jlo, uint32_t jhi, uint64_t B0, uint32_t lane) {
    constexpr int U = kOsBlock / 1024;  // chunks per lane, 1 KB apart
    constexpr int32_t kFar = 1 << 30;
    // window lane j's start / end relative to B0, clamped to +-2^30 (blocks are 2 KB)
    const int64_t ds = (int64_t)(W.s - B0), de = (int64_t)(W.e - B0);
    const int32_t rs = W.s == ~0ull ? kFar : ds < -kFar ? -kFar : ds > kFar ? kFar : (int32_t)ds;
    const int32_t re = W.e == ~0ull ? kFar : de < -kFar ? -kFar : de > kFar ? kFar : (int32_t)de;
    uint32_t j1[U], j2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        j1[u] = 64u;  // none
        j2[u] = 64u;
    }
    for (uint32_t j = jlo; j <= jhi; ++j) {  // uniform
        const int32_t sj = (int32_t)rdl((uint32_t)rs, j), ej = (int32_t)rdl((uint32_t)re, j);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int32_t q = (int32_t)(1024u * u + 16u * lane);
            if (sj <= q) j1[u] = j;
            else if (sj < q + 16 && ej > sj && j2[u] == 64u) j2[u] = j;
        }
    }
    uint32_t c1[U], uu[U], t1[U];
    OsFrame F1[U];
    uint32_t p2[U];
    OsLd L[U];
    uint4 G[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // fields by bpermute, then every load, unconditionally
        const int32_t q = (int32_t)(1024u * u + 16u * lane);
        const uint32_t k1 = j1[u] & 63u, k2 = j2[u] & 63u;
        const int32_t s1 = __shfl(rs, (int)k1), e1 = __shfl(re, (int)k1), s2 = __shfl(rs, (int)k2);
        const bool h1 = j1[u] < 64u && e1 > q, h2 = j2[u] < 64u;
        c1[u] = h1 ? (uint32_t)(e1 - q >= 16 ? 16 : e1 - q) : 0u;
        uu[u] = h2 ? (uint32_t)(s2 - q) : 16u;
        t1[u] = h1 ? (uint32_t)(q - s1) : 0u;
        F1[u].po = (uint64_t)(uint32_t)__shfl((int)(uint32_t)W.po, (int)k1) |
                   ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(W.po >> 32), (int)k1) << 32);
        F1[u].P = (uint32_t)__shfl((int)W.P, (int)k1);
        if (!h1) {  // no frame bytes: the loads read payload[0..16) (a dropped packet's offsets may be anything)
            F1[u].po = 0u;
            F1[u].P = 1u;
        }
        F1[u].p = W.p0 + k1;
        p2[u] = W.p0 + k2;
        L[u] = os_load<NT>(a, heads, nr, F1[u], t1[u]);
        G[u] = heads[p2[u] < a.n ? p2[u] : 0u];
    }
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        v[u] = os_compose(F1[u], L[u], t1[u]);
        if (uu[u] < 16u) {  // F2's first 16 - uu header bytes at chunk offset uu
            const uint4 z = make_uint4(0u, 0u, 0u, 0u);
            const uint4 hv = funnel16_lane(z, G[u], 16u - uu[u]);
            const uint4 mk = rsk::keep_bytes16(make_uint4(~0u, ~0u, ~0u, ~0u), (int)uu[u]);
            v[u] = make_uint4((v[u].x & mk.x) | (hv.x & ~mk.x), (v[u].y & mk.y) | (hv.y & ~mk.y),
                              (v[u].z & mk.z) | (hv.z & ~mk.z), (v[u].w & mk.w) | (hv.w & ~mk.w));
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        uint8_t *d = reinterpret_cast<uint8_t *>(B0 + 1024u * u + 16u * lane);
        if (c1[u] == 16u || (uu[u] < 16u && c1[u] == uu[u])) st16<NT>(d, v[u]);  // the whole chunk is frame bytes
        else {
            if (c1[u]) rsk::store_range16(d, v[u], 0u, c1[u]);
            if (uu[u] < 16u) rsk::store_range16(d, v[u], uu[u], 16u);
        }
    }
}

// Persistent waves, each streaming its own contiguous range of blocks with a sliding window of 64
// packets' descriptors (one block-map load per wave, one descriptor load per 64 packets), or, when the
// header pass flagged the layout, copying packet by packet.
template <int NT>
__global__ __launch_bounds__(kBlock) void k_encode_os(EncArgs a, const uint4 *heads, uint64_t nr, const uint32_t *bfirst,
                                                      const uint32_t *ctl, uint32_t epoch) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint64_t wid = (uint64_t)blockIdx.x * kWavesPerBlock + w, nw = (uint64_t)gridDim.x * kWavesPerBlock;
    if (__hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch) {
        const uint32_t *hr = reinterpret_cast<const uint32_t *>(heads);
        for (uint64_t i0 = wid; i0 < a.n; i0 += nw) {  // packet by packet (k_encode_copy<NT, 1>)
            CopyK<1> c;
            copyk_issue<1, NT>(a, i0, lane, c);
            if (!c.flen[0]) continue;  // uniform
            uint32_t Hj[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) Hj[t] = hr[4 * ((t < 4 ? 0 : nr) + i0) + (t & 3)];
            copyk_store<1, NT>(a, c, 0, lane, Hj);
        }
        return;
    }
    const uint64_t nb = ctl[1];
    const uint64_t r0 = (reinterpret_cast<uintptr_t>(a.frame) + a.frame_off[0]) & ~(uint64_t)(kOsBlock - 1u);
    const uint64_t b0 = nb * wid / nw, b1 = nb * (wid + 1u) / nw;  // this wave's blocks
    if (b0 >= b1) return;
    OsWin W = os_window(a, bfirst[b0], lane);
    for (uint64_t b = b0; b < b1; ++b) {
        const uint64_t B0 = r0 + b * kOsBlock, B1 = B0 + kOsBlock;
        // slide: drop the packets that end at or before the block (the window's first packet that
        // reaches past B0 becomes lane 0) once no packet in the window starts past the block
        for (;;) {
            const uint64_t live = __ballot(W.e > B0);  // frames reaching into or past the block (a suffix)
            const uint64_t past = __ballot(W.s >= B1);  // packets starting past the block
            if (past != 0ull || (W.p0 + 64ull >= a.n)) {
                const uint32_t jlo = live ? (uint32_t)__builtin_ctzll(live) : 64u;
                const uint32_t jhi = past ? (uint32_t)__builtin_ctzll(past) : 64u;  // first starting past
                if (jlo < jhi) os_block<NT>(a, heads, nr, W, jlo, jhi - 1u, B0, lane);
                break;
            }
            // every packet of the window starts inside or before the block: move on by the packets
            // that end before it (at least one, else the whole window is inside the block: by 32)
            const uint32_t adv = live ? (uint32_t)__builtin_ctzll(live) : 64u;
            if (adv == 0u) {  // a block holding 64 packet starts (tiny or dropped packets): by halves
                os_block<NT>(a, heads, nr, W, 0u, 31u, B0, lane);  // packets 0..31, then from 32 on
                W = os_window(a, W.p0 + 32u, lane);
                continue;
            }
            W = os_window(a, W.p0 + adv, lane);
        }
    }
}

// Grouped-interleave mapping (shipped: GRP 8, SBW 1024).  A super-block of SBW consecutive waves owns
// SBW * 64 consecutive packets; wave wl of it takes groups of GRP consecutive packets strided by
// SBW * GRP (lane l: group (l / GRP) * SBW + wl, packet l % GRP in it).  Each wave still frames 64
// packets (descriptor loads coalesced per 8-packet group), but the resident waves copy one compact
// stretch of the arenas at a time (SBW * GRP packets per super-block) instead of each its own region
// 64 packets from the next wave's: C3 -3.7 %, C4 -4.1 %, C2 within 1 % against the tiled mapping
// (profiles/r02_ab_encode_mapping.json; renumbering the blocks so that each XCD's blocks own
// consecutive waves measured no gain, profiles/r01_ab_xcd_map.json).  The grid holds only waves
// that own a packet (enc_grid).
template <int MODE, int PU, int U, int GRP, int SBW, int TG = 0>
__global__ __launch_bounds__(kBlock) void k_encode(EncArgs a, KeySched ks) {
    __shared__ CopyRec recs[kWavesPerBlock][64];
    __shared__ uint32_t cend[kWavesPerBlock][64];
    stage_tags(ks);
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint64_t wg = (uint64_t)blockIdx.x * kWavesPerBlock + w;
    const uint64_t sb = wg / SBW, wl = wg % SBW;
    const uint64_t first = sb * SBW * 64u + wl * GRP;  // the wave's smallest packet
    if (first >= a.n) return;  // wave-uniform
    const uint64_t i = sb * SBW * 64u + ((uint64_t)(lane / GRP) * SBW + wl) * GRP + lane % GRP;
    encode_set<MODE, PU, U, GRP, TG>(a, ks, i < a.n ? i : a.n, lane, recs[w], cend[w]);
}

// ---------------------------------------------------------------------------------------------
// Encode straight to wire packets (RConn::Output + RawTcp::SendRawTcp / libnet)
// ---------------------------------------------------------------------------------------------
struct WireArgs {
    const uint32_t *src, *dst;
    const uint16_t *sp, *dp;
    const uint32_t *seq, *ack;
    const uint8_t *flag;
    const uint16_t *ip_id;
    uint32_t eth[4];  // 14 link-header bytes, LE words
};

// one's-complement sum of the little-endian 16-bit halves of w (RFC 1071 is byte-order agnostic:
// summing LE halfwords and storing ~sum little-endian gives the big-endian checksum bytes)
__device__ __forceinline__ uint32_t hsum(uint32_t w) { return (w & 0xffffu) + (w >> 16); }
// acc + the four words' 16-bit halves: one v_dot2_u32_u16 (halves x (1, 1)) per word
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t hsum4(const uint4 &v, uint32_t acc) {
    const u16x2 one = {1, 1};
    acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, v.x), one, acc, false);
    acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, v.y), one, acc, false);
    acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, v.z), one, acc, false);
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, v.w), one, acc, false);
}
__device__ __forceinline__ uint32_t fold16(uint32_t s) {
    s = (s & 0xffffu) + (s >> 16);
    s = (s & 0xffffu) + (s >> 16);
    return s;
}
// OR `nb` bytes of v (LE) into the byte image PW at byte offset off (all compile-time after inlining)
template <int N>
__device__ __forceinline__ void put_bytes(uint32_t (&PW)[N], int off, uint32_t v, int nb) {
#pragma unroll
    for (int b = 0; b < 4; ++b)
        if (b < nb) PW[(off + b) >> 2] |= ((v >> (8 * b)) & 0xffu) << (8 * ((off + b) & 3));
}

template <int E>  // E = link header bytes before IPv4: 0 (RAW4) or 14 (Ethernet)
struct WireGeom {
    static constexpr int HL = E + 40;                // bytes before the frame
    static constexpr int HB = HL + RSK_HEAD_SIZE;     // bytes before the payload
    static constexpr int NPRE = HB / 16 + 1;          // chunks built from the prefix image
    static constexpr int NPW = 4 * NPRE;              // prefix words (covers HB + 16 payload bytes at least... up to 16*NPRE)
    static constexpr int D0 = 16 * NPRE - HB;         // payload offset of chunk NPRE's first byte
    static constexpr int CK = E + 36;                 // TCP checksum byte offset
    static constexpr int IPC = E + 10;                // IPv4 checksum byte offset
};

// payload bytes [0, 16) of a P-byte payload as 4 LE words (bytes past P zero)
__device__ __forceinline__ void wire_payload_prefix(const uint8_t *pay, uint32_t P, uint32_t (&pw)[4]) {
    rsk::load_window<4>(pay, pay + P - 1, pw);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int k = (int)P - 4 * q;
        pw[q] &= k >= 4 ? 0xffffffffu : (k <= 0 ? 0u : ((1u << (8 * k)) - 1u));
    }
}

// those words into the prefix image at wire offset HB (the part that falls inside the NPRE chunks)
template <int E>
__device__ __forceinline__ void wire_put_prefix(uint32_t (&PW)[WireGeom<E>::NPW], const uint32_t (&pw)[4]) {
    using G = WireGeom<E>;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int off = G::HB + 4 * q;
        const int nb = (off + 4 <= 4 * G::NPW) ? 4 : 4 * G::NPW - off;
        if (nb > 0) put_bytes(PW, off, pw[q], nb);
    }
}

// ---- phase 1 (one lane per packet): the wire prefix image PW = link header, IPv4 header (with its
// checksum), TCP header (checksum 0), frame bytes [0, 31) and payload bytes [0, D0) (masked to P);
// sum_pre = TCP checksum contribution of the pseudo-header and PW from the TCP header on; the
// packet status becomes the wire length.
template <int E>
__device__ __forceinline__ void wire_phase1(const EncArgs &a, const WireArgs &wa, const Lane1 &L, uint64_t i,
                                            uint32_t (&PW)[WireGeom<E>::NPW], uint32_t &sum_pre, int32_t &wst,
                                            bool pre = true) {
    using G = WireGeom<E>;
#pragma unroll
    for (int q = 0; q < G::NPW; ++q) PW[q] = 0;
    sum_pre = 0;
    wst = L.st;
    if (L.st <= 0) return;
    const uint32_t flen = (uint32_t)L.st, P = flen - RSK_HEAD_SIZE;
    const uint32_t wlen = G::HL + flen;
    wst = (int32_t)wlen;
    a.status[i] = wst;
    const uint32_t src = wa.src[i], dst = wa.dst[i], sp = wa.sp[i], dp = wa.dp[i];
    const uint32_t seq = wa.seq[i], ack = wa.ack[i], fl = wa.flag[i], id = wa.ip_id[i];
    if constexpr (E > 0) {
#pragma unroll
        for (int b = 0; b < E; b += 4) put_bytes(PW, b, wa.eth[b >> 2], E - b < 4 ? E - b : 4);
    }
    // IPv4 header (libnet_build_ipv4): 45 00 | len | id | 40 00 | 40 06 | csum | src | dst
    const uint32_t tot = 40u + flen;
    put_bytes(PW, E + 0, 0x45u | (rsk::bswap16(tot) << 16), 4);
    put_bytes(PW, E + 4, rsk::bswap16(id) | (0x0040u << 16), 4);
    put_bytes(PW, E + 8, 64u | (6u << 8), 2);
    put_bytes(PW, E + 12, src, 4);
    put_bytes(PW, E + 16, dst, 4);
    const uint32_t ips = hsum(0x45u | (rsk::bswap16(tot) << 16)) + hsum(rsk::bswap16(id) | (0x0040u << 16)) +
                         hsum(64u | (6u << 8)) + hsum(src) + hsum(dst);
    put_bytes(PW, G::IPC, ~fold16(ips) & 0xffffu, 2);
    // TCP header (libnet_build_tcp): sp dp seq ack | 50 flags | ffff | csum | 0000
    const uint32_t t0 = rsk::bswap16(sp) | (rsk::bswap16(dp) << 16), t1 = rsk::bswap32(seq),
                   t2 = rsk::bswap32(ack), t3 = 0x50u | (fl << 8) | (0xffffu << 16);
    put_bytes(PW, E + 20, t0, 4);
    put_bytes(PW, E + 24, t1, 4);
    put_bytes(PW, E + 28, t2, 4);
    put_bytes(PW, E + 32, t3, 4);
    // frame bytes [0, 31) = tag + EncHead (H[7]'s top byte is payload[0], written below)
#pragma unroll
    for (int q = 0; q < 8; ++q) put_bytes(PW, G::HL + 4 * q, L.H[q], q == 7 ? 3 : 4);
    // payload bytes [0, 16) (bounded by P; bytes past P stay zero); !pre: left to the copy loop
    // (copy_wire_pkt_dpp<..., TAG = true>), which adds them with the tag
    if (pre) {
        uint32_t pw[4];
        wire_payload_prefix(a.payload + L.po, P, pw);
        wire_put_prefix<E>(PW, pw);
    }
    // pseudo-header (src, dst, 0, 6, tcp_len) + TCP header + prefix frame/payload bytes, from the
    // TCP header start (even offset E + 20) to the end of the prefix chunks
    uint32_t s = hsum(src) + hsum(dst) + (6u << 8) + rsk::bswap16(20u + flen);
#pragma unroll
    for (int q = (E + 20) / 4; q < G::NPW; ++q) s += ((E + 20) % 4 && q == (E + 20) / 4) ? (PW[q] >> 16) : hsum(PW[q]);
    sum_pre = s;
}

// Wave-wide sum of v (each lane's value < 2^26): DPP row_shr 1/2/4/8 inclusive scans within each
// 16-lane row (bound_ctrl: lanes shifted in from outside the row read 0), then the four row totals.
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);
    return rdl(v, 15) + rdl(v, 31) + rdl(v, 47) + rdl(v, 63);
}

// A wire packet whose first byte sits r = dst mod 16 (1..15) bytes into a chunk: destination chunk j
// (aligned base d0 = dst - r) holds wire-image bytes [16j - r, 16j - r + 16), i.e. the 16 bytes at
// offset 16 - r of image chunks j - 1 and j.  Image chunks c < NPRE are the prefix image in LDS (the
// TCP checksum ORed into its chunk), c >= NPRE the payload chunks V of the copy (lane c - NPRE, slot
// q; zero past the packet).  Lane l of slot q stores destination chunk NPRE + l + 64q with its
// predecessor from lane l - 1 by a DPP wave shift (lane 0: the last prefix chunk, or lane 63 of slot
// 0), lanes 0 .. NPRE - 1 the prefix chunks; chunk 0 from byte r on, the last up to the packet's
// (padded) end, so packets packed at any byte offset never touch their neighbours.
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);  // wave_shr:1
}
template <int E, int NT>
__device__ __forceinline__ void wire_store_shifted(const EncArgs &a, const uint32_t *img, uint32_t ck, uint8_t *dst,
                                                   uint32_t r, uint32_t wlen, const uint4 (&V)[2], uint32_t lane) {
    using G = WireGeom<E>;
    uint8_t *d0 = dst - r;
    const uint32_t nst = (r + padded_len(dst, wlen, a.pad) + 15u) >> 4;
    const int wend = (int)(r + wlen);  // packet bytes counted from d0
    const bool pad = a.pad != 0u;
    const uint32_t sh = 16u - r;
    // slot 1's lane 0 takes lane 63 of slot 0 (read in uniform flow); slot 0's lane 0 the last prefix chunk
    const uint4 l63 = make_uint4(rdl(V[0].x, 63), rdl(V[0].y, 63), rdl(V[0].z, 63), rdl(V[0].w, 63));
    const uint4 lastpre = *reinterpret_cast<const uint4 *>(img + 4 * (G::NPRE - 1));  // never the checksum chunk
    static_assert(G::CK / 16 < G::NPRE - 1, "checksum chunk below the last prefix chunk");
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        uint4 prev = make_uint4(wave_shr1(V[q].x), wave_shr1(V[q].y), wave_shr1(V[q].z), wave_shr1(V[q].w));
        if (lane == 0u) prev = q == 0 ? lastpre : l63;
        const uint32_t j = G::NPRE + lane + 64u * q;
        if (j < nst) store_last16<NT>(d0 + 16u * j, rsk::funnel16(prev, V[q], sh), wend - 16 * (int)j, pad);
    }
    if (lane < (uint32_t)G::NPRE && lane < nst) {
        uint4 c1 = *reinterpret_cast<const uint4 *>(img + 4u * lane);
        uint4 c0 = lane ? *reinterpret_cast<const uint4 *>(img + 4u * (lane - 1u)) : make_uint4(0u, 0u, 0u, 0u);
        constexpr uint32_t kc = G::CK / 16, kw = (G::CK & 15) >> 2, kb = 8 * (G::CK & 3);
        const uint32_t cw = ck << kb;
        if (lane == kc) {
            if (kw == 0) c1.x |= cw; else if (kw == 1) c1.y |= cw; else if (kw == 2) c1.z |= cw; else c1.w |= cw;
        }
        if (lane == kc + 1u) {
            if (kw == 0) c0.x |= cw; else if (kw == 1) c0.y |= cw; else if (kw == 2) c0.z |= cw; else c0.w |= cw;
        }
        const uint4 d = rsk::funnel16(c0, c1, sh);
        if (lane == 0u) rsk::store_range16(d0, d, r, 16u);
        else store_last16<NT>(d0 + 16u * lane, d, wend - 16 * (int)lane, pad);
    }
}

// ---- the same with one aligned load per chunk: the funnel partner comes from lane + 1 by DPP (as
// copy_pkt_dpp), all PU packets' loads issued before the first shift. ------------------------------
// TAG (sets of long frames, as copy_pkt_dpp_tag): phase 1 left the tag, payload[0] at frame byte
// 31 and the payload prefix bytes out of the prefix images, so that each payload's first line is read
// once, here, next to the chunk loads that fetch it anyway.  Lane p loads packet p's first 16 payload
// bytes before the chunk loads, runs the MD5 while they are in flight, ORs the missing bytes into
// the packet's LDS prefix image and hands their checksum share to the packet's checksum.
template <int E, int PU, int NT, bool TAG = false>
__device__ __forceinline__ void copy_wire_pkt_dpp(const EncArgs &a, const KeySched &ks, const Lane1 &L,
                                                  uint32_t *stage, uint32_t sum_pre, int32_t wst, uint32_t lane,
                                                  uint64_t vm) {
    using G = WireGeom<E>;
    while (vm) {
        uint32_t js[PU];
        bool on[PU];
#pragma unroll
        for (int p = 0; p < PU; ++p) {
            on[p] = vm != 0ull;
            js[p] = on[p] ? (uint32_t)__builtin_ctzll(vm) : 0u;
            if (on[p]) vm &= vm - 1ull;
        }
        uint32_t pw[4] = {0u, 0u, 0u, 0u}, myP = 0, myj = 0;  // TAG: lane p's packet
        if constexpr (TAG) {
            uint64_t mypo = 0;
#pragma unroll
            for (int p = 0; p < PU; ++p) {  // uniform readlanes, per-lane selects
                const uint32_t wl = on[p] ? rdl((uint32_t)wst, js[p]) : 0u;
                const uint64_t po = rdl64(L.po, js[p]);
                if (lane == (uint32_t)p) {
                    myP = on[p] ? wl - G::HB : 0u;
                    mypo = po;
                    myj = js[p];
                }
            }
            if (myP) wire_payload_prefix(a.payload + mypo, myP, pw);
        }
        uint4 A[PU][2];
        uint32_t wlen[PU], shp[PU];
        uint8_t *dstp[PU];
        bool ld1[PU];  // source chunk 64 holds payload bytes (slot 1 loaded; lane 63's funnel partner)
#pragma unroll
        for (int p = 0; p < PU; ++p) {
            wlen[p] = on[p] ? (uint32_t)rdl((uint32_t)wst, js[p]) : 0u;
            const uint32_t P = wlen[p] - G::HB;
            const uint8_t *pay = a.payload + rdl64(L.po, js[p]);
            dstp[p] = a.frame + rdl64(L.fo, js[p]);
            shp[p] = (uint32_t)((reinterpret_cast<uintptr_t>(pay) + G::D0) & 15u);
            const uint8_t *src_al = pay + G::D0 - shp[p];
            const int32_t last_rel = (int32_t)P - 1 - G::D0 + (int32_t)shp[p];
            // round 4: slot 1 skipped for packets that do not reach it -- RAW4 only: measured on
            // Ethernet packets it cost more (SGPR spills 392 -> 450, C4 0.421 -> 0.451 ms) than it saved
            // (RAW4 C4 0.455 -> 0.413 ms, C3 2.339 -> 2.295; profiles/r04_paths_wire.json)
            ld1[p] = E != 0 || (on[p] && last_rel >= 16 * 64);
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const uint32_t m = lane + 64u * q;  // source chunk of frame chunk NPRE + m
                A[p][q] = make_uint4(0u, 0u, 0u, 0u);
                // slot 1 only for payloads reaching source chunk 64 (uniform: most C4 packets do not)
                if (q == 1 && !ld1[p]) continue;
                if (on[p] && (int32_t)(16u * m) <= last_rel) A[p][q] = ld16<0>(src_al + 16u * m);
            }
        }
        uint32_t dsum = 0;  // TAG: lane p, checksum share of the bytes it adds to packet p's prefix image
        if constexpr (TAG) {
            uint32_t t0, t1;
            tag_of(ks, pw[0] & 0xffu, t0, t1);
            uint32_t D[G::NPW];
#pragma unroll
            for (int q = 0; q < G::NPW; ++q) D[q] = 0;
            put_bytes(D, G::HL, t0, 4);
            put_bytes(D, G::HL + 4, t1, 4);
            wire_put_prefix<E>(D, pw);  // payload bytes from wire offset HB (frame byte 31 = payload[0])
            if (myP) {
#pragma unroll
                for (int q = G::HL / 4; q < G::NPW; ++q) {
                    stage[myj * G::NPW + q] |= D[q];
                    dsum += hsum(D[q]);
                }
            }
            wave_lds_sync();
        }
        uint4 v[PU][2];
        uint32_t ck[PU];
#pragma unroll
        for (int p = 0; p < PU; ++p) {
            uint4 B[2];
            B[0] = make_uint4(wave_shl1(A[p][0].x), wave_shl1(A[p][0].y), wave_shl1(A[p][0].z), wave_shl1(A[p][0].w));
            B[1] = make_uint4(0u, 0u, 0u, 0u);
            const uint32_t nch = (wlen[p] + 15u) >> 4;
            // round 4: slot 1's shifts, funnels and sums only for packets that reach it (uniform); a
            // dead slot 1 holds zeros, which is what the zero-pad stores below need
            const bool s1 = E != 0 || nch > (uint32_t)G::NPRE + 64u;  // implies ld1[p]
            if (ld1[p]) {
                const uint4 l0 = make_uint4(rdl(A[p][1].x, 0), rdl(A[p][1].y, 0), rdl(A[p][1].z, 0),
                                            rdl(A[p][1].w, 0));  // read in uniform flow (see k_encode)
                if (lane == 63u) B[0] = l0;
            }
            if (s1)
                B[1] = make_uint4(wave_shl1(A[p][1].x), wave_shl1(A[p][1].y), wave_shl1(A[p][1].z), wave_shl1(A[p][1].w));
            uint32_t part = 0;
            v[p][1] = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                if (q == 1 && !s1) continue;  // uniform
                const uint32_t k = G::NPRE + lane + 64u * q;
                v[p][q] = rsk::funnel16(A[p][q], B[q], shp[p]);
                const int lim = (int)wlen[p] - 16 * (int)k;
                if (k < nch) {
                    if (lim < 16) v[p][q] = rsk::keep_bytes16(v[p][q], lim);
                    part = hsum4(v[p][q], part);
                }
            }
            ck[p] = part;
        }
#pragma unroll
        for (int p = 0; p < PU; ++p)
            ck[p] = ~fold16(wave_sum(ck[p]) + rdl(sum_pre, js[p]) + (TAG ? rdl(dsum, (uint32_t)p) : 0u)) & 0xffffu;
#pragma unroll
        for (int p = 0; p < PU; ++p) {
            if (!on[p]) continue;
            const uint32_t r = (uint32_t)(reinterpret_cast<uintptr_t>(dstp[p]) & 15u);  // uniform
            if (r == 0u) {
                const uint32_t nst = (padded_len(dstp[p], wlen[p], a.pad) + 15u) >> 4;
                if (lane < (uint32_t)G::NPRE && lane < nst) {
                    const uint4 sv = *reinterpret_cast<const uint4 *>(stage + js[p] * G::NPW + 4u * lane);
                    uint32_t w4[4] = {sv.x, sv.y, sv.z, sv.w};
                    if (lane == (uint32_t)(G::CK / 16)) w4[(G::CK & 15) >> 2] |= ck[p] << (8 * (G::CK & 3));
                    store_last16<NT>(dstp[p] + 16u * lane, make_uint4(w4[0], w4[1], w4[2], w4[3]),
                                    (int)wlen[p] - 16 * (int)lane, a.pad != 0u);
                }
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    if (E == 0 && q == 1 && nst <= (uint32_t)G::NPRE + 64u) continue;  // uniform
                    const uint32_t k = G::NPRE + lane + 64u * q;
                    if (k < nst) store_last16<NT>(dstp[p] + 16u * k, v[p][q], (int)wlen[p] - 16 * (int)k, a.pad != 0u);
                }
            } else {
                wire_store_shifted<E, NT>(a, stage + js[p] * G::NPW, ck[p], dstp[p], r, wlen[p], v[p], lane);
            }
        }
    }
}

// ---- flat copy for short packets, two passes over the set: (1) the payload chunks of all packets as
// one flat chunk list (as copy_flat), each lane adding its chunk's halfword sum into the packet's
// LDS slot; (2) the NPRE prefix chunks of every packet as a dense (packet, chunk) grid read from the
// LDS stage, the TCP checksum patched into chunk CK/16 — both passes store coalesced runs.
template <int E, int U>
__device__ __forceinline__ void copy_wire_flat(const EncArgs &a, const Lane1 &L, const uint32_t *stage,
                                               uint32_t sum_pre, int32_t wst, uint32_t lane, bool mine,
                                               CopyRec *recs, uint32_t *cend, uint32_t *psum) {
    using G = WireGeom<E>;
    uint32_t cc = 0;
    CopyRec r;
    r.src_al = nullptr; r.dst = nullptr; r.cstart = 0; r.sh = 0; r.last_rel = 0; r.flen = 0;
    if (mine) {
        uint8_t *dst = a.frame + L.fo;
        const uint32_t wlen = (uint32_t)wst;
        const uint32_t nst = (padded_len(dst, wlen, a.pad) + 15u) >> 4;
        cc = nst > (uint32_t)G::NPRE ? nst - G::NPRE : 0u;
        const uint8_t *pay = a.payload + L.po;
        const uint32_t sh = (uint32_t)((reinterpret_cast<uintptr_t>(pay) + G::D0) & 15u);
        r.src_al = pay + G::D0 - sh;
        r.dst = dst;
        r.sh = sh;
        r.last_rel = (int32_t)(wlen - G::HB) - 1 - G::D0 + (int32_t)sh;
        r.flen = wlen;
    }
    uint32_t inc = cc;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(inc, off);
        if (lane >= (uint32_t)off) inc += v;
    }
    r.cstart = inc - cc;
    recs[lane] = r;
    cend[lane] = inc;
    psum[lane] = sum_pre;
    const uint32_t C = (uint32_t)__shfl((int)inc, 63);
    wave_lds_sync();
    for (uint32_t g0 = 0; g0 < C; g0 += 64u * U) {
        uint4 A[U], B[U];
        uint8_t *dsts[U];
        uint32_t shs[U], pk[U];
        int32_t lims[U];
        bool act[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t g = g0 + 64u * u + lane;
            act[u] = g < C;
            A[u] = make_uint4(0u, 0u, 0u, 0u);
            B[u] = make_uint4(0u, 0u, 0u, 0u);
            shs[u] = 0;
            lims[u] = 0;
            dsts[u] = nullptr;
            pk[u] = 0;
            if (act[u]) {
                uint32_t lo = 0;
#pragma unroll
                for (uint32_t st = 32; st; st >>= 1)
                    if (cend[lo + st - 1] <= g) lo += st;
                const CopyRec rr = recs[lo];
                const uint32_t ro = 16u * (g - rr.cstart);
                lims[u] = (int32_t)rr.flen - 16 * G::NPRE - (int32_t)ro;
                if (lims[u] > 0) {  // chunk holds packet bytes (else pure pad)
                    A[u] = ld16<0>(rr.src_al + ro);
                    if (rr.sh != 0u && (int32_t)(ro + 16u) <= rr.last_rel) B[u] = ld16<0>(rr.src_al + ro + 16);
                }
                shs[u] = rr.sh;
                dsts[u] = rr.dst + 16 * G::NPRE + ro;
                pk[u] = lo;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!act[u]) continue;
            uint4 v = funnel16_lane(A[u], B[u], shs[u]);
            if (lims[u] < 16) v = lims[u] > 0 ? rsk::keep_bytes16(v, lims[u]) : make_uint4(0u, 0u, 0u, 0u);
            const uint32_t s = hsum4(v, 0u);
            if (s) atomicAdd(&psum[pk[u]], s);
            store_last16<0>(dsts[u], v, lims[u], a.pad != 0u);
        }
    }
    wave_lds_sync();
    // pass 2: prefix chunk (j, c) for g = NPRE * j + c
#pragma unroll
    for (int t = 0; t < G::NPRE; ++t) {
        const uint32_t g = 64u * t + lane;
        const uint32_t j = g / G::NPRE, c = g - j * G::NPRE;
        const CopyRec rr = recs[j];
        if (rr.dst == nullptr) continue;  // not a vector-path packet
        const uint32_t nstj = (padded_len(rr.dst, rr.flen, a.pad) + 15u) >> 4;
        if (c >= nstj) continue;
        const uint4 sv = *reinterpret_cast<const uint4 *>(stage + j * G::NPW + 4u * c);
        uint32_t w4[4] = {sv.x, sv.y, sv.z, sv.w};
        if (c == (uint32_t)(G::CK / 16)) {
            const uint32_t ck = ~fold16(psum[j]) & 0xffffu;
            w4[(G::CK & 15) >> 2] |= ck << (8 * (G::CK & 3));
        }
        store_last16<0>(rr.dst + 16u * c, make_uint4(w4[0], w4[1], w4[2], w4[3]), (int)rr.flen - 16 * (int)c,
                        a.pad != 0u);
    }
}

// ---- the flat copy at any packet alignment (sets with an unaligned packet): the flat list holds
// DESTINATION chunks j >= NPRE of every packet (r = dst mod 16; chunk j holds wire-image bytes
// [16j - r, 16j - r + 16), the image chunks j - 1 and j funnelled by 16 - r).  A lane loads the
// source chunks of image chunks j - 1 and j (three aligned loads; image chunk NPRE - 1 is the last
// prefix chunk, from LDS), adds image chunk j's halfword sum to the packet's checksum (each image
// chunk once: the extra destination chunk past the image sums nothing) and stores chunk j whole;
// pass 2 stores the shifted prefix chunks (chunk 0 from byte r on) with the checksum.  Aligned
// packets (r = 0) of such a set take the same path with chunk j = image chunk j.
template <int E, int U>
__device__ __forceinline__ void copy_wire_flat_any(const EncArgs &a, const Lane1 &L, const uint32_t *stage,
                                                   uint32_t sum_pre, int32_t wst, uint32_t lane, bool mine,
                                                   CopyRec *recs, uint32_t *cend, uint32_t *psum) {
    using G = WireGeom<E>;
    uint32_t cc = 0;
    CopyRec r;
    r.src_al = nullptr; r.dst = nullptr; r.cstart = 0; r.sh = 0; r.last_rel = 0; r.flen = 0;
    if (mine) {
        uint8_t *dst = a.frame + L.fo;
        const uint32_t wlen = (uint32_t)wst;
        const uint32_t ro = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15u);
        const uint32_t nst = (ro + padded_len(dst, wlen, a.pad) + 15u) >> 4;  // destination chunks from d0
        cc = nst > (uint32_t)G::NPRE ? nst - G::NPRE : 0u;
        const uint8_t *pay = a.payload + L.po;
        const uint32_t sh = (uint32_t)((reinterpret_cast<uintptr_t>(pay) + G::D0) & 15u);
        r.src_al = pay + G::D0 - sh;
        r.dst = dst;
        r.sh = sh | (ro << 4);
        r.last_rel = (int32_t)(wlen - G::HB) - 1 - G::D0 + (int32_t)sh;
        r.flen = wlen;
    }
    uint32_t inc = cc;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(inc, off);
        if (lane >= (uint32_t)off) inc += v;
    }
    r.cstart = inc - cc;
    recs[lane] = r;
    cend[lane] = inc;
    psum[lane] = sum_pre;
    const uint32_t C = (uint32_t)__shfl((int)inc, 63);
    wave_lds_sync();
    for (uint32_t g0 = 0; g0 < C; g0 += 64u * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t g = g0 + 64u * u + lane;
            if (g >= C) continue;
            uint32_t lo = 0;
#pragma unroll
            for (uint32_t st = 32; st; st >>= 1)
                if (cend[lo + st - 1] <= g) lo += st;
            const CopyRec rr = recs[lo];
            const uint32_t sh = rr.sh & 15u, ro = rr.sh >> 4;
            const uint32_t m = g - rr.cstart;  // image / destination chunk NPRE + m
            // image chunk NPRE + m from source chunks m, m + 1; image chunk NPRE + m - 1 from m - 1, m
            uint4 S0 = make_uint4(0u, 0u, 0u, 0u), S1 = S0, S2 = S0;
            if ((int32_t)(16u * m) <= rr.last_rel) S1 = ld16<0>(rr.src_al + 16u * m);
            if ((int32_t)(16u * m + 16u) <= rr.last_rel) S2 = ld16<0>(rr.src_al + 16u * m + 16u);
            if (ro != 0u && m != 0u) S0 = ld16<0>(rr.src_al + 16u * m - 16u);
            const int32_t limi = (int32_t)rr.flen - 16 * (G::NPRE + (int32_t)m);  // packet bytes in image chunk
            uint4 im = limi > 0 ? funnel16_lane(S1, S2, sh) : make_uint4(0u, 0u, 0u, 0u);
            if (limi > 0 && limi < 16) im = rsk::keep_bytes16(im, limi);
            const uint32_t s = hsum4(im, 0u);
            if (s) atomicAdd(&psum[lo], s);
            uint4 d = im;
            if (ro != 0u) {
                const uint4 ip = m == 0u ? *reinterpret_cast<const uint4 *>(stage + lo * G::NPW + 4 * (G::NPRE - 1))
                                         : funnel16_lane(S0, S1, sh);  // image chunk NPRE + m - 1 (full)
                d = funnel16_lane(ip, im, 16u - ro);
            }
            const uint32_t jj = G::NPRE + m;
            store_last16<0>(rr.dst - ro + 16u * jj, d, (int)(ro + rr.flen) - 16 * (int)jj, a.pad != 0u);
        }
    }
    wave_lds_sync();
    // pass 2: shifted prefix chunk (j, c) for g = NPRE * j + c
    static_assert(G::CK / 16 < G::NPRE - 1, "checksum chunk below the last prefix chunk");
#pragma unroll
    for (int t = 0; t < G::NPRE; ++t) {
        const uint32_t g = 64u * t + lane;
        const uint32_t j = g / G::NPRE, c = g - j * G::NPRE;
        const CopyRec rr = recs[j];
        if (rr.dst == nullptr) continue;  // not framed
        const uint32_t ro = rr.sh >> 4;
        const uint32_t nstj = (ro + padded_len(rr.dst, rr.flen, a.pad) + 15u) >> 4;
        if (c >= nstj) continue;
        const uint32_t ck = ~fold16(psum[j]) & 0xffffu;
        constexpr uint32_t kc = G::CK / 16, kw = (G::CK & 15) >> 2, kb = 8 * (G::CK & 3);
        uint4 c1 = *reinterpret_cast<const uint4 *>(stage + j * G::NPW + 4u * c);
        uint4 c0 = c ? *reinterpret_cast<const uint4 *>(stage + j * G::NPW + 4u * (c - 1u)) : make_uint4(0u, 0u, 0u, 0u);
        const uint32_t cw = ck << kb;
        if (c == kc) {
            if (kw == 0) c1.x |= cw; else if (kw == 1) c1.y |= cw; else if (kw == 2) c1.z |= cw; else c1.w |= cw;
        }
        if (c == kc + 1u) {
            if (kw == 0) c0.x |= cw; else if (kw == 1) c0.y |= cw; else if (kw == 2) c0.z |= cw; else c0.w |= cw;
        }
        uint8_t *d0 = rr.dst - ro;
        if (ro == 0u) store_last16<0>(d0 + 16u * c, c1, (int)rr.flen - 16 * (int)c, a.pad != 0u);
        else if (c == 0u) rsk::store_range16(d0, funnel16_lane(c0, c1, 16u - ro), ro, 16u);
        else store_last16<0>(d0 + 16u * c, funnel16_lane(c0, c1, 16u - ro), (int)(ro + rr.flen) - 16 * (int)c,
                             a.pad != 0u);
    }
}

// The per-set wire build: two launches over the same grid (k_encode's grouped-interleave mapping:
// 8-packet groups across 1024-wave super-blocks, grid by enc_grid).  Each wave derives the set's copy
// path from pay_len alone -- the flat chunk list below a set-mean wire length of kFlatBelowMeanBytes,
// else the per-packet DPP copy -- and returns unless it is its launch's path, so every set is handled
// exactly once and each launch sizes LDS (hence occupancy) for its own path only (one launch holding
// both: C3 2.75 vs 2.52 ms).  MODE 5: the per-packet half (PU packets per iteration), with the tag and
// payload prefix deferred into the copy loop for sets of long frames; MODE 4: the flat half.
template <int E, int MODE>
struct WireLds {
    static constexpr int kStage = 64 * WireGeom<E>::NPW * 4;  // prefix images (both paths)
    static constexpr bool kFlat = MODE == 4;
    static constexpr int kBytes = kStage + (kFlat ? 64 * (int)sizeof(CopyRec) + 2 * 64 * 4 : 0);
};

// Per-wave copy-path choice (identical in both launches).
template <int E>
__device__ __forceinline__ bool wire_flat_choice(bool vec, uint32_t wlen) {
    uint32_t fl = vec ? wlen : 0u;
#pragma unroll
    for (int off = 32; off; off >>= 1) fl += __shfl_xor(fl, off);
    return fl < kFlatBelowMeanBytes * (uint32_t)__popcll(__ballot(vec));
}

template <int E, int MODE, int PU, int U>
__device__ __forceinline__ void encode_wire_set(const EncArgs &a, const WireArgs &wa, const KeySched &ks) {
    static_assert(MODE == 4 || MODE == 5, "the flat half and the per-packet half");
    using G = WireGeom<E>;
    __shared__ uint4 lds[kWavesPerBlock][WireLds<E, MODE>::kBytes / 16];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint64_t wg = (uint64_t)blockIdx.x * kWavesPerBlock + w;
    constexpr uint32_t kGrp = 8u;
    const uint64_t sb = wg / 1024u, wl = wg % 1024u;
    const uint64_t first = sb * 65536u + wl * 8u;
    if (first >= a.n) return;  // wave-uniform; no block barriers below
    const uint64_t gi = sb * 65536u + ((uint64_t)(lane / 8u) * 1024u + wl) * 8u + lane % 8u;
    const uint64_t i = gi < a.n ? gi : a.n;
    {  // is this set ours?
        bool v0 = false;
        uint32_t wlen = 0;
        if (i < a.n) {
            const uint32_t P = a.pay_len[i];
            v0 = P != 0u && P <= (uint32_t)RSK_MAX_PAYLOAD;  // any alignment: both copies take all
            wlen = G::HL + RSK_HEAD_SIZE + P;
        }
        if (wire_flat_choice<E>(v0, wlen) != (MODE == 4)) return;
    }
    Lane1 L = encode_phase1<MODE != 5>(a, ks, i);
    bool defer = false;
    if constexpr (MODE == 5) {  // the set mean frame length decides (as k_encode)
        const bool v = L.st > 0;
        uint32_t fl = v ? (uint32_t)L.st : 0u;
#pragma unroll
        for (int off = 32; off; off >>= 1) fl += __shfl_xor(fl, off);
        defer = fl >= kDeferTagMeanBytes * (uint32_t)__popcll(__ballot(v));
        if (!defer) encode_tag(a, ks, L);
    }
    uint32_t PW[G::NPW];
    uint32_t sum_pre;
    int32_t wst;
    wire_phase1<E>(a, wa, L, i, PW, sum_pre, wst, !defer);
    const bool vec = L.st > 0;  // every framed packet takes a vector path, at any alignment
    const uint64_t vm = __ballot(vec);
    uint8_t *slice = reinterpret_cast<uint8_t *>(lds[w]);
    uint32_t *stage = reinterpret_cast<uint32_t *>(slice);
    if (L.st > 0) {  // every framed packet's prefix image
#pragma unroll
        for (int c = 0; c < G::NPRE; ++c)
            *reinterpret_cast<uint4 *>(stage + lane * G::NPW + 4 * c) =
                make_uint4(PW[4 * c], PW[4 * c + 1], PW[4 * c + 2], PW[4 * c + 3]);
    }
    if constexpr (MODE == 4) {
        CopyRec *recs = reinterpret_cast<CopyRec *>(slice + WireLds<E, MODE>::kStage);
        uint32_t *cend = reinterpret_cast<uint32_t *>(slice + WireLds<E, MODE>::kStage + 64 * sizeof(CopyRec));
        if (__ballot(L.st > 0 && L.slow) != 0ull)  // an unaligned packet: the any-alignment list
            copy_wire_flat_any<E, U>(a, L, stage, sum_pre, wst, lane, L.st > 0, recs, cend, cend + 64);
        else
            copy_wire_flat<E, U>(a, L, stage, sum_pre, wst, lane, vec, recs, cend, cend + 64);
    } else {
        wave_lds_sync();
        // store policy per set, as k_encode: stream the stores when the wire packets leave gaps
        const uint32_t wend = vec ? padded_len(a.frame + L.fo, (uint32_t)wst, a.pad) : 0u;
        const uint64_t end = L.fo + wend;
        const uint64_t nfo = (uint64_t)(uint32_t)__shfl_down((int)(uint32_t)L.fo, 1) |
                             ((uint64_t)(uint32_t)__shfl_down((int)(uint32_t)(L.fo >> 32), 1) << 32);
        const bool nvec = __shfl_down((int)vec, 1) != 0;
        const bool gaps = __ballot(vec && nvec && lane % kGrp != kGrp - 1u && end != nfo) != 0ull;
        if (defer) {
            if (gaps) copy_wire_pkt_dpp<E, PU, 2, true>(a, ks, L, stage, sum_pre, wst, lane, vm);
            else copy_wire_pkt_dpp<E, PU, 0, true>(a, ks, L, stage, sum_pre, wst, lane, vm);
        } else {
            if (gaps) copy_wire_pkt_dpp<E, PU, 2>(a, ks, L, stage, sum_pre, wst, lane, vm);
            else copy_wire_pkt_dpp<E, PU, 0>(a, ks, L, stage, sum_pre, wst, lane, vm);
        }
    }
}

template <int E, int MODE, int PU, int U>
__global__ __launch_bounds__(kBlock) void k_encode_wire(EncArgs a, WireArgs wa, KeySched ks) {
    stage_tags(ks);
    encode_wire_set<E, MODE, PU, U>(a, wa, ks);
}

// The same held to 4 waves per SIMD (<= 128 VGPRs): the deferred-tag build (MODE 5) needs 131 and
// would otherwise drop to 3, which costs the sets that keep the tag in phase 1 (C4 +9 %).
template <int E, int MODE, int PU, int U>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_encode_wire_w4(
    EncArgs a, WireArgs wa, KeySched ks) {
    stage_tags(ks);
    encode_wire_set<E, MODE, PU, U>(a, wa, ks);
}

// ---- the two-pass wire build (round 6): a header pass, one lane per packet (MD5
// tags 64 to a wave), writes each packet's whole header image -- link, IPv4 with its checksum, TCP,
// the 31 frame-head bytes: wire bytes [0, HB), HB = 71 RAW4 / 85 Ethernet -- as Q + 1 = 5 / 6 16-B
// chunks of a record, with the TCP checksum's share of the pseudo-header and the image (from the TCP
// header on) in the last chunk's bytes 12..15, which the payload overwrites; the status is the wire
// length.  Then copy waves of K packets as k_encode_copy's: lane k takes IMAGE chunk k -- wire bytes
// [16k, 16k + 16): the record's chunk (one 16-B load by lanes 0..Q) for k < Q, record and payload for
// k = Q, payload beyond (one aligned load per chunk and the DPP funnel) -- sums the payload halfwords
// on the way into the TCP checksum (a wave reduction), which the lane of the checksum chunk ORs in
// before the stores.  A packet whose first byte is not 16-B aligned (r = dst mod 16) stores
// destination chunk j = image chunks j - 1 and j funnelled by 16 - r (wave_shr:1), so the checksum is
// summed in image coordinates at any alignment.
template <int E>
struct WireRec {
    static constexpr int HB = WireGeom<E>::HB, Q = HB / 16, R = HB % 16;  // RAW4 71 = 4 x 16 + 7; Eth 85 = 5 x 16 + 5
    static constexpr int NC = Q + 1;                                       // record chunks (80 / 96 B)
    static_assert(R != 0 && R <= 12 && WireGeom<E>::CK / 16 < Q, "record layout");
};

// base: the chunk's first packet (a.n = its end); chunk c of packet i at rec[c * stride + i - base]
template <int E>
__global__ __launch_bounds__(kBlock) void k_wire_heads(EncArgs a, WireArgs wa, KeySched ks, uint4 *rec,
                                                       uint32_t *stat, uint64_t base, uint64_t stride) {
    using G = WireGeom<E>;
    using W = WireRec<E>;
    constexpr int NIW = 4 * W::NC;
    stage_tags(ks);
    enc_sample(a.pay_len, a.n, stat);
    const uint64_t i = base + (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const Lane1 L = encode_phase1<true, true, G::HL>(a, ks, i < a.n ? i : a.n);
    if (i >= a.n || L.st <= 0) return;
    const uint32_t flen = (uint32_t)L.st;
    uint32_t PW[NIW];
#pragma unroll
    for (int q = 0; q < NIW; ++q) PW[q] = 0u;
    const uint32_t src = wa.src[i], dst = wa.dst[i], sp = wa.sp[i], dp = wa.dp[i];
    const uint32_t seq = wa.seq[i], ack = wa.ack[i], fl = wa.flag[i], id = wa.ip_id[i];
    if constexpr (E > 0) {
#pragma unroll
        for (int b = 0; b < E; b += 4) put_bytes(PW, b, wa.eth[b >> 2], E - b < 4 ? E - b : 4);
    }
    // IPv4 header (libnet_build_ipv4): 45 00 | len | id | 40 00 | 40 06 | csum | src | dst
    const uint32_t tot = 40u + flen;
    const uint32_t ip0 = 0x45u | (rsk::bswap16(tot) << 16), ip1 = rsk::bswap16(id) | (0x0040u << 16);
    put_bytes(PW, E + 0, ip0, 4);
    put_bytes(PW, E + 4, ip1, 4);
    put_bytes(PW, E + 8, 64u | (6u << 8), 2);
    put_bytes(PW, E + 12, src, 4);
    put_bytes(PW, E + 16, dst, 4);
    const uint32_t ips = hsum(ip0) + hsum(ip1) + hsum(64u | (6u << 8)) + hsum(src) + hsum(dst);
    put_bytes(PW, G::IPC, ~fold16(ips) & 0xffffu, 2);
    // TCP header (libnet_build_tcp): sp dp seq ack | 50 flags | ffff | csum (0 here) | 0000
    put_bytes(PW, E + 20, rsk::bswap16(sp) | (rsk::bswap16(dp) << 16), 4);
    put_bytes(PW, E + 24, rsk::bswap32(seq), 4);
    put_bytes(PW, E + 28, rsk::bswap32(ack), 4);
    put_bytes(PW, E + 32, 0x50u | (fl << 8) | (0xffffu << 16), 4);
    // frame bytes [0, 31) = tag + EncHead (payload[0], H[7]'s top byte, comes with the payload)
#pragma unroll
    for (int q = 0; q < 8; ++q) put_bytes(PW, G::HL + 4 * q, L.H[q], q == 7 ? 3 : 4);
    // the checksum's share: pseudo-header (src, dst, 0, 6, tcp_len) + the image from the TCP header on
    uint32_t s = hsum(src) + hsum(dst) + (6u << 8) + rsk::bswap16(20u + flen);
#pragma unroll
    for (int q = (E + 20) / 4; q < NIW; ++q) s += ((E + 20) % 4 && q == (E + 20) / 4) ? (PW[q] >> 16) : hsum(PW[q]);
    PW[NIW - 1] = s;  // bytes 12..15 of chunk Q: payload positions, overwritten by the copy
    // chunk-major records: each store instruction of the wave writes 1 KB contiguous
#pragma unroll
    for (int c = 0; c < W::NC; ++c)
        rec[(uint64_t)c * stride + (i - base)] = make_uint4(PW[4 * c], PW[4 * c + 1], PW[4 * c + 2], PW[4 * c + 3]);
}

// base: the launch's first packet; rbase / stride: the record chunk's (k_wire_heads)
template <int E, int NT, int K>
__global__ __launch_bounds__(kBlock) void k_wire_copy(EncArgs a, const uint4 *rec, uint64_t base, uint64_t rbase,
                                                      uint64_t stride) {
    using G = WireGeom<E>;
    using W = WireRec<E>;
    constexpr int HB = W::HB, Q = W::Q, R = W::R;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint64_t i0 = base + ((uint64_t)blockIdx.x * kWavesPerBlock + w) * K;
    if (i0 >= a.n) return;
    // descriptors, lanes 0..K-1 (one round trip)
    uint32_t dP = 0;
    uint64_t dpo = 0, dfo = 0;
    {
        const uint64_t il = i0 + lane;
        if (lane < (uint32_t)K && il < a.n) {
            dP = a.pay_len[il];
            dpo = a.pay_off[il];
            dfo = a.frame_off[il];
        }
    }
    uint4 A[K][2], H[K];
    uint32_t Pp[K], shp[K];
#pragma unroll
    for (int p = 0; p < K; ++p) {
        const uint32_t P = rdl(dP, (uint32_t)p);
        const bool on = i0 + p < a.n && P != 0u && P <= (uint32_t)RSK_MAX_PAYLOAD;  // uniform
        Pp[p] = on ? P : 0u;
        // the record chunk of lane k <= Q
        H[p] = on && lane <= (uint32_t)Q ? rec[(uint64_t)lane * stride + (i0 + p - rbase)] : make_uint4(0u, 0u, 0u, 0u);
        const uint8_t *src = a.payload + rdl64(dpo, (uint32_t)p);
        shp[p] = (uint32_t)((reinterpret_cast<uintptr_t>(src) - (uint32_t)R) & 15u);
        const uint8_t *srcp = src - R - shp[p];  // aligned: image chunk k <- source chunks k - Q, k - Q + 1
        const int32_t first_rel = R + (int32_t)shp[p], last_rel = first_rel + (int32_t)P - 1;
        const int32_t m_lo = first_rel >> 4, m_hi = last_rel >> 4;
        const uint32_t nch = (HB + P + 15u) >> 4;  // image chunks
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            A[p][q] = make_uint4(0u, 0u, 0u, 0u);
            if (!on || (q == 1 && nch < 64u)) continue;  // uniform
            const int32_t m = (int32_t)(lane + 64u * q) - Q;
            const int32_t mc = m < m_lo ? m_lo : m > m_hi ? m_hi : m;  // dead lanes re-read a live chunk
            A[p][q] = ld16<NT>(srcp + 16 * mc);
        }
    }
    // Three phases over the K packets, so the packets' dependency chains overlap (round 6: one packet at a
    // time, the wave waited on each packet's funnel -> sum -> reduction chain in turn): (1) each lane's
    // image chunks and payload halfword sums, (2) the K checksums (wave reductions), (3) the stores.
    // Header mask of lane k <= Q (the record's bytes: all of chunk k < Q, the first R of chunk Q).
    const uint4 mh = lane <= (uint32_t)Q ? rsk::keep_bytes16(make_uint4(~0u, ~0u, ~0u, ~0u), lane < (uint32_t)Q ? 16 : R)
                                         : make_uint4(0u, 0u, 0u, 0u);
    uint4 VI[K][2];
    uint32_t part[K];
#pragma unroll
    for (int p = 0; p < K; ++p) {
        VI[p][0] = VI[p][1] = make_uint4(0u, 0u, 0u, 0u);
        part[p] = 0u;
        const uint32_t P = Pp[p];
        if (!P) continue;  // uniform
        const uint32_t wlen = HB + P, nch = (wlen + 15u) >> 4;
        uint4 B[2];
        B[0] = make_uint4(wave_shl1(A[p][0].x), wave_shl1(A[p][0].y), wave_shl1(A[p][0].z), wave_shl1(A[p][0].w));
        B[1] = make_uint4(0u, 0u, 0u, 0u);
        if (nch >= 64u) {  // uniform
            const uint4 l0 = rdl4(A[p][1], 0);
            if (lane == 63u) B[0] = l0;
            B[1] = make_uint4(wave_shl1(A[p][1].x), wave_shl1(A[p][1].y), wave_shl1(A[p][1].z), wave_shl1(A[p][1].w));
        }
        // lane k's image chunk: the record's bytes under mh, the payload's elsewhere (zero past the
        // packet); summed: the payload bytes only (the record's are in its checksum share)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            if (q == 1 && nch <= 64u) continue;  // uniform
            const uint32_t k = lane + 64u * q;
            uint4 v = rsk::funnel16(A[p][q], B[q], shp[p]);
            const int lim = (int)wlen - 16 * (int)k;
            v = lim >= 16 ? v : lim > 0 ? rsk::keep_bytes16(v, lim) : make_uint4(0u, 0u, 0u, 0u);
            if (q == 0) {
                v = make_uint4(v.x & ~mh.x, v.y & ~mh.y, v.z & ~mh.z, v.w & ~mh.w);
                part[p] = hsum4(v, part[p]);
                const uint4 h = H[p];
                v = make_uint4(v.x | (h.x & mh.x), v.y | (h.y & mh.y), v.z | (h.z & mh.z), v.w | (h.w & mh.w));
            } else {
                part[p] = hsum4(v, part[p]);
            }
            VI[p][q] = v;
        }
    }
    uint32_t ck[K];
#pragma unroll
    for (int p = 0; p < K; ++p) ck[p] = ~fold16(wave_sum(part[p]) + rdl(H[p].w, (uint32_t)Q)) & 0xffffu;
#pragma unroll
    for (int p = 0; p < K; ++p) {
        const uint32_t P = Pp[p];
        if (!P) continue;  // uniform
        const uint32_t wlen = HB + P;
        uint8_t *dst = a.frame + rdl64(dfo, (uint32_t)p);
        if (lane == (uint32_t)(G::CK / 16)) {
            constexpr uint32_t kw = (G::CK & 15) >> 2, kb = 8 * (G::CK & 3);
            if (kw == 0) VI[p][0].x |= ck[p] << kb; else if (kw == 1) VI[p][0].y |= ck[p] << kb;
            else if (kw == 2) VI[p][0].z |= ck[p] << kb; else VI[p][0].w |= ck[p] << kb;
        }
        const uint32_t r = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15u);  // uniform
        uint8_t *d0 = dst - r;
        const uint32_t nst = (r + padded_len(dst, wlen, a.pad) + 15u) >> 4;
        const bool pad = a.pad != 0u;
        if (r == 0u) {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const uint32_t k = lane + 64u * q;
                if (q == 1 && nst <= 64u) continue;  // uniform
                if (k < nst) store_last16<NT>(d0 + 16u * k, VI[p][q], (int)wlen - 16 * (int)k, pad);
            }
        } else {
            const uint4 l63 = rdl4(VI[p][0], 63);
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                if (q == 1 && nst <= 64u) continue;  // uniform
                uint4 prev = make_uint4(wave_shr1(VI[p][q].x), wave_shr1(VI[p][q].y), wave_shr1(VI[p][q].z),
                                        wave_shr1(VI[p][q].w));
                if (lane == 0u) prev = q == 0 ? make_uint4(0u, 0u, 0u, 0u) : l63;
                const uint4 d = rsk::funnel16(prev, VI[p][q], 16u - r);
                const uint32_t j = lane + 64u * q;
                if (j >= nst) continue;
                if (j == 0u) rsk::store_range16(d0, d, r, 16u);
                else store_last16<NT>(d0 + 16u * j, d, (int)(r + wlen) - 16 * (int)j, pad);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Decode (shared by k_decode and k_parse_decode)
// ---------------------------------------------------------------------------------------------
struct Dec {
    uint32_t hlen, cmd, id0, id1, conv;
    uint64_t key;
    uint32_t poff, plen;
    int32_t st;
};

// RConn::OnRecv on frame bytes [base, base + nread)  (conn/RConn.cpp:64-85, EncHead.cpp:39-55,
// util/rhash.cpp:71-92).
// SLOT: base is a 32-B header slot (rsk_decode_headers_batch) whose byte 31 holds the hashed byte
// frame[8 + len]; nread is still the frame's length.
template <bool SLOT>
__device__ __forceinline__ Dec decode_frame_t(const uint8_t *base, int nread, bool close,
                                              const KeySched &ks) {
    Dec o = {0, 0, 0, 0, 0, 0, 0, 0, RSK_RECV_DROP};
    if (nread > RSK_HEAD_SIZE) {
        uint32_t w[8];
        if (SLOT || (reinterpret_cast<uintptr_t>(base) & 15u) == 0) {
            const uint4 A = reinterpret_cast<const uint4 *>(base)[0];
            const uint4 B = reinterpret_cast<const uint4 *>(base)[1];
            w[0] = A.x; w[1] = A.y; w[2] = A.z; w[3] = A.w;
            w[4] = B.x; w[5] = B.y; w[6] = B.z; w[7] = B.w;
        } else {
            rsk::load_window16<8>(base, base + nread - 1, w);
        }
        const uint32_t len = w[2] & 0xffu;                 // EncHead len byte (frame[8])
        const int dl = nread - 8 - (int)len;                // data_len handed to hash_equal
        if ((int)len <= nread - 8 && dl > 0) {              // DecodeBuf ok, hash_equal len > 0
            const uint32_t b = (SLOT || len == (uint32_t)RSK_ENC_HEAD_SIZE) ? (w[7] >> 24) : base[8 + len];
            uint32_t t0, t1;
            tag_of<true>(ks, b, t0, t1);
            if (t0 == w[0] && t1 == w[1]) {
                o.st = RSK_RECV_VALID;
                o.hlen = len;
                o.cmd = (w[2] >> 8) & 0xffu;
                o.id0 = (w[2] >> 16) | (w[3] << 16);
                o.id1 = (w[3] >> 16) | (w[4] << 16);
                o.conv = (w[4] >> 16) | (w[5] << 16);
                o.key = (uint64_t)((w[5] >> 16) | (w[6] << 16)) |
                        ((uint64_t)((w[6] >> 16) | (w[7] << 16)) << 32);
                o.poff = 8u + len;
                o.plen = (uint32_t)dl;
            }
        }
    } else if (close) {
        o.st = RSK_RECV_CLOSE;
    }
    return o;
}

__device__ __forceinline__ Dec decode_frame(const uint8_t *base, int nread, bool close, const KeySched &ks) {
    return decode_frame_t<false>(base, nread, close, ks);
}

struct DecOut {
    uint8_t *hlen, *cmd, *id;
    uint32_t *conv;
    uint64_t *key;
    uint16_t *pay_off, *pay_len;
    int8_t *status;
    uint64_t *masks;  // compaction workspace: one VALID ballot per wave (null: no compaction)
};

__device__ __forceinline__ void store_dec(const DecOut &d, uint64_t i, const Dec &o) {
    d.hlen[i] = (uint8_t)o.hlen;
    d.cmd[i] = (uint8_t)o.cmd;
    *reinterpret_cast<uint2 *>(d.id + 8 * i) = make_uint2(o.id0, o.id1);
    d.conv[i] = o.conv;
    d.key[i] = o.key;
    d.pay_off[i] = (uint16_t)o.poff;
    d.pay_len[i] = (uint16_t)o.plen;
    d.status[i] = (int8_t)o.st;
}

// ---- order-stable compaction: the decode launch writes one VALID ballot per wave; k_compact turns
// them into the VALID index list in one pass.  k_compact tile t covers 64 masks (4096 packets):
// it counts them, scans them in one wave, finds the tile's prefix by decoupled look-back over the
// tiles before it, and its lanes write their indices at prefix + rank (valid_idx in index order).
// Tiles are dispatched in index order, so a tile only waits for tiles that are resident or done.
// State word per tile: bits 63..34 the call's epoch, bit 33 taint, bit 32 inclusive, bits 31..0
// the count; a word from another call is not ready, so the state needs no per-call reset.  The
// epoch is a device-side counter (workspace word 0) that every tile reads first and the last tile
// advances when every tile has published its inclusive word (it checks them all, below), so all
// read the same value; the next call on the stream, or the next replay of a captured graph, sees
// the next epoch.  Epochs run 1 .. 2^30 - 1 (0 is the zeroed state).  Device-scope relaxed
// atomics (acquire / release would add an L2 write-back / invalidate per access, rsk_demux.hip);
// a spin that outlives kCmpSpinMax reads gives up (no hang): it sets RSK_DEVERR_LOOKBACK in the
// context's sticky error word and publishes its inclusive word with the taint bit.  The last tile
// waits for every tile's inclusive word of this epoch and writes n_valid = 0xFFFFFFFF instead of the
// count when one is tainted or never arrives, so a wrong VALID list never comes with a count that
// looks valid, whichever tile gave up and whenever (rsk_check_device_errors).  The
// information travels in the words themselves, so relaxed atomics order it.  Round 1 used k_scan (one
// workgroup) + k_scatter; a look-back inside the decode launch itself (one word per 256-packet
// block) was measured slower than both (C2: 40 us vs 31): the block-granular chain is the cost.
constexpr unsigned long long kCmpIncl = 1ull << 32;
constexpr unsigned long long kCmpTaint = 1ull << 33;
constexpr int kCmpEpochShift = 34;
constexpr uint32_t kCmpEpochMod = 0x3fffffffu;  // epochs 1 .. 2^30 - 1
constexpr uint32_t kCmpSpinMax = 1u << 22;

__device__ __forceinline__ unsigned long long cmp_wait(unsigned long long *s, uint32_t epoch, bool &timed_out) {
    unsigned long long v;
    uint32_t spins = 0;
    do {
        v = __hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } while ((uint32_t)(v >> kCmpEpochShift) != epoch && ++spins < kCmpSpinMax);
    if ((uint32_t)(v >> kCmpEpochShift) == epoch) return v;
    timed_out = true;
    return kCmpIncl;
}

// the same for a word that must be INCLUSIVE for this epoch (the last tile's check); false when it
// never became so or carries the taint
__device__ __forceinline__ bool cmp_wait_incl_clean(unsigned long long *s, uint32_t epoch) {
    unsigned long long v;
    uint32_t spins = 0;
    do {
        v = __hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } while (((uint32_t)(v >> kCmpEpochShift) != epoch || !(v & kCmpIncl)) && ++spins < kCmpSpinMax);
    return (uint32_t)(v >> kCmpEpochShift) == epoch && (v & kCmpIncl) && !(v & kCmpTaint);
}

// all 64 lanes of one wave of tile b; agg uniform; returns b's exclusive prefix (uniform); `to`
// (uniform) is set when a predecessor's word never arrived
__device__ uint32_t cmp_lookback(unsigned long long *st, uint32_t b, uint32_t agg, uint32_t lane, uint32_t epoch,
                                 bool &to) {
    const unsigned long long tag = (unsigned long long)epoch << kCmpEpochShift;
    if (b == 0u) {
        if (lane == 0u) __hip_atomic_store(st, tag | kCmpIncl | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0u;
    }
    if (lane == 0u) __hip_atomic_store(st + b, tag | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t excl = 0;
    for (int64_t top = (int64_t)b - 1;; top -= 64) {
        const int64_t j = top - (int64_t)lane;
        bool lto = false;
        const unsigned long long v = j >= 0 ? cmp_wait(st + j, epoch, lto) : kCmpIncl;  // before tile 0: 0
        if (__ballot(lto)) to = true;
        const uint64_t im = __ballot((v & kCmpIncl) != 0ull);
        uint32_t val = (uint32_t)v;
        if (im && lane > (uint32_t)__builtin_ctzll(im)) val = 0u;  // beyond the nearest inclusive word
#pragma unroll
        for (int off = 32; off; off >>= 1) val += __shfl_xor(val, off);
        excl += val;
        if (im) break;
    }
    if (lane == 0u)  // a tile that gave up publishes its (wrong) prefix with the taint bit
        __hip_atomic_store(st + b, tag | kCmpIncl | (to ? kCmpTaint : 0ull) | (excl + agg), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

// The decode launches' epilogue: every thread calls it (no early exit before); i = its packet.
__device__ __forceinline__ void compact_epilogue(const DecOut &d, bool valid, uint64_t i) {
    const uint64_t m = __ballot(valid);
    if ((threadIdx.x & 63u) == 0u) d.masks[i >> 6] = m;
}

struct DecArgs {
    const uint8_t *frame;
    const uint64_t *frame_off;
    const uint16_t *frame_len;
    const uint8_t *close;
    uint32_t n;
};

__global__ __launch_bounds__(kBlock) void k_decode(DecArgs a, DecOut d, KeySched ks) {
    stage_tags(ks);
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    bool valid = false;
    if (i < a.n) {
        const Dec o = decode_frame(a.frame + a.frame_off[i], (int)a.frame_len[i],
                                   a.close ? a.close[i] != 0 : false, ks);
        store_dec(d, i, o);
        valid = o.st == RSK_RECV_VALID;
    }
    if (d.masks) compact_epilogue(d, valid, i);
}

// Header-only decode: 32-B slots (frame bytes [0, 31) + the hashed byte), one lane per frame.
__global__ __launch_bounds__(kBlock) void k_decode_hdr(DecArgs a, DecOut d, KeySched ks) {
    stage_tags(ks);
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    bool valid = false;
    if (i < a.n) {
        const Dec o = decode_frame_t<true>(a.frame + 32u * i, (int)a.frame_len[i], a.close ? a.close[i] != 0 : false,
                                           ks);
        store_dec(d, i, o);
        valid = o.st == RSK_RECV_VALID;
    }
    if (d.masks) compact_epilogue(d, valid, i);
}

// Header-only encode: frame bytes [0, 32) (tag, EncHead, payload[0]) per packet into 32-B slots.
struct EncHdrArgs {
    const uint8_t *b0;
    const uint16_t *pay_len;
    const uint8_t *cmd;
    const uint32_t *conv;
    const uint64_t *conn_key;
    const uint8_t *id;
    uint8_t *hdr;
    int32_t *status;
    uint32_t id_lo, id_hi, n;
};

__global__ __launch_bounds__(kBlock) void k_encode_hdr(EncHdrArgs a, KeySched ks) {
    stage_tags(ks);
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t P = a.pay_len[i];
    const int32_t st = P == 0 ? RSK_SEND_RESET : (P > RSK_MAX_PAYLOAD ? RSK_SEND_OVERSIZE : (int32_t)(RSK_HEAD_SIZE + P));
    uint32_t H[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (st > 0) {  // RConn.cpp:88-105
        const uint32_t b0 = a.b0[i];
        tag_of(ks, b0, H[0], H[1]);
        uint32_t id0 = a.id_lo, id1 = a.id_hi;
        if (a.id) {
            const uint2 v = *reinterpret_cast<const uint2 *>(a.id + 8 * i);
            id0 = v.x;
            id1 = v.y;
        }
        head_words(a.cmd[i], id0, id1, a.conv[i], a.conn_key[i], b0, H);
    }
    st16<0>(a.hdr + 32u * i, make_uint4(H[0], H[1], H[2], H[3]));
    st16<0>(a.hdr + 32u * i + 16u, make_uint4(H[4], H[5], H[6], H[7]));
    a.status[i] = st;
}

// ---------------------------------------------------------------------------------------------
// Fused pcap parse + decode  (conn/RawTcp.cpp:138-244, cap/cap_headers.h:16-32)
// ---------------------------------------------------------------------------------------------
struct ParseArgs {
    const uint8_t *cap;
    const uint64_t *cap_off;
    const uint32_t *wire_len;
    const uint32_t *cap_len;
    uint32_t *src, *dst;
    uint16_t *sp, *dp;
    uint32_t *seq, *ack;
    uint8_t *flag;
    int8_t *pst;
    uint16_t *cpo, *cpl;
    int datalink, flags;
    uint32_t n;
    uint32_t slot;  // SLOT form: packet i's first min(cap_len, slot) bytes at cap + slot * i
};

// L = link header bytes: 14 (DLT_EN10MB) or 4 (DLT_NULL).  One 64-B window (five 16-B loads, bounded
// by cap_len) holds the link, IPv4 and (IHL 5) TCP headers; other IHLs load the TCP header apart.
// SLOT: host-resident capture, only the first min(cap_len, slot) bytes of each packet were staged
// (slot >= 64); every decision still uses the real cap_len, and a packet whose parse or decode needs
// a byte past its slot gets RSK_PARSE_SLOT_SHORT (zero outputs) instead, for a whole resubmission.
// HWIN: hw already holds the packet's first 64 bytes, loaded as below (the fused capture filter).
struct ParseRes {
    int ps;
    uint32_t src, dst, sp, dp, seq, ack, fl, payo, plen;
    Dec o;
};

template <int L, bool SLOT, bool HWIN>
__device__ __forceinline__ ParseRes parse_one(const ParseArgs &a, const uint8_t *pkt, uint32_t wl, uint32_t cl,
                                              uint32_t av, uint32_t (&hw)[16], const KeySched &ks) {
    int ps = RSK_PARSE_DROP;
    uint32_t src = 0, dst = 0, sp = 0, dp = 0, seq = 0, ack = 0, fl = 0, payo = 0, plen = 0;
    Dec o = {0, 0, 0, 0, 0, 0, 0, 0, RSK_RECV_DROP};
    do {
        if (wl < 44u) break;                                   // :139
        const uint8_t *last = pkt + (av ? av - 1u : 0u);
        if (cl < (uint32_t)L) { ps = RSK_PARSE_MALFORMED; break; }
        if (!HWIN) rsk::load_window16<16>(pkt, last, hw);  // HWIN: the caller loaded it
        if (L == 14) {                                          // :144-151
            if ((hw[3] & 0xffffu) != 0x0008u) break;           // OM_PROTO_IP read LE
        } else {                                                // DLT_NULL :152-160
            if (hw[0] != 2u) break;
        }
        constexpr uint32_t ipo = L;
        if (cl < ipo + 20u) { ps = RSK_PARSE_MALFORMED; break; }
        uint32_t ip[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) ip[k] = rsk::funnel(hw[L / 4 + k + 1], hw[L / 4 + k], L & 3);
        if (((ip[2] >> 8) & 0xffu) != 6u) break;               // ip_p :167-172
        const uint32_t ihl = (ip[0] & 15u) * 4u;
        const uint32_t tcpo = ipo + ihl;
        if (cl < tcpo + 20u) { ps = RSK_PARSE_MALFORMED; break; }
        uint32_t th[4];
        if (ihl == 20u) {
            constexpr int T = L + 20;
#pragma unroll
            for (int k = 0; k < 4; ++k) th[k] = rsk::funnel(hw[T / 4 + k + 1], hw[T / 4 + k], T & 3);
        } else {
            if (SLOT && tcpo + 16u > av) { ps = RSK_PARSE_SLOT_SHORT; break; }
            rsk::load_window16<4>(pkt + tcpo, last, th);
        }
        const uint32_t thl = ((th[3] & 0xffu) >> 4) * 4u;
        payo = tcpo + thl;
        const int payload_len = (int)rsk::bswap16(ip[0] >> 16) - (int)(ihl + thl);  // :177
        fl = (th[3] >> 8) & 0xffu;
        src = ip[4];                                            // ip_dst.s_addr :213
        dst = ip[3];                                            // ip_src.s_addr :215
        sp = rsk::bswap16(th[0] >> 16);                         // ntohs(th_dport)
        dp = rsk::bswap16(th[0] & 0xffffu);                     // ntohs(th_sport)
        seq = rsk::bswap32(th[1]);
        ack = rsk::bswap32(th[2]);
        if ((fl & RSK_TH_SYN) && (a.flags & RSK_PARSE_HAS_ACK_POOL)) {  // :221-228
            if (a.flags & RSK_PARSE_IS_SERVER) {
                uint32_t t = src; src = dst; dst = t;
                t = sp; sp = dp; dp = t;
                t = seq; seq = ack; ack = t;
            }
            ps = RSK_PARSE_SYN;
            break;
        }
        const bool close = (fl & (RSK_TH_FIN | RSK_TH_RST)) != 0;
        if (payload_len < RSK_HASH_BUF_SIZE + 1 && !close) break;            // :232-234
        if (payload_len < -32) break;                          // cap2uv size_t wrap :240
        if (payload_len < 0) { ps = RSK_PARSE_MALFORMED; break; }
        if (payload_len + 32 > RSK_MAX_PKT_SIZE) break;        // cap2uv :240-244
        if ((uint64_t)payo + (uint64_t)payload_len > cl) { ps = RSK_PARSE_MALFORMED; break; }
        if (SLOT && payload_len > RSK_HEAD_SIZE) {  // decode reads frame [0, 32) and frame[8 + len]
            if (payo + 32u > av) { ps = RSK_PARSE_SLOT_SHORT; break; }
            const uint32_t len = pkt[payo + 8u];
            if (len != (uint32_t)RSK_ENC_HEAD_SIZE && (int)len < payload_len - 8 && payo + 9u + len > av) {
                ps = RSK_PARSE_SLOT_SHORT;
                break;
            }
        }
        seq += (uint32_t)payload_len;                           // :235
        plen = (uint32_t)payload_len;
        ps = RSK_PARSE_DELIVER;
        o = decode_frame(pkt + payo, payload_len, close, ks);
    } while (false);
    return ParseRes{ps, src, dst, sp, dp, seq, ack, fl, payo, plen, o};
}

__device__ __forceinline__ bool store_parse(const ParseArgs &a, const DecOut &d, uint64_t i, const ParseRes &r) {
    const bool keep = r.ps == RSK_PARSE_DELIVER || r.ps == RSK_PARSE_SYN;
    a.src[i] = keep ? r.src : 0u;
    a.dst[i] = keep ? r.dst : 0u;
    a.sp[i] = (uint16_t)(keep ? r.sp : 0u);
    a.dp[i] = (uint16_t)(keep ? r.dp : 0u);
    a.seq[i] = keep ? r.seq : 0u;
    a.ack[i] = keep ? r.ack : 0u;
    a.flag[i] = (uint8_t)(keep ? r.fl : 0u);
    a.pst[i] = (int8_t)r.ps;
    a.cpo[i] = (uint16_t)(keep ? r.payo : 0u);
    a.cpl[i] = (uint16_t)r.plen;
    store_dec(d, i, r.o);
    return r.o.st == RSK_RECV_VALID;
}

template <int L, bool SLOT>
__global__ __launch_bounds__(kBlock) void k_parse_decode(ParseArgs a, DecOut d, KeySched ks) {
    stage_tags(ks);
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    bool valid = false;
    if (i < a.n) {
        const uint8_t *pkt = SLOT ? a.cap + (uint64_t)a.slot * i : a.cap + a.cap_off[i];
        const uint32_t wl = a.wire_len[i], cl = a.cap_len[i];
        const uint32_t av = SLOT ? (cl < a.slot ? cl : a.slot) : cl;  // bytes present at pkt
        uint32_t hw[16];
        valid = store_parse(a, d, i, parse_one<L, SLOT, false>(a, pkt, wl, cl, av, hw, ks));
    }
    if (d.masks) compact_epilogue(d, valid, i);
}

// ---- RawTcp::syncInput (conn/RawTcp.cpp:262-276) + RConn::OnRecv: the loop thread's side of
// cap2uv's hand-off.  Record i (nread[i] bytes at rec + rec_off[i]) = TcpInfo::Encode's 21 B
// (src LE32 | dst LE32 | sp LE16 | dp LE16 | seq LE32 | ack LE32 | flag; TcpInfo.cpp:20-32,
// ConnInfo.cpp:12-20) then the frame.  A record of fewer than 21 bytes is not decoded (see
// rsk_syncinput_decode_batch); otherwise the frame (nread - 21 bytes) goes through decode_frame
// with is_tcp_close = HasCloseFlag() (TcpInfo.h:31-33).  One lane per record.
struct SyncArgs {
    const uint8_t *rec;
    const uint64_t *rec_off;
    const int32_t *nread;
    uint32_t *src, *dst;
    uint16_t *sp, *dp;
    uint32_t *seq, *ack;
    uint8_t *flag;
    int8_t *pst;
    uint16_t *cpo, *cpl;
    uint32_t n;
};

__global__ __launch_bounds__(kBlock) void k_syncinput_decode(SyncArgs a, DecOut d, KeySched ks) {
    stage_tags(ks);
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    bool valid = false;
    if (i < a.n) {
        const uint8_t *r = a.rec + a.rec_off[i];
        const int nr = a.nread[i];
        uint32_t w[6] = {0u, 0u, 0u, 0u, 0u, 0u};
        Dec o = {0, 0, 0, 0, 0, 0, 0, 0, RSK_RECV_DROP};
        const bool ok = nr >= RSK_TCPINFO_WIRE_SIZE;
        if (ok) {
            rsk::load_window<6>(r, r + (RSK_TCPINFO_WIRE_SIZE - 1), w);
            w[5] &= 0xffu;
            o = decode_frame(r + RSK_TCPINFO_WIRE_SIZE, nr - RSK_TCPINFO_WIRE_SIZE,
                             (w[5] & (RSK_TH_FIN | RSK_TH_RST)) != 0u, ks);
        }
        a.src[i] = w[0];
        a.dst[i] = w[1];
        a.sp[i] = (uint16_t)(w[2] & 0xffffu);
        a.dp[i] = (uint16_t)(w[2] >> 16);
        a.seq[i] = w[3];
        a.ack[i] = w[4];
        a.flag[i] = (uint8_t)w[5];
        a.pst[i] = (int8_t)(ok ? RSK_PARSE_DELIVER : RSK_PARSE_DROP);
        a.cpo[i] = (uint16_t)(ok ? RSK_TCPINFO_WIRE_SIZE : 0);
        a.cpl[i] = (uint16_t)(ok ? nr - RSK_TCPINFO_WIRE_SIZE : 0);
        store_dec(d, i, o);
        valid = o.st == RSK_RECV_VALID;
    }
    if (d.masks) compact_epilogue(d, valid, i);
}

// ---------------------------------------------------------------------------------------------
// Order-stable compaction of VALID indices
// ---------------------------------------------------------------------------------------------
// Exclusive scan of the per-block VALID counts -> offsets (one workgroup; 4 counts per thread per
// pass, wave scans via DPP-backed shuffles, one LDS exchange per pass), plus the total.
// ---------------------------------------------------------------------------------------------
// Capture filter: the pcap predicate BuildFilterStr builds (cap/cap_util.cpp:67-144), SURVEY §8f-4
// (primitive semantics: include/rsk_codec.h).  One lane per captured packet: a 64-B window of the
// link + network headers and a 16-B window at the transport header, both bounded by cap_len; every
// primitive checks the bytes it reads against cap_len and a short read rejects the packet.
// ---------------------------------------------------------------------------------------------
struct FiltArgs {
    const uint8_t *cap;
    const uint64_t *cap_off;
    const uint32_t *cap_len;
    uint8_t *match;
    uint32_t n;
};

template <int L>  // link header bytes: 14 (EN10MB) or 4 (NULL)
struct FPkt {
    uint32_t cl;
    uint32_t w[16];  // packet bytes [0, 64)
    uint32_t t[4];   // transport header bytes [0, 16) (IPv4: at L + 4 IHL; IPv6: at L + 40)
    int lt;          // 4, 6, 0; -1 = link header cut off
    __device__ __forceinline__ uint32_t b(int k) const { return (w[k >> 2] >> (8 * (k & 3))) & 0xffu; }
    __device__ __forceinline__ uint32_t tb(int k) const { return (t[k >> 2] >> (8 * (k & 3))) & 0xffu; }
    __device__ __forceinline__ uint32_t ihl4() const { return 4u * (b(L) & 15u); }
};

__device__ __forceinline__ bool is_tus(uint32_t pr) { return pr == 6u || pr == 17u || pr == 132u; }

template <int L>
__device__ __forceinline__ int fp_tcp(const FPkt<L> &k) {
    if (k.lt < 0) return -1;
    if (k.lt == 4) return k.cl < L + 10u ? -1 : (int)(k.b(L + 9) == 6u);
    if (k.lt == 6) {
        if (k.cl < L + 7u) return -1;
        const uint32_t nxt = k.b(L + 6);
        if (nxt == 6u) return 1;
        if (nxt != 44u) return 0;
        return k.cl < L + 41u ? -1 : (int)(k.b(L + 40) == 6u);
    }
    return 0;
}

template <int L, int OFF>
__device__ __forceinline__ int fp_addr(const FPkt<L> &k, uint32_t val) {
    if (k.lt < 0) return -1;
    if (k.lt != 4) return 0;
    if (k.cl < L + OFF + 4u) return -1;
    const uint32_t a = k.b(L + OFF) | (k.b(L + OFF + 1) << 8) | (k.b(L + OFF + 2) << 16) | (k.b(L + OFF + 3) << 24);
    return (int)(a == val);
}

template <int L>
__device__ __forceinline__ int fp_ports(const FPkt<L> &k, const rsk_port_list &pl, uint32_t dir) {
    if (pl.n_single == 0 && pl.n_range == 0) return 1;
    if (k.lt < 0) return -1;
    uint32_t port;
    if (k.lt == 4) {
        if (k.cl < L + 10u) return -1;
        if (!is_tus(k.b(L + 9)) || (((k.b(L + 6) & 0x1fu) << 8) | k.b(L + 7)) != 0u) return 0;
        if (k.cl < L + k.ihl4() + dir + 2u) return -1;
    } else if (k.lt == 6) {
        if (k.cl < L + 7u) return -1;
        if (!is_tus(k.b(L + 6))) return 0;
        if (k.cl < L + 40u + dir + 2u) return -1;
    } else {
        return 0;
    }
    port = dir ? ((k.tb(2) << 8) | k.tb(3)) : ((k.tb(0) << 8) | k.tb(1));
    bool hit = false;
    for (uint32_t q = 0; q < pl.n_single; ++q) hit |= port == pl.single[q];  // uniform loop bounds
    for (uint32_t q = 0; q < pl.n_range; ++q) hit |= port >= pl.range[q][0] && port <= pl.range[q][1];
    return (int)hit;
}

template <int L>
__device__ __forceinline__ int fp_syn(const FPkt<L> &k, bool want_set) {
    if (k.lt < 0) return -1;
    if (k.lt != 4) return 0;
    if (k.cl < L + 10u) return -1;
    if (k.b(L + 9) != 6u || (((k.b(L + 6) & 0x1fu) << 8) | k.b(L + 7)) != 0u) return 0;
    if (k.cl < L + k.ihl4() + 14u) return -1;
    const bool syn = (k.tb(13) & 2u) != 0u;
    return (int)(want_set ? syn : !syn);
}

template <int L>
__device__ __forceinline__ int fp_main(const FPkt<L> &k, const rsk_capture_filter &f, bool primed) {
    int r = fp_tcp(k);
    if (r != 1) return r;
    if (f.has_src_ip && (r = fp_addr<L, 12>(k, f.src_ip)) != 1) return r;
    if (f.has_dst_ip && (r = primed ? fp_addr<L, 12>(k, f.dst_ip) : fp_addr<L, 16>(k, f.dst_ip)) != 1) return r;
    if ((r = fp_ports(k, f.src_ports, 0u)) != 1) return r;
    return fp_ports(k, f.dst_ports, primed ? 0u : 2u);
}

// the filter's view of one captured packet: the 64-B window at the link header and the 16-B window
// at the transport header, both bounded by cap_len
template <int L>
__device__ __forceinline__ void filter_load(const uint8_t *p, uint32_t cl, FPkt<L> &k) {
    k.cl = cl;
    const uint8_t *last = p + (cl ? cl - 1u : 0u);
    if (cl) rsk::load_window16<16>(p, last, k.w);
    else
#pragma unroll
        for (int q = 0; q < 16; ++q) k.w[q] = 0;
    if (L == 14) {
        k.lt = cl < 14u ? -1 : ({ const uint32_t et = (k.b(12) << 8) | k.b(13); et == 0x0800u ? 4 : et == 0x86ddu ? 6 : 0; });
    } else {
        k.lt = cl < 4u ? -1 : (k.w[0] == 2u ? 4 : (k.w[0] == 24u || k.w[0] == 28u || k.w[0] == 30u) ? 6 : 0);
    }
    const uint32_t th = L + (k.lt == 6 ? 40u : k.ihl4());
#pragma unroll
    for (int q = 0; q < 4; ++q) k.t[q] = 0;
    if (k.lt > 0 && th < cl) rsk::load_window16<4>(p + th, last, k.t);
}

template <int L>
__device__ __forceinline__ bool filter_eval(const FPkt<L> &k, const rsk_capture_filter &f) {
    int r;
    if (!f.is_server) {
        r = fp_main(k, f, false);
    } else {  // ((syn) and F') or (F and (no syn))
        r = fp_syn(k, true);
        if (r == 1) r = fp_main(k, f, true);
        if (r == 0) {
            r = fp_main(k, f, false);
            if (r == 1) r = fp_syn(k, false);
        }
    }
    return r == 1;
}

template <int L>
__global__ __launch_bounds__(kBlock) void k_capture_filter(FiltArgs a, DecOut d, rsk_capture_filter f) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    bool m = false;
    if (i < a.n) {
        FPkt<L> k;
        filter_load<L>(a.cap + a.cap_off[i], a.cap_len[i], k);
        m = filter_eval(k, f);
        a.match[i] = m ? 1 : 0;
    }
    if (d.masks) compact_epilogue(d, m, i);
}

// Capture filter, then RawTcp::RawInput + RConn::OnRecv on the packets it passes, in one pass: the
// parse reuses the filter's 64-B header window.  A packet the filter rejects never reached RawInput
// in the reference (pcap drops it), so it gets match 0, RSK_PARSE_DROP and zero outputs.
template <int L>
__global__ __launch_bounds__(kBlock) void k_filter_parse_decode(ParseArgs a, DecOut d, KeySched ks, uint8_t *match,
                                                                rsk_capture_filter f) {
    stage_tags(ks);
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    bool valid = false;
    if (i < a.n) {
        const uint8_t *pkt = a.cap + a.cap_off[i];
        const uint32_t wl = a.wire_len[i], cl = a.cap_len[i];
        FPkt<L> k;
        filter_load<L>(pkt, cl, k);
        const bool m = filter_eval(k, f);
        match[i] = m ? 1 : 0;
        ParseRes r = {RSK_PARSE_DROP, 0, 0, 0, 0, 0, 0, 0, 0, 0, {0, 0, 0, 0, 0, 0, 0, 0, RSK_RECV_DROP}};
        if (m) r = parse_one<L, false, true>(a, pkt, wl, cl, cl, k.w, ks);
        valid = store_parse(a, d, i, r);
    }
    if (d.masks) compact_epilogue(d, valid, i);
}

// st[0]: the epoch counter; st[1 + t]: tile t's look-back word
__global__ __launch_bounds__(kBlock) void k_compact(const uint64_t *masks, uint32_t nw, unsigned long long *st,
                                                    uint32_t *valid_idx, uint32_t *n_valid, uint32_t *err,
                                                    uint32_t stall_tile) {
    __shared__ uint64_t ms[64];
    __shared__ uint32_t mex[64];
    __shared__ uint32_t pre, s_agg, s_epoch, s_to;
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint64_t mb = (uint64_t)blockIdx.x * 64u;
    const bool last = blockIdx.x == gridDim.x - 1u;
    if (w == 0u) {
        const uint32_t e0 = (uint32_t)__hip_atomic_load(st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t epoch = e0 % kCmpEpochMod + 1u;
        const uint64_t m = mb + lane < nw ? masks[mb + lane] : 0ull;
        const uint32_t c = (uint32_t)__popcll(m);
        uint32_t inc = c;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t v = __shfl_up(inc, off);
            if (lane >= (uint32_t)off) inc += v;
        }
        ms[lane] = m;
        mex[lane] = inc - c;
        const uint32_t agg = (uint32_t)__shfl((int)inc, 63);
        bool to = false;
        // stall_tile (tests only, rsk__inject_compact_stall): that tile publishes nothing, as a tile
        // that never gets scheduled would; the others must time out, flag it and not hang
        const uint32_t p = blockIdx.x == stall_tile ? 0u : cmp_lookback(st + 1, blockIdx.x, agg, lane, epoch, to);
        if (lane == 0u) {
            pre = p;
            s_agg = agg;
            s_epoch = epoch;
            s_to = to ? 1u : 0u;
            // wrong prefix: flag it (sticky); the last tile poisons the count (below)
            if (to) __hip_atomic_fetch_or(err, RSK_DEVERR_LOOKBACK, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    if (last && blockIdx.x != stall_tile) {
        // every earlier tile's word must be inclusive, of this epoch and untainted; the block's 256
        // threads poll them in parallel (bounded, as every spin here).  Only then is the count
        // trustworthy and the epoch advanced: every tile has read it by then.
        bool bad = s_to != 0u;
        for (uint32_t j = t; j + 1u < gridDim.x; j += kBlock)
            if (!cmp_wait_incl_clean(st + 1 + j, s_epoch)) bad = true;
        bad = __syncthreads_or(bad);
        if (t == 0u) {
            if (n_valid) *n_valid = bad ? 0xFFFFFFFFu : pre + s_agg;
            if (bad) __hip_atomic_fetch_or(err, RSK_DEVERR_LOOKBACK, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(st, (unsigned long long)s_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (!valid_idx) return;
#pragma unroll 4
    for (uint32_t r = 0; r < 16u; ++r) {
        const uint32_t j = 4u * r + w;  // wave w takes masks w, w + 4, ... of the tile
        const uint64_t m = ms[j];
        if ((m >> lane) & 1ull)
            valid_idx[pre + mex[j] + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)((mb + j) * 64u + lane);
    }
}

// ---------------------------------------------------------------------------------------------
// TcpInfo 21-B records, staged through LDS so the global stores are 16-B and coalesced
// ---------------------------------------------------------------------------------------------
struct TcpRecArgs {
    const uint32_t *src, *dst;
    const uint16_t *sp, *dp;
    const uint32_t *seq, *ack;
    const uint8_t *flag;
    uint8_t *rec;
    uint32_t n;
};

__global__ __launch_bounds__(kBlock) void k_tcpinfo_encode(TcpRecArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t s[kBlock * RSK_TCPINFO_WIRE_SIZE];
    const uint32_t t = threadIdx.x;
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + t;
    if (i < a.n) {
        uint8_t *r = s + RSK_TCPINFO_WIRE_SIZE * t;
        const uint32_t v32[4] = {a.src[i], a.dst[i], a.seq[i], a.ack[i]};
        const uint32_t v16[2] = {a.sp[i], a.dp[i]};
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            r[0 + b] = (uint8_t)(v32[0] >> (8 * b));
            r[4 + b] = (uint8_t)(v32[1] >> (8 * b));
            r[12 + b] = (uint8_t)(v32[2] >> (8 * b));
            r[16 + b] = (uint8_t)(v32[3] >> (8 * b));
        }
        r[8] = (uint8_t)v16[0];
        r[9] = (uint8_t)(v16[0] >> 8);
        r[10] = (uint8_t)v16[1];
        r[11] = (uint8_t)(v16[1] >> 8);
        r[20] = a.flag[i];
    }
    __syncthreads();
    const uint64_t first = (uint64_t)blockIdx.x * kBlock;
    const uint32_t cnt = (uint32_t)min<uint64_t>(kBlock, a.n - first);
    const uint32_t bytes = cnt * RSK_TCPINFO_WIRE_SIZE;
    uint8_t *out = a.rec + first * RSK_TCPINFO_WIRE_SIZE;
    if ((reinterpret_cast<uintptr_t>(out) & 15u) == 0) {
        for (uint32_t c = t; 16u * c < bytes; c += kBlock) {
            if (16u * c + 16u <= bytes) {
                *reinterpret_cast<uint4 *>(out + 16u * c) = *reinterpret_cast<const uint4 *>(s + 16u * c);
            } else {
                for (uint32_t b = 16u * c; b < bytes; ++b) out[b] = s[b];
            }
        }
    } else {
        for (uint32_t b = t; b < bytes; b += kBlock) out[b] = s[b];
    }
}

// ---------------------------------------------------------------------------------------------
// Single-packet shims (compatibility surface for the reference's per-call signatures)
// ---------------------------------------------------------------------------------------------
}  // namespace
struct ShimIO {
    uint8_t buf[64];   // in: op-specific input bytes; out: op-specific output bytes
    int32_t ret;
};
namespace {

__global__ void k_shim(ShimIO *io, int op, int len_arg, KeySched ks) {
    if (threadIdx.x != 0) return;
    uint8_t *b = io->buf;
    if (op == 0) {  // compute_hash: b[0] = data[0] -> b[8..16) = tag
        uint32_t t0, t1;
        rsk::md5_tag(ks, b[0], t0, t1);
        for (int k = 0; k < 4; ++k) { b[8 + k] = (uint8_t)(t0 >> (8 * k)); b[12 + k] = (uint8_t)(t1 >> (8 * k)); }
        io->ret = 8;
    } else if (op == 1) {  // hash_equal: b[0..8) tag, b[8] = data[0]
        uint32_t t0, t1;
        rsk::md5_tag(ks, b[8], t0, t1);
        uint32_t e0 = 0, e1 = 0;
        for (int k = 0; k < 4; ++k) { e0 |= (uint32_t)b[k] << (8 * k); e1 |= (uint32_t)b[4 + k] << (8 * k); }
        io->ret = (t0 == e0 && t1 == e1) ? 1 : 0;
    } else if (op == 2) {  // enc2buf: b[0]=cmd, b[1..9)=id, b[12..16)=conv, b[16..24)=key -> b[32..55)
        uint32_t id0 = 0, id1 = 0, conv = 0;
        uint64_t key = 0;
        for (int k = 0; k < 4; ++k) {
            id0 |= (uint32_t)b[1 + k] << (8 * k);
            id1 |= (uint32_t)b[5 + k] << (8 * k);
            conv |= (uint32_t)b[12 + k] << (8 * k);
        }
        for (int k = 0; k < 8; ++k) key |= (uint64_t)b[16 + k] << (8 * k);
        uint32_t H[8];
        head_words(b[0], id0, id1, conv, key, 0u, H);
        for (int q = 0; q < 23; ++q) {
            const int f = 8 + q;
            b[32 + q] = (uint8_t)(H[f >> 2] >> (8 * (f & 3)));
        }
        io->ret = RSK_ENC_HEAD_SIZE;
    } else {  // decodebuf: b[0..23) header, len_arg = buf_len -> fields in b[32..)
        const uint32_t len = b[0];
        if (len_arg < RSK_ENC_HEAD_SIZE || (int)len > len_arg) {
            io->ret = -1;
            return;
        }
        for (int q = 0; q < 23; ++q) b[32 + q] = b[q];
        io->ret = (int)len;
    }
}

// The context's 256 tags (see stage_tags): lane b = MD5(key || b)[8..15].
__global__ __launch_bounds__(256) void k_tag_table(KeySched ks, uint2 *tab) {
    uint32_t t0, t1;
    rsk::md5_tag(ks, threadIdx.x, t0, t1);
    tab[threadIdx.x] = make_uint2(t0, t1);
}

// ---------------------------------------------------------------------------------------------
// Synthetic workload generator
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64_at(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1u) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(kBlock) void k_fill_splitmix(uint8_t *dst, uint64_t nbytes, uint64_t seed) {
    const uint64_t nw = nbytes / 8u;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t w = (uint64_t)blockIdx.x * kBlock + threadIdx.x; w < nw; w += stride) {
        const uint64_t v = splitmix64_at(seed, w);
        if ((reinterpret_cast<uintptr_t>(dst) & 7u) == 0) {
            reinterpret_cast<uint64_t *>(dst)[w] = v;
        } else {
            for (int b = 0; b < 8; ++b) dst[8 * w + b] = (uint8_t)(v >> (8 * b));
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && nw * 8u < nbytes) {
        const uint64_t v = splitmix64_at(seed, nw);
        for (uint64_t b = nw * 8u; b < nbytes; ++b) dst[b] = (uint8_t)(v >> (8u * (b - nw * 8u)));
    }
}

// ---------------------------------------------------------------------------------------------
// Host helpers
// ---------------------------------------------------------------------------------------------
void build_sched(const uint8_t *key, uint32_t klen, KeySched &ks) {
    std::memset(&ks, 0, sizeof ks);
    uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    const uint32_t nfull = klen / 64u;  // blocks made only of key bytes
    auto words = [](const uint8_t *p, uint32_t (&m)[16]) {
        for (int w = 0; w < 16; ++w)
            m[w] = (uint32_t)p[4 * w] | ((uint32_t)p[4 * w + 1] << 8) | ((uint32_t)p[4 * w + 2] << 16) |
                   ((uint32_t)p[4 * w + 3] << 24);
    };
    for (uint32_t b = 0; b < nfull; ++b) {
        uint32_t m[16];
        words(key + 64u * b, m);
        rsk::md5_compress(st, m);
    }
    std::memcpy(ks.mid, st, sizeof st);
    uint8_t tail[128];
    std::memset(tail, 0, sizeof tail);
    const uint32_t rem = klen - 64u * nfull;
    if (rem) std::memcpy(tail, key + 64u * nfull, rem);
    tail[rem] = 0;      // payload[0] slot
    tail[rem + 1] = 0x80;
    const bool two = rem + 2u + 8u > 64u;
    const uint32_t tl = two ? 128u : 64u;
    const uint64_t bits = ((uint64_t)klen + 1u) * 8u;
    for (int k = 0; k < 8; ++k) tail[tl - 8 + k] = (uint8_t)(bits >> (8 * k));
    uint32_t m[16];
    words(tail, m);
    std::memcpy(ks.blk, m, sizeof m);
    if (two) {
        words(tail + 64, m);
        std::memcpy(ks.pad, m, sizeof m);
        for (int w = 1; w < 14; ++w) assert(ks.pad[w] == 0u);  // rsk::md5_tag reads words 0, 14, 15 only
    }
    ks.bword = (int32_t)(rem / 4u);
    ks.bshift = (int32_t)(8u * (rem % 4u));
    ks.two_blocks = two ? 1 : 0;
    rsk::md5_prefix_steps(ks.mid, ks.blk, ks.bword, ks.pre);  // rsk::md5_tag_bw starts at step bword
}

inline unsigned grid_for(uint64_t threads) { return (unsigned)((threads + kBlock - 1) / kBlock); }

}  // namespace

thread_local char rsk::g_last_error[256] = "";

namespace {

// Compaction workspace of stream s for n packets.  Layout, fixed by the buffer's capacity (not by
// n, so a call never reads another call's masks as look-back words): word 0 the epoch counter,
// words 1 .. T the look-back words of up to T tiles, then the per-wave ballot masks (T = (cap - 1)
// / 65: room for 64 T masks).  The decode grid has grid_for(n) blocks of 4 waves, one mask each.
struct Compact {
    uint64_t *masks = nullptr;
    unsigned long long *st = nullptr;
    uint32_t nw = 0, ntiles = 0;
};

int ensure_compact(rsk_ctx *c, uint32_t n, hipStream_t s, Compact &k) {
    k.nw = (uint32_t)(((n + kBlock - 1ull) / kBlock) * kWavesPerBlock);
    k.ntiles = (k.nw + 63u) / 64u;
    unsigned long long *p = nullptr;
    size_t cap = 0;
    int r = rsk::stream_compact(c, s, 1u + 65ull * k.ntiles, &p, &cap);
    if (r) return r;
    const size_t T = (cap - 1u) / 65u;
    k.st = p;
    k.masks = reinterpret_cast<uint64_t *>(p + 1u + T);
    return RSK_OK;
}

int run_compaction(rsk_ctx *c, const Compact &k, uint32_t *valid_idx, uint32_t *n_valid, hipStream_t s) {
    const uint32_t stall = c->compact_stall_tile.exchange(~0u, std::memory_order_relaxed);
    hipLaunchKernelGGL(k_compact, dim3(k.ntiles), dim3(kBlock), 0, s, k.masks, k.nw, k.st, valid_idx, n_valid,
                       c->err_dev, stall);
    return launch_check("k_compact");
}

bool filter_ports_bad(const rsk_capture_filter *f) {
    for (const rsk_port_list *pl : {&f->src_ports, &f->dst_ports}) {
        if (pl->n_single > RSK_FILTER_MAX_PORTS || pl->n_range > RSK_FILTER_MAX_PORTS) return true;
        for (uint32_t q = 0; q < pl->n_range; ++q)
            if (pl->range[q][0] >= pl->range[q][1]) return true;  // RPortList::AddPortRange
    }
    return false;
}

// An empty batch (n == 0) is a no-op that may pass null arrays; it still zeroes a given n_valid.
int empty_batch(rsk_ctx *c, uint32_t *n_valid, void *stream) {
    if (!n_valid) return RSK_OK;
    DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    hipError_t e = hipMemsetAsync(n_valid, 0, sizeof(uint32_t), (hipStream_t)stream);
    if (e != hipSuccess) { set_error("hipMemsetAsync", e); return RSK_EDEVICE; }
    return RSK_OK;
}

bool dec_out_ok(const rsk_decode_out *o) {
    return o && o->hlen && o->cmd && o->id && o->conv && o->conn_key && o->pay_off && o->pay_len &&
           o->status && ((reinterpret_cast<uintptr_t>(o->id) & 7u) == 0);
}

DecOut make_dec_out(const rsk_decode_out *o, uint64_t *masks) {
    DecOut d;
    d.hlen = o->hlen; d.cmd = o->cmd; d.id = o->id; d.conv = o->conv; d.key = o->conn_key;
    d.pay_off = o->pay_off; d.pay_len = o->pay_len; d.status = o->status;
    d.masks = masks;
    return d;
}

}  // namespace

// =============================================================================================
// C ABI
// =============================================================================================
namespace {
// Blocks of k_encode<.., GRP, SBW>: every wave that owns at least one packet (the last super-block
// may be partial: its wave wl owns packets iff wl * GRP < the packets left).
unsigned enc_grid(uint64_t n, uint32_t grp, uint32_t sbw) {
    const uint64_t per_sb = (uint64_t)sbw * 64u, rest = n % per_sb;
    const uint64_t waves = n / per_sb * sbw + std::min<uint64_t>(sbw, (rest + grp - 1) / grp);
    return (unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock);
}
}  // namespace

extern "C" {

const char *rsk_last_error(void) { return g_last_error; }

const char *rsk_version(void) { return "rsk 0.1 gfx950"; }


rsk_ctx *rsk_create(const uint8_t *key, uint32_t key_len, int device) {
    if (!key && key_len) { snprintf(g_last_error, sizeof g_last_error, "rsk_create: null key"); return nullptr; }
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0) {
        set_error("hipGetDeviceCount", e == hipSuccess ? hipErrorNoDevice : e);
        return nullptr;
    }
    if (device < 0 || device >= ndev) {
        snprintf(g_last_error, sizeof g_last_error, "rsk_create: device %d out of range", device);
        return nullptr;
    }
    rsk_ctx *c = new rsk_ctx();
    c->device = device;
    c->key.assign(key, key + key_len);
    build_sched(c->key.data(), key_len, c->ks);
    DeviceGuard g(device);
    hipStream_t s = nullptr;
    e = g.ok ? hipMalloc(&c->tag_dev, 256 * sizeof(uint2)) : hipErrorInvalidDevice;
    if (e == hipSuccess) e = hipMalloc(&c->err_dev, sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(c->err_dev, 0, sizeof(uint32_t));
    // the encode path statistic's host-mapped word (enc_path); without it every call takes the per-set
    // kernel unless a path is forced -- not an error
    // (word 1: the demux's table hint, rsk_demux.hip demux_pass)
    if (e == hipSuccess && hipHostMalloc(reinterpret_cast<void **>(&c->enc_stat_host), 2 * sizeof(uint32_t),
                                         hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
        c->enc_stat_host[0] = 0u;
        c->enc_stat_host[1] = 0u;
        if (hipHostGetDevicePointer(reinterpret_cast<void **>(&c->enc_stat_dev), c->enc_stat_host, 0) != hipSuccess) {
            (void)hipHostFree(c->enc_stat_host);
            c->enc_stat_host = nullptr;
            c->enc_stat_dev = nullptr;
        }
    }
    (void)hipGetLastError();  // a failed optional allocation above must not surface as a later launch error
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_tag_table, dim3(1), dim3(256), 0, s, c->ks, c->tag_dev);
        e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(s);
    }
    if (s) (void)hipStreamDestroy(s);
    if (e != hipSuccess) {
        set_error("rsk_create: tag table", e);
        if (c->tag_dev) (void)hipFree(c->tag_dev);
        if (c->err_dev) (void)hipFree(c->err_dev);
        if (c->enc_stat_host) (void)hipHostFree(c->enc_stat_host);
        delete c;
        return nullptr;
    }
    c->ks.tab = c->tag_dev;
    return c;
}

int rsk_set_tag_mode(rsk_ctx *c, int mode) {
    if (!c) return RSK_EINVAL;
    if (mode != RSK_TAG_MD5 && mode != RSK_TAG_TABLE) return RSK_EINVAL;
    c->ks.tag_mode = mode;
    return RSK_OK;
}

int rsk_get_tag_mode(const rsk_ctx *c) { return c ? c->ks.tag_mode : RSK_EINVAL; }

void rsk_destroy(rsk_ctx *c) {
    if (!c) return;
    DeviceGuard g(c->device);
    rsk::free_ws(c);
    if (c->shim_dev) (void)hipFree(c->shim_dev);
    if (c->tag_dev) (void)hipFree(c->tag_dev);
    if (c->err_dev) (void)hipFree(c->err_dev);
    if (c->enc_stat_host) (void)hipHostFree(c->enc_stat_host);
    if (c->shim_host) (void)hipHostFree(c->shim_host);
    if (c->shim_stream) (void)hipStreamDestroy(c->shim_stream);
    delete c;
}

int rsk_reserve(rsk_ctx *c, uint32_t n_max) { return rsk_reserve_stream(c, n_max, nullptr); }

int rsk_release_stream(rsk_ctx *c, void *stream) {
    if (!c) return RSK_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    return rsk::release_ws(c, (hipStream_t)stream);
}

// Encode path of this context's calls (rsk_codec.h): RSK_ENC_PATH_AUTO (chosen per call, enc_path),
// RSK_ENC_PATH_PER_SET (k_encode), RSK_ENC_PATH_TWO_PASS (k_encode_heads + k_encode_copy).
int rsk_set_encode_path(rsk_ctx *c, int path) {
    if (!c || path < RSK_ENC_PATH_AUTO || path > RSK_ENC_PATH_SHORT) return RSK_EINVAL;
    c->enc_path = path;
    return RSK_OK;
}

// Internal (tests, tools): the two-pass copy's packets per wave k (1, 2, 4; -1 = the output-stationary
// copy k_encode_os; 0 = from the sampled statistic, copy_k below).
int rsk__set_copy_k(rsk_ctx *c, int k) {
    if (!c || !(k == -1 || k == 0 || k == 1 || k == 2 || k == 4)) return RSK_EINVAL;
    c->copy_k = k;
    return RSK_OK;
}

// Internal (tests, bench): packets per copy wave of the context's last two-pass encode (0 before any).
int rsk__last_copy_k(const rsk_ctx *c) { return c ? c->enc_last_k.load(std::memory_order_relaxed) : RSK_EINVAL; }

// Internal (tests, tools): the two-pass form in chunks of `packets` (0: the whole batch in one pass each)
int rsk__set_two_pass_chunk(rsk_ctx *c, uint32_t packets) {
    if (!c) return RSK_EINVAL;
    c->tp_chunk = packets;
    return RSK_OK;
}

// Internal (tests, bench): the path the context's last rsk_encode_batch took (RSK_ENC_PATH_PER_SET,
// _TWO_PASS or _SHORT: 1, 2 or 3; 0 before any).
int rsk__last_encode_path(const rsk_ctx *c) { return c ? c->enc_last_path.load(std::memory_order_relaxed) : RSK_EINVAL; }

// Internal (tests): the next compaction launch of this context runs with tile `tile` publishing
// nothing (a stalled tile), to exercise the look-back timeout, the sticky flag and the recovery.
int rsk__inject_compact_stall(rsk_ctx *c, uint32_t tile) {
    if (!c) return RSK_EINVAL;
    c->compact_stall_tile = tile;
    return RSK_OK;
}

// Internal (CPU tests): the per-lane tag path of the device kernels (KeySched from build_sched,
// rsk::md5_tag_lane: the payload-word-specialised step schedule starting from KeySched::pre) run on
// the host, so its schedule is checked against the oracle without a GPU.
int rsk__host_tag(const uint8_t *key, uint32_t key_len, uint32_t b, uint32_t *t01) {
    if ((!key && key_len) || !t01 || b > 255u) return RSK_EINVAL;
    KeySched ks;
    build_sched(key, key_len, ks);
    rsk::md5_tag_lane(ks, b, t01[0], t01[1]);
    return RSK_OK;
}

int rsk_check_device_errors(rsk_ctx *c, uint32_t *flags) {
    if (!c) return RSK_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    uint32_t f = 0;
    // the context's streams only: the flags are raised by look-back kernels, which run on
    // streams the context has scratch for; other contexts' and torch's work is not waited for
    hipError_t e = rsk::sync_ctx_streams(c);
    if (e == hipSuccess) e = hipMemcpy(&f, c->err_dev, sizeof f, hipMemcpyDeviceToHost);
    if (e == hipSuccess && f) e = hipMemset(c->err_dev, 0, sizeof f);
    if (e != hipSuccess) { set_error("rsk_check_device_errors", e); return RSK_EDEVICE; }
    if (flags) *flags = f;
    if (!f) return RSK_OK;
    rsk::invalidate_compact(c);
    snprintf(g_last_error, sizeof g_last_error,
             "device error flags 0x%x (RSK_DEVERR_LOOKBACK: a look-back gave up; RSK_DEVERR_TABLE: a demux "
             "probe found no slot)", f);
    return RSK_EDEVICE;
}

int rsk_forget_captures(rsk_ctx *c) {
    if (!c) return RSK_EINVAL;
    c->captured.store(false, std::memory_order_relaxed);
    return RSK_OK;
}

int rsk_reserve_stream(rsk_ctx *c, uint32_t n_max, void *stream) {
    if (!c) return RSK_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    Compact ck;
    const int r = ensure_compact(c, n_max, (hipStream_t)stream, ck);
    // the two-pass encode's header records (32 B per packet), for a context that encodes: held to the
    // two-pass path, or AUTO with an encode call behind it (a decode- or demux-only context
    // does not pay 32 B per packet for them).  A capture cannot allocate them: without this reserve
    // bench.py's graph captured the per-set kernel (r05z kernel trace).
    const bool encodes = c->enc_path == RSK_ENC_PATH_TWO_PASS ||
                         (c->enc_path == RSK_ENC_PATH_AUTO && c->enc_last_path.load(std::memory_order_relaxed) != 0);
    if (r || n_max < kTwoPassMinPackets || !encodes) return r;
    // A failed allocation is not an error: eager calls allocate on demand, a captured call
    // takes the per-set kernel.
    void *p = nullptr;
    // (and the two-pass wire build's: 96 B per packet of one 2^20-packet chunk, k_wire_heads)
    const uint64_t wire_rec = 96ull * std::min<uint64_t>(n_max, 1ull << 20);
    if (rsk::stream_ws(c, (hipStream_t)stream, rsk::WS_ENC, std::max<uint64_t>(enc_ws_bytes(n_max), wire_rec), &p) !=
        RSK_OK) {
        (void)hipGetLastError();
        g_last_error[0] = 0;
    }
    return RSK_OK;
}

// The batch statistic behind AUTO (enc_sample: k_encode_heads in every two-pass call, k_enc_sample
// behind every other uncaptured call of >= kTwoPassMinPackets packets; enc_path samples before the
// first such call on a context).  Every path gives identical bytes.
// The context's last sampled mean payload (bit 31 set: valid), or 0.
static uint32_t sampled_mean(const rsk_ctx *c) {
    const uint32_t s = c->enc_stat_host ? __atomic_load_n(c->enc_stat_host, __ATOMIC_RELAXED) : 0u;
    return s;
}

// packets per copy wave of the two-pass form: forced (rsk__set_copy_k), else by the sampled mean payload
static int copy_k(rsk_ctx *c) {
    if (c->copy_k) return c->copy_k;
    const uint32_t s = sampled_mean(c);
    const uint32_t mean = (s & kStatValid) ? s & kStatMean : 1400u;
    // byte-packed frames of the four-packet range: the output-stationary copy (C4 0.420 vs 0.429 ms);
    // long ones keep the one-packet waves (C3 byte-packed 2.59 vs 3.01 ms: profiles/r06_layouts_os.json)
    if ((s & kStatValid) && (s & kStatPacked) && mean < kAutoK4Below && c->tp_chunk == 0u) return -1;
    return mean < kAutoK4Below ? 4 : mean < kAutoK2Below ? 2 : 1;
}

// Encode path per call: the context's forced path (rsk_set_encode_path), else AUTO's table above.
// The first AUTO call of >= kTwoPassMinPackets packets on a context samples its own batch and waits
// for an event behind that one 64-thread launch on its stream, so it already takes the table's path
// (without that, back-to-back eager calls ran the per-set kernel until the first sample landed: 5
// calls in gpurun_out/r05f1/c3).  The event, not the stream: nothing queued on the
// stream after the sample is waited for, and a failed wait is the call's error.  A capture never
// waits: it takes the per-set kernel when no sample exists.  Returns the path, or RSK_EDEVICE.
static int enc_path(rsk_ctx *c, uint32_t n, const uint16_t *pay_len, hipStream_t st,
                    const uint64_t *frame_off = nullptr, uint32_t pad = 0u) {
    if (c->enc_path) return c->enc_path;
    // Not on the legacy NULL stream: work there synchronises with every blocking stream, so
    // the wait could join -- and invalidate -- another stream's capture; its first call takes the
    // per-set kernel and the sample launched behind it serves the next calls.  Elsewhere the wait runs
    // with this thread's capture mode relaxed, so another thread's global-mode capture does not turn it
    // into an error (the event and the sample are on this call's own, uncaptured stream).
    if (n >= kTwoPassMinPackets && c->enc_stat_dev && !(sampled_mean(c) & kStatValid) && st != nullptr &&
        !rsk::capturing(st)) {
        hipLaunchKernelGGL(k_enc_sample, dim3(1), dim3(64), 0, st, pay_len, n, c->enc_stat_dev, frame_off, pad);
        hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
        const bool swapped = hipThreadExchangeStreamCaptureMode(&mode) == hipSuccess;
        hipEvent_t ev = nullptr;
        hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventRecord(ev, st);
        if (e == hipSuccess) e = hipEventSynchronize(ev);
        if (ev) (void)hipEventDestroy(ev);
        if (swapped) (void)hipThreadExchangeStreamCaptureMode(&mode);  // restore the caller's mode
        if (e != hipSuccess) { set_error("enc_path: waiting for the batch sample", e); return RSK_EDEVICE; }
    }
    const uint32_t s = sampled_mean(c);
    if (n < kTwoPassMinPackets || !(s & kStatValid)) return RSK_ENC_PATH_PER_SET;
    const uint32_t mean = s & kStatMean;
    return mean <= kAutoShortMax      ? RSK_ENC_PATH_SHORT
           : mean < kAutoPerSetBelow  ? RSK_ENC_PATH_PER_SET
           : mean < kAutoShortBelow   ? RSK_ENC_PATH_SHORT
                                      : RSK_ENC_PATH_TWO_PASS;
}

// k_encode_os's persistent grid: every workgroup resident at once (its waves own static block ranges,
// so a workgroup that waited for a slot would run its range after the others: a tail)
static unsigned os_grid(int device) {
    static std::atomic<unsigned> cached[64];
    const int d = device >= 0 && device < 64 ? device : 0;
    unsigned g = cached[d].load(std::memory_order_relaxed);
    if (g) return g;
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_encode_os<3>, kBlock, 0) != hipSuccess || per_cu < 1)
        per_cu = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus < 1) cus = 256;
    (void)hipGetLastError();
    g = (unsigned)(per_cu * cus);
    cached[d].store(g, std::memory_order_relaxed);
    return g;
}

int rsk_encode_batch(rsk_ctx *c, uint32_t n, const rsk_encode_in *in, const rsk_encode_out *out,
                     void *stream) {
    if (!c || !in || !out) return RSK_EINVAL;
    if (n == 0) return RSK_OK;
    if (n > RSK_MAX_BATCH) return RSK_EINVAL;  // grids of one lane per packet
    if (!in->payload_arena || !in->pay_off || !in->pay_len || !in->cmd || !in->conv || !in->conn_key ||
        !out->frame_arena || !out->frame_off || !out->status)
        return RSK_EINVAL;
    if (in->id && (reinterpret_cast<uintptr_t>(in->id) & 7u)) return RSK_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    EncArgs a;
    a.payload = in->payload_arena; a.pay_off = in->pay_off; a.pay_len = in->pay_len; a.cmd = in->cmd;
    a.conv = in->conv; a.conn_key = in->conn_key; a.id = in->id;
    a.frame = out->frame_arena; a.frame_off = out->frame_off; a.status = out->status;
    std::memcpy(&a.id_lo, in->id_uniform, 4);
    std::memcpy(&a.id_hi, in->id_uniform + 4, 4);
    a.n = n;
    a.pad = (out->flags & RSK_ENC_ZERO_PAD128) ? 7u : (out->flags & RSK_ENC_ZERO_PAD16) ? 4u : 0u;
    const uint64_t waves = (n + 63ull) / 64ull;
    const unsigned grid = (unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock);
    hipStream_t st = (hipStream_t)stream;
    const dim3 gd(grid), bd(kBlock);
    (void)gd;
    const int path = enc_path(c, n, in->pay_len, st, out->frame_off, a.pad);
    if (path < 0) return path;
    if (path == RSK_ENC_PATH_TWO_PASS) {
        // the two-pass form (batches of long frames): header records, then one wave per packet
        void *hp = nullptr;
        if (rsk::stream_ws_if(c, st, rsk::WS_ENC, enc_ws_bytes(n), &hp) == RSK_OK) {
            const int ck = copy_k(c);
            if (ck < 0) {  // frames back to back: the output-stationary copy (k_encode_os)
                OsMap m;
                m.bfirst = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(hp) + 32ull * n);
                m.ctl = m.bfirst + os_bcap(n);
                m.bcap = os_bcap(n);
                m.epoch = ++c->os_epoch;
                hipLaunchKernelGGL(k_encode_heads_os<0>, dim3(grid_for(n)), bd, 0, st, a, c->ks, static_cast<uint4 *>(hp),
                                   c->enc_stat_dev, (uint64_t)n, m);
                hipLaunchKernelGGL(k_encode_os<3>, dim3(os_grid(c->device)), bd, 0, st, a, static_cast<const uint4 *>(hp),
                                   (uint64_t)n, m.bfirst, m.ctl, m.epoch);
                c->enc_last_path.store(2, std::memory_order_relaxed);
                c->enc_last_k.store(-1, std::memory_order_relaxed);
                return launch_check("k_encode_heads_os / k_encode_os");
            }
            // chunked (rsk__set_two_pass_chunk): heads then copy per chunk, so a chunk's records and
            // first payload lines may still be in the Infinity Cache when its copy reads them
            const uint64_t chunk = c->tp_chunk ? c->tp_chunk : (uint64_t)n;
            for (uint64_t c0 = 0; c0 < n; c0 += chunk) {
                EncArgs ac = a;
                ac.n = (uint32_t)std::min<uint64_t>(n, c0 + chunk);
                hipLaunchKernelGGL(k_encode_heads<0>, dim3(grid_for(ac.n - c0)), bd, 0, st, ac, c->ks,
                                   static_cast<uint4 *>(hp), c0 == 0 ? c->enc_stat_dev : nullptr, c0, (uint64_t)n);
                for (uint64_t b0 = c0; b0 < ac.n; b0 += kCopyMaxPackets) {  // one launch up to 2^25 packets
                    const uint64_t m = ac.n - b0 < kCopyMaxPackets ? ac.n - b0 : kCopyMaxPackets;
                    const dim3 cg((unsigned)((m + 4ull * ck - 1ull) / (4ull * ck)));
                    const uint32_t *hr = static_cast<const uint32_t *>(hp);
                    const uint64_t nr = n;
                    if (ck == 2) hipLaunchKernelGGL((k_encode_copy<3, 2>), cg, bd, 0, st, ac, hr, b0, nr);
                    else if (ck == 4) hipLaunchKernelGGL((k_encode_copy<3, 4>), cg, bd, 0, st, ac, hr, b0, nr);
                    else hipLaunchKernelGGL((k_encode_copy<3, 1>), cg, bd, 0, st, ac, hr, b0, nr);
                }
            }
            c->enc_last_path.store(2, std::memory_order_relaxed);
            c->enc_last_k.store(ck, std::memory_order_relaxed);
            return launch_check("k_encode_heads / k_encode_copy");
        }
        g_last_error[0] = 0;  // no records (a capture that would grow them, or no memory): one pass
    }
    if (path == RSK_ENC_PATH_SHORT) {
        // batches of short frames: the per-set kernel with every set on the flat chunk list, compiled
        // without the per-packet copy (fewer VGPRs, more waves per SIMD; profiles/r04ac_short_path.json)
        hipLaunchKernelGGL((k_encode<19, 4, 2, 8, 1024>), dim3(enc_grid(n, 8, 1024)), bd, 0, st, a, c->ks);
        c->enc_last_path.store(RSK_ENC_PATH_SHORT, std::memory_order_relaxed);
    } else {
        // the per-set kernel: per-wave hybrid (flat chunk list for short frames, with the tag behind the
        // first chunk loads; software-pipelined one-load DPP per-packet copy, 4 packets per batch, for
        // the rest), tag in the copy loop for long-frame sets, per-set store policy
        hipLaunchKernelGGL((k_encode<11, 4, 4, 8, 1024>), dim3(enc_grid(n, 8, 1024)), bd, 0, st, a, c->ks);
        c->enc_last_path.store(RSK_ENC_PATH_PER_SET, std::memory_order_relaxed);
    }
    // the statistic for the next call, on every call this path takes (a sample every 256th
    // call left a context that switched from short to long frames on the flat-only kernel for up to 255
    // calls), unless the call is being captured (a graph replays the path it was captured with).  One
    // 64-thread launch behind the encode: the per-set kernel itself carries no pointer for it (one more
    // argument cost C4 12 % through SGPR spills, gpurun_out/r04o).
    if (c->enc_path == 0 && c->enc_stat_dev && n >= kTwoPassMinPackets && !rsk::capturing(st))
        hipLaunchKernelGGL(k_enc_sample, dim3(1), dim3(64), 0, st, in->pay_len, n, c->enc_stat_dev, out->frame_off,
                           a.pad);
    return launch_check("k_encode");
}

// The wire build's choice (round 6; tools/path_threshold.py --wire raw4 / eth, profiles/r06_wire_paths.json):
// under AUTO the per-set wire kernels below a mean payload of kWireTwoPassFrom, and for Ethernet packets
// from kWireEthPerSetFrom (4M x 1400 B: per-set 2.285, two-pass 2.296-2.373 ms); the two-pass form
// otherwise, with 4 packets per copy wave, RAW4 from kWireK2From 2 (4M x 1400 B: 2.200 vs 2.230 for 1,
// 2.288 per-set).
constexpr uint32_t kWireTwoPassFrom = 160;
constexpr uint32_t kWireEthPerSetFrom = 1300;
constexpr uint32_t kWireK2From = 1080;
constexpr uint64_t kWireChunk = 1ull << 20;
static int wire_path(rsk_ctx *c, uint32_t n, const uint16_t *pay_len, hipStream_t st, bool eth) {
    if (c->enc_path) return c->enc_path == RSK_ENC_PATH_TWO_PASS ? RSK_ENC_PATH_TWO_PASS : RSK_ENC_PATH_PER_SET;
    const int ep = enc_path(c, n, pay_len, st);  // the first-call sample, and the statistic
    if (ep < 0) return ep;
    const uint32_t s = sampled_mean(c);
    if (n < kTwoPassMinPackets || !(s & kStatValid)) return RSK_ENC_PATH_PER_SET;
    const uint32_t mean = s & kStatMean;
    return mean < kWireTwoPassFrom || (eth && mean >= kWireEthPerSetFrom) ? RSK_ENC_PATH_PER_SET
                                                                          : RSK_ENC_PATH_TWO_PASS;
}
static int wire_k(rsk_ctx *c, bool eth) {
    if (c->copy_k) return c->copy_k;
    const uint32_t s = sampled_mean(c);
    const uint32_t mean = (s & kStatValid) ? s & kStatMean : 1400u;
    return eth || mean < kWireK2From ? 4 : 2;
}

int rsk_encode_wire_batch(rsk_ctx *c, uint32_t n, const rsk_encode_in *in, const rsk_wire_in *wire,
                          const rsk_encode_out *out, void *stream) {
    if (!c || !in || !wire || !out) return RSK_EINVAL;
    if (n == 0) return RSK_OK;
    if (n > RSK_MAX_BATCH) return RSK_EINVAL;  // grids of one lane per packet
    if (!in->payload_arena || !in->pay_off || !in->pay_len || !in->cmd || !in->conv || !in->conn_key ||
        !out->frame_arena || !out->frame_off || !out->status || !wire->src || !wire->dst || !wire->sp ||
        !wire->dp || !wire->seq || !wire->ack || !wire->flag || !wire->ip_id)
        return RSK_EINVAL;
    if (in->id && (reinterpret_cast<uintptr_t>(in->id) & 7u)) return RSK_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    EncArgs a;
    a.payload = in->payload_arena; a.pay_off = in->pay_off; a.pay_len = in->pay_len; a.cmd = in->cmd;
    a.conv = in->conv; a.conn_key = in->conn_key; a.id = in->id;
    a.frame = out->frame_arena; a.frame_off = out->frame_off; a.status = out->status;
    std::memcpy(&a.id_lo, in->id_uniform, 4);
    std::memcpy(&a.id_hi, in->id_uniform + 4, 4);
    a.n = n;
    a.pad = (out->flags & RSK_ENC_ZERO_PAD128) ? 7u : (out->flags & RSK_ENC_ZERO_PAD16) ? 4u : 0u;
    WireArgs w;
    w.src = wire->src; w.dst = wire->dst; w.sp = wire->sp; w.dp = wire->dp; w.seq = wire->seq;
    w.ack = wire->ack; w.flag = wire->flag; w.ip_id = wire->ip_id;
    uint8_t eth[16] = {0};
    std::memcpy(eth, wire->eth, 14);
    std::memcpy(w.eth, eth, 16);
    const unsigned grid = enc_grid(n, 8, 1024);
    const hipStream_t st = (hipStream_t)stream;
    const bool eth14 = wire->with_eth != 0;
    // the encode path the context is held to (rsk_set_encode_path: two-pass, or else the per-set wire
    // kernels), or AUTO's wire table (wire_path): the two-pass form -- k_wire_heads (header images,
    // 80 / 96-B records in the stream's scratch) + k_wire_copy with 1, 2 or 4 packets per copy wave
    // (round 6) -- from a mean payload of 160 B (Ethernet: up to 1300 B), the per-set kernels otherwise
    const int path = wire_path(c, n, in->pay_len, st, eth14);
    if (path < 0) return path;
    if (path == RSK_ENC_PATH_TWO_PASS) {
        void *hp = nullptr;
        const uint64_t recb = 16ull * (eth14 ? WireRec<14>::NC : WireRec<0>::NC);  // 96 / 80 B per packet
        // header pass then copy per chunk of kWireChunk packets: one chunk's records (80 / 96 MB at 1M)
        // stay in the Infinity Cache until its copy reads them (a whole C3 batch's, 320 MB, do not)
        const uint64_t chunk = n < kWireChunk ? (uint64_t)n : kWireChunk;
        if (rsk::stream_ws_if(c, st, rsk::WS_ENC, recb * chunk, &hp) == RSK_OK) {
            const int ck = wire_k(c, eth14);
            const dim3 bd(kBlock);
            uint4 *rec = static_cast<uint4 *>(hp);
            for (uint64_t c0 = 0; c0 < n; c0 += chunk) {
                EncArgs ac = a;
                ac.n = (uint32_t)std::min<uint64_t>(n, c0 + chunk);
                const uint64_t m = ac.n - c0;
                uint32_t *stat = c0 == 0 ? c->enc_stat_dev : nullptr;
                if (eth14) hipLaunchKernelGGL(k_wire_heads<14>, dim3(grid_for(m)), bd, 0, st, ac, w, c->ks, rec, stat, c0, chunk);
                else hipLaunchKernelGGL(k_wire_heads<0>, dim3(grid_for(m)), bd, 0, st, ac, w, c->ks, rec, stat, c0, chunk);
                const dim3 cg((unsigned)((m + 4ull * ck - 1ull) / (4ull * ck)));  // m <= kWireChunk: one launch
#define RSK_WCOPY(E, K) hipLaunchKernelGGL((k_wire_copy<E, 3, K>), cg, bd, 0, st, ac, rec, c0, c0, chunk)
                if (eth14) {
                    if (ck == 2) RSK_WCOPY(14, 2); else if (ck == 4) RSK_WCOPY(14, 4); else RSK_WCOPY(14, 1);
                } else {
                    if (ck == 2) RSK_WCOPY(0, 2); else if (ck == 4) RSK_WCOPY(0, 4); else RSK_WCOPY(0, 1);
                }
#undef RSK_WCOPY
            }
            c->enc_last_path.store(RSK_ENC_PATH_TWO_PASS, std::memory_order_relaxed);
            c->enc_last_k.store(ck, std::memory_order_relaxed);
            return launch_check("k_wire_heads / k_wire_copy");
        }
        g_last_error[0] = 0;  // no records (a capture that would grow them, or no memory): one pass
    }
#define RSK_WIRE(E, M, PU, U) hipLaunchKernelGGL((k_encode_wire<E, M, PU, U>), dim3(grid), dim3(kBlock), 0, st, a, w, c->ks)
#define RSK_WIRE4(E, M, PU, U) hipLaunchKernelGGL((k_encode_wire_w4<E, M, PU, U>), dim3(grid), dim3(kBlock), 0, st, a, w, c->ks)
    // the per-set kernels: per-packet half (DPP copy, 8 packets per iteration, tag + payload prefix in
    // the copy loop for long-frame sets, 4 waves/SIMD) then the flat half
    if (eth14) { RSK_WIRE4(14, 5, 8, 2); RSK_WIRE(14, 4, 2, 2); }
    else { RSK_WIRE4(0, 5, 8, 2); RSK_WIRE(0, 4, 2, 2); }
#undef RSK_WIRE
#undef RSK_WIRE4
    c->enc_last_path.store(RSK_ENC_PATH_PER_SET, std::memory_order_relaxed);
    // the statistic for the next call's choice (as rsk_encode_batch)
    if (c->enc_path == 0 && c->enc_stat_dev && n >= kTwoPassMinPackets && !rsk::capturing(st))
        hipLaunchKernelGGL(k_enc_sample, dim3(1), dim3(64), 0, st, in->pay_len, n, c->enc_stat_dev,
                           (const uint64_t *)nullptr, 0u);
    return launch_check("k_encode_wire");
}

int rsk_decode_batch(rsk_ctx *c, uint32_t n, const uint8_t *frame_arena, const uint64_t *frame_off,
                     const uint16_t *frame_len, const uint8_t *is_tcp_close, const rsk_decode_out *out,
                     void *stream) {
    if (!c || !out) return RSK_EINVAL;
    if (n == 0) return empty_batch(c, out->n_valid, stream);
    if (n > RSK_MAX_BATCH) return RSK_EINVAL;  // grids of one lane per packet
    if (!frame_arena || !frame_off || !frame_len || !dec_out_ok(out)) return RSK_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    const bool compact = out->valid_idx || out->n_valid;
    Compact ck;
    if (compact) {
        int r = ensure_compact(c, n, (hipStream_t)stream, ck);
        if (r) return r;
    }
    DecArgs a{frame_arena, frame_off, frame_len, is_tcp_close, n};
    DecOut d = make_dec_out(out, ck.masks);
    hipLaunchKernelGGL(k_decode, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, a, d, c->ks);
    int r = launch_check("k_decode");
    if (r || !compact) return r;
    return run_compaction(c, ck, out->valid_idx, out->n_valid, (hipStream_t)stream);
}

int rsk_encode_headers_batch(rsk_ctx *c, uint32_t n, const rsk_encode_hdr_in *in, uint8_t *hdr, int32_t *status,
                             void *stream) {
    if (!c || !in) return RSK_EINVAL;
    if (n == 0) return RSK_OK;
    if (n > RSK_MAX_BATCH) return RSK_EINVAL;  // grids of one lane per packet
    if (!in->first_byte || !in->pay_len || !in->cmd || !in->conv || !in->conn_key || !hdr || !status)
        return RSK_EINVAL;
    if ((reinterpret_cast<uintptr_t>(hdr) & 15u) || (in->id && (reinterpret_cast<uintptr_t>(in->id) & 7u)))
        return RSK_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    EncHdrArgs a;
    a.b0 = in->first_byte; a.pay_len = in->pay_len; a.cmd = in->cmd; a.conv = in->conv; a.conn_key = in->conn_key;
    a.id = in->id; a.hdr = hdr; a.status = status; a.n = n;
    std::memcpy(&a.id_lo, in->id_uniform, 4);
    std::memcpy(&a.id_hi, in->id_uniform + 4, 4);
    hipLaunchKernelGGL(k_encode_hdr, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, a, c->ks);
    return launch_check("k_encode_hdr");
}

int rsk_decode_headers_batch(rsk_ctx *c, uint32_t n, const uint8_t *hdr, const uint16_t *frame_len,
                             const uint8_t *is_tcp_close, const rsk_decode_out *out, void *stream) {
    if (!c || !out) return RSK_EINVAL;
    if (n == 0) return empty_batch(c, out->n_valid, stream);
    if (n > RSK_MAX_BATCH) return RSK_EINVAL;  // grids of one lane per packet
    if (!hdr || !frame_len || !dec_out_ok(out)) return RSK_EINVAL;
    if (reinterpret_cast<uintptr_t>(hdr) & 15u) return RSK_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    const bool compact = out->valid_idx || out->n_valid;
    Compact ck;
    if (compact) {
        int r = ensure_compact(c, n, (hipStream_t)stream, ck);
        if (r) return r;
    }
    DecArgs a{hdr, nullptr, frame_len, is_tcp_close, n};
    DecOut d = make_dec_out(out, ck.masks);
    hipLaunchKernelGGL(k_decode_hdr, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, a, d, c->ks);
    int r = launch_check("k_decode_hdr");
    if (r || !compact) return r;
    return run_compaction(c, ck, out->valid_idx, out->n_valid, (hipStream_t)stream);
}

// Host: the 32-B decode slot of one received frame (EncHead::DecodeBuf reads frame[8] = len; the
// hashed byte is frame[8 + len] when that lies inside the frame, RConn.cpp:64-75).
void rsk_stage_decode_header(const uint8_t *frame, int nread, uint8_t *slot) {
    const int k = nread < 0 ? 0 : (nread < 32 ? nread : 32);
    std::memcpy(slot, frame, (size_t)k);
    if (k < 32) std::memset(slot + k, 0, (size_t)(32 - k));
    if (nread > 8) {
        const int at = 8 + frame[8];
        if (at < nread) slot[31] = frame[at];
    }
}

namespace {
int parse_decode(rsk_ctx *c, uint32_t n, const uint8_t *cap_arena, const uint64_t *cap_off, uint32_t slot,
                 const uint32_t *wire_len, const uint32_t *cap_len, int datalink, int flags,
                 const rsk_tcpinfo_out *tcp, const rsk_decode_out *dec, void *stream) {
    if (!c || !tcp || !dec) return RSK_EINVAL;
    if (datalink != RSK_DLT_EN10MB && datalink != RSK_DLT_NULL) return RSK_EINVAL;  // RawTcp.cpp:161-164
    if (n == 0) return empty_batch(c, dec->n_valid, stream);
    if (n > RSK_MAX_BATCH) return RSK_EINVAL;  // grids of one lane per packet
    if (!cap_arena || (!slot && !cap_off) || !wire_len || !cap_len || !dec_out_ok(dec)) return RSK_EINVAL;
    if (!tcp->src || !tcp->dst || !tcp->sp || !tcp->dp || !tcp->seq || !tcp->ack || !tcp->flag ||
        !tcp->parse_status || !tcp->cap_pay_off || !tcp->cap_pay_len)
        return RSK_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    const bool compact = dec->valid_idx || dec->n_valid;
    Compact ck;
    if (compact) {
        int r = ensure_compact(c, n, (hipStream_t)stream, ck);
        if (r) return r;
    }
    ParseArgs a;
    a.cap = cap_arena; a.cap_off = cap_off; a.wire_len = wire_len; a.cap_len = cap_len;
    a.src = tcp->src; a.dst = tcp->dst; a.sp = tcp->sp; a.dp = tcp->dp; a.seq = tcp->seq; a.ack = tcp->ack;
    a.flag = tcp->flag; a.pst = tcp->parse_status; a.cpo = tcp->cap_pay_off; a.cpl = tcp->cap_pay_len;
    a.datalink = datalink; a.flags = flags; a.n = n;
    DecOut d = make_dec_out(dec, ck.masks);
    a.slot = slot;
    const bool sl = slot != 0;
    const hipStream_t st = (hipStream_t)stream;
    const dim3 gd(grid_for(n)), bd(kBlock);
    if (datalink == RSK_DLT_EN10MB) {
        if (sl) hipLaunchKernelGGL((k_parse_decode<14, true>), gd, bd, 0, st, a, d, c->ks);
        else hipLaunchKernelGGL((k_parse_decode<14, false>), gd, bd, 0, st, a, d, c->ks);
    } else {
        if (sl) hipLaunchKernelGGL((k_parse_decode<4, true>), gd, bd, 0, st, a, d, c->ks);
        else hipLaunchKernelGGL((k_parse_decode<4, false>), gd, bd, 0, st, a, d, c->ks);
    }
    int r = launch_check("k_parse_decode");
    if (r || !compact) return r;
    return run_compaction(c, ck, dec->valid_idx, dec->n_valid, (hipStream_t)stream);
}
}  // namespace

int rsk_parse_decode_batch(rsk_ctx *c, uint32_t n, const uint8_t *cap_arena, const uint64_t *cap_off,
                           const uint32_t *wire_len, const uint32_t *cap_len, int datalink, int flags,
                           const rsk_tcpinfo_out *tcp, const rsk_decode_out *dec, void *stream) {
    return parse_decode(c, n, cap_arena, cap_off, 0u, wire_len, cap_len, datalink, flags, tcp, dec, stream);
}

int rsk_parse_decode_slots_batch(rsk_ctx *c, uint32_t n, const uint8_t *slots, uint32_t slot,
                                 const uint32_t *wire_len, const uint32_t *cap_len, int datalink, int flags,
                                 const rsk_tcpinfo_out *tcp, const rsk_decode_out *dec, void *stream) {
    if (slot < RSK_CAP_SLOT_MIN || (slot & 15u) || (reinterpret_cast<uintptr_t>(slots) & 15u)) return RSK_EINVAL;
    return parse_decode(c, n, slots, nullptr, slot, wire_len, cap_len, datalink, flags, tcp, dec, stream);
}

int rsk_syncinput_decode_batch(rsk_ctx *c, uint32_t n, const uint8_t *rec_arena, const uint64_t *rec_off,
                               const int32_t *nread, const rsk_tcpinfo_out *tcp, const rsk_decode_out *dec,
                               void *stream) {
    if (!c || !tcp || !dec) return RSK_EINVAL;
    if (n == 0) return empty_batch(c, dec->n_valid, stream);
    if (n > RSK_MAX_BATCH) return RSK_EINVAL;  // grids of one lane per packet
    if (!rec_arena || !rec_off || !nread || !dec_out_ok(dec)) return RSK_EINVAL;
    if (!tcp->src || !tcp->dst || !tcp->sp || !tcp->dp || !tcp->seq || !tcp->ack || !tcp->flag ||
        !tcp->parse_status || !tcp->cap_pay_off || !tcp->cap_pay_len)
        return RSK_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    const bool compact = dec->valid_idx || dec->n_valid;
    Compact ck;
    if (compact) {
        int r = ensure_compact(c, n, (hipStream_t)stream, ck);
        if (r) return r;
    }
    SyncArgs a;
    a.rec = rec_arena; a.rec_off = rec_off; a.nread = nread;
    a.src = tcp->src; a.dst = tcp->dst; a.sp = tcp->sp; a.dp = tcp->dp; a.seq = tcp->seq; a.ack = tcp->ack;
    a.flag = tcp->flag; a.pst = tcp->parse_status; a.cpo = tcp->cap_pay_off; a.cpl = tcp->cap_pay_len;
    a.n = n;
    const DecOut d = make_dec_out(dec, ck.masks);
    hipLaunchKernelGGL(k_syncinput_decode, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, a, d, c->ks);
    int r = launch_check("k_syncinput_decode");
    if (r || !compact) return r;
    return run_compaction(c, ck, dec->valid_idx, dec->n_valid, (hipStream_t)stream);
}

int rsk_filter_parse_decode_batch(rsk_ctx *c, uint32_t n, const uint8_t *cap_arena, const uint64_t *cap_off,
                                  const uint32_t *wire_len, const uint32_t *cap_len, int datalink, int flags,
                                  const rsk_capture_filter *f, uint8_t *match, const rsk_tcpinfo_out *tcp,
                                  const rsk_decode_out *dec, void *stream) {
    if (!c || !f || !tcp || !dec) return RSK_EINVAL;
    if (datalink != RSK_DLT_EN10MB && datalink != RSK_DLT_NULL) return RSK_EINVAL;
    if (filter_ports_bad(f)) return RSK_EINVAL;
    if (n == 0) return empty_batch(c, dec->n_valid, stream);
    if (n > RSK_MAX_BATCH) return RSK_EINVAL;  // grids of one lane per packet
    if (!cap_arena || !cap_off || !wire_len || !cap_len || !match || !dec_out_ok(dec)) return RSK_EINVAL;
    if (!tcp->src || !tcp->dst || !tcp->sp || !tcp->dp || !tcp->seq || !tcp->ack || !tcp->flag ||
        !tcp->parse_status || !tcp->cap_pay_off || !tcp->cap_pay_len)
        return RSK_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    const bool compact = dec->valid_idx || dec->n_valid;
    Compact ck;
    if (compact) {
        int r = ensure_compact(c, n, (hipStream_t)stream, ck);
        if (r) return r;
    }
    ParseArgs a;
    a.cap = cap_arena; a.cap_off = cap_off; a.wire_len = wire_len; a.cap_len = cap_len;
    a.src = tcp->src; a.dst = tcp->dst; a.sp = tcp->sp; a.dp = tcp->dp; a.seq = tcp->seq; a.ack = tcp->ack;
    a.flag = tcp->flag; a.pst = tcp->parse_status; a.cpo = tcp->cap_pay_off; a.cpl = tcp->cap_pay_len;
    a.datalink = datalink; a.flags = flags; a.n = n; a.slot = 0;
    DecOut d = make_dec_out(dec, ck.masks);
    const hipStream_t st = (hipStream_t)stream;
    if (datalink == RSK_DLT_EN10MB)
        hipLaunchKernelGGL(k_filter_parse_decode<14>, dim3(grid_for(n)), dim3(kBlock), 0, st, a, d, c->ks, match, *f);
    else
        hipLaunchKernelGGL(k_filter_parse_decode<4>, dim3(grid_for(n)), dim3(kBlock), 0, st, a, d, c->ks, match, *f);
    int r = launch_check("k_filter_parse_decode");
    if (r || !compact) return r;
    return run_compaction(c, ck, dec->valid_idx, dec->n_valid, (hipStream_t)stream);
}

int rsk_capture_filter_batch(rsk_ctx *c, uint32_t n, const uint8_t *cap_arena, const uint64_t *cap_off,
                             const uint32_t *cap_len, int datalink, const rsk_capture_filter *f, uint8_t *match,
                             uint32_t *match_idx, uint32_t *n_match, void *stream) {
    if (!c || !f || (n && (!cap_arena || !cap_off || !cap_len || !match))) return RSK_EINVAL;
    if (datalink != RSK_DLT_EN10MB && datalink != RSK_DLT_NULL) return RSK_EINVAL;
    if (filter_ports_bad(f)) return RSK_EINVAL;
    if (n == 0) return empty_batch(c, n_match, stream);
    if (n > RSK_MAX_BATCH) return RSK_EINVAL;  // grids of one lane per packet
    DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    const bool compact = match_idx || n_match;
    Compact ck;
    if (compact) {
        int r = ensure_compact(c, n, (hipStream_t)stream, ck);
        if (r) return r;
    }
    FiltArgs a;
    a.cap = cap_arena; a.cap_off = cap_off; a.cap_len = cap_len; a.match = match; a.n = n;
    DecOut d;
    std::memset(&d, 0, sizeof d);
    d.masks = ck.masks;
    if (datalink == RSK_DLT_EN10MB)
        hipLaunchKernelGGL(k_capture_filter<14>, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, a, d, *f);
    else
        hipLaunchKernelGGL(k_capture_filter<4>, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, a, d, *f);
    int r = launch_check("k_capture_filter");
    if (r || !compact) return r;
    return run_compaction(c, ck, match_idx, n_match, (hipStream_t)stream);
}

// BuildFilterStr (cap/cap_util.cpp:67-144) with proto "tcp" (cap/RCap.cpp:64)
int rsk_filter_str(const rsk_capture_filter *f, char *buf, size_t buf_len) {
    if (!f || !buf) return -1;
    auto ip = [](uint32_t v) {
        return std::to_string(v & 255u) + "." + std::to_string((v >> 8) & 255u) + "." +
               std::to_string((v >> 16) & 255u) + "." + std::to_string(v >> 24);
    };
    auto ports = [](const rsk_port_list &pl, const char *dir) -> std::string {
        if (pl.n_single == 0 && pl.n_range == 0) return "";
        std::string s = "(";
        for (uint32_t q = 0; q < pl.n_single && q < RSK_FILTER_MAX_PORTS; ++q)
            s += std::string(" or ") + dir + " port " + std::to_string(pl.single[q]);
        for (uint32_t q = 0; q < pl.n_range && q < RSK_FILTER_MAX_PORTS; ++q)
            s += std::string(" or ") + dir + " portrange " + std::to_string(pl.range[q][0]) + "-" +
                 std::to_string(pl.range[q][1]);
        s += " )";
        s.replace(s.find("or"), 2, "");  // the reference removes the first "or"
        return " and " + s;
    };
    std::string out = "tcp";
    if (f->has_src_ip) out += " and  (ip src " + ip(f->src_ip) + ")";
    if (f->has_dst_ip) out += " and  (ip dst " + ip(f->dst_ip) + ")";
    out += ports(f->src_ports, "src");
    out += ports(f->dst_ports, "dst");
    if (f->is_server) {
        std::string s = out;
        for (size_t pos = s.find("dst"); pos != std::string::npos; pos = s.find("dst")) s.replace(pos, 3, "src");
        out = "((tcp[tcpflags] & tcp-syn != 0) and " + s + ") or (" + out + "and (tcp[tcpflags] & (tcp-syn) == 0))";
    }
    if (out.size() + 1 > buf_len) return -1;
    std::memcpy(buf, out.c_str(), out.size() + 1);
    return (int)out.size();
}

int rsk_tcpinfo_encode_batch(rsk_ctx *c, uint32_t n, const uint32_t *src, const uint32_t *dst,
                             const uint16_t *sp, const uint16_t *dp, const uint32_t *seq,
                             const uint32_t *ack, const uint8_t *flag, uint8_t *rec, void *stream) {
    if (!c) return RSK_EINVAL;
    if (n == 0) return RSK_OK;
    if (n > RSK_MAX_BATCH) return RSK_EINVAL;  // grids of one lane per packet
    if (!src || !dst || !sp || !dp || !seq || !ack || !flag || !rec) return RSK_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    TcpRecArgs a{src, dst, sp, dp, seq, ack, flag, rec, n};
    hipLaunchKernelGGL(k_tcpinfo_encode, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream, a);
    return launch_check("k_tcpinfo_encode");
}

int rsk_fill_splitmix(void *dst, uint64_t nbytes, uint64_t seed, void *stream) {
    if (!dst && nbytes) return RSK_EINVAL;
    if (nbytes == 0) return RSK_OK;
    const uint64_t nw = nbytes / 8u + 1u;
    const unsigned grid = (unsigned)std::min<uint64_t>((nw + kBlock - 1) / kBlock, 8192u);
    hipLaunchKernelGGL(k_fill_splitmix, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream,
                       reinterpret_cast<uint8_t *>(dst), nbytes, seed);
    return launch_check("k_fill_splitmix");
}

uint64_t rsk_key_for_tcp(uint16_t sp, uint16_t dp) {
    return 0x10000000ull | ((uint64_t)dp << 16) | (uint64_t)sp;  // KeyGenerator.cpp:16-25
}
uint64_t rsk_key_for_udp(uint16_t sp, uint16_t dp) {
    return 0x20000000ull | ((uint64_t)dp << 16) | (uint64_t)sp;  // KeyGenerator.cpp:27-36
}

}  // extern "C"

// ---- single-packet shims ----------------------------------------------------------------------
namespace {
int shim_init(rsk_ctx *c) {
    if (c->shim_dev && c->shim_host && c->shim_stream) return RSK_OK;
    DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    hipError_t e;
    if (!c->shim_dev && (e = hipMalloc(&c->shim_dev, sizeof(ShimIO))) != hipSuccess) { set_error("hipMalloc", e); return RSK_ENOMEM; }
    if (!c->shim_host && (e = hipHostMalloc(&c->shim_host, sizeof(ShimIO))) != hipSuccess) { set_error("hipHostMalloc", e); return RSK_ENOMEM; }
    if (!c->shim_stream && (e = hipStreamCreateWithFlags(&c->shim_stream, hipStreamNonBlocking)) != hipSuccess) {
        set_error("hipStreamCreate", e);
        return RSK_EDEVICE;
    }
    return RSK_OK;
}

int shim_run(rsk_ctx *c, int op, int len_arg) {
    DeviceGuard g(c->device);
    if (!g.ok) return RSK_EDEVICE;
    hipError_t e;
    if ((e = hipMemcpyAsync(c->shim_dev, c->shim_host, sizeof(ShimIO), hipMemcpyHostToDevice, c->shim_stream)) != hipSuccess) {
        set_error("hipMemcpyAsync", e);
        return RSK_EDEVICE;
    }
    hipLaunchKernelGGL(k_shim, dim3(1), dim3(64), 0, c->shim_stream, c->shim_dev, op, len_arg, c->ks);
    if (launch_check("k_shim")) return RSK_EDEVICE;
    if ((e = hipMemcpyAsync(c->shim_host, c->shim_dev, sizeof(ShimIO), hipMemcpyDeviceToHost, c->shim_stream)) != hipSuccess) {
        set_error("hipMemcpyAsync", e);
        return RSK_EDEVICE;
    }
    if ((e = hipStreamSynchronize(c->shim_stream)) != hipSuccess) { set_error("hipStreamSynchronize", e); return RSK_EDEVICE; }
    return RSK_OK;
}
}  // namespace

extern "C" {

uint8_t *rsk_compute_hash(rsk_ctx *c, uint8_t *tag_out, const uint8_t *data, int data_len) {
    if (!c || !tag_out || !data || data_len <= 0) return nullptr;  // rhash.cpp:21 asserts this
    std::lock_guard<std::mutex> lk(c->shim_mu);
    if (shim_init(c) != RSK_OK) return nullptr;
    c->shim_host->buf[0] = data[0];
    if (shim_run(c, 0, 0) != RSK_OK) return nullptr;
    std::memcpy(tag_out, c->shim_host->buf + 8, 8);
    return tag_out + RSK_HASH_BUF_SIZE;
}

int rsk_hash_equal(rsk_ctx *c, const uint8_t *tag, const uint8_t *data, int data_len) {
    if (!c || !tag || !data || data_len <= 0) return 0;  // rhash.cpp:73-75
    std::lock_guard<std::mutex> lk(c->shim_mu);
    if (shim_init(c) != RSK_OK) return 0;
    std::memcpy(c->shim_host->buf, tag, 8);
    c->shim_host->buf[8] = data[0];
    if (shim_run(c, 1, 0) != RSK_OK) return 0;
    return c->shim_host->ret;
}

uint8_t *rsk_enchead_enc2buf(rsk_ctx *c, uint8_t *p, int buf_len, uint8_t cmd, const uint8_t id[8],
                             uint32_t conv, uint64_t conn_key) {
    if (!c || !p || buf_len < RSK_ENC_HEAD_SIZE || !id) return nullptr;  // EncHead.cpp:10
    std::lock_guard<std::mutex> lk(c->shim_mu);
    if (shim_init(c) != RSK_OK) return nullptr;
    uint8_t *b = c->shim_host->buf;
    b[0] = cmd;
    std::memcpy(b + 1, id, 8);
    std::memcpy(b + 12, &conv, 4);
    std::memcpy(b + 16, &conn_key, 8);
    if (shim_run(c, 2, 0) != RSK_OK) return nullptr;
    std::memcpy(p, c->shim_host->buf + 32, RSK_ENC_HEAD_SIZE);
    return p + RSK_ENC_HEAD_SIZE;
}

const uint8_t *rsk_enchead_decodebuf(rsk_ctx *c, const uint8_t *p, int buf_len, uint8_t *len,
                                     uint8_t *cmd, uint8_t id[8], uint32_t *conv, uint64_t *conn_key) {
    if (!c || !p || buf_len < RSK_ENC_HEAD_SIZE) return nullptr;  // EncHead.cpp:40
    std::lock_guard<std::mutex> lk(c->shim_mu);
    if (shim_init(c) != RSK_OK) return nullptr;
    std::memcpy(c->shim_host->buf, p, RSK_ENC_HEAD_SIZE);
    if (shim_run(c, 3, buf_len) != RSK_OK || c->shim_host->ret < 0) return nullptr;
    const uint8_t *h = c->shim_host->buf + 32;
    if (len) *len = h[0];
    if (cmd) *cmd = h[1];
    if (id) std::memcpy(id, h + 2, 8);
    if (conv) std::memcpy(conv, h + 10, 4);
    if (conn_key) std::memcpy(conn_key, h + 14, 8);
    return p + c->shim_host->ret;
}

}  // extern "C"
