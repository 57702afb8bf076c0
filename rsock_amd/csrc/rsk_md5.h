// rsk_md5.h — MD5 compression (RFC 1321 §3.4) for the tag path, host + device.
//
// The tag is MD5(key || payload[0])[8..15] (util/rhash.cpp:20-41).  On the device the key part of
// the message schedule is uniform per launch (kernel arguments -> SGPRs) and only the word holding
// payload[0] differs per lane, so one tag costs one compression for key_len <= 54 (two otherwise).
// Round constants and rotations are compile-time literals: after full unrolling every K[i] is an
// instruction immediate, which needs no LDS traffic and no VGPRs ("MD5 constants:
// immediates vs LDS": an LDS-staged table measured slower, profiles/r03_ab_md5_lds.json).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsk {

struct Md5Consts {
    static constexpr uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
        0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
        0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
        0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
        0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
        0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
        0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
        0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
};

__host__ __device__ __forceinline__ uint32_t rotl(uint32_t x, int s) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(x, x, 32 - s);  // v_alignbit_b32: funnel shift == rotate
#else
    return (x << s) | (x >> (32 - s));
#endif
}

// Where the round constants come from.  KImm (shipped): K[I] is a compile-time literal, so after full
// unrolling it is an instruction immediate.  A kernel may pass another source with a get<I>() (an
// LDS-staged table, as round 3 measured for the north star's "constants in LDS").
struct KImm {
    template <int I>
    __host__ __device__ __forceinline__ uint32_t get() const { return Md5Consts::K[I]; }
};

// One MD5 step; the round function and message index are resolved at compile time.
template <int I, class KS = KImm>
__host__ __device__ __forceinline__ void md5_step(uint32_t &a, uint32_t b, uint32_t c, uint32_t d,
                                                  const uint32_t (&m)[16], const KS &ksrc = KS()) {
    constexpr int R = I / 16;
    constexpr int G = R == 0 ? I : R == 1 ? (5 * I + 1) & 15 : R == 2 ? (3 * I + 5) & 15 : (7 * I) & 15;
    constexpr int S0[4] = {7, 12, 17, 22}, S1[4] = {5, 9, 14, 20}, S2[4] = {4, 11, 16, 23},
                  S3[4] = {6, 10, 15, 21};
    constexpr int S = R == 0 ? S0[I & 3] : R == 1 ? S1[I & 3] : R == 2 ? S2[I & 3] : S3[I & 3];
    uint32_t f;
    if constexpr (R == 0) f = d ^ (b & (c ^ d));        // F = (b&c) | (~b&d)
    else if constexpr (R == 1) f = c ^ (d & (b ^ c));   // G = (b&d) | (c&~d)
    else if constexpr (R == 2) f = b ^ c ^ d;           // H
    else f = c ^ (b | ~d);                              // I
    a = b + rotl(a + f + ksrc.template get<I>() + m[G], S);
}

template <int I, class KS>
__host__ __device__ __forceinline__ void md5_steps(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d,
                                                   const uint32_t (&m)[16], const KS &ksrc) {
    if constexpr (I < 64) {
        // state rotation a<-d, d<-c, c<-b, b<-new: expressed by rotating the argument roles
        md5_step<I + 0>(a, b, c, d, m, ksrc);
        md5_step<I + 1>(d, a, b, c, m, ksrc);
        md5_step<I + 2>(c, d, a, b, m, ksrc);
        md5_step<I + 3>(b, c, d, a, m, ksrc);
        md5_steps<I + 4>(a, b, c, d, m, ksrc);
    }
}

// st <- compress(st, m)
template <class KS = KImm>
__host__ __device__ __forceinline__ void md5_compress(uint32_t (&st)[4], const uint32_t (&m)[16],
                                                      const KS &ksrc = KS()) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    md5_steps<0>(a, b, c, d, m, ksrc);
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
}

// Per-key message schedule, precomputed on the host by rsk_create (rsk_kernels.hip).
struct KeySched {
    uint32_t mid[4];   // chaining state after every block that holds only key bytes
    uint32_t blk[16];  // words of the block that holds payload[0], with that byte = 0
    uint32_t pad[16];  // the following padding/length block (used when two_blocks)
    uint32_t pre[4];   // (a, b, c, d) after steps 0 .. bword - 1 of the last compression (md5_prefix_steps)
    int32_t bword;     // word index of payload[0] inside blk
    int32_t bshift;    // bit position of payload[0] inside that word
    int32_t two_blocks;
    // How the framing / verifying kernels obtain a tag (rsk_set_tag_mode): RSK_TAG_MD5 (0, default)
    // runs the MD5 compression per lane; RSK_TAG_TABLE (1) stages `tab` in LDS and looks the tag up.
    // Uniform per launch (a kernel argument), so the choice is a scalar branch.
    int32_t tag_mode;
    // Device table of the 256 tags this key can produce (tag = f(key, payload[0]) only): entry b =
    // (t0, t1) for payload[0] = b, built on the GPU by k_tag_table at rsk_create.
    const uint2 *tab;
};

// ---- the per-lane form (round 4): payload[0]'s word index BW is a template parameter, so every
// message word but one is uniform.  A step whose word is uniform folds K[i] + m[g] into one scalar
// add and costs 4 VALU (the round function as one v_bitop3_b32, v_add3_u32(a, f, K + m),
// v_alignbit_b32, v_add_u32); only the 4 steps that read word BW (one per round) add the per-lane
// word.  Steps 0 .. BW - 1 read key words only and start from the key's midstate, so the host runs
// them (build_sched -> KeySched::pre) and the device starts at step BW.  The generic md5_tag above
// had every message word in a VGPR (word BW selected at run time): 5 VALU per step
// (profiles/r04_ab_md5_isa.json).
template <int I>
struct Md5Step {
    static constexpr int R = I / 16;
    static constexpr int G = R == 0 ? I : R == 1 ? (5 * I + 1) & 15 : R == 2 ? (3 * I + 5) & 15 : (7 * I) & 15;
    static constexpr int S = R == 0 ? (I % 4 == 0 ? 7 : I % 4 == 1 ? 12 : I % 4 == 2 ? 17 : 22)
                           : R == 1 ? (I % 4 == 0 ? 5 : I % 4 == 1 ? 9 : I % 4 == 2 ? 14 : 20)
                           : R == 2 ? (I % 4 == 0 ? 4 : I % 4 == 1 ? 11 : I % 4 == 2 ? 16 : 23)
                                    : (I % 4 == 0 ? 6 : I % 4 == 1 ? 10 : I % 4 == 2 ? 15 : 21);
    __host__ __device__ static __forceinline__ uint32_t f(uint32_t b, uint32_t c, uint32_t d) {
        if constexpr (R == 0) return d ^ (b & (c ^ d));
        else if constexpr (R == 1) return c ^ (d & (b ^ c));
        else if constexpr (R == 2) return b ^ c ^ d;
        else return c ^ (b | ~d);
    }
};

// steps I .. 63 on (a, b, c, d); mw = the per-lane word BW; returns the final c and d (the tag's words
// before the feed-forward; step 63's b is not needed and the compiler drops it)
template <int I, int BW>
__host__ __device__ __forceinline__ void md5_steps_bw(uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                                                      const uint32_t *blk, uint32_t mw, uint32_t &oc, uint32_t &od) {
    if constexpr (I == 64) {
        oc = c;
        od = d;
    } else {
        using St = Md5Step<I>;
        const uint32_t fv = St::f(b, c, d);
        uint32_t x;
        if constexpr (St::G == BW) x = a + fv + mw + Md5Consts::K[I];
        else x = a + fv + (Md5Consts::K[I] + blk[St::G]);  // K + m: one scalar add
        const uint32_t nb = b + rotl(x, St::S);
        md5_steps_bw<I + 1, BW>(d, nb, b, c, blk, mw, oc, od);  // (a, b, c, d) <- (d, new, b, c)
    }
}

// host: state (a, b, c, d) after steps 0 .. bw - 1 from the midstate (round 0 reads m[i] at step i,
// all key words for i < bw)
inline void md5_prefix_steps(const uint32_t mid[4], const uint32_t blk[16], int bw, uint32_t out[4]) {
    uint32_t a = mid[0], b = mid[1], c = mid[2], d = mid[3];
    static const int S0[4] = {7, 12, 17, 22};
    for (int i = 0; i < bw; ++i) {
        const uint32_t f = d ^ (b & (c ^ d));
        const uint32_t x = a + f + Md5Consts::K[i] + blk[i];
        const uint32_t nb = b + ((x << S0[i & 3]) | (x >> (32 - S0[i & 3])));
        a = d;
        d = c;
        c = b;
        b = nb;
    }
    out[0] = a;
    out[1] = b;
    out[2] = c;
    out[3] = d;
}

// Tag words (digest bytes 8..11 and 12..15, little-endian) for payload byte b.
template <class KS = KImm>
__host__ __device__ __forceinline__ void md5_tag(const KeySched &ks, uint32_t b, uint32_t &t0,
                                                 uint32_t &t1, const KS &ksrc = KS()) {
    uint32_t m[16];
    const uint32_t bb = b << ks.bshift;
#pragma unroll
    for (int w = 0; w < 16; ++w) m[w] = ks.blk[w] | (w == ks.bword ? bb : 0u);
    uint32_t st[4] = {ks.mid[0], ks.mid[1], ks.mid[2], ks.mid[3]};
    md5_compress(st, m, ksrc);
    if (ks.two_blocks) {
        // the padding block of a key with 55..63 bytes past its last whole block: at most 0x80 in
        // word 0 and the bit length in words 14..15, zeros elsewhere (build_sched) -- literal zeros
        // keep 13 words out of the SGPRs of the kernels that inline this
        uint32_t p[16];
#pragma unroll
        for (int w = 0; w < 16; ++w) p[w] = (w == 0 || w >= 14) ? ks.pad[w] : 0u;
        md5_compress(st, p, ksrc);
    }
    t0 = st[2];
    t1 = st[3];
}

// The per-lane tag with payload[0] in word BW (== ks.bword): starts from ks.pre at step BW.
template <int BW>
__host__ __device__ __forceinline__ void md5_tag_bw(const KeySched &ks, uint32_t b, uint32_t &t0, uint32_t &t1) {
    const uint32_t mw = ks.blk[BW] | (b << ks.bshift);
    uint32_t c, d;
    if (BW < 13 || !ks.two_blocks) {  // a two-block tail puts payload[0] in byte 55..63: word 13..15
        md5_steps_bw<BW, BW>(ks.pre[0], ks.pre[1], ks.pre[2], ks.pre[3], ks.blk, mw, c, d);
        t0 = ks.mid[2] + c;
        t1 = ks.mid[3] + d;
        return;
    }
    // 55..63 key bytes past the last whole block (BW = 13 .. 15): the full state of the first
    // compression feeds the padding block's
    uint32_t m[16];
#pragma unroll
    for (int w = 0; w < 16; ++w) m[w] = w == BW ? mw : ks.blk[w];
    uint32_t st[4] = {ks.mid[0], ks.mid[1], ks.mid[2], ks.mid[3]};
    md5_compress(st, m);
    uint32_t p[16];
#pragma unroll
    for (int w = 0; w < 16; ++w) p[w] = (w == 0 || w >= 14) ? ks.pad[w] : 0u;
    md5_compress(st, p);
    t0 = st[2];
    t1 = st[3];
}

// Dispatch on the key's payload word (uniform per launch: one scalar branch).
__host__ __device__ __forceinline__ void md5_tag_lane(const KeySched &ks, uint32_t b, uint32_t &t0, uint32_t &t1) {
    switch (ks.bword) {
#define RSK_MD5_BW(W) \
    case W: md5_tag_bw<W>(ks, b, t0, t1); return;
        RSK_MD5_BW(0) RSK_MD5_BW(1) RSK_MD5_BW(2) RSK_MD5_BW(3) RSK_MD5_BW(4) RSK_MD5_BW(5) RSK_MD5_BW(6)
        RSK_MD5_BW(7) RSK_MD5_BW(8) RSK_MD5_BW(9) RSK_MD5_BW(10) RSK_MD5_BW(11) RSK_MD5_BW(12) RSK_MD5_BW(13)
        RSK_MD5_BW(14)
#undef RSK_MD5_BW
        default: md5_tag_bw<15>(ks, b, t0, t1); return;
    }
}

}  // namespace rsk
