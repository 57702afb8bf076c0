// rsk_device.h — byte-movement and header helpers shared by the codec kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsk {

// Global (address space 1) views of generic pointers.  Pointers that pass through LDS records,
// readlane'd offsets or selects lose their address space and would otherwise be accessed with
// flat_* instructions, which count against both vmcnt and lgkmcnt and force conservative waits.
#define RSK_GLOBAL __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ RSK_GLOBAL T *gptr(T *p) {
    return (RSK_GLOBAL T *)p;
}
template <typename T>
__device__ __forceinline__ const RSK_GLOBAL T *gptr(const T *p) {
    return (const RSK_GLOBAL T *)p;
}

// bytes [r, r+4) of the 8-byte little-endian pair {hi:lo}  (v_alignbyte_b32)
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t r) {
    return __builtin_amdgcn_alignbyte(hi, lo, r);
}

// 16 bytes starting at byte `sh` (0..15) of the 32-byte little-endian concatenation A||B.
// sh is uniform per packet, so the switch is a scalar branch.
__device__ __forceinline__ uint4 funnel16(const uint4 &A, const uint4 &B, uint32_t sh) {
    const uint32_t r = sh & 3u;
    uint4 o;
    switch (sh >> 2) {
        case 0:
            o.x = funnel(A.y, A.x, r); o.y = funnel(A.z, A.y, r);
            o.z = funnel(A.w, A.z, r); o.w = funnel(B.x, A.w, r);
            break;
        case 1:
            o.x = funnel(A.z, A.y, r); o.y = funnel(A.w, A.z, r);
            o.z = funnel(B.x, A.w, r); o.w = funnel(B.y, B.x, r);
            break;
        case 2:
            o.x = funnel(A.w, A.z, r); o.y = funnel(B.x, A.w, r);
            o.z = funnel(B.y, B.x, r); o.w = funnel(B.z, B.y, r);
            break;
        default:
            o.x = funnel(B.x, A.w, r); o.y = funnel(B.y, B.x, r);
            o.z = funnel(B.z, B.y, r); o.w = funnel(B.w, B.z, r);
            break;
    }
    return o;
}

// Store bytes [lo, hi) of the 16-byte chunk v at p (16-byte aligned, 0 <= lo < hi <= 16) with the
// fewest stores: a byte and a short up to the first dword boundary, one dword / dwordx2 / dwordx3 /
// dwordx4 for the whole dwords, then a short and a byte.  Neighbouring frames may own the rest of
// the 16-B chunk, so nothing outside [lo, hi) is written.  lo / hi may be per lane.
__device__ __forceinline__ uint32_t word_at(const uint4 &v, uint32_t d) {
    // dword d (0..3) as AND/OR of masks: a select chain on a per-lane index is turned into a
    // dynamic vector extract, which the backend lowers through scratch memory
    auto m = [d](uint32_t i) { return (uint32_t)((int32_t)((d ^ i) - 1u) >> 31); };
    return (v.x & m(0)) | (v.y & m(1)) | (v.z & m(2)) | (v.w & m(3));
}
__device__ __forceinline__ void store_range16(uint8_t *p, const uint4 &v, uint32_t lo, uint32_t hi) {
    RSK_GLOBAL uint8_t *g = gptr(p);
    uint32_t x = lo;
    if ((x & 1u) && x < hi) {
        g[x] = (uint8_t)(word_at(v, x >> 2) >> (8u * (x & 3u)));
        x += 1u;
    }
    if ((x & 2u) && x + 2u <= hi) {
        *reinterpret_cast<RSK_GLOBAL uint16_t *>(g + x) = (uint16_t)(word_at(v, x >> 2) >> 16);
        x += 2u;
    }
    const uint32_t nd = x < hi ? (hi - x) >> 2 : 0u;  // x is a multiple of 4 here when nd > 0
    const uint32_t d = x >> 2;
    typedef uint32_t v2 __attribute__((ext_vector_type(2)));
    typedef uint32_t v3 __attribute__((ext_vector_type(3)));
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    if (nd == 4u) {
        const v4 q = {v.x, v.y, v.z, v.w};
        *reinterpret_cast<RSK_GLOBAL v4 *>(g) = q;
    } else if (nd == 3u) {
        const v3 q = {word_at(v, d), word_at(v, d + 1u), word_at(v, d + 2u)};
        *reinterpret_cast<RSK_GLOBAL v3 *>(g + x) = q;
    } else if (nd == 2u) {
        const v2 q = {word_at(v, d), word_at(v, d + 1u)};
        *reinterpret_cast<RSK_GLOBAL v2 *>(g + x) = q;
    } else if (nd == 1u) {
        *reinterpret_cast<RSK_GLOBAL uint32_t *>(g + x) = word_at(v, d);
    }
    x += 4u * nd;
    if (x + 2u <= hi) {
        *reinterpret_cast<RSK_GLOBAL uint16_t *>(g + x) = (uint16_t)(word_at(v, x >> 2) >> (8u * (x & 3u)));
        x += 2u;
    }
    if (x < hi) g[x] = (uint8_t)(word_at(v, x >> 2) >> (8u * (x & 3u)));
}

// Store bytes [0, lim) of v at p (16-byte aligned, 0 < lim < 16).
__device__ __forceinline__ void store_partial16(uint8_t *p, const uint4 &v, int lim) {
    store_range16(p, v, 0u, (uint32_t)lim);
}

// v with bytes [lim, 16) cleared (0 < lim < 16)
__device__ __forceinline__ uint4 keep_bytes16(const uint4 &v, int lim) {
    auto m = [lim](int d) -> uint32_t {
        const int k = lim - 4 * d;
        return k >= 4 ? 0xffffffffu : (k <= 0 ? 0u : ((1u << (8 * k)) - 1u));
    };
    return make_uint4(v.x & m(0), v.y & m(1), v.z & m(2), v.w & m(3));
}

// Store the last chunk of a frame: bytes [0, lim) of v at p (16-B aligned).  With pad, the whole
// chunk is written with the tail zeroed (RSK_ENC_ZERO_PAD16); without, only [0, lim).
typedef uint32_t gu32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store16(uint8_t *p, const uint4 &v) {
    const gu32x4 w = {v.x, v.y, v.z, v.w};
    *reinterpret_cast<RSK_GLOBAL gu32x4 *>(gptr(p)) = w;
}
__device__ __forceinline__ void store_tail16(uint8_t *p, const uint4 &v, int lim, bool pad) {
    if (lim >= 16) store16(p, v);
    else if (pad) store16(p, keep_bytes16(v, lim));
    else store_partial16(p, v, lim);
}

// NW dwords of bytes starting at an arbitrary byte address p; aligned dwords whose address is
// past `last` (the last byte the caller may touch) are not loaded (read as 0).  An aligned dword
// that contains a valid byte never crosses a page, so no load can fault.
template <int NW>
__device__ __forceinline__ void load_window(const uint8_t *p, const uint8_t *last, uint32_t (&w)[NW]) {
    const uint32_t r = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3u);
    const RSK_GLOBAL uint32_t *q = reinterpret_cast<const RSK_GLOBAL uint32_t *>(gptr(p - r));
    const intptr_t lim = last - (p - r);                             // last valid byte, rel. to q
    uint32_t raw[NW + 1];
#pragma unroll
    for (int j = 0; j <= NW; ++j) raw[j] = (4 * j <= lim) ? q[j] : 0u;
#pragma unroll
    for (int j = 0; j < NW; ++j) w[j] = funnel(raw[j + 1], raw[j], r);
}

// As load_window, with aligned 16-B loads: (4 NW + 30) / 16 chunk loads instead of NW + 1 dword
// loads.  Chunks wholly past `last` are not loaded (read as 0); a 16-B chunk holding a valid byte
// never crosses a page.  Bytes past `last` inside a loaded chunk are whatever memory holds: callers
// bound every field they use by the packet length themselves.
template <int NW>
__device__ __forceinline__ void load_window16(const uint8_t *p, const uint8_t *last, uint32_t (&w)[NW]) {
    constexpr int NC = (4 * NW + 30) / 16;
    const uint32_t r = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 15u);
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    const RSK_GLOBAL v4 *q = reinterpret_cast<const RSK_GLOBAL v4 *>(gptr(p - r));
    const intptr_t lim = last - (p - r);
    uint32_t raw[4 * NC + 4];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        v4 v = {0u, 0u, 0u, 0u};
        if (16 * c <= lim) v = q[c];
        raw[4 * c] = v.x; raw[4 * c + 1] = v.y; raw[4 * c + 2] = v.z; raw[4 * c + 3] = v.w;
    }
#pragma unroll
    for (int k = 4 * NC; k < 4 * NC + 4; ++k) raw[k] = 0u;
    const uint32_t dq = r >> 2, rb = r & 3u;
#pragma unroll
    for (int j = 0; j < NW; ++j) {
        const uint32_t lo = dq == 0 ? raw[j] : dq == 1 ? raw[j + 1] : dq == 2 ? raw[j + 2] : raw[j + 3];
        const uint32_t hi = dq == 0 ? raw[j + 1] : dq == 1 ? raw[j + 2] : dq == 2 ? raw[j + 3] : raw[j + 4];
        w[j] = funnel(hi, lo, rb);
    }
}

__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// byte k (0..31) of an 8-word little-endian window, k compile-time
template <int K>
__device__ __forceinline__ uint32_t byte_of(const uint32_t (&w)[8]) {
    return (w[K >> 2] >> (8 * (K & 3))) & 0xffu;
}

}  // namespace rsk
