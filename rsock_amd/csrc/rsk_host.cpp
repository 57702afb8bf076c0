// rsk_host.cpp — host-side batch helpers of the header-only path (include/rsk_codec.h): staging
// the 32-B decode slots of received frames and assembling frames from encoded header slots and
// payloads, each over contiguous shards on std::threads.  Pure host code (no HIP calls).
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/rsk_codec.h"

namespace {

template <typename F>
void for_shards(uint32_t n, int nthreads, F f) {
    if (nthreads <= 1 || n < 4096) {
        f(0u, n);
        return;
    }
    std::vector<std::thread> ts;
    const uint32_t per = (n + (uint32_t)nthreads - 1) / (uint32_t)nthreads;
    for (uint32_t lo = 0; lo < n; lo += per) ts.emplace_back(f, lo, lo + per < n ? lo + per : n);
    for (auto &t : ts) t.join();
}

}  // namespace

extern "C" int rsk_stage_decode_headers(uint32_t n, const uint8_t *arena, const uint64_t *frame_off,
                                        const uint16_t *frame_len, uint8_t *slots, int nthreads) {
    if (n && (!arena || !frame_off || !frame_len || !slots)) return RSK_EINVAL;
    for_shards(n, nthreads, [=](uint32_t lo, uint32_t hi) {
        for (uint32_t i = lo; i < hi; ++i)
            rsk_stage_decode_header(arena + frame_off[i], (int)frame_len[i], slots + 32ull * i);
    });
    return RSK_OK;
}

extern "C" int rsk_assemble_frames(uint32_t n, const uint8_t *hdr, const int32_t *status, const uint8_t *payload_arena,
                                   const uint64_t *pay_off, uint8_t *frame_arena, const uint64_t *frame_off,
                                   int nthreads) {
    if (n && (!hdr || !status || !payload_arena || !pay_off || !frame_arena || !frame_off)) return RSK_EINVAL;
    for_shards(n, nthreads, [=](uint32_t lo, uint32_t hi) {
        for (uint32_t i = lo; i < hi; ++i) {
            const int32_t st = status[i];
            if (st <= 0) continue;
            uint8_t *f = frame_arena + frame_off[i];
            std::memcpy(f, hdr + 32ull * i, RSK_HEAD_SIZE);                                   // RConn.cpp:101-103
            std::memcpy(f + RSK_HEAD_SIZE, payload_arena + pay_off[i], (size_t)(st - RSK_HEAD_SIZE));  // :104
        }
    });
    return RSK_OK;
}

extern "C" int rsk_stage_capture_slots(uint32_t n, const uint8_t *arena, const uint64_t *cap_off, const uint32_t *cap_len,
                                       uint32_t slot, uint8_t *slots, int nthreads) {
    if (slot < RSK_CAP_SLOT_MIN || (slot & 15u)) return RSK_EINVAL;
    if (n && (!arena || !cap_off || !cap_len || !slots)) return RSK_EINVAL;
    for_shards(n, nthreads, [=](uint32_t lo, uint32_t hi) {
        for (uint32_t i = lo; i < hi; ++i) {
            const uint32_t k = cap_len[i] < slot ? cap_len[i] : slot;
            uint8_t *d = slots + (uint64_t)slot * i;
            std::memcpy(d, arena + cap_off[i], k);
            std::memset(d + k, 0, slot - k);
        }
    });
    return RSK_OK;
}
