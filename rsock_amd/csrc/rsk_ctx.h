// Internal (not installed): the rsk_ctx handle and host helpers shared by the librsk translation
// units (rsk_kernels.hip: codec; rsk_demux.hip: receive demux).
#pragma once

#include <hip/hip_runtime.h>

#include <array>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../../include/rsk_codec.h"
#include "rsk_md5.h"

struct ShimIO;  // rsk_kernels.hip

namespace rsk {
// Device scratch of one kind for the calls ordered on one stream.
enum WsKind { WS_COMPACT = 0, WS_SEQ = 1, WS_DEMUX = 2, WS_ENC = 3, WS_KINDS = 4 };
struct WsBuf {
    void *p = nullptr;
    size_t bytes = 0;
    // WS_COMPACT: zero-filled since (re)allocation (see stream_compact); WS_DEMUX: its table flag word
    // was initialised (rsk_demux.hip k_dm_fill / k_dm_final keep it from there)
    bool zeroed = false;
};
}  // namespace rsk

struct rsk_ctx {
    int device = 0;
    // encode path (rsk_encode_batch): 0 = chosen per call from the previous batch's statistic, else
    // RSK_ENC_PATH_* (rsk_set_encode_path)
    int enc_path = 0;
    int copy_k = 0;  // the two-pass copy's packets per wave (-1: output-stationary; 0: by the sampled statistic; rsk__set_copy_k)
    uint32_t os_epoch = 0;  // per output-stationary call: the value k_encode_heads_os flags a failed layout check with
    uint32_t tp_chunk = 0;  // the two-pass form's chunk of packets (0: whole batch; rsk__set_two_pass_chunk)
    std::atomic<int> enc_last_path{0};  // the path the last rsk_encode_batch took (rsk__last_encode_path)
    std::atomic<int> enc_last_k{0};     // its packets per copy wave, two-pass form (rsk__last_copy_k)
    // set once any call of this context was captured into a graph: its replays may run on streams the
    // context never saw, so rsk_check_device_errors waits for the device instead of its streams
    std::atomic<bool> captured{false};
    // host-mapped word the batch statistic is stored to (enc_sample: k_encode_heads, k_enc_sample) and
    // its device address; read without synchronisation by later calls (a stale value only picks the
    // slower path, never different bytes)
    uint32_t *enc_stat_host = nullptr;  // [2]: the batch statistic, then the demux's table hint (rsk_demux.hip)
    uint32_t *enc_stat_dev = nullptr;
    std::vector<uint8_t> key;
    rsk::KeySched ks;
    // Scratch per stream (compaction look-back state, send-seq tables, demux tables): calls on
    // different streams never share scratch, calls on one stream are ordered by it (rsk_codec.h).
    std::mutex ws_mu;
    std::unordered_map<hipStream_t, std::array<rsk::WsBuf, rsk::WS_KINDS>> ws;
    bool sq_force_groupby = false;  // see rsk__set_send_seq_groupby
    int sq_scan_variant = 0;
    // single-packet shim buffers
    ShimIO *shim_dev = nullptr;
    uint2 *tag_dev = nullptr;  // 256-entry tag table (rsk::KeySched::tab)
    uint32_t *err_dev = nullptr;  // sticky device error flags (RSK_DEVERR_*, rsk_check_device_errors)
    // see rsk__inject_compact_stall (tests): consumed by exchange, so host threads driving one
    // context on several streams never race on it
    std::atomic<uint32_t> compact_stall_tile{~0u};
    ShimIO *shim_host = nullptr;
    hipStream_t shim_stream = nullptr;
    std::mutex shim_mu;
};

namespace rsk {

extern thread_local char g_last_error[256];

inline void set_error(const char *what, hipError_t e) {
    snprintf(g_last_error, sizeof g_last_error, "%s: %s", what, hipGetErrorString(e));
}

inline int launch_check(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error(what, e);
        return RSK_EDEVICE;
    }
    return 0;
}

struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) {
            hipError_t e = hipSetDevice(dev);
            if (e != hipSuccess) {
                set_error("hipSetDevice", e);
                ok = false;
            }
        }
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// True when s is being captured into a graph (stream operations are recorded, not run).
inline bool capturing(hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

// At least `need` bytes of `kind` scratch for stream s.  Growing waits for s to drain (the old
// buffer may still be read by work queued on s) and then reallocates; neither can happen while s is
// being captured (RSK_EINVAL: reserve before the capture, rsk_codec.h).
inline int stream_ws(rsk_ctx *c, hipStream_t s, int kind, size_t need, void **out) {
    std::lock_guard<std::mutex> lk(c->ws_mu);
    if (capturing(s)) c->captured.store(true, std::memory_order_relaxed);
    WsBuf &b = c->ws[s][kind];
    if (!b.p || b.bytes < need) {
        if (capturing(s)) {
            snprintf(g_last_error, sizeof g_last_error,
                     "scratch of a capturing stream must be reserved before the capture (rsk_reserve_stream)");
            return RSK_EINVAL;
        }
        if (b.p) {
            hipError_t e = hipStreamSynchronize(s);
            if (e != hipSuccess) { set_error("hipStreamSynchronize", e); return RSK_EDEVICE; }
            (void)hipFree(b.p);
            b.p = nullptr;
            b.bytes = 0;
        }
        hipError_t e = hipMalloc(&b.p, need);
        if (e != hipSuccess) { set_error("hipMalloc(workspace)", e); b.p = nullptr; return RSK_ENOMEM; }
        b.bytes = need;
        b.zeroed = false;  // fresh memory: stream_compact zeroes it before first use
    }
    *out = b.p;
    return RSK_OK;
}

// As stream_ws, but a buffer that would have to grow while s is being captured is refused quietly
// (RSK_EINVAL, no error text): for scratch whose caller has a path that needs none.
inline int stream_ws_if(rsk_ctx *c, hipStream_t s, int kind, size_t need, void **out) {
    if (capturing(s)) {
        c->captured.store(true, std::memory_order_relaxed);
        std::lock_guard<std::mutex> lk(c->ws_mu);
        auto it = c->ws.find(s);
        if (it == c->ws.end() || !it->second[kind].p || it->second[kind].bytes < need) return RSK_EINVAL;
        *out = it->second[kind].p;
        return RSK_OK;
    }
    return stream_ws(c, s, kind, need, out);
}

// Workspace of the compaction for stream s: `words` 64-bit words, zeroed when (re)allocated.  Its
// first word is the device-side call counter k_compact keeps (see rsk_kernels.hip), so the state
// needs no host-side reset per call and a captured graph replays correctly.
inline int stream_compact(rsk_ctx *c, hipStream_t s, size_t words, unsigned long long **out, size_t *cap) {
    void *p = nullptr;
    int r = stream_ws(c, s, WS_COMPACT, words * sizeof(unsigned long long), &p);
    if (r) return r;
    std::lock_guard<std::mutex> lk(c->ws_mu);
    WsBuf &b = c->ws[s][WS_COMPACT];
    if (!b.zeroed) {
        if (capturing(s)) {  // a captured memset has not run yet: an eager call would read stale state
            snprintf(g_last_error, sizeof g_last_error,
                     "compaction state of a capturing stream must be initialised by an eager call first");
            return RSK_EINVAL;
        }
        hipError_t e = hipMemsetAsync(b.p, 0, b.bytes, s);
        if (e != hipSuccess) { set_error("hipMemsetAsync(compaction state)", e); return RSK_EDEVICE; }
        b.zeroed = true;
    }
    *out = reinterpret_cast<unsigned long long *>(p);
    *cap = b.bytes / sizeof(unsigned long long);
    return RSK_OK;
}

// After a look-back timeout (RSK_DEVERR_LOOKBACK) a stalled tile may publish words under a later
// call's epoch: every stream's compaction state is zeroed again at its next use.
inline void invalidate_compact(rsk_ctx *c) {
    std::lock_guard<std::mutex> lk(c->ws_mu);
    for (auto &kv : c->ws) {
        kv.second[WS_COMPACT].zeroed = false;
        kv.second[WS_DEMUX].zeroed = false;  // a demux call that gave up may leave slots claimed: fill again
    }
}

// The `zeroed` flag of stream s's `kind` scratch (after stream_ws sized it), under the lock.
inline bool ws_clean(rsk_ctx *c, hipStream_t s, int kind) {
    std::lock_guard<std::mutex> lk(c->ws_mu);
    return c->ws[s][kind].zeroed;
}
inline void set_ws_clean(rsk_ctx *c, hipStream_t s, int kind, bool v) {
    std::lock_guard<std::mutex> lk(c->ws_mu);
    c->ws[s][kind].zeroed = v;
}

// Wait for the work whose device error flags rsk_check_device_errors reads.  Normally the streams
// this context has scratch on (its look-back kernels ran there) and its shim stream -- the context's
// own work, not the device.  Two cases fall back to the whole device: a
// context that ever had a call captured (its graphs may be replayed on streams ordered with the
// capture stream, which the context never saw), and a scratch stream whose handle is no longer valid
// (destroyed without rsk_release_stream: its scratch is freed and its entry dropped, so later calls
// do not fail on it again).
inline hipError_t sync_ctx_streams(rsk_ctx *c) {
    if (c->captured.load(std::memory_order_relaxed)) return hipDeviceSynchronize();
    std::vector<hipStream_t> ss;
    {
        std::lock_guard<std::mutex> lk(c->ws_mu);
        for (auto &kv : c->ws) ss.push_back(kv.first);
    }
    bool stale = false;
    for (hipStream_t s : ss) {
        hipError_t e = hipStreamSynchronize(s);
        if (e == hipErrorInvalidHandle || e == hipErrorContextIsDestroyed || e == hipErrorInvalidResourceHandle) {
            (void)hipGetLastError();
            stale = true;
            std::lock_guard<std::mutex> lk(c->ws_mu);
            auto it = c->ws.find(s);
            if (it != c->ws.end()) {
                for (WsBuf &b : it->second)
                    if (b.p) (void)hipFree(b.p);
                c->ws.erase(it);
            }
        } else if (e != hipSuccess) {
            return e;
        }
    }
    if (c->shim_stream) {
        hipError_t e = hipStreamSynchronize(c->shim_stream);
        if (e != hipSuccess) return e;
    }
    return stale ? hipDeviceSynchronize() : hipSuccess;
}

// Sync s, then free its scratch (rsk_release_stream).  Graphs captured on s point at that scratch:
// they must be destroyed first (rsk_codec.h, rsk_release_stream).
inline int release_ws(rsk_ctx *c, hipStream_t s) {
    std::lock_guard<std::mutex> lk(c->ws_mu);
    auto it = c->ws.find(s);
    if (it == c->ws.end()) return RSK_OK;
    hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) { set_error("hipStreamSynchronize", e); return RSK_EDEVICE; }
    for (WsBuf &b : it->second)
        if (b.p) (void)hipFree(b.p);
    c->ws.erase(it);
    return RSK_OK;
}

inline void free_ws(rsk_ctx *c) {
    std::lock_guard<std::mutex> lk(c->ws_mu);
    for (auto &kv : c->ws)
        for (WsBuf &b : kv.second)
            if (b.p) (void)hipFree(b.p);
    c->ws.clear();
}

}  // namespace rsk
