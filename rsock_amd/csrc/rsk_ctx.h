// Internal (not installed): the rsk_ctx handle and host helpers shared by the librsk translation
// units (rsk_kernels.hip: codec; rsk_demux.hip: receive demux).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <mutex>
#include <vector>

#include "../../include/rsk_codec.h"
#include "rsk_md5.h"

struct ShimIO;  // rsk_kernels.hip

struct rsk_ctx {
    int device = 0;
    int enc_variant = 0;   // see rsk__set_encode_variant
    int wire_variant = 0;  // see rsk__set_wire_variant
    std::vector<uint8_t> key;
    rsk::KeySched ks;
    // compaction workspace
    void *ws = nullptr;
    uint32_t ws_n = 0;
    // connection-state workspace (rsk_tcp_send_seq_batch, rsk_demux.hip)
    void *sq_ws = nullptr;
    size_t sq_ws_bytes = 0;
    bool sq_force_groupby = false;  // see rsk__set_send_seq_groupby
    int sq_scan_variant = 0;
    // demux workspace (rsk_demux.hip)
    void *dm_ws = nullptr;
    size_t dm_ws_bytes = 0;
    // single-packet shim buffers
    ShimIO *shim_dev = nullptr;
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

}  // namespace rsk
