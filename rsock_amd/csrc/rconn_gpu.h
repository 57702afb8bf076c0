// rconn_gpu.h — RConn-shaped batching adapter over the rsk C ABI (host C++, MI355X).
//
// The reference frames and verifies one packet per call on the libuv thread
// (conn/RConn.cpp:64-128).  RConnGpu keeps RConn's per-packet surface and return contract but
// queues the packets and runs each full batch (or an explicit Flush) through the header-only
// entry points rsk_encode_headers_batch / rsk_decode_headers_batch, double-buffered: while batch k
// is on the GPU (H2D -> kernel -> D2H on its own stream), batch k+1 is being filled.  Only
// payload[0] + descriptors go to the GPU on the send side and only the 32-B header slot on the
// receive side; payloads stay in host frame slots (Output copies the payload to offset 31 of its
// slot, as RConn.cpp:104 copies it into the stack frame; the 31 header bytes land in front at
// delivery).  Results are delivered through callbacks in input order, i.e. the order RConn would
// have produced them.
//
//   Output(nread, base, head, user)      <- RConn::Output(nread, rbuf) with rbuf.data->head
//       nread < 0  -> returns nread (RConn.cpp:127)
//       nread == 0 -> reset_cb(user), returns its value (RConn.cpp:119-123)
//       31 + nread > 1500 -> returns -1 (RConn.cpp:94-98)
//       else queued; returns 31 + nread; send_cb(frame, 31 + nread, user) runs at delivery
//   OnRecv(nread, base, tcp_close, user) <- RConn::OnRecv(nread, rbuf)
//       queued; recv_cb(result) runs at delivery with result.status = RSK_RECV_VALID (payload
//       forwarded, IGroup::OnRecv), RSK_RECV_CLOSE (NotifyTcpFinOrRst) or RSK_RECV_DROP
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <sys/types.h>

#include <functional>
#include <string>
#include <vector>

#include "../../include/rsk_codec.h"

namespace rsk {

struct EncHeadFields {  // the fields of bean/EncHead.h:24-29 that Enc2Buf writes
    uint8_t cmd = RSK_CMD_DATA;
    uint8_t id[RSK_ID_BUF_SIZE] = {0};
    uint32_t conv = 0;
    uint64_t conn_key = 0;
};

struct RecvResult {
    int status;         // RSK_RECV_*
    uint8_t hlen, cmd;  // decoded EncHead (VALID only)
    uint8_t id[RSK_ID_BUF_SIZE];
    uint32_t conv;
    uint64_t conn_key;
    const char *payload;  // base + 8 + hlen inside the adapter's copy of the frame (valid during the callback)
    int payload_len;
    void *user;
};

class RConnGpu {
public:
    using SendFn = std::function<int(const char *frame, int len, void *user)>;  // RawTcp::Send / BtmUdpConn
    using ResetFn = std::function<int(void *user)>;                            // RConnReset::SendReset
    using RecvFn = std::function<int(const RecvResult &)>;                     // IGroup::OnRecv

    RConnGpu(const std::string &hash_key, int device, uint32_t batch = 4096);
    ~RConnGpu();
    RConnGpu(const RConnGpu &) = delete;
    RConnGpu &operator=(const RConnGpu &) = delete;

    bool ok() const { return ok_; }
    void SetSendCb(SendFn f) { send_cb_ = std::move(f); }
    void SetResetCb(ResetFn f) { reset_cb_ = std::move(f); }
    void SetRecvCb(RecvFn f) { recv_cb_ = std::move(f); }

    int Output(ssize_t nread, const char *base, const EncHeadFields &head, void *user);
    int OnRecv(ssize_t nread, const char *base, bool tcp_close, void *user);
    // Launch whatever is queued and deliver every outstanding result.  Returns 0 or RSK_E*.
    int Flush();

    uint64_t frames_sent() const { return n_sent_; }
    // send / reset callbacks that returned < 0 since creation (RConn::Output returns the callee's
    // result synchronously, RConn.cpp:108-123; here the callbacks run at delivery, so their failures
    // are counted instead)
    uint64_t callback_failures() const { return n_cb_fail_; }
    uint64_t frames_received() const { return n_recv_; }

private:
    static constexpr uint32_t kPayPitch = 1472;   // >= 1469, 16-B multiple
    static constexpr uint32_t kFramePitch = 1504;  // >= 1500, 16-B multiple (RSK_ENC_ZERO_PAD16 safe)

    struct EncSlot {
        uint32_t count = 0;
        bool in_flight = false;
        hipStream_t stream = nullptr;
        hipEvent_t done = nullptr;
        uint8_t *frame = nullptr;  // host frames (pinned pages): payload copied to +31 at Output, header at delivery
        // pinned host
        uint8_t *h_b0 = nullptr, *h_cmd = nullptr, *h_id = nullptr, *h_hdr = nullptr;
        uint64_t *h_key = nullptr;
        uint16_t *h_len = nullptr;
        uint32_t *h_conv = nullptr;
        int32_t *h_status = nullptr;
        std::vector<void *> user;
        // device
        uint8_t *d_b0 = nullptr, *d_cmd = nullptr, *d_id = nullptr, *d_hdr = nullptr;
        uint64_t *d_key = nullptr;
        uint16_t *d_len = nullptr;
        uint32_t *d_conv = nullptr;
        int32_t *d_status = nullptr;
    };
    struct DecSlot {
        uint32_t count = 0;
        bool in_flight = false;
        hipStream_t stream = nullptr;
        hipEvent_t done = nullptr;
        uint8_t *frame = nullptr;            // host copies of the frames (payload hand-off; pinned pages)
        std::vector<std::vector<char>> big;  // full copies of frames longer than a slot
        uint8_t *h_slot = nullptr, *h_close = nullptr;  // pinned: 32-B header slots
        uint16_t *h_len = nullptr;
        uint8_t *h_out = nullptr;  // packed SoA outputs (see dec_ptrs)
        std::vector<void *> user;
        uint8_t *d_slot = nullptr, *d_close = nullptr, *d_out = nullptr;
        uint16_t *d_len = nullptr;
    };

    int alloc_slots();
    void free_slots();
    int launch_enc(EncSlot &s);
    int launch_dec(DecSlot &s);
    int deliver_enc(EncSlot &s);
    int deliver_dec(DecSlot &s);
    int rotate_enc();
    int rotate_dec();
    size_t dec_out_bytes() const;
    void dec_ptrs(uint8_t *base, rsk_decode_out &o) const;

    rsk_ctx *ctx_ = nullptr;
    int device_ = 0;
    uint32_t batch_ = 0;
    bool ok_ = false;
    EncSlot enc_[2];
    DecSlot dec_[2];
    int enc_cur_ = 0, dec_cur_ = 0;
    SendFn send_cb_;
    ResetFn reset_cb_;
    RecvFn recv_cb_;
    uint64_t n_sent_ = 0, n_recv_ = 0, n_cb_fail_ = 0;
};

}  // namespace rsk
