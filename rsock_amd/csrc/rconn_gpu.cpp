// rconn_gpu.cpp — RConnGpu (see rconn_gpu.h) and its C ABI (include/rsk_rconn.h).
#include "rconn_gpu.h"

#include <cstring>

#include "../../include/rsk_rconn.h"

namespace rsk {

namespace {
template <typename T>
int hmalloc(T **p, size_t n) {
    return hipHostMalloc(reinterpret_cast<void **>(p), n * sizeof(T) + 16, hipHostMallocDefault) == hipSuccess ? 0 : -1;
}
template <typename T>
int dmalloc(T **p, size_t n) {
    return hipMalloc(reinterpret_cast<void **>(p), n * sizeof(T) + 16) == hipSuccess ? 0 : -1;
}
template <typename T>
void hfree(T *&p) {
    if (p) (void)hipHostFree(p);
    p = nullptr;
}
template <typename T>
void dfree(T *&p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}
size_t up8(size_t x) { return (x + 15) & ~size_t(15); }
}  // namespace

RConnGpu::RConnGpu(const std::string &hash_key, int device, uint32_t batch) : device_(device), batch_(batch) {
    if (batch_ == 0) batch_ = 1;
    ctx_ = rsk_create(reinterpret_cast<const uint8_t *>(hash_key.data()), (uint32_t)hash_key.size(), device);
    if (!ctx_) return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device_);
    // no compaction scratch to reserve: decodes run on the slot streams without valid_idx / n_valid
    ok_ = alloc_slots() == 0;
    (void)hipSetDevice(prev);
}

RConnGpu::~RConnGpu() {
    if (ok_) (void)Flush();
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device_);
    free_slots();
    (void)hipSetDevice(prev);
    if (ctx_) rsk_destroy(ctx_);
}

size_t RConnGpu::dec_out_bytes() const {
    const size_t n = batch_;
    return up8(8 * n) + up8(4 * n) + up8(4 * n) + up8(2 * n) * 2 + up8(8 * n) + up8(n) * 3 + 16;
}

// one device (or pinned host) block holds every SoA output of a decode batch
void RConnGpu::dec_ptrs(uint8_t *b, rsk_decode_out &o) const {
    const size_t n = batch_;
    o.conn_key = reinterpret_cast<uint64_t *>(b);
    b += up8(8 * n);
    o.conv = reinterpret_cast<uint32_t *>(b);
    b += up8(4 * n);
    o.valid_idx = reinterpret_cast<uint32_t *>(b);
    b += up8(4 * n);
    o.pay_off = reinterpret_cast<uint16_t *>(b);
    b += up8(2 * n);
    o.pay_len = reinterpret_cast<uint16_t *>(b);
    b += up8(2 * n);
    o.id = b;
    b += up8(8 * n);
    o.hlen = b;
    b += up8(n);
    o.cmd = b;
    b += up8(n);
    o.status = reinterpret_cast<int8_t *>(b);
    b += up8(n);
    o.n_valid = reinterpret_cast<uint32_t *>(b);
}

int RConnGpu::alloc_slots() {
    const size_t n = batch_;
    for (auto &s : enc_) {
        if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess) return -1;
        if (hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess) return -1;
        if (hmalloc(&s.h_b0, n) || hmalloc(&s.h_cmd, n) || hmalloc(&s.h_id, 8 * n) || hmalloc(&s.h_hdr, 32 * n) ||
            hmalloc(&s.h_key, n) || hmalloc(&s.h_len, n) || hmalloc(&s.h_conv, n) || hmalloc(&s.h_status, n))
            return -1;
        if (dmalloc(&s.d_b0, n) || dmalloc(&s.d_cmd, n) || dmalloc(&s.d_id, 8 * n) || dmalloc(&s.d_hdr, 32 * n) ||
            dmalloc(&s.d_key, n) || dmalloc(&s.d_len, n) || dmalloc(&s.d_conv, n) || dmalloc(&s.d_status, n))
            return -1;
        if (hmalloc(&s.frame, n * kFramePitch)) return -1;
        s.user.resize(n);
    }
    for (auto &s : dec_) {
        if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess) return -1;
        if (hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess) return -1;
        if (hmalloc(&s.h_slot, 32 * n) || hmalloc(&s.h_close, n) || hmalloc(&s.h_len, n) ||
            hmalloc(&s.h_out, dec_out_bytes()))
            return -1;
        if (dmalloc(&s.d_slot, 32 * n) || dmalloc(&s.d_close, n) || dmalloc(&s.d_len, n) ||
            dmalloc(&s.d_out, dec_out_bytes()))
            return -1;
        if (hmalloc(&s.frame, n * kFramePitch)) return -1;
        s.user.resize(n);
        s.big.resize(n);
    }
    return 0;
}

void RConnGpu::free_slots() {
    for (auto &s : enc_) {
        if (s.stream) (void)hipStreamSynchronize(s.stream);
        hfree(s.frame); hfree(s.h_b0); hfree(s.h_cmd); hfree(s.h_id); hfree(s.h_hdr); hfree(s.h_key); hfree(s.h_len);
        hfree(s.h_conv); hfree(s.h_status);
        dfree(s.d_b0); dfree(s.d_cmd); dfree(s.d_id); dfree(s.d_hdr); dfree(s.d_key); dfree(s.d_len);
        dfree(s.d_conv); dfree(s.d_status);
        if (s.done) (void)hipEventDestroy(s.done);
        if (s.stream) (void)hipStreamDestroy(s.stream);
        s.done = nullptr;
        s.stream = nullptr;
    }
    for (auto &s : dec_) {
        if (s.stream) (void)hipStreamSynchronize(s.stream);
        hfree(s.frame); hfree(s.h_slot); hfree(s.h_close); hfree(s.h_len); hfree(s.h_out);
        dfree(s.d_slot); dfree(s.d_close); dfree(s.d_len); dfree(s.d_out);
        if (s.done) (void)hipEventDestroy(s.done);
        if (s.stream) (void)hipStreamDestroy(s.stream);
        s.done = nullptr;
        s.stream = nullptr;
    }
}

// ---- send side -------------------------------------------------------------------------------
int RConnGpu::Output(ssize_t nread, const char *base, const EncHeadFields &head, void *user) {
    if (nread < 0) return (int)nread;                                   // RConn.cpp:127
    if (RSK_HEAD_SIZE + nread > RSK_MAX_PKT_SIZE) return RSK_SEND_OVERSIZE;  // RConn.cpp:94-98
    if (!ok_) return RSK_EDEVICE;
    // nread == 0 is RConnReset::SendReset (RConn.cpp:119-123).  It is queued like a frame (the kernel
    // gives it status RSK_SEND_RESET) so that deliver_enc fires the reset callback in input order,
    // after the frames queued before it, as the reference's synchronous Output would.
    EncSlot &s = enc_[enc_cur_];
    const uint32_t i = s.count;
    if (nread) std::memcpy(s.frame + (size_t)i * kFramePitch + RSK_HEAD_SIZE, base, (size_t)nread);  // RConn.cpp:104
    s.h_b0[i] = nread ? (uint8_t)base[0] : 0;
    s.h_len[i] = (uint16_t)nread;
    s.h_cmd[i] = head.cmd;
    std::memcpy(s.h_id + 8 * (size_t)i, head.id, 8);
    s.h_conv[i] = head.conv;
    s.h_key[i] = head.conn_key;
    s.user[i] = user;
    if (++s.count == batch_) {
        const int r = rotate_enc();
        if (r) return r;
    }
    return nread == 0 ? 0 : (int)(RSK_HEAD_SIZE + nread);
}

int RConnGpu::launch_enc(EncSlot &s) {
    const size_t n = s.count;
    hipStream_t st = s.stream;
    if (hipMemcpyAsync(s.d_b0, s.h_b0, n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(s.d_len, s.h_len, 2 * n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(s.d_cmd, s.h_cmd, n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(s.d_id, s.h_id, 8 * n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(s.d_conv, s.h_conv, 4 * n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(s.d_key, s.h_key, 8 * n, hipMemcpyHostToDevice, st) != hipSuccess)
        return RSK_EDEVICE;
    rsk_encode_hdr_in in{};
    in.first_byte = s.d_b0; in.pay_len = s.d_len; in.cmd = s.d_cmd; in.conv = s.d_conv; in.conn_key = s.d_key;
    in.id = s.d_id;
    int r = rsk_encode_headers_batch(ctx_, (uint32_t)n, &in, s.d_hdr, s.d_status, st);
    if (r) return r;
    if (hipMemcpyAsync(s.h_hdr, s.d_hdr, 32 * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(s.h_status, s.d_status, 4 * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipEventRecord(s.done, st) != hipSuccess)
        return RSK_EDEVICE;
    s.in_flight = true;
    return 0;
}

int RConnGpu::deliver_enc(EncSlot &s) {
    if (!s.in_flight) return 0;
    if (hipEventSynchronize(s.done) != hipSuccess) return RSK_EDEVICE;
    for (uint32_t i = 0; i < s.count; ++i) {
        const int st = s.h_status[i];
        char *f = reinterpret_cast<char *>(s.frame) + (size_t)i * kFramePitch;
        if (st > 0) std::memcpy(f, s.h_hdr + 32 * (size_t)i, RSK_HEAD_SIZE);  // tag | EncHead (RConn.cpp:101-103)
        if (st > 0 && send_cb_ && send_cb_(f, st, s.user[i]) < 0) ++n_cb_fail_;
        if (st == RSK_SEND_RESET && reset_cb_ && reset_cb_(s.user[i]) < 0) ++n_cb_fail_;
        ++n_sent_;
    }
    s.count = 0;
    s.in_flight = false;
    return 0;
}

// launch the current slot, then make the other slot (the older batch) current after delivering it
int RConnGpu::rotate_enc() {
    EncSlot &cur = enc_[enc_cur_];
    int r = launch_enc(cur);
    if (r) return r;
    enc_cur_ ^= 1;
    return deliver_enc(enc_[enc_cur_]);
}

// ---- receive side ----------------------------------------------------------------------------
int RConnGpu::OnRecv(ssize_t nread, const char *base, bool tcp_close, void *user) {
    if (!ok_) return RSK_EDEVICE;
    if (nread < 0) nread = 0;
    if (nread > 0xFFFF) nread = 0xFFFF;  // frame_len is u16 (a UDP datagram is at most 65507 B)
    DecSlot &s = dec_[dec_cur_];
    const uint32_t i = s.count;
    // the caller may reuse `base` after the call: keep a copy for the payload hand-off (frames
    // longer than a slot on the heap); only the 32-B header slot goes to the GPU
    const size_t cp = (size_t)nread < kFramePitch ? (size_t)nread : kFramePitch;
    if (cp) std::memcpy(s.frame + (size_t)i * kFramePitch, base, cp);
    if ((size_t)nread > kFramePitch) s.big[i].assign(base, base + nread);
    rsk_stage_decode_header(reinterpret_cast<const uint8_t *>(base), (int)nread, s.h_slot + 32 * (size_t)i);
    s.h_len[i] = (uint16_t)nread;
    s.h_close[i] = tcp_close ? 1 : 0;
    s.user[i] = user;
    if (++s.count == batch_) return rotate_dec();
    return 0;
}

int RConnGpu::launch_dec(DecSlot &s) {
    const size_t n = s.count;
    hipStream_t st = s.stream;
    if (hipMemcpyAsync(s.d_slot, s.h_slot, 32 * n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(s.d_len, s.h_len, 2 * n, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(s.d_close, s.h_close, n, hipMemcpyHostToDevice, st) != hipSuccess)
        return RSK_EDEVICE;
    rsk_decode_out o{};
    dec_ptrs(s.d_out, o);
    o.valid_idx = nullptr;  // delivery walks every frame in order; no compaction needed
    o.n_valid = nullptr;
    int r = rsk_decode_headers_batch(ctx_, (uint32_t)n, s.d_slot, s.d_len, s.d_close, &o, st);
    if (r) return r;
    if (hipMemcpyAsync(s.h_out, s.d_out, dec_out_bytes(), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipEventRecord(s.done, st) != hipSuccess)
        return RSK_EDEVICE;
    s.in_flight = true;
    return 0;
}

int RConnGpu::deliver_dec(DecSlot &s) {
    if (!s.in_flight) return 0;
    if (hipEventSynchronize(s.done) != hipSuccess) return RSK_EDEVICE;
    rsk_decode_out o{};
    dec_ptrs(s.h_out, o);
    for (uint32_t i = 0; i < s.count; ++i) {
        RecvResult rr{};
        rr.status = o.status[i];
        rr.user = s.user[i];
        if (rr.status == RSK_RECV_VALID) {
            rr.hlen = o.hlen[i];
            rr.cmd = o.cmd[i];
            std::memcpy(rr.id, o.id + 8 * (size_t)i, 8);
            rr.conv = o.conv[i];
            rr.conn_key = o.conn_key[i];
            const char *fb = s.big[i].empty() ? reinterpret_cast<const char *>(s.frame) + (size_t)i * kFramePitch
                                              : s.big[i].data();
            rr.payload = fb + o.pay_off[i];
            rr.payload_len = o.pay_len[i];
        }
        if (recv_cb_) recv_cb_(rr);
        ++n_recv_;
        if (!s.big[i].empty()) std::vector<char>().swap(s.big[i]);
    }
    s.count = 0;
    s.in_flight = false;
    return 0;
}

int RConnGpu::rotate_dec() {
    DecSlot &cur = dec_[dec_cur_];
    int r = launch_dec(cur);
    if (r) return r;
    dec_cur_ ^= 1;
    return deliver_dec(dec_[dec_cur_]);
}

int RConnGpu::Flush() {
    if (!ok_) return RSK_EDEVICE;
    int r = 0;
    // older batch (the other slot) first, then the current one: input order is preserved
    if ((r = deliver_enc(enc_[enc_cur_ ^ 1]))) return r;
    if (enc_[enc_cur_].count) {
        if ((r = launch_enc(enc_[enc_cur_]))) return r;
        if ((r = deliver_enc(enc_[enc_cur_]))) return r;
    }
    if ((r = deliver_dec(dec_[dec_cur_ ^ 1]))) return r;
    if (dec_[dec_cur_].count) {
        if ((r = launch_dec(dec_[dec_cur_]))) return r;
        if ((r = deliver_dec(dec_[dec_cur_]))) return r;
    }
    return 0;
}

}  // namespace rsk

// ---- C ABI (include/rsk_rconn.h) --------------------------------------------------------------
struct rsk_rconn {
    rsk::RConnGpu impl;
    rsk_rconn(const std::string &k, int dev, uint32_t b) : impl(k, dev, b) {}
};

extern "C" {

rsk_rconn *rsk_rconn_create(const uint8_t *key, uint32_t key_len, int device, uint32_t batch) {
    auto *r = new rsk_rconn(std::string(reinterpret_cast<const char *>(key), key_len), device, batch);
    if (!r->impl.ok()) {
        delete r;
        return nullptr;
    }
    return r;
}

void rsk_rconn_destroy(rsk_rconn *r) { delete r; }

void rsk_rconn_set_callbacks(rsk_rconn *r, rsk_send_fn send, rsk_reset_fn reset, rsk_recv_fn recv, void *cb_arg) {
    if (!r) return;
    r->impl.SetSendCb([send, cb_arg](const char *f, int len, void *user) { return send ? send(f, len, user, cb_arg) : 0; });
    r->impl.SetResetCb([reset, cb_arg](void *user) { return reset ? reset(user, cb_arg) : 0; });
    r->impl.SetRecvCb([recv, cb_arg](const rsk::RecvResult &x) {
        return recv ? recv(x.status, x.hlen, x.cmd, x.id, x.conv, x.conn_key, x.payload, x.payload_len, x.user, cb_arg)
                    : 0;
    });
}

int rsk_rconn_output(rsk_rconn *r, int64_t nread, const char *base, uint8_t cmd, const uint8_t id[8], uint32_t conv,
                     uint64_t conn_key, void *user) {
    if (!r) return RSK_EINVAL;
    rsk::EncHeadFields h;
    h.cmd = cmd;
    if (id) std::memcpy(h.id, id, 8);
    h.conv = conv;
    h.conn_key = conn_key;
    return r->impl.Output((ssize_t)nread, base, h, user);
}

int rsk_rconn_onrecv(rsk_rconn *r, int64_t nread, const char *base, int tcp_close, void *user) {
    if (!r) return RSK_EINVAL;
    return r->impl.OnRecv((ssize_t)nread, base, tcp_close != 0, user);
}

int rsk_rconn_flush(rsk_rconn *r) { return r ? r->impl.Flush() : RSK_EINVAL; }

uint64_t rsk_rconn_callback_failures(const rsk_rconn *r) { return r ? r->impl.callback_failures() : 0; }

}  // extern "C"
