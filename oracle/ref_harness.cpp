/*
 * ref_harness.cpp — TEST INFRASTRUCTURE ONLY.
 *
 * C-ABI harness over the REFERENCE's own codec objects (compiled from /root/reference by
 * oracle/Makefile into oracle/_ref/librsk_ref.so; nothing from the reference is copied here).
 * It exposes the reference functions to Python (tests/golden/make_golden.py, the oracle pin tests)
 * and times them for bench.py's cpu_baseline leg (kind "reference").
 *
 * RConn itself cannot be linked standalone (IGroup/RawTcp/libnet/libuv loop), so ref_rconn_output
 * and ref_rconn_onrecv replay RConn.cpp's statement sequence around the reference's compute_hash,
 * EncHead::Enc2Buf, EncHead::DecodeBuf and hash_equal — the same loop the SURVEY (§6) timed.
 */
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "rscomm.h"
#include "rstype.h"
#include "bean/EncHead.h"
#include "bean/TcpInfo.h"
#include "src/util/KeyGenerator.h"
#include "util/rhash.h"

extern "C" {

/* util/rhash.cpp:20-41 */
int ref_compute_hash(char *tag, const char *key, int key_len, const char *data, int data_len) {
    std::string k(key, (size_t)key_len);
    char *p = compute_hash(tag, k, data, data_len);
    return (int)(p - tag);
}

/* util/rhash.cpp:71-92 */
int ref_hash_equal(const char *tag, const char *key, int key_len, const char *data, int data_len) {
    std::string k(key, (size_t)key_len);
    return hash_equal(tag, k, data, data_len) ? 1 : 0;
}

/* bean/EncHead.cpp:9-24 — returns bytes advanced or -1 */
int ref_enc2buf(char *p, int buf_len, uint8_t cmd, const char *id, uint32_t conv, uint64_t key) {
    EncHead h;
    h.SetCmd(cmd);
    IdBufType ib;
    std::memcpy(ib.data(), id, ID_BUF_SIZE);
    h.SetIdBuf(ib);
    h.SetConv(conv);
    h.SetConnKey(key);
    char *r = h.Enc2Buf(p, buf_len);
    return r ? (int)(r - p) : -1;
}

/* bean/EncHead.cpp:39-55 — returns len (p + len - p) or -1 */
int ref_decodebuf(const char *p, int buf_len, uint8_t *cmd, char *id, uint32_t *conv, uint64_t *key) {
    EncHead h;
    const char *r = EncHead::DecodeBuf(h, p, buf_len);
    if (!r) return -1;
    *cmd = h.Cmd();
    IdBufType ib = h.IdBuf();
    std::memcpy(id, ib.data(), ID_BUF_SIZE);
    *conv = h.Conv();
    *key = h.ConnKey();
    return (int)(r - p);
}

/* conn/RConn.cpp:87-105 statement sequence; frame gets the bytes RConn would hand to RawTcp::Send.
 * Returns frame length, -1 (oversize) or 0 (nread == 0: reset path). */
int ref_rconn_output(const char *key, int key_len, const char *payload, int nread, uint8_t cmd,
                     const char *id, uint32_t conv, uint64_t ckey, char *frame) {
    if (nread == 0) return 0;
    if (nread < 0) return nread;
    EncHead head;
    head.SetCmd(cmd);
    IdBufType ib;
    std::memcpy(ib.data(), id, ID_BUF_SIZE);
    head.SetIdBuf(ib);
    head.SetConv(conv);
    head.SetConnKey(ckey);
    const int ENC_SIZE = head.GetSize();
    if (HASH_BUF_SIZE + ENC_SIZE + nread > OM_MAX_PKT_SIZE) return -1;
    std::string k(key, (size_t)key_len);
    char base[OM_MAX_PKT_SIZE] = {0};
    char *p = compute_hash(base, k, payload, nread);
    p = head.Enc2Buf(p, OM_MAX_PKT_SIZE - (int)(p - base));
    std::memcpy(p, payload, (size_t)nread);
    p += nread;
    int len = (int)(p - base);
    std::memcpy(frame, base, (size_t)len);
    return len;
}

/* conn/RConn.cpp:64-85.  Returns 1 valid (fields filled), 0 close-notify, -1 drop. */
int ref_rconn_onrecv(const char *key, int key_len, const char *frame, int nread, int is_tcp_close,
                     uint8_t *hlen, uint8_t *cmd, char *id, uint32_t *conv, uint64_t *ckey,
                     int *pay_off, int *pay_len) {
    const int MIN_LEN = HASH_BUF_SIZE + EncHead::GetMinEncSize();
    std::string k(key, (size_t)key_len);
    if (nread > MIN_LEN) {
        EncHead head;
        const char *p = frame + HASH_BUF_SIZE;
        p = EncHead::DecodeBuf(head, p, nread - HASH_BUF_SIZE);
        if (p && hash_equal(frame, k, p, nread - (int)(p - frame))) {
            *hlen = (uint8_t)(p - frame - HASH_BUF_SIZE);
            *cmd = head.Cmd();
            IdBufType ib = head.IdBuf();
            std::memcpy(id, ib.data(), ID_BUF_SIZE);
            *conv = head.Conv();
            *ckey = head.ConnKey();
            *pay_off = (int)(p - frame);
            *pay_len = nread - (int)(p - frame);
            return 1;
        }
    } else if (is_tcp_close) {
        return 0;
    }
    return -1;
}

/* src/util/KeyGenerator.cpp:16-25 via a TcpInfo */
uint64_t ref_key_for_tcp(uint16_t sp, uint16_t dp) {
    TcpInfo info;
    info.sp = sp;
    info.dp = dp;
    return KeyGenerator::KeyForTcp(info);
}

/* src/util/KeyGenerator.cpp:27-36 via a (UDP) ConnInfo */
uint64_t ref_key_for_udp(uint16_t sp, uint16_t dp) {
    ConnInfo info;
    info.sp = sp;
    info.dp = dp;
    return KeyGenerator::KeyForUdp(info);
}

/* bean/TcpInfo.cpp:20-32 — returns bytes written or -1 */
int ref_tcpinfo_encode(uint32_t src, uint32_t dst, uint16_t sp, uint16_t dp, uint32_t seq,
                       uint32_t ack, uint8_t flag, char *rec, int len) {
    TcpInfo t;
    t.src = src; t.dst = dst; t.sp = sp; t.dp = dp; t.seq = seq; t.ack = ack; t.flag = flag;
    char *r = t.Encode(rec, len);
    return r ? (int)(r - rec) : -1;
}

/* bean/TcpInfo.cpp:35-45 */
int ref_tcpinfo_decode(const char *rec, int len, uint32_t *out7 /* src,dst,sp,dp,seq,ack,flag */) {
    TcpInfo t;
    const char *r = t.Decode(rec, len);
    if (!r) return -1;
    out7[0] = t.src; out7[1] = t.dst; out7[2] = t.sp; out7[3] = t.dp;
    out7[4] = t.seq; out7[5] = t.ack; out7[6] = t.flag;
    return (int)(r - rec);
}

/* CPU baseline: for each packet i in [0, n): RConn::Output framing into a zeroed 1500-B stack
 * buffer (as RConn.cpp:100-104 does), then RConn::OnRecv's DecodeBuf + hash_equal on that frame.
 * Payloads are read from payload_arena + pay_off[i]; frames are also stored to frame_arena +
 * frame_off[i] (the device path's output) so the whole job is comparable.  Returns the number of
 * verified packets.  Threads take contiguous shards. */
uint64_t ref_bench_codec(const char *key, int key_len, uint32_t n, const char *payload_arena,
                         const uint64_t *pay_off, const uint16_t *pay_len, const uint8_t *cmd,
                         const uint32_t *conv, const uint64_t *ckey, const char *id,
                         char *frame_arena, const uint64_t *frame_off, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    std::string k(key, (size_t)key_len);
    std::vector<uint64_t> ok((size_t)nthreads, 0);
    auto work = [&](int t) {
        uint32_t lo = (uint32_t)((uint64_t)n * t / nthreads), hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
        IdBufType ib;
        std::memcpy(ib.data(), id, ID_BUF_SIZE);
        uint64_t good = 0;
        for (uint32_t i = lo; i < hi; i++) {
            const char *pl = payload_arena + pay_off[i];
            int nread = pay_len[i];
            EncHead head;
            head.SetCmd(cmd[i]);
            head.SetIdBuf(ib);
            head.SetConv(conv[i]);
            head.SetConnKey(ckey[i]);
            if (nread <= 0 || HASH_BUF_SIZE + head.GetSize() + nread > OM_MAX_PKT_SIZE) continue;
            char base[OM_MAX_PKT_SIZE] = {0};
            char *p = compute_hash(base, k, pl, nread);
            p = head.Enc2Buf(p, OM_MAX_PKT_SIZE - (int)(p - base));
            std::memcpy(p, pl, (size_t)nread);
            p += nread;
            int flen = (int)(p - base);
            std::memcpy(frame_arena + frame_off[i], base, (size_t)flen);
            /* receive side on the stored frame */
            const char *fr = frame_arena + frame_off[i];
            if (flen > HASH_BUF_SIZE + EncHead::GetMinEncSize()) {
                EncHead dh;
                const char *q = EncHead::DecodeBuf(dh, fr + HASH_BUF_SIZE, flen - HASH_BUF_SIZE);
                if (q && hash_equal(fr, k, q, flen - (int)(q - fr))) good++;
            }
        }
        ok[(size_t)t] = good;
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; t++) th.emplace_back(work, t);
    work(0);
    for (auto &x : th) x.join();
    uint64_t s = 0;
    for (auto v : ok) s += v;
    return s;
}

}  // extern "C"
