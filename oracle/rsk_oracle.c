/*
 * rsk_oracle.c — TEST INFRASTRUCTURE ONLY (see rsk_oracle.h).
 *
 * Clean-room CPU restatement of the rsock framing-codec path, written from RFC 1321 and from the
 * behaviour of the reference files cited per function.  Plain C99 + pthreads; no reference code.
 */
#define _GNU_SOURCE
#include "rsk_oracle.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rsk_codec.h"

/* ------------------------------------------------------------------------------------------------
 * MD5, RFC 1321 §3.  Follows thirdparty/md5.c:105-294 in result: little-endian message words,
 * 0x80 pad, 64-bit little-endian bit count at bytes 56..63, little-endian digest (OUT macro :254).
 * Written here as the textbook table-driven loop, not as the reference's unrolled macros.
 * --------------------------------------------------------------------------------------------- */
static const uint32_t K_[64] = {
    /* K[i] = floor(2^32 * |sin(i + 1)|), RFC 1321 §3.4 */
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
static const uint8_t S_[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                               5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                               4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                               6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};

static uint32_t rotl32(uint32_t x, unsigned s) { return (x << s) | (x >> (32u - s)); }

static void md5_compress(uint32_t st[4], const uint8_t blk[64]) {
    uint32_t m[16];
    for (int i = 0; i < 16; i++)
        m[i] = (uint32_t)blk[4 * i] | ((uint32_t)blk[4 * i + 1] << 8) |
               ((uint32_t)blk[4 * i + 2] << 16) | ((uint32_t)blk[4 * i + 3] << 24);
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    for (int i = 0; i < 64; i++) {
        uint32_t f;
        int g;
        if (i < 16) {
            f = (b & c) | (~b & d);
            g = i;
        } else if (i < 32) {
            f = (d & b) | (~d & c);
            g = (5 * i + 1) & 15;
        } else if (i < 48) {
            f = b ^ c ^ d;
            g = (3 * i + 5) & 15;
        } else {
            f = c ^ (b | ~d);
            g = (7 * i) & 15;
        }
        uint32_t t = d;
        d = c;
        c = b;
        b = b + rotl32(a + f + K_[i] + m[g], S_[i]);
        a = t;
    }
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
}

void orc_md5(const uint8_t *msg, size_t len, uint8_t digest[16]) {
    uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u}; /* md5.c:212-221 */
    size_t off = 0;
    for (; off + 64 <= len; off += 64) md5_compress(st, msg + off);
    uint8_t tail[128];
    size_t rem = len - off;
    memset(tail, 0, sizeof tail);
    if (rem) memcpy(tail, msg + off, rem);
    tail[rem] = 0x80;
    size_t tl = (rem + 1 + 8 <= 64) ? 64 : 128;
    uint64_t bits = (uint64_t)len << 3;
    for (int i = 0; i < 8; i++) tail[tl - 8 + i] = (uint8_t)(bits >> (8 * i));
    md5_compress(st, tail);
    if (tl == 128) md5_compress(st, tail + 64);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) digest[4 * i + j] = (uint8_t)(st[i] >> (8 * j));
}

/* ------------------------------------------------------------------------------------------------
 * Tag: util/rhash.cpp:20-41 (compute_hash) — MD5_Update(key) then MD5_Update(data, 1): only the
 * FIRST payload byte is hashed; the tag is digest bytes [16-8 .. 16) (rhash.cpp:34-35).
 * --------------------------------------------------------------------------------------------- */
void orc_compute_hash(uint8_t tag[8], const uint8_t *key, size_t key_len, uint8_t data0) {
    uint8_t stackbuf[256];
    uint8_t *msg = key_len + 1 <= sizeof stackbuf ? stackbuf : (uint8_t *)malloc(key_len + 1);
    if (key_len) memcpy(msg, key, key_len);
    msg[key_len] = data0;
    uint8_t dg[16];
    orc_md5(msg, key_len + 1, dg);
    memcpy(tag, dg + 8, 8);
    if (msg != stackbuf) free(msg);
}

/* util/rhash.cpp:71-92 (hash_equal): false if data == NULL or data_len <= 0 (:73-75). */
int orc_hash_equal(const uint8_t tag[8], const uint8_t *key, size_t key_len, const uint8_t *data,
                   int data_len) {
    if (!data || data_len <= 0) return 0;
    uint8_t t[8];
    orc_compute_hash(t, key, key_len, data[0]);
    return memcmp(t, tag, 8) == 0;
}

/* ------------------------------------------------------------------------------------------------
 * EncHead wire record (bean/EncHead.h:12-63): len u8 | cmd u8 | IdBuf[8] | conv u32 LE |
 * connKey u64 LE (KeyGenerator::EncodeKey, KeyGenerator.cpp:63) | reserved u8 (always 0).
 * All multi-byte fields little-endian (util/enc.c:28-36, :103-109 store natively on LE hosts).
 * --------------------------------------------------------------------------------------------- */
static void put_le(uint8_t *p, uint64_t v, int n) {
    for (int i = 0; i < n; i++) p[i] = (uint8_t)(v >> (8 * i));
}
static uint64_t get_le(const uint8_t *p, int n) {
    uint64_t v = 0;
    for (int i = 0; i < n; i++) v |= (uint64_t)p[i] << (8 * i);
    return v;
}

/* EncHead::Enc2Buf (EncHead.cpp:9-24): writes len = GetSize() = 23. */
int orc_enchead_encode(uint8_t *p, int buf_len, uint8_t cmd, const uint8_t id[8], uint32_t conv,
                       uint64_t conn_key) {
    if (!p || buf_len < RSK_ENC_HEAD_SIZE) return -1;
    p[0] = RSK_ENC_HEAD_SIZE;
    p[1] = cmd;
    memcpy(p + 2, id, 8);
    put_le(p + 10, conv, 4);
    put_le(p + 14, conn_key, 8);
    p[22] = 0;
    return RSK_ENC_HEAD_SIZE;
}

/* EncHead::DecodeBuf (EncHead.cpp:39-55): needs buf_len >= 23; fails if len byte > buf_len;
 * reads every other field at its FIXED offset; the payload starts at p + len (not p + 23). */
int orc_enchead_decode(const uint8_t *p, int buf_len, uint8_t *len, uint8_t *cmd, uint8_t id[8],
                       uint32_t *conv, uint64_t *conn_key) {
    if (!p || buf_len < RSK_ENC_HEAD_SIZE) return -1;
    uint8_t l = p[0];
    if ((int)l > buf_len) return -1;
    if (len) *len = l;
    if (cmd) *cmd = p[1];
    if (id) memcpy(id, p + 2, 8);
    if (conv) *conv = (uint32_t)get_le(p + 10, 4);
    if (conn_key) *conn_key = get_le(p + 14, 8);
    return l;
}

/* ------------------------------------------------------------------------------------------------
 * RConn::Output framing (conn/RConn.cpp:87-105):
 *   nread > 0: drop (-1) if 8 + 23 + nread > 1500 (:94-98); else tag = compute_hash(payload) at
 *   frame[0..8) (:101), EncHead at frame[8..31) (:102), payload at frame[31..) (:104).
 *   nread == 0: SendReset path (:119-123) -> status 0, nothing framed.
 * --------------------------------------------------------------------------------------------- */
int orc_rconn_output(const uint8_t *key, size_t key_len, const uint8_t *payload, int nread,
                     uint8_t cmd, const uint8_t id[8], uint32_t conv, uint64_t conn_key,
                     uint8_t *frame) {
    if (nread < 0) return nread;
    if (nread == 0) return RSK_SEND_RESET;
    if (RSK_HEAD_SIZE + nread > RSK_MAX_PKT_SIZE) return RSK_SEND_OVERSIZE;
    orc_compute_hash(frame, key, key_len, payload[0]);
    orc_enchead_encode(frame + 8, RSK_MAX_PKT_SIZE - 8, cmd, id, conv, conn_key);
    memcpy(frame + RSK_HEAD_SIZE, payload, (size_t)nread);
    return RSK_HEAD_SIZE + nread;
}

/* ------------------------------------------------------------------------------------------------
 * RConn::OnRecv (conn/RConn.cpp:64-85):
 *   nread > 31 (:68): p = DecodeBuf(frame + 8, nread - 8) (:71); valid iff p != NULL and
 *     hash_equal(frame, key, p, nread - (p - frame)) (:72) -> forward (p, nread-8-len) (:73-75).
 *     A frame of > 31 bytes that fails verification is dropped even with FIN/RST set.
 *   else: TCP with FIN|RST -> NotifyTcpFinOrRst, return 0 (:77-82).
 *   otherwise return -1.
 * --------------------------------------------------------------------------------------------- */
int orc_rconn_onrecv(const uint8_t *key, size_t key_len, const uint8_t *frame, int nread,
                     int is_tcp_close, orc_dec *out) {
    memset(out, 0, sizeof *out);
    out->status = RSK_RECV_DROP;
    if (nread > RSK_HEAD_SIZE) {
        orc_dec d;
        memset(&d, 0, sizeof d);
        int l = orc_enchead_decode(frame + 8, nread - 8, &d.hlen, &d.cmd, d.id, &d.conv, &d.conn_key);
        if (l >= 0) {
            int data_len = nread - 8 - l;
            if (orc_hash_equal(frame, key, key_len, frame + 8 + l, data_len)) {
                d.pay_off = (uint16_t)(8 + l);
                d.pay_len = (uint16_t)data_len;
                d.status = RSK_RECV_VALID;
                *out = d;
            }
        }
    } else if (is_tcp_close) {
        out->status = RSK_RECV_CLOSE;
    }
    return out->status;
}

/* ------------------------------------------------------------------------------------------------
 * RawTcp::RawInput (conn/RawTcp.cpp:138-237) + cap2uv size check (:239-244), cap_headers.h:16-32.
 *   1. hdr->len (wire length) < 44 -> drop (:139)
 *   2. EN10MB: u16 at 12 read little-endian must be 0x0008 (OM_PROTO_IP), ip at 14 (:144-151);
 *      NULL: u32 at 0 read little-endian must be 2, ip at 4 (:152-160)
 *   3. ip[9] (ip_p) != 6 -> drop (:167-172)
 *   4. tcp = ip + (ip[0]&15)*4; payload = tcp + (tcp[12]>>4)*4;
 *      payload_len = ntohs(ip[2..4]) - (payload - ip) (:174-177)
 *   5. TcpInfo = reversed "self" view (:213-219)
 *   6. SYN with ack pool -> AddInfoFromPeer (server: Reverse first), return 0 (:221-228)
 *   7. payload_len < 9 && !(FIN|RST) -> drop (:232-234); seq += payload_len (:235)
 *   8. cap2uv: payload_len + 2*sizeof(sockaddr_in) > 1500 -> drop (:240-244)
 * Deviations (defined where the reference is undefined): any header byte or payload byte beyond
 * cap_len, and negative payload_len with FIN|RST (memcpy of a negative length at :251), give
 * RSK_PARSE_MALFORMED.
 * --------------------------------------------------------------------------------------------- */
static uint32_t be16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | p[1]; }
static uint32_t be32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

int orc_rawinput(const uint8_t *pkt, uint32_t wire_len, uint32_t cap_len, int datalink, int flags,
                 orc_tcpinfo *o) {
    memset(o, 0, sizeof *o);
    o->parse_status = RSK_PARSE_DROP;
    if (wire_len < 44) return o->parse_status;
    uint32_t ipo;
    if (datalink == RSK_DLT_EN10MB) {
        if (cap_len < 14) return o->parse_status = RSK_PARSE_MALFORMED;
        if (get_le(pkt + 12, 2) != 0x0008) return o->parse_status;
        ipo = 14;
    } else if (datalink == RSK_DLT_NULL) {
        if (cap_len < 4) return o->parse_status = RSK_PARSE_MALFORMED;
        if (get_le(pkt, 4) != 2) return o->parse_status;
        ipo = 4;
    } else {
        return o->parse_status; /* the batch API rejects other datalinks up front */
    }
    if (cap_len < ipo + 20) return o->parse_status = RSK_PARSE_MALFORMED;
    const uint8_t *ip = pkt + ipo;
    if (ip[9] != 6) return o->parse_status;
    uint32_t ihl = (uint32_t)(ip[0] & 15) * 4;
    uint32_t tcpo = ipo + ihl;
    if (cap_len < tcpo + 20) return o->parse_status = RSK_PARSE_MALFORMED;
    const uint8_t *tcp = pkt + tcpo;
    uint32_t thl = (uint32_t)(tcp[12] >> 4) * 4;
    uint32_t payo = tcpo + thl;
    int payload_len = (int)be16(ip + 2) - (int)(ihl + thl);
    uint8_t fl = tcp[13];
    uint32_t src = (uint32_t)get_le(ip + 16, 4), dst = (uint32_t)get_le(ip + 12, 4);
    uint16_t sp = (uint16_t)be16(tcp + 2), dp = (uint16_t)be16(tcp + 0);
    uint32_t seq = be32(tcp + 4), ack = be32(tcp + 8);
    if ((fl & RSK_TH_SYN) && (flags & RSK_PARSE_HAS_ACK_POOL)) {
        if (flags & RSK_PARSE_IS_SERVER) { /* TcpInfo::Reverse, TcpInfo.cpp:60-63 */
            uint32_t t32 = src; src = dst; dst = t32;
            uint16_t t16 = sp; sp = dp; dp = t16;
            t32 = seq; seq = ack; ack = t32;
        }
        o->src = src; o->dst = dst; o->sp = sp; o->dp = dp; o->seq = seq; o->ack = ack; o->flag = fl;
        o->cap_pay_off = (uint16_t)payo;
        return o->parse_status = RSK_PARSE_SYN;
    }
    int close = (fl & (RSK_TH_FIN | RSK_TH_RST)) != 0;
    if (payload_len < RSK_HASH_BUF_SIZE + 1 && !close) return o->parse_status;
    /* cap2uv computes payload_len + 2*sizeof(SA4) in size_t (:240): a negative payload_len below
     * -32 wraps to a huge value and is dropped there; -32..-1 reaches memcpy with a negative
     * length (UB) and is MALFORMED here. */
    if (payload_len < -32) return o->parse_status;
    if (payload_len < 0) return o->parse_status = RSK_PARSE_MALFORMED;
    if (payload_len + 32 > RSK_MAX_PKT_SIZE) return o->parse_status;
    if ((uint64_t)payo + (uint64_t)payload_len > cap_len) return o->parse_status = RSK_PARSE_MALFORMED;
    o->src = src; o->dst = dst; o->sp = sp; o->dp = dp;
    o->seq = seq + (uint32_t)payload_len; o->ack = ack; o->flag = fl;
    o->cap_pay_off = (uint16_t)payo;
    o->cap_pay_len = (uint16_t)payload_len;
    return o->parse_status = RSK_PARSE_DELIVER;
}

/* TcpInfo::Encode (TcpInfo.cpp:20-32 -> ConnInfo::Encode ConnInfo.cpp:12-20): src, dst LE32,
 * sp, dp LE16, seq, ack LE32, flag. */
int orc_tcpinfo_encode(const orc_tcpinfo *t, uint8_t rec[21]) {
    put_le(rec + 0, t->src, 4);
    put_le(rec + 4, t->dst, 4);
    put_le(rec + 8, t->sp, 2);
    put_le(rec + 10, t->dp, 2);
    put_le(rec + 12, t->seq, 4);
    put_le(rec + 16, t->ack, 4);
    rec[20] = t->flag;
    return 21;
}

/* TcpInfo::Decode (TcpInfo.cpp:35-45, ConnInfo.cpp:23-32): needs 12 bytes for the ConnInfo part.
 * The reference's second length check (TcpInfo.cpp:40, `p - buf < 9`) compares the CONSUMED
 * length, which is always 12, so it never fails: a 12..20-byte record reads past its end there.
 * Here a record shorter than 21 bytes is rejected (documented deviation on a malformed input). */
int orc_tcpinfo_decode(const uint8_t *rec, int len, orc_tcpinfo *t) {
    if (len < 21) return -1;
    memset(t, 0, sizeof *t);
    t->src = (uint32_t)get_le(rec + 0, 4);
    t->dst = (uint32_t)get_le(rec + 4, 4);
    t->sp = (uint16_t)get_le(rec + 8, 2);
    t->dp = (uint16_t)get_le(rec + 10, 2);
    t->seq = (uint32_t)get_le(rec + 12, 4);
    t->ack = (uint32_t)get_le(rec + 16, 4);
    t->flag = rec[20];
    return 21;
}

/* RawTcp::syncInput (conn/RawTcp.cpp:262-276) + RConn::OnRecv: the loop thread's side of cap2uv's
 * hand-off.  A record is the 21-B TcpInfo followed by the frame.  nread <= 0 never reaches Decode;
 * a failed Decode returns -1 before Input (both: parse_status DROP, dec DROP); otherwise
 * Input(nread - 21) reaches RConn::OnRecv with is_tcp_close = HasCloseFlag() (TcpInfo.h:31-33). */
int orc_syncinput(const uint8_t *key, size_t key_len, const uint8_t *rec, int nread, orc_tcpinfo *t,
                  orc_dec *d) {
    memset(t, 0, sizeof *t);
    memset(d, 0, sizeof *d);
    d->status = RSK_RECV_DROP;
    t->parse_status = RSK_PARSE_DROP;
    if (nread <= 0 || orc_tcpinfo_decode(rec, nread, t) < 0) return RSK_PARSE_DROP;
    t->parse_status = RSK_PARSE_DELIVER;
    t->cap_pay_off = 21;
    t->cap_pay_len = (uint16_t)(nread - 21);
    orc_rconn_onrecv(key, key_len, rec + 21, nread - 21, (t->flag & (RSK_TH_FIN | RSK_TH_RST)) != 0, d);
    return RSK_PARSE_DELIVER;
}

/* ------------------------------------------------------------------------------------------------
 * Send-side wire build: RawTcp::SendRawTcp (conn/RawTcp.cpp:280-341) = libnet_build_tcp(sp, dp,
 * seq, ack, flag, win 65535, sum 0 = auto, urg 0, len = 20 + frame) + libnet_build_ipv4(
 * 40 + frame, tos 0, id = mIpId++, IP_DF, TTL_OUT 64, IPPROTO_TCP, sum 0 = auto, src, dst).
 * Checksums per RFC 791 / RFC 793 (pseudo-header) with the RFC 1071 one's-complement sum.  libnet
 * 1.1.6 is present only as the reference's prebuilt .a, so this restatement is pinned to the RFCs
 * (and an independent Python restatement in tests), not to libnet output.
 * --------------------------------------------------------------------------------------------- */
uint16_t orc_inet_csum(const uint8_t *p, size_t n, uint32_t init) {
    uint64_t s = init;
    size_t i = 0;
    for (; i + 1 < n; i += 2) s += ((uint32_t)p[i] << 8) | p[i + 1];
    if (i < n) s += (uint32_t)p[i] << 8;
    while (s >> 16) s = (s & 0xffff) + (s >> 16);
    return (uint16_t)~s;
}

int orc_build_wire(const uint8_t *frame, int frame_len, uint32_t src, uint32_t dst, uint16_t sp,
                   uint16_t dp, uint32_t seq, uint32_t ack, uint8_t flag, uint16_t ip_id,
                   const uint8_t *eth, uint8_t *wire) {
    int o = 0;
    if (eth) {
        memcpy(wire, eth, 14);
        o = 14;
    }
    uint8_t *ip = wire + o, *tcp = ip + 20;
    const int tot = 40 + frame_len;
    ip[0] = 0x45; ip[1] = 0;
    ip[2] = (uint8_t)(tot >> 8); ip[3] = (uint8_t)tot;
    ip[4] = (uint8_t)(ip_id >> 8); ip[5] = (uint8_t)ip_id;
    ip[6] = 0x40; ip[7] = 0x00; /* IP_DF */
    ip[8] = 64; ip[9] = 6;
    ip[10] = ip[11] = 0;
    put_le(ip + 12, src, 4); /* stored network-order word, copied as is */
    put_le(ip + 16, dst, 4);
    const uint16_t ic = orc_inet_csum(ip, 20, 0);
    ip[10] = (uint8_t)(ic >> 8); ip[11] = (uint8_t)ic;
    tcp[0] = (uint8_t)(sp >> 8); tcp[1] = (uint8_t)sp;
    tcp[2] = (uint8_t)(dp >> 8); tcp[3] = (uint8_t)dp;
    for (int k = 0; k < 4; k++) tcp[4 + k] = (uint8_t)(seq >> (24 - 8 * k));
    for (int k = 0; k < 4; k++) tcp[8 + k] = (uint8_t)(ack >> (24 - 8 * k));
    tcp[12] = 0x50; tcp[13] = flag;
    tcp[14] = 0xff; tcp[15] = 0xff;
    tcp[16] = tcp[17] = 0;
    tcp[18] = tcp[19] = 0;
    memcpy(tcp + 20, frame, (size_t)frame_len);
    /* pseudo-header: src, dst, zero, proto, TCP length */
    uint8_t ph[12];
    memcpy(ph, ip + 12, 8);
    ph[8] = 0; ph[9] = 6;
    ph[10] = (uint8_t)((20 + frame_len) >> 8); ph[11] = (uint8_t)(20 + frame_len);
    uint64_t s = 0;
    for (int i = 0; i < 12; i += 2) s += ((uint32_t)ph[i] << 8) | ph[i + 1];
    while (s >> 16) s = (s & 0xffff) + (s >> 16);
    const uint16_t tc = orc_inet_csum(tcp, (size_t)(20 + frame_len), (uint32_t)s);
    tcp[16] = (uint8_t)(tc >> 8); tcp[17] = (uint8_t)tc;
    return o + tot;
}

/* KeyGenerator.cpp:16-36 and KeyGenerator.h:21-23,51: INIT_KEY 0 | TYPE | (dp << 16) | sp. */
uint64_t orc_key_for_tcp(uint16_t sp, uint16_t dp) {
    return 0x10000000ull | ((uint64_t)dp << 16) | (uint64_t)sp;
}
uint64_t orc_key_for_udp(uint16_t sp, uint16_t dp) {
    return 0x20000000ull | ((uint64_t)dp << 16) | (uint64_t)sp;
}

/* splitmix64 (Steele, Lea, Flood 2014): output i of the generator seeded with `seed`. */
uint64_t orc_splitmix64_at(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void orc_fill_splitmix(uint8_t *dst, uint64_t nbytes, uint64_t seed) {
    uint64_t w = 0;
    for (; (w + 1) * 8 <= nbytes; w++) put_le(dst + 8 * w, orc_splitmix64_at(seed, w), 8);
    if (w * 8 < nbytes) {
        uint64_t v = orc_splitmix64_at(seed, w);
        for (uint64_t b = w * 8; b < nbytes; b++) dst[b] = (uint8_t)(v >> (8 * (b - w * 8)));
    }
}

/* ------------------------------------------------------------------------------------------------
 * Batch forms (SoA, same layout and semantics as include/rsk_codec.h).
 * --------------------------------------------------------------------------------------------- */
typedef struct {
    const uint8_t *key;
    size_t key_len;
    uint32_t lo, hi;
    const uint8_t *payload_arena;
    const uint64_t *pay_off;
    const uint16_t *pay_len;
    const uint8_t *cmd;
    const uint32_t *conv;
    const uint64_t *conn_key;
    const uint8_t *id;
    const uint8_t *id_uniform;
    uint8_t *frame_arena;
    const uint64_t *frame_off;
    int32_t *status;
} enc_job;

static void *enc_run(void *arg) {
    enc_job *j = (enc_job *)arg;
    for (uint32_t i = j->lo; i < j->hi; i++) {
        const uint8_t *id = j->id ? j->id + 8ull * i : j->id_uniform;
        j->status[i] = orc_rconn_output(j->key, j->key_len, j->payload_arena + j->pay_off[i],
                                        j->pay_len[i], j->cmd[i], id, j->conv[i], j->conn_key[i],
                                        j->frame_arena + j->frame_off[i]);
    }
    return NULL;
}

void orc_encode_batch(const uint8_t *key, size_t key_len, uint32_t n, const uint8_t *payload_arena,
                      const uint64_t *pay_off, const uint16_t *pay_len, const uint8_t *cmd,
                      const uint32_t *conv, const uint64_t *conn_key, const uint8_t *id,
                      const uint8_t id_uniform[8], uint8_t *frame_arena, const uint64_t *frame_off,
                      int32_t *status, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if ((uint32_t)nthreads > n) nthreads = n ? (int)n : 1;
    enc_job *jobs = (enc_job *)calloc((size_t)nthreads, sizeof *jobs);
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof *th);
    for (int t = 0; t < nthreads; t++) {
        enc_job j = {key, key_len, (uint32_t)((uint64_t)n * t / nthreads),
                     (uint32_t)((uint64_t)n * (t + 1) / nthreads), payload_arena, pay_off, pay_len,
                     cmd, conv, conn_key, id, id_uniform, frame_arena, frame_off, status};
        jobs[t] = j;
    }
    for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, enc_run, &jobs[t]);
    enc_run(&jobs[0]);
    for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
    free(jobs);
    free(th);
}

typedef struct {
    const uint8_t *key;
    size_t key_len;
    uint32_t lo, hi;
    const uint8_t *payload_arena;
    const uint64_t *pay_off;
    const uint16_t *pay_len;
    const uint8_t *cmd;
    const uint32_t *conv;
    const uint64_t *conn_key;
    const uint8_t *id;
    uint8_t *frame_arena;
    const uint64_t *frame_off;
    uint64_t good;
} bench_job;

static void *bench_run(void *arg) {
    bench_job *j = (bench_job *)arg;
    uint64_t good = 0;
    for (uint32_t i = j->lo; i < j->hi; i++) {
        uint8_t base[RSK_MAX_PKT_SIZE];
        memset(base, 0, sizeof base); /* RConn.cpp:100: char base[OM_MAX_PKT_SIZE] = {0} */
        int st = orc_rconn_output(j->key, j->key_len, j->payload_arena + j->pay_off[i], j->pay_len[i], j->cmd[i],
                                  j->id, j->conv[i], j->conn_key[i], base);
        if (st <= 0) continue;
        uint8_t *fr = j->frame_arena + j->frame_off[i];
        memcpy(fr, base, (size_t)st);
        orc_dec d;
        if (orc_rconn_onrecv(j->key, j->key_len, fr, st, 0, &d) == RSK_RECV_VALID) good++;
    }
    j->good = good;
    return NULL;
}

uint64_t orc_bench_codec(const uint8_t *key, size_t key_len, uint32_t n, const uint8_t *payload_arena,
                         const uint64_t *pay_off, const uint16_t *pay_len, const uint8_t *cmd,
                         const uint32_t *conv, const uint64_t *conn_key, const uint8_t id[8],
                         uint8_t *frame_arena, const uint64_t *frame_off, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if ((uint32_t)nthreads > n) nthreads = n ? (int)n : 1;
    bench_job *jobs = (bench_job *)calloc((size_t)nthreads, sizeof *jobs);
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof *th);
    for (int t = 0; t < nthreads; t++) {
        bench_job j = {key, key_len, (uint32_t)((uint64_t)n * t / nthreads), (uint32_t)((uint64_t)n * (t + 1) / nthreads),
                       payload_arena, pay_off, pay_len, cmd, conv, conn_key, id, frame_arena, frame_off, 0};
        jobs[t] = j;
    }
    for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, bench_run, &jobs[t]);
    bench_run(&jobs[0]);
    uint64_t good = jobs[0].good;
    for (int t = 1; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        good += jobs[t].good;
    }
    free(jobs);
    free(th);
    return good;
}

typedef struct {
    const uint8_t *key;
    size_t key_len;
    uint32_t lo, hi;
    const uint8_t *frame_arena;
    const uint64_t *frame_off;
    const uint16_t *frame_len;
    const uint8_t *is_tcp_close;
    uint8_t *hlen, *cmd, *id;
    uint32_t *conv;
    uint64_t *conn_key;
    uint16_t *pay_off, *pay_len;
    int8_t *status;
    uint32_t nvalid;
} dec_job;

static void dec_one(dec_job *j, uint32_t i, const orc_dec *d) {
    j->hlen[i] = d->hlen;
    j->cmd[i] = d->cmd;
    memcpy(j->id + 8ull * i, d->id, 8);
    j->conv[i] = d->conv;
    j->conn_key[i] = d->conn_key;
    j->pay_off[i] = d->pay_off;
    j->pay_len[i] = d->pay_len;
    j->status[i] = d->status;
}

static void *dec_run(void *arg) {
    dec_job *j = (dec_job *)arg;
    uint32_t nv = 0;
    for (uint32_t i = j->lo; i < j->hi; i++) {
        orc_dec d;
        orc_rconn_onrecv(j->key, j->key_len, j->frame_arena + j->frame_off[i], j->frame_len[i],
                         j->is_tcp_close ? j->is_tcp_close[i] : 0, &d);
        dec_one(j, i, &d);
        nv += d.status == RSK_RECV_VALID;
    }
    j->nvalid = nv;
    return NULL;
}

void orc_decode_batch(const uint8_t *key, size_t key_len, uint32_t n, const uint8_t *frame_arena,
                      const uint64_t *frame_off, const uint16_t *frame_len,
                      const uint8_t *is_tcp_close, uint8_t *hlen, uint8_t *cmd, uint8_t *id,
                      uint32_t *conv, uint64_t *conn_key, uint16_t *pay_off, uint16_t *pay_len,
                      int8_t *status, uint32_t *valid_idx, uint32_t *n_valid, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if ((uint32_t)nthreads > n) nthreads = n ? (int)n : 1;
    dec_job *jobs = (dec_job *)calloc((size_t)nthreads, sizeof *jobs);
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof *th);
    for (int t = 0; t < nthreads; t++) {
        dec_job j = {key, key_len, (uint32_t)((uint64_t)n * t / nthreads),
                     (uint32_t)((uint64_t)n * (t + 1) / nthreads), frame_arena, frame_off,
                     frame_len, is_tcp_close, hlen, cmd, id, conv, conn_key, pay_off, pay_len,
                     status, 0};
        jobs[t] = j;
    }
    for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, dec_run, &jobs[t]);
    dec_run(&jobs[0]);
    for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
    /* order-stable compaction of the VALID indices */
    uint32_t nv = 0;
    for (uint32_t i = 0; i < n; i++)
        if (status[i] == RSK_RECV_VALID) {
            if (valid_idx) valid_idx[nv] = i;
            nv++;
        }
    if (n_valid) *n_valid = nv;
    free(jobs);
    free(th);
}

void orc_parse_decode_batch(const uint8_t *key, size_t key_len, uint32_t n, const uint8_t *cap_arena,
                            const uint64_t *cap_off, const uint32_t *wire_len,
                            const uint32_t *cap_len, int datalink, int flags, uint32_t *src,
                            uint32_t *dst, uint16_t *sp, uint16_t *dp, uint32_t *seq, uint32_t *ack,
                            uint8_t *flag, int8_t *parse_status, uint16_t *cap_pay_off,
                            uint16_t *cap_pay_len, uint8_t *hlen, uint8_t *cmd, uint8_t *id,
                            uint32_t *conv, uint64_t *conn_key, uint16_t *pay_off,
                            uint16_t *pay_len, int8_t *status, uint32_t *valid_idx,
                            uint32_t *n_valid) {
    uint32_t nv = 0;
    for (uint32_t i = 0; i < n; i++) {
        orc_tcpinfo t;
        const uint8_t *pkt = cap_arena + cap_off[i];
        orc_rawinput(pkt, wire_len[i], cap_len[i], datalink, flags, &t);
        src[i] = t.src; dst[i] = t.dst; sp[i] = t.sp; dp[i] = t.dp;
        seq[i] = t.seq; ack[i] = t.ack; flag[i] = t.flag;
        parse_status[i] = t.parse_status;
        cap_pay_off[i] = t.parse_status == RSK_PARSE_DELIVER || t.parse_status == RSK_PARSE_SYN
                             ? t.cap_pay_off : 0;
        cap_pay_len[i] = t.cap_pay_len;
        orc_dec d;
        memset(&d, 0, sizeof d);
        d.status = RSK_RECV_DROP;
        if (t.parse_status == RSK_PARSE_DELIVER)
            orc_rconn_onrecv(key, key_len, pkt + t.cap_pay_off, t.cap_pay_len,
                             (t.flag & (RSK_TH_FIN | RSK_TH_RST)) != 0, &d);
        hlen[i] = d.hlen; cmd[i] = d.cmd; memcpy(id + 8ull * i, d.id, 8);
        conv[i] = d.conv; conn_key[i] = d.conn_key; pay_off[i] = d.pay_off; pay_len[i] = d.pay_len;
        status[i] = d.status;
        if (d.status == RSK_RECV_VALID) {
            if (valid_idx) valid_idx[nv] = i;
            nv++;
        }
    }
    if (n_valid) *n_valid = nv;
}

/* ---- receive demux ------------------------------------------------------------ */
typedef struct orc_dkey {
    uint32_t epoch, conv, dst, used;
    uint64_t id, key;
    uint32_t seg;
} orc_dkey;

static uint64_t orc_dkey_hash(const orc_dkey *k) {
    uint64_t h = k->epoch * 0x9E3779B97F4A7C15ull ^ k->id * 0xC2B2AE3D27D4EB4Full ^
                 k->key * 0x165667B19E3779F9ull ^ ((uint64_t)k->conv | (uint64_t)k->dst << 32) * 0xD6E8FEB86659FD93ull;
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    return h;
}

int orc_demux_batch(uint32_t n, const int8_t *status, const uint8_t *cmd, const uint8_t *id,
                    const uint32_t *conv, const uint64_t *conn_key, const uint32_t *dst,
                    uint32_t fields, uint32_t *perm, uint32_t *seg_off, uint32_t *seg_first,
                    uint32_t *n_seg, uint32_t *n_valid) {
    uint64_t cap = 2;
    while (cap < 2ull * n) cap <<= 1;
    orc_dkey *tab = (orc_dkey *)calloc(cap, sizeof(orc_dkey));
    uint32_t *seg_of = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
    uint32_t *cnt = (uint32_t *)calloc(n + 1, sizeof(uint32_t));
    if (!tab || !seg_of || !cnt) {
        free(tab); free(seg_of); free(cnt);
        return -12;
    }
    const int barrier = (fields & RSK_DEMUX_CMD_BARRIER) != 0;
    const int gbarrier = (fields & RSK_DEMUX_GROUP_BARRIER) != 0;
    /* GROUP_BARRIER: the epoch of a DATA packet counts the control packets of its own IdBuf before
       it (per-IdBuf counters in a second table, `epoch` = the count, `key` = the IdBuf) */
    orc_dkey *gtab = gbarrier ? (orc_dkey *)calloc(cap, sizeof(orc_dkey)) : NULL;
    if (gbarrier && !gtab) {
        free(tab); free(seg_of); free(cnt);
        return -12;
    }
    uint32_t epoch = 0, S = 0, nv = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (status[i] != RSK_RECV_VALID) continue;
        nv++;
        orc_dkey *grp = NULL;
        if (gbarrier) {
            uint64_t gid;
            memcpy(&gid, id + 8ull * i, 8);
            orc_dkey gk;
            memset(&gk, 0, sizeof gk);
            gk.id = gid;
            uint64_t h = orc_dkey_hash(&gk) & (cap - 1);
            while (gtab[h].used && gtab[h].id != gid) h = (h + 1) & (cap - 1);
            grp = &gtab[h];
            grp->used = 1;
            grp->id = gid;
        }
        if ((barrier || gbarrier) && cmd[i] != RSK_CMD_DATA) {  /* singleton segment, then a new epoch */
            seg_first[S] = i;
            seg_of[i] = S++;
            if (grp) grp->epoch++;
            else epoch++;
            continue;
        }
        orc_dkey k;
        memset(&k, 0, sizeof k);
        k.epoch = grp ? grp->epoch : epoch;
        if (fields & RSK_DEMUX_ID) memcpy(&k.id, id + 8ull * i, 8);
        if (fields & RSK_DEMUX_CONN_KEY) k.key = conn_key[i];
        if (fields & RSK_DEMUX_CONV) k.conv = conv[i];
        if (fields & RSK_DEMUX_DST) k.dst = dst[i];
        uint64_t h = orc_dkey_hash(&k) & (cap - 1);
        for (;;) {
            orc_dkey *t = &tab[h];
            if (!t->used) {  /* first occurrence: the reference would create the conn here */
                *t = k;
                t->used = 1;
                t->seg = S;
                seg_first[S] = i;
                S++;
                break;
            }
            if (t->epoch == k.epoch && t->id == k.id && t->key == k.key && t->conv == k.conv && t->dst == k.dst)
                break;
            h = (h + 1) & (cap - 1);
        }
        seg_of[i] = tab[h].seg;
    }
    for (uint32_t i = 0; i < n; i++)
        if (status[i] == RSK_RECV_VALID) cnt[seg_of[i]]++;
    uint32_t run = 0;
    for (uint32_t s = 0; s < S; s++) {
        seg_off[s] = run;
        run += cnt[s];
        cnt[s] = seg_off[s];
    }
    seg_off[S] = run;
    for (uint32_t i = 0; i < n; i++)
        if (status[i] == RSK_RECV_VALID) perm[cnt[seg_of[i]]++] = i;
    *n_seg = S;
    *n_valid = nv;
    free(tab); free(gtab); free(seg_of); free(cnt);
    return 0;
}

/* ---- capture filter ----------------------------------------------------------- */
/* Each primitive returns 1 / 0, or -1 when a byte it reads lies past cap_len (the BPF program then
 * returns 0 for the packet: libpcap bpf_filter's out-of-bounds load). */
typedef struct orc_fpkt {
    const uint8_t *p;
    uint32_t cl;
    uint32_t L;   /* link header bytes: 14 (EN10MB) or 4 (NULL) */
    int datalink;
} orc_fpkt;

static int orc_f_link(const orc_fpkt *k) {  /* 4, 6, 0 or -1 */
    if (k->datalink == RSK_DLT_EN10MB) {
        if (k->cl < 14) return -1;
        const unsigned et = ((unsigned)k->p[12] << 8) | k->p[13];
        return et == 0x0800 ? 4 : et == 0x86dd ? 6 : 0;
    }
    if (k->cl < 4) return -1;
    const uint32_t fam = (uint32_t)k->p[0] | (uint32_t)k->p[1] << 8 | (uint32_t)k->p[2] << 16 | (uint32_t)k->p[3] << 24;
    return fam == 2 ? 4 : (fam == 24 || fam == 28 || fam == 30) ? 6 : 0;
}

static int orc_f_tcp(const orc_fpkt *k) {  /* "tcp" */
    const int lt = orc_f_link(k);
    if (lt < 0) return -1;
    if (lt == 4) {
        if (k->cl < k->L + 10) return -1;
        return k->p[k->L + 9] == 6;
    }
    if (lt == 6) {
        if (k->cl < k->L + 7) return -1;
        const uint8_t nxt = k->p[k->L + 6];
        if (nxt == 6) return 1;
        if (nxt != 44) return 0;
        if (k->cl < k->L + 41) return -1;
        return k->p[k->L + 40] == 6;
    }
    return 0;
}

static int orc_f_addr(const orc_fpkt *k, uint32_t off, uint32_t val) {  /* "ip src|dst A" */
    const int lt = orc_f_link(k);
    if (lt < 0) return -1;
    if (lt != 4) return 0;
    if (k->cl < k->L + off + 4) return -1;
    const uint8_t *q = k->p + k->L + off;
    return ((uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 | (uint32_t)q[3] << 24) == val;
}

static int orc_is_tus(uint8_t pr) { return pr == 6 || pr == 17 || pr == 132; }

/* "( [src|dst] port p or ... [src|dst] portrange a-b ... )"; dir = 0 (src) or 2 (dst) */
static int orc_f_ports(const orc_fpkt *k, const rsk_port_list *pl, uint32_t dir) {
    if (pl->n_single == 0 && pl->n_range == 0) return 1;  /* no clause */
    const int lt = orc_f_link(k);
    if (lt < 0) return -1;
    int have = 0;
    unsigned port = 0;
    if (lt == 4) {
        if (k->cl < k->L + 10) return -1;
        if (orc_is_tus(k->p[k->L + 9])) {
            const unsigned frag = ((unsigned)(k->p[k->L + 6] & 0x1f) << 8) | k->p[k->L + 7];
            if (frag == 0) {
                const uint32_t th = k->L + 4u * (k->p[k->L] & 15u);
                if (k->cl < th + dir + 2) return -1;
                port = ((unsigned)k->p[th + dir] << 8) | k->p[th + dir + 1];
                have = 1;
            }
        }
    } else if (lt == 6) {
        if (k->cl < k->L + 7) return -1;
        if (orc_is_tus(k->p[k->L + 6])) {
            const uint32_t th = k->L + 40;
            if (k->cl < th + dir + 2) return -1;
            port = ((unsigned)k->p[th + dir] << 8) | k->p[th + dir + 1];
            have = 1;
        }
    }
    if (!have) return 0;
    for (unsigned q = 0; q < pl->n_single; q++)
        if (port == pl->single[q]) return 1;
    for (unsigned q = 0; q < pl->n_range; q++)
        if (port >= pl->range[q][0] && port <= pl->range[q][1]) return 1;
    return 0;
}

static int orc_f_syn(const orc_fpkt *k, int want_set) {  /* tcp[tcpflags] & tcp-syn != 0 / == 0 */
    const int lt = orc_f_link(k);
    if (lt < 0) return -1;
    if (lt != 4) return 0;
    if (k->cl < k->L + 10) return -1;
    if (k->p[k->L + 9] != 6) return 0;
    const unsigned frag = ((unsigned)(k->p[k->L + 6] & 0x1f) << 8) | k->p[k->L + 7];
    if (frag != 0) return 0;
    const uint32_t th = k->L + 4u * (k->p[k->L] & 15u);
    if (k->cl < th + 14) return -1;
    const int syn = (k->p[th + 13] & 0x02) != 0;
    return want_set ? syn : !syn;
}

/* F (primed = 0) or F' ("dst" -> "src", primed = 1), left to right with short-circuit */
static int orc_f_main(const orc_fpkt *k, const rsk_capture_filter *f, int primed) {
    int r = orc_f_tcp(k);
    if (r != 1) return r;
    if (f->has_src_ip && (r = orc_f_addr(k, 12, f->src_ip)) != 1) return r;
    if (f->has_dst_ip && (r = orc_f_addr(k, primed ? 12 : 16, f->dst_ip)) != 1) return r;
    if ((r = orc_f_ports(k, &f->src_ports, 0)) != 1) return r;
    return orc_f_ports(k, &f->dst_ports, primed ? 0 : 2);
}

int orc_capture_filter(const uint8_t *pkt, uint32_t cap_len, int datalink, const rsk_capture_filter *f) {
    orc_fpkt k = {pkt, cap_len, datalink == RSK_DLT_EN10MB ? 14u : 4u, datalink};
    int r;
    if (!f->is_server) {
        r = orc_f_main(&k, f, 0);
    } else {  /* ((syn) and F') or (F and (no syn)) */
        r = orc_f_syn(&k, 1);
        if (r == 1) r = orc_f_main(&k, f, 1);
        if (r == 0) {
            r = orc_f_main(&k, f, 0);
            if (r == 1) r = orc_f_syn(&k, 0);
        }
    }
    return r == 1;
}

/* BuildFilterStr (cap/cap_util.cpp:67-144) */
static size_t orc_put(char *buf, size_t cap, size_t at, const char *s) {
    size_t n = strlen(s);
    if (at + n < cap) memcpy(buf + at, s, n + 1);
    return at + n;
}

static size_t orc_put_ports(char *buf, size_t cap, size_t at, const rsk_port_list *pl, const char *dir) {
    if (pl->n_single == 0 && pl->n_range == 0) return at;
    char tmp[64];
    at = orc_put(buf, cap, at, " and ");
    at = orc_put(buf, cap, at, "(");
    int first = 1;  /* the reference deletes the first "or" (cap_util.cpp:116-121) */
    for (unsigned q = 0; q < pl->n_single; q++, first = 0) {
        snprintf(tmp, sizeof tmp, " %s %s port %u", first ? "" : "or", dir, (unsigned)pl->single[q]);
        at = orc_put(buf, cap, at, tmp);
    }
    for (unsigned q = 0; q < pl->n_range; q++, first = 0) {
        snprintf(tmp, sizeof tmp, " %s %s portrange %u-%u", first ? "" : "or", dir, (unsigned)pl->range[q][0],
                 (unsigned)pl->range[q][1]);
        at = orc_put(buf, cap, at, tmp);
    }
    return orc_put(buf, cap, at, " )");
}

static size_t orc_base_str(const rsk_capture_filter *f, char *buf, size_t cap) {
    char ip[40];
    size_t at = orc_put(buf, cap, 0, "tcp");
    if (f->has_src_ip) {
        snprintf(ip, sizeof ip, " and  (ip src %u.%u.%u.%u)", f->src_ip & 255, (f->src_ip >> 8) & 255,
                 (f->src_ip >> 16) & 255, f->src_ip >> 24);
        at = orc_put(buf, cap, at, ip);
    }
    if (f->has_dst_ip) {
        snprintf(ip, sizeof ip, " and  (ip dst %u.%u.%u.%u)", f->dst_ip & 255, (f->dst_ip >> 8) & 255,
                 (f->dst_ip >> 16) & 255, f->dst_ip >> 24);
        at = orc_put(buf, cap, at, ip);
    }
    at = orc_put_ports(buf, cap, at, &f->src_ports, "src");
    return orc_put_ports(buf, cap, at, &f->dst_ports, "dst");
}

int orc_filter_str(const rsk_capture_filter *f, char *buf, size_t buf_len) {
    char base[8192];
    const size_t bl = orc_base_str(f, base, sizeof base);
    if (bl >= sizeof base) return -1;
    if (!f->is_server) {
        if (bl + 1 > buf_len) return -1;
        memcpy(buf, base, bl + 1);
        return (int)bl;
    }
    char primed[8192];
    size_t o = 0;
    for (size_t q = 0; q < bl;) {  /* every "dst" -> "src" */
        if (q + 3 <= bl && memcmp(base + q, "dst", 3) == 0) {
            memcpy(primed + o, "src", 3);
            o += 3;
            q += 3;
        } else {
            primed[o++] = base[q++];
        }
    }
    primed[o] = 0;
    size_t at = orc_put(buf, buf_len, 0, "((tcp[tcpflags] & tcp-syn != 0) and ");
    at = orc_put(buf, buf_len, at, primed);
    at = orc_put(buf, buf_len, at, ") or (");
    at = orc_put(buf, buf_len, at, base);
    at = orc_put(buf, buf_len, at, "and (tcp[tcpflags] & (tcp-syn) == 0))");
    if (at + 1 > buf_len) return -1;
    return (int)at;
}

/* ---- fake-TCP connection state (restated from the reference, one packet at a time) ---------- */
/* FakeTcp::Output (conn/FakeTcp.cpp:43-49): after INetConn::Output returns n >= 0 (the frame was
 * sent), mInfo.UpdateSeq(nread + mInfo.seq + RConn::HEAD_SIZE); the packet carried the seq before
 * the update.  RawTcp::Output (conn/RawTcp.cpp:111-121): SendRawTcp(..., mIpId++, ...) per sent
 * packet.  Packets RConn::Output did not frame (status <= 0) are not sent through RawTcp. */
void orc_tcp_send_seq_batch(uint32_t n, const uint32_t *conn, const int32_t *status, uint32_t n_conn,
                            uint32_t *conn_seq, uint16_t *ip_id_next, uint32_t *seq, uint16_t *ip_id) {
    for (uint32_t i = 0; i < n; ++i) {
        seq[i] = 0;
        ip_id[i] = 0;
        if (status[i] <= 0) continue;
        ip_id[i] = (*ip_id_next)++;
        if (conn[i] >= n_conn) continue;
        seq[i] = conn_seq[conn[i]];
        conn_seq[conn[i]] = conn_seq[conn[i]] + (uint32_t)status[i];
    }
}

/* FakeTcp::OnRecv (conn/FakeTcp.cpp:52-66): if (n >= 0) { if (mInfo.ack < info->seq) UpdateAck(info->seq); } */
void orc_tcp_recv_ack_batch(uint32_t n, const uint32_t *conn, const uint8_t *delivered, const uint32_t *seq,
                            uint32_t n_conn, uint32_t *conn_ack) {
    for (uint32_t i = 0; i < n; ++i) {
        if (!delivered[i] || conn[i] >= n_conn) continue;
        if (conn_ack[conn[i]] < seq[i]) conn_ack[conn[i]] = seq[i];
    }
}
