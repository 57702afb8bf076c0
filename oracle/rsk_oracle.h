/*
 * rsk_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of rsock's framing-codec path (EncHead + MD5 hash-tag, RConn send/recv framing,
 * RawTcp eth/IPv4/TCP receive parse).  This is the parity checker for the HIP path and the "port"
 * CPU baseline.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it;
 * the product library (rsock_amd/librsk.so) never links or calls it.
 *
 * Pinning: the codec functions are checked bit-for-bit against oracle/_ref (the reference's own
 * md5.c / enc.c / rhash.cpp / EncHead.cpp / KeyGenerator.cpp / TcpInfo.cpp / ConnInfo.cpp compiled
 * from /root/reference by oracle/Makefile.ref) through tests/golden fixtures, against the RFC 1321
 * MD5 test suite and against the SURVEY's live-capture known answers.  The pcap parse (RawInput)
 * cannot be compiled from the reference here (it needs libnet/libpcap, which exist only as the
 * reference's prebuilt .a files); it is pinned by the SURVEY's verified live parse vector and by
 * hand-built packets — see DESIGN.md §Parity.
 *
 * Semantics are identical to include/rsk_codec.h; status codes are shared.
 */
#ifndef RSK_ORACLE_H
#define RSK_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/rsk_codec.h"

#ifdef __cplusplus
extern "C" {
#endif

/* RFC 1321 MD5 of msg[0..len) (thirdparty/md5.c:105-294). */
void orc_md5(const uint8_t *msg, size_t len, uint8_t digest[16]);

/* tag = MD5(key || data0)[8..15]  (util/rhash.cpp:20-41) */
void orc_compute_hash(uint8_t tag[8], const uint8_t *key, size_t key_len, uint8_t data0);
/* util/rhash.cpp:71-92: 0 when data == NULL or data_len <= 0 */
int orc_hash_equal(const uint8_t tag[8], const uint8_t *key, size_t key_len, const uint8_t *data,
                   int data_len);

/* EncHead::Enc2Buf (bean/EncHead.cpp:9-24): returns 23 (bytes written) or -1 */
int orc_enchead_encode(uint8_t *p, int buf_len, uint8_t cmd, const uint8_t id[8], uint32_t conv,
                       uint64_t conn_key);
/* EncHead::DecodeBuf (bean/EncHead.cpp:39-55): returns len (payload offset from p) or -1 */
int orc_enchead_decode(const uint8_t *p, int buf_len, uint8_t *len, uint8_t *cmd, uint8_t id[8],
                       uint32_t *conv, uint64_t *conn_key);

/* RConn::Output framing (conn/RConn.cpp:87-105): frame must have room for 31+P bytes.
 * Returns 31+P, -1 (oversize) or 0 (P == 0: reset). */
int orc_rconn_output(const uint8_t *key, size_t key_len, const uint8_t *payload, int nread,
                     uint8_t cmd, const uint8_t id[8], uint32_t conv, uint64_t conn_key,
                     uint8_t *frame);

/* RConn::OnRecv (conn/RConn.cpp:64-85).  Returns RSK_RECV_*; fields zero unless VALID. */
typedef struct orc_dec {
    uint8_t hlen, cmd, id[8];
    uint32_t conv;
    uint64_t conn_key;
    uint16_t pay_off, pay_len;
    int8_t status;
} orc_dec;
int orc_rconn_onrecv(const uint8_t *key, size_t key_len, const uint8_t *frame, int nread,
                     int is_tcp_close, orc_dec *out);

/* RawTcp::RawInput + cap2uv size check (conn/RawTcp.cpp:138-244). */
typedef struct orc_tcpinfo {
    uint32_t src, dst;
    uint16_t sp, dp;
    uint32_t seq, ack;
    uint8_t flag;
    int8_t parse_status;
    uint16_t cap_pay_off, cap_pay_len;
} orc_tcpinfo;
int orc_rawinput(const uint8_t *pkt, uint32_t wire_len, uint32_t cap_len, int datalink, int flags,
                 orc_tcpinfo *out);

/* TcpInfo::Encode / Decode (bean/TcpInfo.cpp:20-45, bean/ConnInfo.cpp:12-32): 21-byte record. */
int orc_tcpinfo_encode(const orc_tcpinfo *t, uint8_t rec[21]);
int orc_tcpinfo_decode(const uint8_t *rec, int len, orc_tcpinfo *t);
/* RawTcp::syncInput (conn/RawTcp.cpp:262-276) -> RConn::OnRecv on one hand-off record (21-B TcpInfo
 * + frame, nread bytes).  Returns the parse status (DELIVER when Decode succeeded). */
int orc_syncinput(const uint8_t *key, size_t key_len, const uint8_t *rec, int nread, orc_tcpinfo *t,
                  orc_dec *d);

/* RawTcp::SendRawTcp (conn/RawTcp.cpp:280-341) through libnet 1.1.6: the wire packet for one frame.
 * [eth 14 if eth != NULL] | IPv4 20 (v4, IHL 5, tos 0, tot_len, id, DF, ttl 64, proto 6, checksum,
 * src, dst) | TCP 20 (sp, dp, seq, ack, doff 5, flags, win 65535, checksum, urg 0) | frame.
 * src/dst are the stored network-byte-order words (TcpInfo::src/dst); sp, dp, seq, ack host order.
 * Returns the wire length. */
int orc_build_wire(const uint8_t *frame, int frame_len, uint32_t src, uint32_t dst, uint16_t sp,
                   uint16_t dp, uint32_t seq, uint32_t ack, uint8_t flag, uint16_t ip_id,
                   const uint8_t *eth, uint8_t *wire);
/* RFC 1071 Internet checksum of bytes (as stored on the wire), returned in network byte order
 * value (i.e. the 16-bit value whose big-endian bytes go into the header). */
uint16_t orc_inet_csum(const uint8_t *p, size_t n, uint32_t init);

/* Receive demux (semantics in include/rsk_codec.h rsk_demux_batch): the reference's
 * per-packet conn lookups (INetGroup.cpp:57-83 by connKey, IAppGroup.cpp:76-96 by cmd,
 * ServerGroup.cpp:44-60 by IdBuf, SubGroup.cpp:31-50 by (dst, conv), ClientGroup.cpp:66-80 by conv)
 * restated as a sequential walk: each VALID packet looks its key up in a map (new key -> next
 * segment id), control packets (cmd != 0) under RSK_DEMUX_CMD_BARRIER open a new epoch, under
 * RSK_DEMUX_GROUP_BARRIER a new epoch of their own IdBuf only (ServerGroup.cpp:44-60 hands a packet
 * to its IdBuf's SubGroup alone).  Pointers for unselected fields may be NULL.  Returns 0, or -12 on
 * allocation failure. */
int orc_demux_batch(uint32_t n, const int8_t *status, const uint8_t *cmd, const uint8_t *id,
                    const uint32_t *conv, const uint64_t *conn_key, const uint32_t *dst,
                    uint32_t fields, uint32_t *perm, uint32_t *seg_off, uint32_t *seg_first,
                    uint32_t *n_seg, uint32_t *n_valid);

/* Capture filter (semantics in include/rsk_codec.h rsk_capture_filter_batch): the
 * pcap filter BuildFilterStr (cap/cap_util.cpp:67-144) builds, evaluated on one captured packet
 * with libpcap's meaning of each primitive.  Returns 1 (match) or 0. */
int orc_capture_filter(const uint8_t *pkt, uint32_t cap_len, int datalink, const rsk_capture_filter *f);
/* BuildFilterStr("tcp", srcIp, dstIp, srcPorts, dstPorts, isServer) for this filter. */
int orc_filter_str(const rsk_capture_filter *f, char *buf, size_t buf_len);

/* KeyGenerator::KeyForTcp / KeyForUdp (src/util/KeyGenerator.cpp:16-36) */
/* FakeTcp::Output seq advance + RawTcp::Output mIpId++ / FakeTcp::OnRecv ack (sequential loops) */
void orc_tcp_send_seq_batch(uint32_t n, const uint32_t *conn, const int32_t *status, uint32_t n_conn,
                            uint32_t *conn_seq, uint16_t *ip_id_next, uint32_t *seq, uint16_t *ip_id);
void orc_tcp_recv_ack_batch(uint32_t n, const uint32_t *conn, const uint8_t *delivered, const uint32_t *seq,
                            uint32_t n_conn, uint32_t *conn_ack);

uint64_t orc_key_for_tcp(uint16_t sp, uint16_t dp);
uint64_t orc_key_for_udp(uint16_t sp, uint16_t dp);

/* i-th output of a splitmix64 generator seeded with `seed` (synthetic workloads). */
uint64_t orc_splitmix64_at(uint64_t seed, uint64_t i);
void orc_fill_splitmix(uint8_t *dst, uint64_t nbytes, uint64_t seed);

/* ---- batch forms over the same SoA layout as include/rsk_codec.h (host memory) ------------- */
/* nthreads <= 1 runs on the calling thread; otherwise contiguous shards on pthreads. */
void orc_encode_batch(const uint8_t *key, size_t key_len, uint32_t n, const uint8_t *payload_arena,
                      const uint64_t *pay_off, const uint16_t *pay_len, const uint8_t *cmd,
                      const uint32_t *conv, const uint64_t *conn_key, const uint8_t *id,
                      const uint8_t id_uniform[8], uint8_t *frame_arena, const uint64_t *frame_off,
                      int32_t *status, int nthreads);

/* CPU baseline (bench.py cpu_baseline, kind "port"): per packet i in [0, n), RConn::Output framing
 * into a zeroed 1500-B stack buffer (RConn.cpp:100-104), the frame stored to frame_arena +
 * frame_off[i], then RConn::OnRecv (DecodeBuf + hash_equal) on the stored frame.  Contiguous shards
 * over nthreads pthreads; returns the number of verified packets. */
uint64_t orc_bench_codec(const uint8_t *key, size_t key_len, uint32_t n, const uint8_t *payload_arena,
                         const uint64_t *pay_off, const uint16_t *pay_len, const uint8_t *cmd,
                         const uint32_t *conv, const uint64_t *conn_key, const uint8_t id[8],
                         uint8_t *frame_arena, const uint64_t *frame_off, int nthreads);

void orc_decode_batch(const uint8_t *key, size_t key_len, uint32_t n, const uint8_t *frame_arena,
                      const uint64_t *frame_off, const uint16_t *frame_len,
                      const uint8_t *is_tcp_close, uint8_t *hlen, uint8_t *cmd, uint8_t *id,
                      uint32_t *conv, uint64_t *conn_key, uint16_t *pay_off, uint16_t *pay_len,
                      int8_t *status, uint32_t *valid_idx, uint32_t *n_valid, int nthreads);

void orc_parse_decode_batch(const uint8_t *key, size_t key_len, uint32_t n, const uint8_t *cap_arena,
                            const uint64_t *cap_off, const uint32_t *wire_len,
                            const uint32_t *cap_len, int datalink, int flags, uint32_t *src,
                            uint32_t *dst, uint16_t *sp, uint16_t *dp, uint32_t *seq, uint32_t *ack,
                            uint8_t *flag, int8_t *parse_status, uint16_t *cap_pay_off,
                            uint16_t *cap_pay_len, uint8_t *hlen, uint8_t *cmd, uint8_t *id,
                            uint32_t *conv, uint64_t *conn_key, uint16_t *pay_off,
                            uint16_t *pay_len, int8_t *status, uint32_t *valid_idx,
                            uint32_t *n_valid);

#ifdef __cplusplus
}
#endif
#endif
